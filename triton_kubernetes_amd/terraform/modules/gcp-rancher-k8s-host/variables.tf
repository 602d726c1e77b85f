variable "hostname" {
}

variable "rancher_api_url" {
}

variable "rancher_cluster_registration_token" {
  sensitive   = true
}

variable "rancher_cluster_ca_checksum" {
}

variable "rancher_host_labels" {
  type        = map(string)
  description = "A single-key map: {worker|etcd|control = \"true\"}"
}

variable "docker_engine_install_url" {
  description = "The URL to the shell script to install the docker engine."
  default     = "https://releases.rancher.com/install-docker/24.0.sh"
}

variable "rancher_agent_image" {
  description = "The Rancher Agent image to use."
  default     = "rancher/rancher-agent:v2.8.5"
}

variable "rancher_registry" {
  description = "The docker registry to use for rancher server and agent images"
  default     = ""
}

variable "rancher_registry_username" {
  description = "The username to login as."
  default     = ""
}

variable "rancher_registry_password" {
  description = "The password to use."
  default     = ""
  sensitive   = true
}

variable "gcp_path_to_credentials" {
}

variable "gcp_compute_region" {
}

variable "gcp_project_id" {
}

variable "gcp_machine_type" {
  default     = "n1-standard-4"
}

variable "gcp_instance_zone" {
}

variable "gcp_image" {
  default     = "ubuntu-os-cloud/ubuntu-2204-lts"
}

variable "gcp_compute_network_name" {
}

variable "gcp_compute_firewall_host_tag" {
}

variable "gcp_disk_type" {
  default     = ""
}

variable "gcp_disk_size" {
  default     = ""
}

variable "gcp_disk_mount_path" {
  default     = ""
}
