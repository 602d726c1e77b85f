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

variable "vsphere_user" {
}

variable "vsphere_password" {
  sensitive   = true
}

variable "vsphere_server" {
}

variable "vsphere_datacenter_name" {
}

variable "vsphere_datastore_name" {
}

variable "vsphere_resource_pool_name" {
}

variable "vsphere_network_name" {
}

variable "vsphere_template_name" {
}

variable "ssh_user" {
  default     = "ubuntu"
}

variable "key_path" {
  default     = "~/.ssh/id_rsa"
}

variable "vsphere_num_cpus" {
  default     = "2"
}

variable "vsphere_memory_mb" {
  default     = "2048"
}
