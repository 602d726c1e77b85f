variable "name" {
  description = "Human readable name used as prefix to generated names."
}

variable "rancher_admin_password" {
  description = "The Rancher admin password"
  sensitive   = true
}

variable "docker_engine_install_url" {
  description = "The URL to the shell script to install the docker engine."
  default     = "https://releases.rancher.com/install-docker/24.0.sh"
}

variable "rancher_server_image" {
  description = "The Rancher Server image to use."
  default     = "rancher/rancher:v2.8.5"
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
  default     = "n1-standard-2"
}

variable "gcp_instance_zone" {
}

variable "gcp_image" {
  default     = "ubuntu-os-cloud/ubuntu-2204-lts"
}

variable "gcp_ssh_user" {
  default     = "ubuntu"
}

variable "gcp_public_key_path" {
  default     = "~/.ssh/id_rsa.pub"
}

variable "gcp_private_key_path" {
  default     = "~/.ssh/id_rsa"
}
