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

variable "triton_account" {
}

variable "triton_key_path" {
}

variable "triton_key_id" {
}

variable "triton_url" {
  default     = "https://us-east-1.api.joyent.com"
}

variable "triton_network_names" {
  type        = list(string)
  default     = [
  "Joyent-SDC-Public"
]
}

variable "triton_image_name" {
  default     = "ubuntu-certified-22.04"
}

variable "triton_image_version" {
}

variable "triton_ssh_user" {
  default     = "ubuntu"
}

variable "master_triton_machine_package" {
  default     = "k4-highcpu-kvm-3.75G"
}
