variable "name" {
  description = "Human readable name used as prefix to generated names."
  type        = string
}

variable "rancher_admin_password" {
  description = "The Rancher admin password"
  type        = string
  sensitive   = true
}

variable "docker_engine_install_url" {
  description = "The URL to the shell script to install the docker engine."
  type        = string
  default     = "https://releases.rancher.com/install-docker/24.0.sh"
}

variable "rancher_server_image" {
  description = "The Rancher Server image to use."
  type        = string
  default     = "rancher/rancher:v2.8.5"
}

variable "rancher_agent_image" {
  description = "The Rancher Agent image to use."
  type        = string
  default     = "rancher/rancher-agent:v2.8.5"
}

variable "rancher_registry" {
  description = "The docker registry to use for rancher server and agent images"
  type        = string
  default     = ""
}

variable "rancher_registry_username" {
  description = "The username to login as."
  type        = string
  default     = ""
}

variable "rancher_registry_password" {
  description = "The password to use."
  type        = string
  default     = ""
  sensitive   = true
}

variable "ssh_user" {
  description = "SSH login user."
  type        = string
  default     = "ubuntu"
}

variable "host" {
  description = "Address of the machine reached over SSH."
  type        = string
}

variable "bastion_host" {
  description = "Optional SSH jump host (empty: direct)."
  type        = string
  default     = ""
}

variable "key_path" {
  description = "Private key used for SSH."
  type        = string
  default     = "~/.ssh/id_rsa"
}
