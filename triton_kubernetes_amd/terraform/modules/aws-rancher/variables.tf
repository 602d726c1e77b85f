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

variable "aws_access_key" {
}

variable "aws_secret_key" {
  sensitive   = true
}

variable "aws_region" {
}

variable "aws_vpc_cidr" {
  default     = "10.0.0.0/16"
}

variable "aws_subnet_cidr" {
  default     = "10.0.2.0/24"
}

variable "aws_ami_id" {
}

variable "aws_instance_type" {
  default     = "t3.medium"
}

variable "aws_key_name" {
}

variable "aws_public_key_path" {
  default     = "~/.ssh/id_rsa.pub"
}

variable "aws_private_key_path" {
  default     = "~/.ssh/id_rsa"
}

variable "aws_ssh_user" {
  default     = "ubuntu"
}
