variable "name" {
  description = "Human readable name used as prefix to generated names."
}

variable "rancher_api_url" {
}

variable "rancher_access_key" {
}

variable "rancher_secret_key" {
  sensitive   = true
}

variable "k8s_version" {
  default     = "v1.9.5-rancher1-1"
}

variable "k8s_network_provider" {
  default     = "flannel"
}

variable "rancher_registry" {
  default     = ""
}

variable "rancher_registry_username" {
  default     = ""
}

variable "rancher_registry_password" {
  default     = ""
  sensitive   = true
}

variable "k8s_registry" {
  default     = ""
}

variable "k8s_registry_username" {
  default     = ""
}

variable "k8s_registry_password" {
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

variable "aws_public_key_path" {
  default     = "~/.ssh/id_rsa.pub"
}

variable "aws_key_name" {
}
