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

variable "gcp_path_to_credentials" {
}

variable "gcp_compute_region" {
}

variable "gcp_project_id" {
}
