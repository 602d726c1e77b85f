variable "name" {
}

variable "rancher_api_url" {
}

variable "rancher_access_key" {
}

variable "rancher_secret_key" {
  sensitive   = true
}

variable "rancher_cluster_id" {
}

variable "device_plugin_image" {
  default     = "rocm/k8s-device-plugin:latest"
}

variable "node_labeller_image" {
  default     = "rocm/k8s-device-plugin:labeller-latest"
}

variable "rccl_probe_image" {
  default     = ""
}

variable "rccl_gate" {
  default     = "true"
}
