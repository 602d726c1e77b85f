variable "name" {
  description = "Name."
  type        = string
}

variable "rancher_api_url" {
  description = "Base URL of the Rancher server (the cluster manager's rancher_url output)."
  type        = string
}

variable "rancher_access_key" {
  description = "Rancher API access key (cluster manager output)."
  type        = string
}

variable "rancher_secret_key" {
  description = "Rancher API secret key (cluster manager output)."
  type        = string
  sensitive   = true
}

variable "rancher_cluster_id" {
  description = "Rancher cluster id."
  type        = string
}

variable "device_plugin_image" {
  description = "Device plugin image."
  type        = string
  default     = "rocm/k8s-device-plugin:1.31.0.6"
}

variable "node_labeller_image" {
  description = "Node labeller image."
  type        = string
  default     = "rocm/k8s-device-plugin:labeller-1.31.0.6"
}

variable "rccl_probe_image" {
  description = "Rccl probe image."
  type        = string
  default     = ""
}

variable "rccl_gate" {
  description = "Rccl gate."
  type        = string
  default     = "true"
}
