variable "name" {
  description = "Name."
  type        = string
}

variable "rancher_api_url" {
  description = "Base URL of the Rancher server (the cluster manager's rancher_url output)."
  type        = string

  validation {
    condition     = length(regexall("^https?://[][A-Za-z0-9._:-]+(/[A-Za-z0-9._/-]*)?$", var.rancher_api_url)) > 0
    error_message = "rancher_api_url must be an http(s) URL."
  }
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

variable "tk_rancher_ca" {
  description = "PEM CA bundle the Rancher server is verified against (the manager's pinned CA, rendered by the CLI; empty: a publicly trusted certificate)"
  type        = string
  default     = ""
}

variable "device_plugin_image" {
  description = "Device plugin image."
  type        = string
  default     = "rocm/k8s-device-plugin:1.31.0.6"
}

variable "node_labeller_image" {
  description = "ROCm node labeller image, opt-in (e.g. rocm/k8s-device-plugin:labeller-1.31.0.6); it writes only keys the bootstrap labeller does not. Empty: no labeller DaemonSet or its RBAC."
  type        = string
  default     = ""
}

variable "rccl_probe_image" {
  description = "Image of the node-level rccl-ready Job (runs the node's installed tools)."
  type        = string
  default     = "ubuntu:22.04"
}

variable "webhook_image" {
  description = "Python image running the RCCL-env injector webhook."
  type        = string
  default     = "python:3.11-slim"
}

variable "rccl_gate" {
  description = "Apply the rccl-ready Job (true/false)."
  type        = string
  default     = "true"
}

variable "rccl_env_injector" {
  description = "Inject the rccl-env values into every pod requesting amd.com/gpu (mutating webhook; true/false)."
  type        = string
  default     = "true"
}
