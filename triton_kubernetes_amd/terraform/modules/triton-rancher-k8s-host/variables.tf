variable "hostname" {
  description = "Host name given to the node."
  type        = string
}

variable "rancher_api_url" {
  description = "Base URL of the Rancher server (the cluster manager's rancher_url output)."
  type        = string
}

variable "k8s_distribution" {
  description = "the cluster's distribution: rke2 joins with the server's system-agent installer, rke1 with docker run rancher/rancher-agent"
  type        = string
  default     = "rke2"

  validation {
    condition     = contains(["rke2", "rke1"], var.k8s_distribution)
    error_message = "k8s_distribution must be rke2 or rke1."
  }
}

variable "rancher_cluster_registration_token" {
  description = "Registration token of the cluster the node joins."
  type        = string
  sensitive   = true
}

variable "rancher_cluster_ca_checksum" {
  description = "SHA-256 of the Rancher CA bundle, pinned by the agent."
  type        = string
}

variable "rancher_host_labels" {
  description = "A single-key map: {worker|etcd|control = \"true\"}"
  type        = map(string)

  validation {
    condition     = length(var.rancher_host_labels) == 1 && contains(["worker", "etcd", "control"], keys(var.rancher_host_labels)[0])
    error_message = "rancher_host_labels must hold exactly one of worker, etcd or control."
  }
}

variable "docker_engine_install_url" {
  description = "The URL to the shell script to install the docker engine."
  type        = string
  default     = "https://releases.rancher.com/install-docker/24.0.sh"
}

variable "docker_install_sha256" {
  description = "SHA-256 the downloaded runtime install script must match (empty: not checked)."
  type        = string
  default     = ""
}

variable "rancher_agent_image" {
  description = "The Rancher Agent image to use."
  type        = string
  default     = "rancher/rancher-agent:v2.10.3"
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

variable "triton_account" {
  description = "Triton account."
  type        = string
}

variable "triton_key_path" {
  description = "Triton key path."
  type        = string
}

variable "triton_key_id" {
  description = "Triton key id."
  type        = string
}

variable "triton_url" {
  description = "Triton url."
  type        = string
  default     = "https://us-east-1.api.joyent.com"
}

variable "triton_network_names" {
  description = "Triton network names."
  type        = list(string)
  default     = [
  "Joyent-SDC-Public"
]
}

variable "triton_image_name" {
  description = "Triton image name."
  type        = string
  default     = "ubuntu-certified-22.04"
}

variable "triton_image_version" {
  description = "Triton image version."
  type        = string
}

variable "triton_ssh_user" {
  description = "Triton ssh user."
  type        = string
  default     = "ubuntu"
}

variable "triton_machine_package" {
  description = "Triton machine package."
  type        = string
  default     = "k4-highcpu-kvm-7.75G"
}
