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

variable "host_key" {
  description = "Pinned SSH host key of host (\"<type> <base64>\", set by the executor; empty: not pinned yet)."
  type        = string
  default     = ""
}

variable "bastion_host_key" {
  description = "Pinned SSH host key of bastion_host (set by the executor; empty: not pinned yet)."
  type        = string
  default     = ""
}
