variable "hostname" {
  description = "Host name given to the node."
  type        = string

  validation {
    condition     = length(regexall("^[A-Za-z0-9]([-A-Za-z0-9.]{0,251}[A-Za-z0-9])?$", var.hostname)) > 0
    error_message = "hostname must be a DNS host name."
  }
}

variable "rancher_api_url" {
  description = "Base URL of the Rancher server (the cluster manager's rancher_url output)."
  type        = string

  validation {
    condition     = length(regexall("^https?://[][A-Za-z0-9._:-]+(/[A-Za-z0-9._/-]*)?$", var.rancher_api_url)) > 0
    error_message = "rancher_api_url must be an http(s) URL."
  }
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

  validation {
    condition     = length(regexall("^[A-Za-z0-9._:-]{1,512}$", var.rancher_cluster_registration_token)) > 0
    error_message = "rancher_cluster_registration_token must be a Rancher registration token."
  }
}

variable "rancher_cluster_ca_checksum" {
  description = "SHA-256 of the Rancher CA bundle, pinned by the agent."
  type        = string

  validation {
    condition     = length(regexall("^[A-Za-z0-9]{0,128}$", var.rancher_cluster_ca_checksum)) > 0
    error_message = "rancher_cluster_ca_checksum must be a hex checksum (or empty)."
  }
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

  validation {
    condition     = length(regexall("^(https?://[][A-Za-z0-9._:-]+(/[A-Za-z0-9._/~%+=-]*)?)?$", var.docker_engine_install_url)) > 0
    error_message = "docker_engine_install_url must be an http(s) URL (or empty)."
  }
}

variable "docker_install_sha256" {
  description = "SHA-256 the downloaded runtime install script must match (empty: not checked)."
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("^[A-Fa-f0-9]{0,64}$", var.docker_install_sha256)) > 0
    error_message = "docker_install_sha256 must be a sha256 hex digest (or empty)."
  }
}

variable "rancher_agent_image" {
  description = "The Rancher Agent image to use."
  type        = string
  default     = "rancher/rancher-agent:v2.10.3"

  validation {
    condition     = length(regexall("^[A-Za-z0-9][A-Za-z0-9._/:@-]{0,254}$", var.rancher_agent_image)) > 0
    error_message = "rancher_agent_image must be a container image reference."
  }
}

variable "rancher_registry" {
  description = "The docker registry to use for rancher server and agent images"
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("^([A-Za-z0-9][A-Za-z0-9._/:@-]{0,254})?$", var.rancher_registry)) > 0
    error_message = "rancher_registry must be a registry host (or empty)."
  }
}

variable "rancher_registry_username" {
  description = "The username to login as."
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("['\"\\\\]", var.rancher_registry_username)) == 0
    error_message = "rancher_registry_username must not contain quotes or backslashes."
  }
}

variable "rancher_registry_password" {
  description = "The password to use."
  type        = string
  default     = ""
  sensitive   = true

  validation {
    condition     = length(regexall("['\"\\\\]", var.rancher_registry_password)) == 0
    error_message = "rancher_registry_password must not contain quotes or backslashes."
  }
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

variable "node_cleanup" {
  description = "on destroy, take the host out of its cluster: uninstall rancher-system-agent and RKE2 (or the RKE1 containers) and remove their state, keeping the node tools and the container runtime (bare metal outlives its cluster; node/cleanup.py)"
  type        = bool
  default     = true
}
