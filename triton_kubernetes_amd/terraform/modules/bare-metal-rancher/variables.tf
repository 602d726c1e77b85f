variable "name" {
  description = "Human readable name used as prefix to generated names."
  type        = string
}

variable "rancher_admin_password" {
  description = "The Rancher admin password"
  type        = string
  sensitive   = true

  validation {
    condition     = length(var.rancher_admin_password) >= 12 && length(regexall("['\"\\\\]", var.rancher_admin_password)) == 0
    error_message = "rancher_admin_password must be at least 12 characters (Rancher >= 2.6) without quotes or backslashes."
  }
}

variable "rancher_bootstrap_password" {
  description = "First-login password of the Rancher server (CATTLE_BOOTSTRAP_PASSWORD); empty: derived from name and rancher_admin_password."
  type        = string
  default     = ""
  sensitive   = true

  validation {
    condition     = length(regexall("['\"\\\\]", var.rancher_bootstrap_password)) == 0
    error_message = "rancher_bootstrap_password must not contain quotes or backslashes."
  }
}

variable "tk_operation" {
  description = "Which CLI operation runs this configuration (set by the executor through the root variable of the same name): apply runs the create-side data sources in full; destroy and read make them find-only and tolerant of hosts that are gone."
  type        = string
  default     = "apply"

  validation {
    condition     = contains(["apply", "destroy", "read"], var.tk_operation)
    error_message = "tk_operation must be apply, destroy or read."
  }
}

variable "tk_known_hosts" {
  description = "known_hosts lines of the cluster manager's pinned SSH host keys (set by the executor through the root variable of the same name, parallel/hostkeys.py)."
  type        = string
  default     = ""
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

variable "rancher_server_image" {
  description = "The Rancher Server image to use."
  type        = string
  default     = "rancher/rancher:v2.10.3"
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
