variable "name" {
  description = "Human readable name used as prefix to generated names."
  type        = string
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

variable "k8s_distribution" {
  description = "rke2 (provisioning.cattle.io/v1 custom cluster, nodes join with rancher-system-agent) or rke1 (v3 cluster + rancher-agent; reference-era documents)"
  type        = string
  default     = "rke2"

  validation {
    condition     = contains(["rke2", "rke1"], var.k8s_distribution)
    error_message = "k8s_distribution must be rke2 or rke1."
  }
}

variable "k8s_version" {
  description = "RKE Kubernetes version."
  type        = string
  default     = "v1.31.6+rke2r1"

  validation {
    condition     = (contains(["v1.31", "v1.30", "v1.29"], join(".", slice(split(".", var.k8s_version), 0, 2))) && length(regexall("[+]rke2r[0-9]+$", var.k8s_version)) > 0) || (contains(["v1.31", "v1.30", "v1.29", "v1.28"], join(".", slice(split(".", var.k8s_version), 0, 2))) && length(regexall("-rancher[0-9]+-[0-9]+$", var.k8s_version)) > 0)
    error_message = "k8s_version must be an RKE2 (v1.31.6+rke2r1, v1.30.10+rke2r1, v1.29.14+rke2r1) or RKE1 (v1.31.6-rancher1-1, v1.30.10-rancher1-1, v1.29.14-rancher1-1, v1.28.15-rancher1-1) release of Rancher v2.10.3."
  }
}

variable "k8s_network_provider" {
  description = "CNI plugin of the cluster."
  type        = string
  default     = "canal"

  validation {
    condition     = contains(["canal", "calico", "cilium", "flannel", "weave"], var.k8s_network_provider)
    error_message = "k8s_network_provider must be one of canal, calico, cilium, flannel (RKE2) or weave (RKE1)."
  }
}

variable "tk_rancher_ca" {
  description = "PEM CA bundle the Rancher server is verified against (the manager's pinned CA, rendered by the CLI; empty: a publicly trusted certificate)"
  type        = string
  default     = ""
}

variable "rancher_registry" {
  description = "Private registry serving the Rancher images (empty: Docker Hub)."
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("^([A-Za-z0-9][A-Za-z0-9._/:@-]{0,254})?$", var.rancher_registry)) > 0
    error_message = "rancher_registry must be a registry host (or empty)."
  }
}

variable "rancher_registry_username" {
  description = "User for rancher_registry."
  type        = string
  default     = ""

  validation {
    condition     = length(regexall("['\"\\\\]", var.rancher_registry_username)) == 0
    error_message = "rancher_registry_username must not contain quotes or backslashes."
  }
}

variable "rancher_registry_password" {
  description = "Password for rancher_registry."
  type        = string
  default     = ""
  sensitive   = true

  validation {
    condition     = length(regexall("['\"\\\\]", var.rancher_registry_password)) == 0
    error_message = "rancher_registry_password must not contain quotes or backslashes."
  }
}

variable "k8s_registry" {
  description = "Private registry for the Kubernetes system images (empty: default)."
  type        = string
  default     = ""
}

variable "k8s_registry_username" {
  description = "User for k8s_registry."
  type        = string
  default     = ""
}

variable "k8s_registry_password" {
  description = "Password for k8s_registry."
  type        = string
  default     = ""
  sensitive   = true
}

variable "aws_access_key" {
  description = "AWS access key."
  type        = string
}

variable "aws_secret_key" {
  description = "AWS secret key."
  type        = string
  sensitive   = true
}

variable "aws_region" {
  description = "AWS region."
  type        = string
}

variable "aws_vpc_cidr" {
  description = "AWS vpc cidr."
  type        = string
  default     = "10.0.0.0/16"
}

variable "aws_subnet_cidr" {
  description = "AWS subnet cidr."
  type        = string
  default     = "10.0.2.0/24"
}

variable "aws_public_key_path" {
  description = "AWS public key path."
  type        = string
  default     = "~/.ssh/id_rsa.pub"
}

variable "aws_key_name" {
  description = "AWS key name."
  type        = string
}

variable "aws_ami_id" {
  description = "Accepted for compatibility; the hosts' AMI is set per node."
  type        = string
  default     = ""
}
