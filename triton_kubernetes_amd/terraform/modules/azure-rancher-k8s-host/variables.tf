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

variable "azure_subscription_id" {
  description = "Azure subscription id."
  type        = string
  default     = ""
}

variable "azure_client_id" {
  description = "Azure client id."
  type        = string
  default     = ""
}

variable "azure_client_secret" {
  description = "Azure client secret."
  type        = string
  default     = ""
  sensitive   = true
}

variable "azure_tenant_id" {
  description = "Azure tenant id."
  type        = string
  default     = ""
}

variable "azure_environment" {
  description = "Azure environment."
  type        = string
  default     = "public"
}

variable "azure_location" {
  description = "Azure location."
  type        = string
  default     = "westus2"
}

variable "azure_image_publisher" {
  description = "Azure image publisher."
  type        = string
  default     = "Canonical"
}

variable "azure_image_offer" {
  description = "Azure image offer."
  type        = string
  default     = "0001-com-ubuntu-server-jammy"
}

variable "azure_image_sku" {
  description = "Azure image sku."
  type        = string
  default     = "22_04-lts-gen2"
}

variable "azure_image_version" {
  description = "Azure image version."
  type        = string
  default     = "latest"
}

variable "azure_resource_group_name" {
  description = "Azure resource group name."
  type        = string
}

variable "azure_network_security_group_id" {
  description = "Azure network security group id."
  type        = string
}

variable "azure_subnet_id" {
  description = "Azure subnet id."
  type        = string
}

variable "azure_size" {
  description = "Azure size."
  type        = string
  default     = "Standard_D4s_v5"
}

variable "azure_ssh_user" {
  description = "Azure ssh user."
  type        = string
  default     = "ubuntu"
}

variable "azure_public_key_path" {
  description = "Azure public key path."
  type        = string
  default     = "~/.ssh/id_rsa.pub"
}

variable "azure_disk_mount_path" {
  description = "Azure disk mount path."
  type        = string
  default     = ""
}

variable "azure_disk_size" {
  description = "Azure disk size."
  type        = string
  default     = ""
}
