variable "hostname" {
}

variable "rancher_api_url" {
}

variable "rancher_cluster_registration_token" {
  sensitive   = true
}

variable "rancher_cluster_ca_checksum" {
}

variable "rancher_host_labels" {
  type        = map(string)
  description = "A single-key map: {worker|etcd|control = \"true\"}"
}

variable "docker_engine_install_url" {
  description = "The URL to the shell script to install the docker engine."
  default     = "https://releases.rancher.com/install-docker/24.0.sh"
}

variable "rancher_agent_image" {
  description = "The Rancher Agent image to use."
  default     = "rancher/rancher-agent:v2.8.5"
}

variable "rancher_registry" {
  description = "The docker registry to use for rancher server and agent images"
  default     = ""
}

variable "rancher_registry_username" {
  description = "The username to login as."
  default     = ""
}

variable "rancher_registry_password" {
  description = "The password to use."
  default     = ""
  sensitive   = true
}

variable "azure_subscription_id" {
  default     = ""
}

variable "azure_client_id" {
  default     = ""
}

variable "azure_client_secret" {
  default     = ""
  sensitive   = true
}

variable "azure_tenant_id" {
  default     = ""
}

variable "azure_environment" {
  default     = "public"
}

variable "azure_location" {
  default     = "westus2"
}

variable "azure_image_publisher" {
  default     = "Canonical"
}

variable "azure_image_offer" {
  default     = "0001-com-ubuntu-server-jammy"
}

variable "azure_image_sku" {
  default     = "22_04-lts-gen2"
}

variable "azure_image_version" {
  default     = "latest"
}

variable "azure_resource_group_name" {
}

variable "azure_network_security_group_id" {
}

variable "azure_subnet_id" {
}

variable "azure_size" {
  default     = "Standard_D4s_v5"
}

variable "azure_ssh_user" {
  default     = "ubuntu"
}

variable "azure_public_key_path" {
  default     = "~/.ssh/id_rsa.pub"
}

variable "azure_disk_mount_path" {
  default     = ""
}

variable "azure_disk_size" {
  default     = ""
}
