variable "name" {
  description = "Human readable name used as prefix to generated names."
}

variable "rancher_api_url" {
}

variable "rancher_access_key" {
}

variable "rancher_secret_key" {
  sensitive   = true
}

variable "k8s_version" {
  default     = "v1.9.5-rancher1-1"
}

variable "k8s_network_provider" {
  default     = "flannel"
}

variable "rancher_registry" {
  default     = ""
}

variable "rancher_registry_username" {
  default     = ""
}

variable "rancher_registry_password" {
  default     = ""
  sensitive   = true
}

variable "k8s_registry" {
  default     = ""
}

variable "k8s_registry_username" {
  default     = ""
}

variable "k8s_registry_password" {
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

variable "azure_virtual_network_name" {
  default     = "k8s-network"
}

variable "azure_virtual_network_address_space" {
  default     = "10.0.0.0/16"
}

variable "azure_subnet_name" {
  default     = "k8s-subnet"
}

variable "azure_subnet_address_prefix" {
  default     = "10.0.2.0/24"
}

variable "azurerm_network_security_group_name" {
  default     = "k8s-firewall"
}
