output "rancher_cluster_id" {
  description = "Rancher id of the cluster (found by name or created)."
  value       = data.external.cluster.result["cluster_id"]
}

output "rancher_cluster_registration_token" {
  description = "Token nodes present when they register."
  value       = data.external.cluster.result["registration_token"]
  sensitive   = true
}

output "rancher_cluster_ca_checksum" {
  description = "Checksum of the Rancher CA bundle that agents pin."
  value       = data.external.cluster.result["ca_checksum"]
}

output "azure_resource_group_name" {
  description = "Azure resource group name."
  value       = azurerm_resource_group.resource_group.name
}

output "azure_network_security_group_id" {
  description = "Azure network security group id."
  value       = azurerm_network_security_group.rke_ports.id
}

output "azure_subnet_id" {
  description = "Azure subnet id."
  value       = azurerm_subnet.subnet.id
}
