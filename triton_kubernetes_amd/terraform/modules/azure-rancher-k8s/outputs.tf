output "rancher_cluster_id" {
  value = data.external.rancher_cluster.result.cluster_id
}

output "rancher_cluster_registration_token" {
  value = data.external.rancher_cluster.result.registration_token
  sensitive = true
}

output "rancher_cluster_ca_checksum" {
  value = data.external.rancher_cluster.result.ca_checksum
}

output "azure_resource_group_name" {
  value = azurerm_resource_group.resource_group.name
}

output "azure_network_security_group_id" {
  value = azurerm_network_security_group.rke_ports.id
}

output "azure_subnet_id" {
  value = azurerm_subnet.subnet.id
}
