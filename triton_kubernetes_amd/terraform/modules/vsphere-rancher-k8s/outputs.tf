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

output "vsphere_datacenter_name" {
  description = "VSphere datacenter name."
  value       = data.vsphere_datacenter.dc.name
}

output "vsphere_datastore_name" {
  description = "VSphere datastore name."
  value       = data.vsphere_datastore.datastore.name
}

output "vsphere_resource_pool_name" {
  description = "VSphere resource pool name."
  value       = data.vsphere_resource_pool.pool.name
}

output "vsphere_network_name" {
  description = "VSphere network name."
  value       = data.vsphere_network.network.name
}
