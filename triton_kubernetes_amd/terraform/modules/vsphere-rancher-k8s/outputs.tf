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

output "vsphere_datacenter_name" {
  value = data.vsphere_datacenter.dc.name
}

output "vsphere_datastore_name" {
  value = data.vsphere_datastore.datastore.name
}

output "vsphere_resource_pool_name" {
  value = data.vsphere_resource_pool.pool.name
}

output "vsphere_network_name" {
  value = data.vsphere_network.network.name
}
