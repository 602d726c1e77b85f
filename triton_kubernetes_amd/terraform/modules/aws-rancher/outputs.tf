output "rancher_url" {
  value = "https://${local.rancher_master_ip}"
}

output "rancher_access_key" {
  value = data.external.rancher_api_key.result.access_key
}

output "rancher_secret_key" {
  value = data.external.rancher_api_key.result.secret_key
  sensitive = true
}
