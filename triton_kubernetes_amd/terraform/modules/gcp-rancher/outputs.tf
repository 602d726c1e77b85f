output "rancher_url" {
  description = "URL of the Rancher server."
  value       = "https://${local.rancher_master_ip}"
}

output "rancher_access_key" {
  description = "API access key created for triton-kubernetes."
  value       = data.external.rancher_api_key.result.access_key
}

output "rancher_secret_key" {
  description = "API secret key created for triton-kubernetes."
  value       = data.external.rancher_api_key.result.secret_key
  sensitive   = true
}

output "tk_ssh_known_hosts" {
  description = "known_hosts lines of the hosts this module's SSH reads contacted (pinned by the CLI)."
  value       = data.external.rancher_api_key.result.known_hosts
}

output "tk_rancher_ca_certs" {
  description = "The Rancher server's CA bundle as its host serves it (pinned by the CLI; empty: public CA)."
  value       = data.external.rancher_api_key.result.ca_certs
}
