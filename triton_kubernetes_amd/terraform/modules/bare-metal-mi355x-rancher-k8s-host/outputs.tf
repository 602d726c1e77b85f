output "gpu_node_labels" {
  description = "Gpu node labels."
  value       = data.external.gpu_labels.result.labels
}

output "tk_ssh_known_hosts" {
  description = "known_hosts lines of the hosts this module's SSH reads contacted (pinned by the CLI)."
  value       = data.external.gpu_labels.result.known_hosts
}
