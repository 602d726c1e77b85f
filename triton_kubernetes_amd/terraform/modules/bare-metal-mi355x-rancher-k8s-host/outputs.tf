output "gpu_node_labels" {
  description = "Gpu node labels."
  value       = data.external.gpu_labels.result.labels
}
