output "gpu_node_labels" {
  value = data.external.gpu_labels.result.labels
}
