output "addons_applied" {
  description = "Addons applied."
  value       = tostring(terraform_data.apply_addons.output)
}
