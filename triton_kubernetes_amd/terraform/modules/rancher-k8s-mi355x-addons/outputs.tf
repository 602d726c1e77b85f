output "addons_applied" {
  value = tostring(terraform_data.apply_addons.output)
}
