output "resource_group_name" {
  value = local.resource_group_name
}

output "kubernetes_cluster_name" {
  value = azurerm_kubernetes_cluster.holoscan.name
}

output "client_certificate" {
  sensitive = true
  value     = azurerm_kubernetes_cluster.holoscan.kube_config[0].client_certificate
}

output "kube_config" {
  value     = azurerm_kubernetes_cluster.holoscan.kube_config_raw
  sensitive = true
}

output "location" {
  value = azurerm_kubernetes_cluster.holoscan.location
}

/****************************
AMD GPU stack outputs (new)
****************************/
output "gpu_operator_namespace" {
  value = module.amd_gpu_stack.namespace
}

output "gpu_validation_job" {
  value = module.amd_gpu_stack.validation_job_name
}
