output "kubernetes_cluster_name" {
  description = "AKS cluster name."
  value       = azurerm_kubernetes_cluster.this.name
}

output "resource_group_name" {
  description = "Resource group holding the cluster."
  value       = local.rg.name
}

output "location" {
  description = "Azure region of the cluster."
  value       = azurerm_kubernetes_cluster.this.location
}

output "kube_config" {
  description = "Raw admin kubeconfig (Entra ID clusters still need kubelogin for user tokens)."
  value       = azurerm_kubernetes_cluster.this.kube_config_raw
  sensitive   = true
}

output "client_certificate" {
  description = "Client certificate from the admin kubeconfig."
  value       = azurerm_kubernetes_cluster.this.kube_config[0].client_certificate
  sensitive   = true
}

output "gpu_operator_namespace" {
  description = "Namespace of the GPU stack and the validation Job."
  value       = module.amd_gpu_stack.namespace
}

output "gpu_validation_job" {
  description = "Name of the validation Job."
  value       = module.amd_gpu_stack.validation_job_name
}
