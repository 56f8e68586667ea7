output "prometheus-query-url" {
  description = "PromQL endpoint of the Azure Monitor workspace."
  value       = local.monitor_props.metrics.prometheusQueryEndpoint
}

output "az-monitor-client-id" {
  description = "Client id of the remote_write identity (for the Prometheus config)."
  value       = azurerm_user_assigned_identity.remote_write.client_id
}

output "cluster_managed-client-id" {
  description = "Client id of the cluster's kubelet identity."
  value       = data.azurerm_user_assigned_identity.kubelet.client_id
}

output "fluentbit-secret-name" {
  description = "Secret holding the Log Analytics workspace id and key (null when disabled)."
  value       = var.fluentbit_enabled ? kubernetes_secret_v1.fluentbit["fluentbit"].metadata[0].name : null
}

output "fluentbit-secret-namespace" {
  description = "Namespace of that secret (null when disabled)."
  value       = var.fluentbit_enabled ? kubernetes_namespace_v1.monitoring["fluentbit"].metadata[0].name : null
}
