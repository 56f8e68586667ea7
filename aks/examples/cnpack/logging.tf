# Log Analytics for Fluent Bit, and the workspace credentials as a Kubernetes
# secret - created through the provider, only when fluentbit_enabled (the
# upstream example ran kubectl with the key on its command line, whatever the
# flag said).

resource "azurerm_log_analytics_workspace" "fluentbit" {
  for_each            = local.logging_instances
  name                = var.fluentbit-workspace-name
  location            = module.mi355x_aks.location
  resource_group_name = module.mi355x_aks.resource_group_name
  sku                 = var.azure_log_analytics_sku
  retention_in_days   = var.azure_log_analytics_retention_in_days
}

resource "kubernetes_namespace_v1" "monitoring" {
  for_each = local.logging_instances
  metadata {
    name   = local.monitoring_ns
    labels = { "app.kubernetes.io/managed-by" = "terraform" }
  }
}

resource "kubernetes_secret_v1" "fluentbit" {
  for_each = local.logging_instances
  type     = "Opaque"
  metadata {
    name      = "fluentbit-secrets"
    namespace = kubernetes_namespace_v1.monitoring[each.key].metadata[0].name
  }
  data = {
    WorkspaceId = azurerm_log_analytics_workspace.fluentbit[each.key].workspace_id
    SharedKey   = azurerm_log_analytics_workspace.fluentbit[each.key].primary_shared_key
  }
}
