/*******************************************
Fluent Bit -> Azure Log Analytics
The reference created the namespace + secret with `kubectl` in a
null_resource (key on the command line and in state, ungated, create-only).
Here: kubernetes provider resources, gated on fluentbit_enabled.
*******************************************/
resource "azurerm_log_analytics_workspace" "cnpack-fluentbit-workspace" {
  count               = var.fluentbit_enabled ? 1 : 0
  name                = var.fluentbit-workspace-name
  location            = module.holoscan-ready-aks.location
  resource_group_name = module.holoscan-ready-aks.resource_group_name
  sku                 = var.azure_log_analytics_sku
  retention_in_days   = var.azure_log_analytics_retention_in_days
}

resource "kubernetes_namespace_v1" "monitoring" {
  count = var.fluentbit_enabled ? 1 : 0
  metadata {
    name = local.monitoring_namespace
    labels = {
      "app.kubernetes.io/managed-by" = "terraform"
    }
  }
}

resource "kubernetes_secret_v1" "fluentbit" {
  count = var.fluentbit_enabled ? 1 : 0
  metadata {
    name      = "fluentbit-secrets"
    namespace = kubernetes_namespace_v1.monitoring[0].metadata[0].name
  }
  data = {
    WorkspaceId = azurerm_log_analytics_workspace.cnpack-fluentbit-workspace[0].workspace_id
    SharedKey   = azurerm_log_analytics_workspace.cnpack-fluentbit-workspace[0].primary_shared_key
  }
  type = "Opaque"
}

output "fluentbit-secret-name" {
  value = var.fluentbit_enabled ? kubernetes_secret_v1.fluentbit[0].metadata[0].name : null
}

output "fluentbit-secret-namespace" {
  value = var.fluentbit_enabled ? kubernetes_namespace_v1.monitoring[0].metadata[0].name : null
}
