# 1. user-assigned identity for Prometheus remote-write
# 2. Azure Monitor workspace (managed Prometheus)
# 3. Monitoring Metrics Publisher on the workspace's default DCR for the
#    cluster's kubelet identity and the user-assigned identity
# 4. outputs: query URL + client ids for the monitoring stack config

data "azurerm_user_assigned_identity" "cnpack-cluster-managed-id" {
  depends_on          = [module.holoscan-ready-aks]
  name                = "${module.holoscan-ready-aks.kubernetes_cluster_name}-agentpool"
  resource_group_name = local.node_resource_group
}

output "cluster_managed-client-id" {
  value = data.azurerm_user_assigned_identity.cnpack-cluster-managed-id.client_id
}

data "azurerm_resource_group" "prometheus" {
  depends_on = [module.holoscan-ready-aks]
  name       = var.prometheus_resource_group_name == "" ? local.node_resource_group : var.prometheus_resource_group_name
}

resource "azurerm_user_assigned_identity" "az-monitor" {
  name                = var.az_monitor-user-managed-id
  resource_group_name = data.azurerm_resource_group.prometheus.name
  location            = data.azurerm_resource_group.prometheus.location
}

resource "azapi_resource" "prometheus-cnpack" {
  depends_on                = [module.holoscan-ready-aks]
  type                      = "microsoft.monitor/accounts@2023-04-03"
  name                      = var.prometheus-name
  schema_validation_enabled = false
  parent_id                 = data.azurerm_resource_group.prometheus.id
  location                  = data.azurerm_resource_group.prometheus.location
  response_export_values    = ["*"]
}

locals {
  prometheus_properties = jsondecode(azapi_resource.prometheus-cnpack.output).properties
}

output "prometheus-query-url" {
  value = local.prometheus_properties.metrics.prometheusQueryEndpoint
}

output "az-monitor-client-id" {
  value = azurerm_user_assigned_identity.az-monitor.client_id
}

resource "azurerm_role_assignment" "cnpack-prometheus-role" {
  scope                = local.prometheus_properties.defaultIngestionSettings.dataCollectionRuleResourceId
  role_definition_name = "Monitoring Metrics Publisher"
  principal_id         = data.azurerm_user_assigned_identity.cnpack-cluster-managed-id.principal_id
}

resource "azurerm_role_assignment" "az-monitor-prometheus-role" {
  scope                = local.prometheus_properties.defaultIngestionSettings.dataCollectionRuleResourceId
  role_definition_name = "Monitoring Metrics Publisher"
  principal_id         = azurerm_user_assigned_identity.az-monitor.principal_id
}
