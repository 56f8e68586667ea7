# Azure Monitor managed Prometheus: a monitor workspace, a user-assigned
# identity for remote_write, and "Monitoring Metrics Publisher" on the
# workspace's default data collection rule for that identity and for the
# cluster's kubelet identity (<cluster>-agentpool in the node resource group).

locals {
  monitor_rg_name = coalesce(var.prometheus_resource_group_name, local.aks_node_rg)
}

data "azurerm_resource_group" "monitor" {
  name       = local.monitor_rg_name
  depends_on = [module.mi355x_aks]
}

data "azurerm_user_assigned_identity" "kubelet" {
  name                = "${module.mi355x_aks.kubernetes_cluster_name}-agentpool"
  resource_group_name = local.aks_node_rg
  depends_on          = [module.mi355x_aks]
}

resource "azurerm_user_assigned_identity" "remote_write" {
  name                = var.az_monitor-user-managed-id
  location            = data.azurerm_resource_group.monitor.location
  resource_group_name = data.azurerm_resource_group.monitor.name
}

resource "azapi_resource" "monitor_workspace" {
  type                      = "microsoft.monitor/accounts@2023-04-03"
  name                      = var.prometheus-name
  parent_id                 = data.azurerm_resource_group.monitor.id
  location                  = data.azurerm_resource_group.monitor.location
  schema_validation_enabled = false
  response_export_values    = ["*"]
  depends_on                = [module.mi355x_aks]
}

locals {
  monitor_props = jsondecode(azapi_resource.monitor_workspace.output).properties
  publishers = {
    kubelet      = data.azurerm_user_assigned_identity.kubelet.principal_id
    remote_write = azurerm_user_assigned_identity.remote_write.principal_id
  }
}

resource "azurerm_role_assignment" "metrics_publisher" {
  for_each             = local.publishers
  scope                = local.monitor_props.defaultIngestionSettings.dataCollectionRuleResourceId
  role_definition_name = "Monitoring Metrics Publisher"
  principal_id         = each.value
}
