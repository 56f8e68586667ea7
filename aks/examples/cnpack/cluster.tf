# The MI355X AKS cluster and what the add-ons need to know about it.

module "mi355x_aks" {
  source = "../../"

  cluster_name           = var.cluster_name
  location               = var.location
  admin_group_object_ids = var.admin_group_object_ids
  gpu_machine_type       = var.gpu_machine_type
}

# re-read after creation: API endpoint + CA for the kubernetes provider
data "azurerm_kubernetes_cluster" "cnpack" {
  name                = module.mi355x_aks.kubernetes_cluster_name
  resource_group_name = module.mi355x_aks.resource_group_name
  depends_on          = [module.mi355x_aks]
}

locals {
  kube              = data.azurerm_kubernetes_cluster.cnpack.kube_config[0]
  monitoring_ns     = "amd-monitoring"
  aks_node_rg       = "MC_${module.mi355x_aks.resource_group_name}_${module.mi355x_aks.kubernetes_cluster_name}_${module.mi355x_aks.location}"
  logging_instances = var.fluentbit_enabled ? { fluentbit = true } : {}
}
