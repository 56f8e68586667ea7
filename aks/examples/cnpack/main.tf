module "holoscan-ready-aks" {
  source                 = "../../" # path or git URL of this repo's aks module
  cluster_name           = var.cluster_name
  admin_group_object_ids = var.admin_group_object_ids
  location               = var.location
  gpu_machine_type       = var.gpu_machine_type
}

# Used to configure the kubernetes provider of this example (dead in the reference)
data "azurerm_kubernetes_cluster" "holoscancluster" {
  name                = module.holoscan-ready-aks.kubernetes_cluster_name
  resource_group_name = module.holoscan-ready-aks.resource_group_name
  depends_on          = [module.holoscan-ready-aks]
}

locals {
  monitoring_namespace = "amd-monitoring"
  node_resource_group  = "MC_${module.holoscan-ready-aks.resource_group_name}_${module.holoscan-ready-aks.kubernetes_cluster_name}_${module.holoscan-ready-aks.location}"
}
