# AKS with Entra ID RBAC; the default pool is the system (CPU) pool and the
# MI355X devices come in a separate, tainted user pool. No provisioners: the
# upstream module shelled out to `az aks get-credentials` and `kubelogin
# convert-kubeconfig` here, rewriting the operator's ~/.kube/config.

resource "terraform_data" "gpu_machine_type_guard" {
  input = var.gpu_machine_type
  lifecycle {
    precondition {
      condition     = var.gpu_machine_type != ""
      error_message = "Set gpu_machine_type to an Azure VM size with 8x AMD Instinct MI355X."
    }
  }
}

resource "azurerm_kubernetes_cluster" "this" {
  name                = var.cluster_name
  dns_prefix          = var.cluster_name
  resource_group_name = local.rg.name
  location            = local.rg.location
  kubernetes_version  = var.kubernetes_version
  tags                = local.tags

  identity {
    type = "SystemAssigned"
  }

  azure_active_directory_role_based_access_control {
    managed                = true
    azure_rbac_enabled     = true
    admin_group_object_ids = var.admin_group_object_ids
  }

  default_node_pool {
    name                 = "cpu"
    vm_size              = var.cpu_machine_type
    os_sku               = var.cpu_os_sku
    os_disk_size_gb      = var.cpu_node_pool_disk_size
    orchestrator_version = var.kubernetes_version
    enable_auto_scaling  = true
    node_count           = var.cpu_node_pool_count
    min_count            = var.cpu_node_pool_min_count
    max_count            = var.cpu_node_pool_max_count
    node_labels          = { "node.kubernetes.io/pool" = "cpu" }
  }
}

resource "azurerm_kubernetes_cluster_node_pool" "mi355x" {
  name                  = "mi355x"
  kubernetes_cluster_id = azurerm_kubernetes_cluster.this.id
  vm_size               = var.gpu_machine_type
  os_sku                = var.gpu_os_sku
  os_disk_size_gb       = var.gpu_node_pool_disk_size
  orchestrator_version  = var.kubernetes_version
  enable_auto_scaling   = true
  node_count            = var.gpu_node_pool_count
  min_count             = var.gpu_node_pool_min_count
  max_count             = var.gpu_node_pool_max_count
  # + the startup taint the node-prep DaemonSet removes after a verified prep
  node_taints = concat(["amd.com/gpu=present:NoSchedule"],
  var.gpu_node_prep_taint ? ["${local.prep_taint_key}=pending:NoSchedule"] : [])
  tags = local.tags
  node_labels = {
    "node.kubernetes.io/pool" = "gpu"
    "amd.com/gpu.present"     = "true"
    "amd.com/gpu.family"      = "mi355x"
    "amd.com/gpu.arch"        = "gfx950"
  }

  depends_on = [terraform_data.gpu_machine_type_guard]
}
