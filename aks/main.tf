data "azurerm_resource_group" "existing" {
  count = var.existing_resource_group_name == null ? 0 : 1
  name  = var.existing_resource_group_name
}

resource "azurerm_resource_group" "holoscan" {
  count    = var.existing_resource_group_name == null ? 1 : 0
  name     = "${var.cluster_name}-rg"
  location = var.location
  tags = {
    group      = "amd-instinct"
    managed_by = "Terraform"
  }
}

locals {
  resource_group_name     = var.existing_resource_group_name == null ? azurerm_resource_group.holoscan[0].name : data.azurerm_resource_group.existing[0].name
  resource_group_location = var.existing_resource_group_name == null ? azurerm_resource_group.holoscan[0].location : data.azurerm_resource_group.existing[0].location
  tags = {
    group      = "amd-instinct"
    managed_by = "Terraform"
  }
}

resource "terraform_data" "gpu_machine_type_guard" {
  input = var.gpu_machine_type

  lifecycle {
    precondition {
      condition     = var.gpu_machine_type != ""
      error_message = "Set gpu_machine_type to an Azure VM size with 8x AMD Instinct MI355X."
    }
  }
}

resource "azurerm_kubernetes_cluster" "holoscan" {
  name                = var.cluster_name
  kubernetes_version  = var.kubernetes_version
  resource_group_name = local.resource_group_name
  location            = local.resource_group_location
  dns_prefix          = var.cluster_name

  default_node_pool {
    name                 = "cpu"
    node_count           = var.cpu_node_pool_count
    enable_auto_scaling  = true
    min_count            = var.cpu_node_pool_min_count
    max_count            = var.cpu_node_pool_max_count
    vm_size              = var.cpu_machine_type
    os_disk_size_gb      = var.cpu_node_pool_disk_size
    os_sku               = var.cpu_os_sku
    node_labels          = { "node.kubernetes.io/pool" = "cpu" }
    orchestrator_version = var.kubernetes_version
  }

  azure_active_directory_role_based_access_control {
    managed                = true
    azure_rbac_enabled     = true
    admin_group_object_ids = var.admin_group_object_ids
  }

  identity {
    type = "SystemAssigned"
  }

  tags = local.tags

  # No local-exec: the reference ran `az aks get-credentials` + `kubelogin
  # convert-kubeconfig` here (aks/main.tf:51-58), mutating the operator's
  # ~/.kube/config. The helm/kubernetes providers below authenticate with
  # kubelogin exec tokens instead.
}

/****************************
MI355X GPU node pool
****************************/
resource "azurerm_kubernetes_cluster_node_pool" "holoscan" {
  name                  = "mi355x"
  kubernetes_cluster_id = azurerm_kubernetes_cluster.holoscan.id
  node_count            = var.gpu_node_pool_count
  enable_auto_scaling   = true
  min_count             = var.gpu_node_pool_min_count
  max_count             = var.gpu_node_pool_max_count
  vm_size               = var.gpu_machine_type
  os_disk_size_gb       = var.gpu_node_pool_disk_size
  os_sku                = var.gpu_os_sku
  orchestrator_version  = var.kubernetes_version
  node_labels = {
    "node.kubernetes.io/pool" = "gpu"
    "amd.com/gpu.present"     = "true"
    "amd.com/gpu.family"      = "mi355x"
    "amd.com/gpu.arch"        = "gfx950"
  }
  node_taints = ["amd.com/gpu=present:NoSchedule"]
  tags        = local.tags

  depends_on = [terraform_data.gpu_machine_type_guard]
}

/****************************
AMD GPU stack. AKS node images carry no amdgpu driver, so unlike the
reference (`--set driver.enabled=false`, aks/main.tf:89-91) the driver is
installed by the stack. The release is tracked in Terraform state (the
reference's helm CLI provisioner was invisible to state and ran on create
only, so gpu_operator_version changes did nothing).
****************************/
module "amd_gpu_stack" {
  source = "../modules/amd-gpu-stack"

  cluster_name                = var.cluster_name
  gpu_stack_mode              = var.gpu_stack_mode
  gpu_operator_version        = var.gpu_operator_version
  gpu_operator_driver_version = var.gpu_operator_driver_version
  gpu_operator_namespace      = var.gpu_operator_namespace
  gpu_node_selector           = { "amd.com/gpu.present" = "true" }
  gpu_node_pool_ids           = [azurerm_kubernetes_cluster_node_pool.holoscan.id]
  validation_enabled          = var.gpu_validation_enabled
  validation_image            = var.gpu_validation_image
  validation_gpu_count        = var.gpus_per_node

  # Only the validation Job waits for the GPU pool (via gpu_node_pool_ids): the
  # operator installs on the default CPU pool while MI355X nodes boot.
}
