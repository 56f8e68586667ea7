# AMD GPU stack on AKS. The node images ship no amdgpu driver, so the stack
# installs it (upstream passed driver.enabled=false, which only works where a
# vendor driver is preinstalled). Everything is a tracked Terraform resource
# - version bumps apply in place - instead of a create-only helm provisioner.
# Only the validation Job waits for the MI355X pool (gpu_node_pool_ids).

module "amd_gpu_stack" {
  source = "../modules/amd-gpu-stack"

  cluster_name                = var.cluster_name
  gpu_stack_mode              = var.gpu_stack_mode
  gpu_operator_version        = var.gpu_operator_version
  gpu_operator_driver_version = var.gpu_operator_driver_version
  gpu_operator_namespace      = var.gpu_operator_namespace

  driver_enabled              = !var.gpu_driver_preinstalled
  node_prep_iommu_mode        = var.gpu_node_iommu_passthrough
  validation_require_iommu_pt = var.gpu_node_iommu_passthrough == "reboot"

  # the pools' startup taint: the Job schedules only on verified-prepared nodes
  node_prep_startup_taint = var.gpu_node_prep_taint
  node_prep_taint_key     = local.prep_taint_key

  gpu_node_selector = { "amd.com/gpu.present" = "true" }
  gpu_node_pool_ids = [azurerm_kubernetes_cluster_node_pool.mi355x.id]

  validation_enabled      = var.gpu_validation_enabled
  validation_image        = var.gpu_validation_image
  validation_tflops_floor = var.gpu_validation_tflops_floor
  validation_gpu_count    = var.gpus_per_node
  validation_node_count   = max(1, var.gpu_node_pool_count)
}
