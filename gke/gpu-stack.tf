# AMD GPU stack on GKE. critical_pod_quota: GKE admits system-*-critical pods
# outside kube-system only under a ResourceQuota scoped to those classes, and
# the device plugin / driver DaemonSets use them. Depending on the system pool
# only (the Job alone waits for the MI355X pool) lets the stack install while
# GPU nodes boot; the namespace is owned by the module, so destroy needs no
# manual `terraform state rm`.

module "amd_gpu_stack" {
  source = "../modules/amd-gpu-stack"

  cluster_name                = var.cluster_name
  gpu_stack_mode              = var.gpu_stack_mode
  gpu_operator_version        = var.gpu_operator_version
  gpu_operator_driver_version = var.gpu_operator_driver_version
  gpu_operator_namespace      = var.gpu_operator_namespace
  critical_pod_quota          = true

  driver_enabled              = !var.gpu_driver_preinstalled
  node_prep_iommu_mode        = var.gpu_node_iommu_passthrough
  validation_require_iommu_pt = var.gpu_node_iommu_passthrough == "reboot"

  # the pools' startup taint: the Job schedules only on verified-prepared nodes
  node_prep_startup_taint = var.gpu_node_prep_taint
  node_prep_taint_key     = local.prep_taint_key

  gpu_node_selector = { "amd.com/gpu.present" = "true" }
  gpu_node_pool_ids = [google_container_node_pool.mi355x.id]

  validation_enabled      = var.gpu_validation_enabled
  validation_image        = var.gpu_validation_image
  validation_tflops_floor = var.gpu_validation_tflops_floor
  validation_gpu_count    = tonumber(var.gpu_count)
  validation_node_count   = max(1, var.num_gpu_nodes * length(var.node_zones))

  depends_on = [google_container_node_pool.system]
}
