# AMD GPU enablement (operator or DKMS + device plugin), metrics exporter and
# the validation Job that apply waits for. Only the Job is tied to the MI355X
# node group (gpu_node_pool_ids); the rest depends on the control plane and the
# system pool and installs while the GPU nodes boot (the reference meant to
# gate on running GPU nodes, /root/reference/eks/main.tf:186, and gated the
# whole operator instead).

module "amd_gpu_stack" {
  source = "../modules/amd-gpu-stack"

  cluster_name   = var.cluster_name
  gpu_stack_mode = var.gpu_stack_mode

  gpu_operator_version        = var.gpu_operator_version
  gpu_operator_driver_version = var.gpu_operator_driver_version
  gpu_operator_namespace      = var.gpu_operator_namespace

  driver_enabled = !var.gpu_driver_preinstalled
  # the pre-bootstrap user data applies the host prep (incl. the iommu=pt
  # reboot); the DaemonSet re-applies it idempotently and the Job checks it
  node_prep_iommu_mode        = "check"
  validation_require_iommu_pt = var.gpu_node_iommu_passthrough != "off"

  # the pools' startup taint: the Job schedules only on verified-prepared nodes
  node_prep_startup_taint = var.gpu_node_prep_taint
  node_prep_taint_key     = local.prep_taint_key

  gpu_node_selector = { "amd.com/gpu.present" = "true" }
  gpu_node_pool_ids = [module.gpu_node_pool.node_group_id]

  validation_enabled      = var.gpu_validation_enabled
  validation_image        = var.gpu_validation_image
  validation_gpu_count    = var.gpus_per_node
  validation_node_count   = max(1, var.desired_count_gpu_nodes)
  validation_tflops_floor = var.gpu_validation_tflops_floor

  depends_on = [module.eks, module.cpu_node_pool]
}
