output "namespace" {
  value       = local.namespace
  description = "Namespace holding the AMD GPU stack and the validation Job."
}

output "gpu_resource_name" {
  value       = local.gpu_resource
  description = "Extended resource name workloads request (amd.com/gpu)."
}

output "gpu_stack_mode" {
  value       = var.gpu_stack_mode
  description = "operator or daemonsets."
}

output "operator_release" {
  value = local.operator_mode ? {
    name    = helm_release.amd_gpu_operator[0].name
    version = helm_release.amd_gpu_operator[0].version
    status  = helm_release.amd_gpu_operator[0].status
  } : null
  description = "AMD GPU Operator Helm release (operator mode)."
}

output "device_config_name" {
  value       = local.operator_mode ? local.device_config_values.name : null
  description = "Name of the DeviceConfig custom resource (operator mode)."
}

output "validation_job_name" {
  value       = var.validation_enabled ? kubernetes_job_v1.gpu_validation[0].metadata[0].name : null
  description = "Name of the post-provision validation Job (kubectl logs job/<name> for its JSON report)."
}

output "gpu_node_selector" {
  value       = var.gpu_node_selector
  description = "Labels that select MI355X nodes."
}

output "node_prep_gate" {
  value = local.prep_gate ? {
    taint_key            = var.node_prep_taint_key
    reconcile_interval_s = var.node_prep_gate_interval_s
    image                = var.node_prep_gate_image
  } : null
  description = "The node-prep startup-taint gate (node_prep_startup_taint): the taint its reconciler removes from each GPU node after verifying the host prep, and how often it re-checks; null when off."

  precondition {
    condition     = !var.node_prep_startup_taint || var.node_prep_enabled
    error_message = "node_prep_startup_taint needs node_prep_enabled: the node-prep DaemonSet is what removes the startup taint, and without it every GPU node would stay NoSchedule for the validation Job and every workload."
  }
}
