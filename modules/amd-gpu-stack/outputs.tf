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
