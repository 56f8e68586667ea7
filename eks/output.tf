output "private_subnet_ids" {
  value       = module.vpc[*].private_subnets
  description = "Private subnets of the created VPC (empty list when existing_vpc_details is used)."
}

output "public_subnet_ids" {
  value       = module.vpc[*].public_subnets
  description = "Public subnets of the created VPC (empty list when existing_vpc_details is used)."
}

output "nodes" {
  value       = data.aws_instances.nodes.public_ips
  description = "Public IPs of the running MI355X GPU nodes."
}

output "cluster_endpoint" {
  value = module.eks.cluster_endpoint
}

output "cpu_node_role_name" {
  description = "IAM Node Role Name for CPU node pools"
  value       = module.eks.eks_managed_node_groups.cpu_node_pool.iam_role_name
}

output "gpu_node_role_name" {
  description = "IAM Node Role Name for GPU node pools"
  value       = module.eks.eks_managed_node_groups.gpu_node_pool.iam_role_name
}

output "oidc_endpoint" {
  value = module.eks.oidc_provider
}

output "cluster_ca_certificate" {
  value     = module.eks.cluster_certificate_authority_data
  sensitive = true
}

output "kube_exec_api_version" {
  value = local.kube_exec_api_version
}

output "kube_exec_command" {
  value = "aws"
}

output "kube_exec_args" {
  value = local.kube_exec_args
}

/************************
  AMD GPU stack outputs (new)
*************************/
output "gpu_operator_namespace" {
  value = module.amd_gpu_stack.namespace
}

output "gpu_resource_name" {
  value = module.amd_gpu_stack.gpu_resource_name
}

output "gpu_validation_job" {
  value       = module.amd_gpu_stack.validation_job_name
  description = "kubectl -n <gpu_operator_namespace> logs job/<this> prints the validation JSON (TFLOP/s, HBM GB/s, RCCL busbw)."
}
