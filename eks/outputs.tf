# Outputs. The first eleven keep the reference module's names (CNPack and
# other callers consume them); the last three describe the AMD GPU stack.

data "aws_instances" "nodes" {
  instance_state_names = ["running"]
  filter {
    name   = "tag:aws:autoscaling:groupName"
    values = module.gpu_node_pool.node_group_autoscaling_group_names
  }
}

output "cluster_endpoint" {
  description = "HTTPS endpoint of the Kubernetes API."
  value       = module.eks.cluster_endpoint
}

output "cluster_ca_certificate" {
  description = "Base64 CA bundle of the API server."
  value       = module.eks.cluster_certificate_authority_data
  sensitive   = true
}

output "oidc_endpoint" {
  description = "OIDC issuer (without https://) for IRSA trust policies."
  value       = module.eks.oidc_provider
}

output "gpu_node_role_name" {
  description = "IAM role of the MI355X node group (attach node-level policies here)."
  value       = module.gpu_node_pool.iam_role_name
}

output "cpu_node_role_name" {
  description = "IAM role of the system node group."
  value       = module.cpu_node_pool.iam_role_name
}

output "nodes" {
  description = "Public addresses of the MI355X nodes running now."
  value       = data.aws_instances.nodes.public_ips
}

output "private_subnet_ids" {
  description = "Private subnets this module created (empty list with existing_vpc_details)."
  value       = module.vpc[*].private_subnets
}

output "public_subnet_ids" {
  description = "Public subnets this module created (empty list with existing_vpc_details)."
  value       = module.vpc[*].public_subnets
}

output "kube_exec_command" {
  description = "Program for a kubeconfig exec credential."
  value       = "aws"
}

output "kube_exec_args" {
  description = "Arguments for kube_exec_command (cluster, region, optional profile)."
  value       = local.kube_exec_args
}

output "kube_exec_api_version" {
  description = "client.authentication API version the exec credential speaks - the same one the providers use."
  value       = local.kube_exec_api_version
}

output "gpu_operator_namespace" {
  description = "Namespace of the GPU stack and the validation Job."
  value       = module.amd_gpu_stack.namespace
}

output "gpu_resource_name" {
  description = "Extended resource pods request for MI355X devices."
  value       = module.amd_gpu_stack.gpu_resource_name
}

output "gpu_validation_job" {
  description = "Name of the validation Job (one pod per GPU node); each pod's termination message holds its node's one-line verdict."
  value       = module.amd_gpu_stack.validation_job_name
}
