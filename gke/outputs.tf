/***************************
Outputs
***************************/

output "region" {
  value       = var.region
  description = "Region the resources of this module are created in"
}

output "project_id" {
  value       = var.project_id
  description = "GCloud Project ID"
}

/***************************
VPC Network Outputs
***************************/

output "vpc_project" {
  value       = google_compute_network.holoscan-vpc[*].project
  description = "Project of the VPC network (can be different from the project launching Kubernetes resources)"
}

output "subnet_cidr_range" {
  value       = google_compute_subnetwork.holoscan-subnet[*].ip_cidr_range
  description = "The IPs and CIDRs of the subnets"
}

output "subnet_region" {
  value       = google_compute_subnetwork.holoscan-subnet[*].region
  description = "The region of the VPC subnet used in this module"
}

/***************************
GKE Outputs
***************************/
output "kubernetes_cluster_name" {
  value       = google_container_cluster.holoscan.name
  description = "MI355X-ready GKE cluster name"
}

output "kubernetes_cluster_endpoint_ip" {
  value       = google_container_cluster.holoscan.endpoint
  description = "GKE Cluster IP Endpoint"
}

output "kubernetes_config_file" {
  value       = google_container_cluster.holoscan.master_auth[0].cluster_ca_certificate
  description = "GKE cluster CA certificate (base64)"
  sensitive   = true
}

output "rapid_channel_latest_gke_version" {
  value       = data.google_container_engine_versions.latest.release_channel_latest_version["RAPID"]
  description = "The latest available version of GKE when using the RAPID channel"
}

output "stable_channel_latest_gke_version" {
  value       = data.google_container_engine_versions.latest.release_channel_latest_version["STABLE"]
  description = "The latest available version of GKE when using the STABLE channel"
}

/***************************
AMD GPU stack outputs (new)
***************************/
output "gpu_operator_namespace" {
  value = module.amd_gpu_stack.namespace
}

output "gpu_validation_job" {
  value = module.amd_gpu_stack.validation_job_name
}
