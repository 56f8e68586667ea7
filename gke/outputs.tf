# Reference output names first (CNPack's providers read the endpoint and CA
# from here), then the AMD GPU stack.

output "project_id" {
  description = "Project that owns the cluster."
  value       = var.project_id
}

output "region" {
  description = "Region of the cluster and its network."
  value       = var.region
}

output "kubernetes_cluster_name" {
  description = "GKE cluster name."
  value       = google_container_cluster.this.name
}

output "kubernetes_cluster_endpoint_ip" {
  description = "Address of the Kubernetes API (no scheme)."
  value       = google_container_cluster.this.endpoint
}

output "kubernetes_config_file" {
  description = "Base64 CA certificate of the API server, for kubeconfig / providers."
  value       = google_container_cluster.this.master_auth[0].cluster_ca_certificate
  sensitive   = true
}

output "vpc_project" {
  description = "Project of the network this root created (empty list when vpc_enabled = false)."
  value       = google_compute_network.this[*].project
}

output "subnet_cidr_range" {
  description = "Primary range of the created node subnet (list; empty without vpc_enabled)."
  value       = google_compute_subnetwork.nodes[*].ip_cidr_range
}

output "subnet_region" {
  description = "Region of the created node subnet (list; empty without vpc_enabled)."
  value       = google_compute_subnetwork.nodes[*].region
}

output "rapid_channel_latest_gke_version" {
  description = "Newest GKE version offered on the RAPID channel in this region."
  value       = data.google_container_engine_versions.latest.release_channel_latest_version["RAPID"]
}

output "stable_channel_latest_gke_version" {
  description = "Newest GKE version offered on the STABLE channel in this region."
  value       = data.google_container_engine_versions.latest.release_channel_latest_version["STABLE"]
}

output "gpu_operator_namespace" {
  description = "Namespace of the GPU stack and the validation Job."
  value       = module.amd_gpu_stack.namespace
}

output "gpu_validation_job" {
  description = "Name of the validation Job."
  value       = module.amd_gpu_stack.validation_job_name
}
