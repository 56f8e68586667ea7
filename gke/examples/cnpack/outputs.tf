output "gcp_service_account_email_for_prometheus" {
  description = "Annotate the Prometheus KSA with this (iam.gke.io/gcp-service-account); null when disabled."
  value       = var.gke_managed_prometheus_enabled ? google_service_account.prometheus["gmp"].email : null
}

output "gpu_validation_job" {
  description = "Validation Job of the cluster's AMD GPU stack."
  value       = module.mi355x_gke.gpu_validation_job
}
