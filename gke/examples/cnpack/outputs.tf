/*******************************************
CNPack-equivalent Example Outputs
*******************************************/
output "gcp_service_account_email_for_prometheus" {
  value = var.gke_managed_prometheus_enabled ? google_service_account.prometheus_service_account[0].email : null
}

output "gpu_validation_job" {
  value = module.holoscan-ready-gke.gpu_validation_job
}
