/*******************************************
GKE Workload Identity for the in-cluster Prometheus (amd-monitoring KSA)
*******************************************/
module "managed-prometheus-workload-identity" {
  count               = var.gke_managed_prometheus_enabled ? 1 : 0
  source              = "terraform-google-modules/kubernetes-engine/google//modules/workload-identity"
  version             = "~> 33.0"
  use_existing_gcp_sa = true
  use_existing_k8s_sa = true
  annotate_k8s_sa     = false
  name                = google_service_account.prometheus_service_account[count.index].account_id
  k8s_sa_name         = local.prometheus_serviceaccount
  namespace           = local.monitoring_namespace
  project_id          = var.project_id
  depends_on          = [google_service_account.prometheus_service_account]
}

/*******************************************
Prometheus Service Account Config
*******************************************/
resource "random_string" "gke" {
  count   = var.gke_managed_prometheus_enabled ? 1 : 0
  length  = 3
  special = false
  upper   = false
}

resource "google_service_account" "prometheus_service_account" {
  count        = var.gke_managed_prometheus_enabled ? 1 : 0
  account_id   = "amd-prometheus-${random_string.gke[count.index].result}"
  display_name = "Prometheus Service Account (AMD GPU metrics)"
  project      = var.project_id
}

# Non-authoritative member grant. The reference used google_project_iam_binding
# (gcp-prometheus.tf:33-38), which is AUTHORITATIVE for the role and strips
# every other metricWriter in the project.
resource "google_project_iam_member" "prometheus_service_account" {
  count   = var.gke_managed_prometheus_enabled ? 1 : 0
  project = var.project_id
  role    = "roles/monitoring.metricWriter"
  member  = "serviceAccount:${google_service_account.prometheus_service_account[count.index].email}"
}

resource "google_service_account_iam_member" "prometheus_service_account" {
  count              = var.gke_managed_prometheus_enabled ? 1 : 0
  service_account_id = google_service_account.prometheus_service_account[count.index].name
  role               = "roles/iam.workloadIdentityUser"
  member             = "serviceAccount:${var.project_id}.svc.id.goog[${local.monitoring_namespace}/${local.prometheus_serviceaccount}]"
}
