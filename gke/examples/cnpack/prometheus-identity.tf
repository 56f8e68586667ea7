# Google Managed Prometheus identity: a Google service account allowed to
# write metrics, bound to the Prometheus KSA through Workload Identity.
# The metricWriter grant is a non-authoritative *member*; upstream used an
# authoritative binding, which removes every other holder of the role in
# the whole project.

resource "random_string" "gsa_suffix" {
  for_each = local.prom_enabled
  length   = 3
  upper    = false
  special  = false
}

resource "google_service_account" "prometheus" {
  for_each     = local.prom_enabled
  project      = var.project_id
  account_id   = "amd-prometheus-${random_string.gsa_suffix[each.key].result}"
  display_name = "Prometheus for AMD GPU metrics (CNPack)"
}

resource "google_project_iam_member" "metric_writer" {
  for_each = local.prom_enabled
  project  = var.project_id
  role     = "roles/monitoring.metricWriter"
  member   = google_service_account.prometheus[each.key].member
}

resource "google_service_account_iam_member" "ksa_impersonation" {
  for_each           = local.prom_enabled
  service_account_id = google_service_account.prometheus[each.key].name
  role               = "roles/iam.workloadIdentityUser"
  member             = "serviceAccount:${var.project_id}.svc.id.goog[${local.prom_namespace}/${local.prom_ksa}]"
}

# Registers the pairing with the GKE workload-identity module (both
# accounts already exist; the KSA is annotated by the Helm chart that
# creates it).
module "prometheus_workload_identity" {
  for_each = local.prom_enabled
  source   = "terraform-google-modules/kubernetes-engine/google//modules/workload-identity"
  version  = "~> 33.0"

  project_id          = var.project_id
  namespace           = local.prom_namespace
  k8s_sa_name         = local.prom_ksa
  name                = google_service_account.prometheus[each.key].account_id
  use_existing_gcp_sa = true
  use_existing_k8s_sa = true
  annotate_k8s_sa     = false
}
