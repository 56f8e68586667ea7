# The reference also read data.google_container_cluster with location =
# var.region (wrong for zonal clusters) and never used it
# (/root/reference/gke/data.tf:4-8); dropped.

data "google_client_config" "provider" {}

data "google_project" "cluster" {
  project_id = var.project_id
}
