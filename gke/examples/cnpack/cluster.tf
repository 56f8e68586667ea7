# The MI355X GKE cluster (point `source` at a git tag when running elsewhere).

module "mi355x_gke" {
  source = "../../"

  project_id        = var.project_id
  region            = var.region
  node_zones        = var.node_zones
  cluster_name      = var.cluster_name
  gpu_instance_type = var.gpu_instance_type
}

locals {
  # Kubernetes identity of the in-cluster Prometheus that scrapes the AMD
  # device-metrics exporter and forwards to Google Managed Prometheus
  prom_namespace = "amd-monitoring"
  prom_ksa       = "amd-prometheus-prometheus"
  prom_enabled   = var.gke_managed_prometheus_enabled ? { gmp = true } : {}
}
