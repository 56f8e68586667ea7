/***************************
CNPack-equivalent example: MI355X GKE cluster + GKE Managed Prometheus identity
***************************/
module "holoscan-ready-gke" {
  source            = "../../" # or the git URL + tag when running remotely
  cluster_name      = var.cluster_name
  project_id        = var.project_id
  region            = var.region
  node_zones        = var.node_zones
  gpu_instance_type = var.gpu_instance_type
}

locals {
  monitoring_namespace      = "amd-monitoring"
  prometheus_serviceaccount = "amd-prometheus-prometheus"
}
