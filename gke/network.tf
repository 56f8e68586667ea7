# Dedicated VPC-native network (vpc_enabled), or the caller's network and
# subnetwork. The node range is sized by subnet_cidr_range (upstream fixed a
# /24); pods and services get their own secondary ranges.

resource "google_compute_network" "this" {
  count                   = var.vpc_enabled ? 1 : 0
  project                 = var.project_id
  name                    = "${var.cluster_name}-vpc"
  auto_create_subnetworks = false
}

resource "google_compute_subnetwork" "nodes" {
  count         = var.vpc_enabled ? 1 : 0
  project       = var.project_id
  region        = var.region
  name          = "${var.cluster_name}-subnet"
  network       = google_compute_network.this[0].name
  ip_cidr_range = var.subnet_cidr_range

  dynamic "secondary_ip_range" {
    for_each = local.secondary_ranges
    content {
      range_name    = secondary_ip_range.key
      ip_cidr_range = secondary_ip_range.value
    }
  }
}

locals {
  pods_range_name     = "${var.cluster_name}-pods"
  services_range_name = "${var.cluster_name}-services"
  secondary_ranges = {
    (local.pods_range_name)     = var.pods_cidr_range
    (local.services_range_name) = var.services_cidr_range
  }
  network_name    = var.vpc_enabled ? google_compute_network.this[0].name : var.network
  subnetwork_name = var.vpc_enabled ? google_compute_subnetwork.nodes[0].name : var.subnetwork
}
