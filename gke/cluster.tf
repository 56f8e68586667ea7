# GKE cluster with Workload Identity and two pools: "system" (operator
# controllers, monitoring) and "mi355x". One zone in node_zones makes a zonal
# cluster, several a regional one spread over those zones.
#
# There is no AMD guest_accelerator type on GKE, so the MI355X pool carries
# no accelerator block: the machine shape (gpu_instance_type) brings the
# GPUs, and nodes are labelled / tainted for the AMD GPU stack instead.

data "google_project" "cluster" {
  project_id = var.project_id
}

data "google_container_engine_versions" "latest" {
  provider = google-beta
  project  = var.project_id
  location = var.region
}

resource "terraform_data" "gpu_instance_type_guard" {
  input = var.gpu_instance_type
  lifecycle {
    precondition {
      condition     = var.gpu_instance_type != ""
      error_message = "Set gpu_instance_type to a machine type with AMD Instinct MI355X attached."
    }
  }
}

locals {
  zonal          = length(var.node_zones) == 1
  location       = local.zonal ? one(var.node_zones) : var.region
  node_locations = local.zonal ? null : var.node_zones

  node_scopes = [for s in ["logging.write", "monitoring", "devstorage.read_only", "compute"] :
  "https://www.googleapis.com/auth/${s}"]
  base_labels = { part_of = var.cluster_name, env = var.project_id, managed_by = "terraform" }
  base_tags   = ["tf-managed", var.cluster_name]

  prep_taint_key = "startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep"
}

resource "google_container_cluster" "this" {
  project  = var.project_id
  name     = var.cluster_name
  location = local.location

  network    = local.network_name
  subnetwork = local.subnetwork_name

  release_channel {
    channel = var.release_channel
  }

  # GKE insists on an initial pool; it is dropped once the cluster exists
  initial_node_count       = 1
  remove_default_node_pool = true
  deletion_protection      = false

  dynamic "ip_allocation_policy" {
    for_each = var.vpc_enabled ? ["vpc-native"] : []
    content {
      cluster_secondary_range_name  = local.pods_range_name
      services_secondary_range_name = local.services_range_name
    }
  }

  workload_identity_config {
    workload_pool = "${data.google_project.cluster.project_id}.svc.id.goog"
  }
}

resource "google_container_node_pool" "system" {
  project        = var.project_id
  cluster        = google_container_cluster.this.name
  name           = "tf-${var.cluster_name}-cpu-pool"
  location       = local.location
  node_locations = local.node_locations
  node_count     = var.num_cpu_nodes

  autoscaling {
    min_node_count = var.cpu_min_node_count
    max_node_count = var.cpu_max_node_count
  }

  node_config {
    machine_type = var.cpu_instance_type
    image_type   = "UBUNTU_CONTAINERD"
    disk_size_gb = var.disk_size_gb
    spot         = var.use_cpu_spot_instances
    oauth_scopes = local.node_scopes
    tags         = local.base_tags # the GPU tags stay on the GPU pool
    labels       = merge(local.base_labels, { "node.kubernetes.io/pool" = "cpu" })
    metadata     = { disable-legacy-endpoints = "true" }
    workload_metadata_config {
      mode = "GKE_METADATA"
    }
  }

  timeouts {
    create = "30m"
    update = "20m"
  }
}

resource "google_container_node_pool" "mi355x" {
  project        = var.project_id
  cluster        = google_container_cluster.this.name
  name           = "tf-${var.cluster_name}-gpu-pool"
  location       = local.location
  node_locations = local.node_locations
  node_count     = var.num_gpu_nodes

  autoscaling {
    min_node_count = var.gpu_min_node_count
    max_node_count = var.gpu_max_node_count
  }

  node_config {
    machine_type = var.gpu_instance_type
    image_type   = "UBUNTU_CONTAINERD" # amdgpu-dkms builds against Ubuntu kernel headers
    disk_size_gb = var.disk_size_gb
    spot         = var.use_gpu_spot_instances
    oauth_scopes = local.node_scopes
    tags         = concat(local.base_tags, var.gpu_instance_tags)
    labels = merge(local.base_labels, {
      "node.kubernetes.io/pool" = "gpu"
      "amd.com/gpu.present"     = "true"
      "amd.com/gpu.family"      = "mi355x"
      "amd.com/gpu.arch"        = "gfx950"
      "amd.com/gpu.model"       = var.gpu_type
      "amd.com/gpu.count"       = tostring(var.gpu_count)
    })
    metadata = { disable-legacy-endpoints = "true" }
    taint {
      key    = "amd.com/gpu"
      value  = "present"
      effect = "NO_SCHEDULE"
    }
    # startup taint, removed by the node-prep DaemonSet after a verified prep
    dynamic "taint" {
      for_each = var.gpu_node_prep_taint ? [local.prep_taint_key] : []
      content {
        key    = taint.value
        value  = "pending"
        effect = "NO_SCHEDULE"
      }
    }
    workload_metadata_config {
      mode = "GKE_METADATA"
    }
  }

  timeouts {
    create = "30m"
    update = "20m"
  }

  depends_on = [terraform_data.gpu_instance_type_guard]
}
