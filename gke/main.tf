/***************************
VPC Network Configuration
***************************/
resource "google_compute_network" "holoscan-vpc" {
  count                   = var.vpc_enabled ? 1 : 0
  name                    = "${var.cluster_name}-vpc"
  auto_create_subnetworks = false
  project                 = var.project_id
}

/***************************
Subnet Configuration (VPC-native: pod + service secondary ranges)
***************************/
resource "google_compute_subnetwork" "holoscan-subnet" {
  count         = var.vpc_enabled ? 1 : 0
  name          = "${var.cluster_name}-subnet"
  region        = var.region
  network       = google_compute_network.holoscan-vpc[0].name
  ip_cidr_range = var.subnet_cidr_range
  project       = var.project_id

  secondary_ip_range {
    range_name    = "${var.cluster_name}-pods"
    ip_cidr_range = var.pods_cidr_range
  }
  secondary_ip_range {
    range_name    = "${var.cluster_name}-services"
    ip_cidr_range = var.services_cidr_range
  }
}

/***************************
GKE Configuration
***************************/

locals {
  location       = length(var.node_zones) == 1 ? one(var.node_zones) : var.region
  node_locations = length(var.node_zones) > 1 ? var.node_zones : null
  oauth_scopes = [
    "https://www.googleapis.com/auth/logging.write",
    "https://www.googleapis.com/auth/monitoring",
    "https://www.googleapis.com/auth/devstorage.read_only",
    "https://www.googleapis.com/auth/compute",
  ]
  node_labels = {
    part_of    = var.cluster_name
    env        = var.project_id
    managed_by = "terraform"
  }
}

# latest versions per channel, for the version outputs
data "google_container_engine_versions" "latest" {
  provider = google-beta
  location = var.region
  project  = var.project_id
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

resource "google_container_cluster" "holoscan" {
  name     = var.cluster_name
  project  = var.project_id
  location = local.location
  release_channel {
    channel = var.release_channel
  }
  # A default pool is mandatory at creation; it is replaced by the pools below.
  remove_default_node_pool = true
  initial_node_count       = 1
  deletion_protection      = false

  network    = var.vpc_enabled ? google_compute_network.holoscan-vpc[0].name : var.network
  subnetwork = var.vpc_enabled ? google_compute_subnetwork.holoscan-subnet[0].name : var.subnetwork

  dynamic "ip_allocation_policy" {
    for_each = var.vpc_enabled ? [1] : []
    content {
      cluster_secondary_range_name  = "${var.cluster_name}-pods"
      services_secondary_range_name = "${var.cluster_name}-services"
    }
  }

  workload_identity_config {
    workload_pool = "${data.google_project.cluster.project_id}.svc.id.goog"
  }
}

/***************************
GKE CPU Node Pool Config
***************************/
resource "google_container_node_pool" "cpu_nodes" {
  name           = "tf-${var.cluster_name}-cpu-pool"
  project        = var.project_id
  location       = local.location
  node_locations = local.node_locations
  cluster        = google_container_cluster.holoscan.name
  node_count     = var.num_cpu_nodes
  autoscaling {
    min_node_count = var.cpu_min_node_count
    max_node_count = var.cpu_max_node_count
  }
  node_config {
    image_type   = "UBUNTU_CONTAINERD"
    oauth_scopes = local.oauth_scopes
    spot         = var.use_cpu_spot_instances
    machine_type = var.cpu_instance_type
    disk_size_gb = var.disk_size_gb
    # the reference tagged CPU nodes with var.gpu_instance_tags (gke/main.tf:83)
    tags = ["tf-managed", var.cluster_name]
    metadata = {
      disable-legacy-endpoints = "true"
    }
    labels = merge(local.node_labels, { "node.kubernetes.io/pool" = "cpu" })
    workload_metadata_config {
      mode = "GKE_METADATA"
    }
  }
  timeouts {
    create = "30m"
    update = "20m"
  }
}

/***************************
GKE GPU Node Pool Config (AMD Instinct MI355X)
No guest_accelerator: GKE has no AMD accelerator type; the machine shape
carries the GPUs. Nodes are labelled + tainted for the AMD GPU stack.
***************************/
resource "google_container_node_pool" "gpu_nodes" {
  name           = "tf-${var.cluster_name}-gpu-pool"
  project        = var.project_id
  location       = local.location
  node_locations = local.node_locations
  cluster        = google_container_cluster.holoscan.name
  node_count     = var.num_gpu_nodes
  autoscaling {
    min_node_count = var.gpu_min_node_count
    max_node_count = var.gpu_max_node_count
  }
  node_config {
    image_type   = "UBUNTU_CONTAINERD" # amdgpu-dkms needs the Ubuntu kernel headers
    oauth_scopes = local.oauth_scopes
    spot         = var.use_gpu_spot_instances
    machine_type = var.gpu_instance_type
    disk_size_gb = var.disk_size_gb
    tags         = concat(["tf-managed", var.cluster_name], var.gpu_instance_tags)
    metadata = {
      disable-legacy-endpoints = "true"
    }
    labels = merge(local.node_labels, {
      "node.kubernetes.io/pool" = "gpu"
      "amd.com/gpu.present"     = "true"
      "amd.com/gpu.family"      = "mi355x"
      "amd.com/gpu.arch"        = "gfx950"
      "amd.com/gpu.model"       = var.gpu_type
      "amd.com/gpu.count"       = tostring(var.gpu_count)
    })
    taint {
      key    = "amd.com/gpu"
      value  = "present"
      effect = "NO_SCHEDULE"
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

/***************************
AMD GPU stack (namespace + critical-priority ResourceQuota + device plugin /
operator + exporter + validation Job). The quota is required on GKE for
system-*-critical pods outside kube-system (reference gke/main.tf:173-191).
Destroy no longer needs `terraform state rm` (reference gke/README.md:59):
the Job, DaemonSets / CRs and the namespace are all ordered inside the
module and torn down before the node pool and the cluster.
***************************/
module "amd_gpu_stack" {
  source = "../modules/amd-gpu-stack"

  cluster_name                = var.cluster_name
  gpu_stack_mode              = var.gpu_stack_mode
  gpu_operator_version        = var.gpu_operator_version
  gpu_operator_driver_version = var.gpu_operator_driver_version
  gpu_operator_namespace      = var.gpu_operator_namespace
  critical_pod_quota          = true
  gpu_node_selector           = { "amd.com/gpu.present" = "true" }
  gpu_node_pool_ids           = [google_container_node_pool.gpu_nodes.id]
  validation_enabled          = var.gpu_validation_enabled
  validation_image            = var.gpu_validation_image
  validation_gpu_count        = tonumber(var.gpu_count)

  # operator controller needs the CPU pool; only the validation Job (through
  # gpu_node_pool_ids) waits for the GPU pool -> operator install overlaps
  # with MI355X node boot instead of following it.
  depends_on = [google_container_node_pool.cpu_nodes]
}
