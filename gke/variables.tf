# Call surface of /root/reference/gke/variables.tf: all 25 names, required
# ones unchanged (project_id, region, cluster_name, node_zones).

/***************************
GCP Variables
***************************/
variable "project_id" {
  type        = string
  description = "GCP Project ID for the VPC and K8s Cluster. Shared VPC host projects are not supported."
}

variable "region" {
  type        = string
  description = "The Region resources (VPC, GKE, Compute Nodes) will be created in"
}

variable "vpc_enabled" {
  default     = true
  type        = bool
  description = "Create a dedicated VPC + subnet (false: use network/subnetwork)."
}

variable "network" {
  default     = ""
  type        = string
  description = "Existing VPC network name (used when vpc_enabled = false)."
}

variable "subnetwork" {
  type        = string
  default     = ""
  description = "Existing subnet name used for k8s cluster nodes (when vpc_enabled = false)."
}

/***************************
GKE Variables
***************************/

variable "cluster_name" {
  description = "Name of the Kubernetes Cluster to provision"
  type        = string
}

variable "node_zones" {
  description = "Zones for the node pools (same region as above). Exactly one zone = zonal cluster."
  type        = list(any)
}

variable "release_channel" {
  type        = string
  default     = "REGULAR"
  description = "GKE release channel (RAPID, REGULAR, STABLE)."

  validation {
    condition     = contains(["RAPID", "REGULAR", "STABLE", "UNSPECIFIED"], var.release_channel)
    error_message = "release_channel must be RAPID, REGULAR, STABLE or UNSPECIFIED."
  }
}

/***************************
GKE CPU Node Pool Variables
***************************/

variable "cpu_min_node_count" {
  default     = "1"
  description = "Minimum number of CPU nodes in the CPU node pool"
}

variable "cpu_max_node_count" {
  default     = "5"
  description = "Max Number of CPU nodes in CPU nodepool"
}

variable "use_cpu_spot_instances" {
  type        = bool
  default     = false
  description = "Use Spot instances for the CPU pool"
}

variable "cpu_instance_type" {
  default     = "n2-standard-8"
  description = "Machine Type for CPU node pool"
}

variable "num_cpu_nodes" {
  default     = 1
  description = "Number of CPU nodes when pool is created"
}

/***************************
GKE GPU Node Pool Variables
***************************/

variable "gpu_type" {
  type        = string
  default     = "amd-instinct-mi355x"
  description = "Accelerator of the GPU pool. GKE has no AMD guest_accelerator type: AMD Instinct machine shapes bundle their GPUs, so this value only labels the nodes and no guest_accelerator block is emitted."

  validation {
    condition     = can(regex("^amd-instinct-mi3[0-9]{2}x?$", var.gpu_type))
    error_message = "gpu_type must name an AMD Instinct accelerator (e.g. amd-instinct-mi355x); this module provisions AMD GPUs only."
  }
}

variable "gpu_min_node_count" {
  default     = "1"
  description = "Min number of GPU nodes in GPU nodepool"
}

variable "gpu_max_node_count" {
  default     = "5"
  description = "Max Number of GPU nodes in GPU nodepool"
}

variable "use_gpu_spot_instances" {
  type        = bool
  default     = false
  description = "Use Spot instances for the GPU pool"
}

variable "num_gpu_nodes" {
  default     = 1
  description = "Number of GPU nodes when pool is created"
}

variable "gpu_count" {
  default     = "8"
  description = "MI355X GPUs per GPU node (the validation Job requests this many)."

  validation {
    condition     = contains(["1", "2", "4", "8"], tostring(var.gpu_count))
    error_message = "gpu_count must be 1, 2, 4 or 8."
  }
}

variable "gpu_instance_type" {
  type        = string
  default     = ""
  description = "Machine type with AMD Instinct MI355X attached (required for apply; no public GKE default exists)."
}

variable "gpu_instance_tags" {
  type        = list(string)
  default     = []
  description = "Network tags for GPU instance nodes"
}

variable "disk_size_gb" {
  default     = "1024"
  type        = string
  description = "Boot disk size of every node (GB); ROCm images are multi-GB."
}

/***************************
GPU Operator Variables
***************************/

variable "gpu_operator_version" {
  type        = string
  default     = "v1.3.0"
  description = "AMD GPU Operator Helm chart version"
}

variable "gpu_operator_driver_version" {
  type        = string
  default     = "7.0.2"
  description = "amdgpu driver / ROCm release for the GPU nodes (>= 7.0 for gfx950)"
}

variable "gpu_operator_namespace" {
  type        = string
  default     = "kube-amd-gpu"
  description = "The namespace to deploy the AMD GPU stack into"
}

/***************************
New (not in the reference surface)
***************************/
variable "subnet_cidr_range" {
  type        = string
  default     = "10.150.0.0/20"
  description = "Primary range of the created subnet (the reference hard-coded a /24)."
}

variable "pods_cidr_range" {
  type        = string
  default     = "10.160.0.0/14"
  description = "Secondary range for pods (VPC-native cluster)."
}

variable "services_cidr_range" {
  type        = string
  default     = "10.150.64.0/20"
  description = "Secondary range for services."
}

variable "gpu_stack_mode" {
  type        = string
  default     = "daemonsets"
  description = "\"daemonsets\" (amdgpu-dkms + rocm/k8s-device-plugin; default on GKE's Ubuntu images) or \"operator\"."
}

variable "gpu_validation_enabled" {
  type        = bool
  default     = true
  description = "Run the MI355X validation Job and make apply wait for it."
}

variable "gpu_validation_image" {
  type        = string
  default     = "ghcr.io/amd-instinct-terraform-modules/amdgpu-validate:0.1.0"
  description = "Image built from validation/image/Dockerfile."
}
