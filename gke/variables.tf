# Inputs of the GKE root. The names (and which are required: project_id,
# region, cluster_name, node_zones) follow the reference call surface; the
# rest - types, defaults, wording, validation - is this module's own.

# --- where -------------------------------------------------------------------

variable "project_id" {
  description = "Project that owns the network, the cluster and its nodes (shared-VPC hosts are not supported)."
  type        = string
}

variable "region" {
  description = "Region of the network and, for multi-zone clusters, of the cluster itself."
  type        = string
}

variable "node_zones" {
  description = "Zones for the node pools, all in `region`. One entry gives a zonal cluster; several give a regional cluster limited to those zones."
  type        = list(any)
  validation {
    condition     = length(var.node_zones) > 0
    error_message = "List at least one zone."
  }
}

variable "cluster_name" {
  description = "Cluster name; also the prefix of the VPC, subnet and pool names."
  type        = string
}

variable "release_channel" {
  description = "GKE release channel that drives control-plane and node upgrades."
  type        = string
  default     = "REGULAR"
  validation {
    condition     = contains(["RAPID", "REGULAR", "STABLE", "UNSPECIFIED"], var.release_channel)
    error_message = "release_channel must be RAPID, REGULAR, STABLE or UNSPECIFIED."
  }
}

# --- network -------------------------------------------------------------------

variable "vpc_enabled" {
  description = "Create a dedicated VPC-native network; false attaches the cluster to `network` / `subnetwork`."
  type        = bool
  default     = true
}

variable "network" {
  description = "Name of an existing VPC (only read when vpc_enabled is false)."
  type        = string
  default     = ""
}

variable "subnetwork" {
  description = "Name of an existing subnet for the nodes (only read when vpc_enabled is false)."
  type        = string
  default     = ""
}

variable "subnet_cidr_range" {
  description = "Node range of the created subnet; a /20 leaves room for growth where a /24 would not."
  type        = string
  default     = "10.150.0.0/20"
}

variable "pods_cidr_range" {
  description = "Secondary range for pod IPs."
  type        = string
  default     = "10.160.0.0/14"
}

variable "services_cidr_range" {
  description = "Secondary range for ClusterIP services."
  type        = string
  default     = "10.150.64.0/20"
}

# --- system pool -----------------------------------------------------------

variable "cpu_instance_type" {
  description = "Machine type of the system pool."
  type        = string
  default     = "n2-standard-8"
}

variable "num_cpu_nodes" {
  description = "System-pool size at creation (per zone for regional clusters)."
  type        = number
  default     = 1
}

variable "cpu_min_node_count" {
  description = "Autoscaler floor of the system pool."
  type        = number
  default     = 1
}

variable "cpu_max_node_count" {
  description = "Autoscaler ceiling of the system pool."
  type        = number
  default     = 5
}

variable "use_cpu_spot_instances" {
  description = "Run the system pool on Spot VMs."
  type        = bool
  default     = false
}

# --- MI355X pool -----------------------------------------------------------

variable "gpu_instance_type" {
  description = "Machine type that brings AMD Instinct MI355X GPUs. GKE publishes no default; plan stops until it is set."
  type        = string
  default     = ""
}

variable "gpu_type" {
  description = "Accelerator model recorded on the nodes as amd.com/gpu.model. GKE has no AMD guest_accelerator type, so no accelerator block is emitted; the machine shape carries the GPUs."
  type        = string
  default     = "amd-instinct-mi355x"
  validation {
    condition     = can(regex("^amd-instinct-mi3[0-9]{2}x?$", var.gpu_type))
    error_message = "Name an AMD Instinct accelerator such as amd-instinct-mi355x; this module provisions AMD GPUs only."
  }
}

variable "gpu_count" {
  description = "MI355X devices per node; the validation Job requests all of them."
  type        = number
  default     = 8
  validation {
    condition     = contains([1, 2, 4, 8], var.gpu_count)
    error_message = "gpu_count must be 1, 2, 4 or 8."
  }
}

variable "num_gpu_nodes" {
  description = "MI355X pool size at creation."
  type        = number
  default     = 1
}

variable "gpu_min_node_count" {
  description = "Autoscaler floor of the MI355X pool."
  type        = number
  default     = 1
}

variable "gpu_max_node_count" {
  description = "Autoscaler ceiling of the MI355X pool."
  type        = number
  default     = 5
}

variable "use_gpu_spot_instances" {
  description = "Run the MI355X pool on Spot VMs."
  type        = bool
  default     = false
}

variable "gpu_instance_tags" {
  description = "Extra network tags for MI355X nodes only (firewall targeting)."
  type        = list(string)
  default     = []
}

variable "disk_size_gb" {
  description = "Boot disk of every node in GB; ROCm images are several GB each."
  type        = number
  default     = 1024
}

# --- AMD GPU stack and validation ---------------------------------------------

variable "gpu_stack_mode" {
  description = "\"daemonsets\" (amdgpu-dkms + rocm/k8s-device-plugin; the default for GKE's Ubuntu nodes) or \"operator\" (AMD GPU Operator + DeviceConfig)."
  type        = string
  default     = "daemonsets"
  validation {
    condition     = contains(["operator", "daemonsets"], var.gpu_stack_mode)
    error_message = "Either operator or daemonsets."
  }
}

variable "gpu_operator_version" {
  description = "AMD GPU Operator chart version (operator mode)."
  type        = string
  default     = "v1.3.0"
}

variable "gpu_operator_driver_version" {
  description = "amdgpu / ROCm release installed on MI355X nodes (7.0 or newer for gfx950)."
  type        = string
  default     = "7.0.2"
}

variable "gpu_operator_namespace" {
  description = "Namespace of the GPU stack, its exporter and the validation Job."
  type        = string
  default     = "kube-amd-gpu"
}

variable "gpu_validation_enabled" {
  description = "Make apply wait for the MI355X validation Job."
  type        = bool
  default     = true
}

variable "gpu_validation_image" {
  description = "Registry path of the image built from validation/image/Dockerfile and pushed where the GPU nodes can pull it. Required while gpu_validation_enabled (no public default)."
  type        = string
  default     = ""
}

variable "gpu_validation_tflops_floor" {
  description = "Fail the Job when any GPU's bf16 GEMM rate drops below this many TFLOP/s."
  type        = number
  default     = 1000
}

variable "gpu_driver_preinstalled" {
  description = "The MI355X node image already ships the amdgpu driver for gfx950: skip the driver install (operator: no KMM build/load; daemonsets: no DKMS DaemonSet) and run only the device plugin + labeller (reference parity: driver.enabled=false, /root/reference/aks/main.tf:89-91). Only for a node image that really has it - the managed images of this cloud do not today (README \"Preinstalled driver\"); the validation Job fails if no GPU comes up."
  type        = bool
  default     = false
}

variable "gpu_node_iommu_passthrough" {
  description = "iommu=pt on the MI355X nodes (xGMI / PCIe peer DMA), applied by the module's node-prep DaemonSet: \"check\" (record whether the node image booted with it), \"reboot\" (add it to GRUB and reboot each node once) or \"off\". The managed node images take no kernel arguments, so \"reboot\" is the only in-cluster lever. WARNING: switching an EXISTING cluster to \"reboot\" reboots every GPU node that lacks iommu=pt at the same moment, without cordon or drain, killing the workloads on them; new nodes are safe (they join behind the gpu_node_prep_taint startup taint, so nothing runs on them yet). Roll it out by replacing nodes (e.g. a new node pool) rather than in place."
  type        = string
  default     = "check"
  validation {
    condition     = contains(["check", "reboot", "off"], var.gpu_node_iommu_passthrough)
    error_message = "gpu_node_iommu_passthrough must be check, reboot or off."
  }
}

variable "gpu_node_prep_taint" {
  type        = bool
  default     = true
  description = "GPU nodes join with the startup taint startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep=pending:NoSchedule, which the node-prep DaemonSet removes once the MI355X host prep is verified on the node (NUMA balancing off, containerd running with LimitMEMLOCK=infinity). The GPU stack tolerates it, the validation Job does not, so the Job never races the prep. A cloud operation that re-applies the taint to a running node is undone by the prep pod's gate reconciler within 30 s, after the same verification."
}
