# Inputs of the AKS root. Names and required-ness (location,
# admin_group_object_ids) follow the reference call surface; wording, types,
# defaults and validation are this module's own.

# --- placement and access ---------------------------------------------------

variable "location" {
  description = "Azure region for the resource group (when created) and the cluster."
  type        = string
}

variable "existing_resource_group_name" {
  description = "Deploy into this resource group instead of creating <cluster_name>-rg."
  type        = string
  default     = null
}

variable "admin_group_object_ids" {
  description = "Object ids (GUIDs, not names or e-mails) of Entra ID groups that become cluster admins. Attaching them requires the Azure Owner role, Contributor is not enough."
  type        = list(any)
}

variable "cluster_name" {
  description = "AKS cluster name and DNS prefix."
  type        = string
  default     = "mi355x-cluster"
}

variable "kubernetes_version" {
  description = "Kubernetes version of the control plane and both pools (see `az aks get-versions -l <location>`)."
  type        = string
  default     = "1.31"
}

# --- system (default) pool ------------------------------------------------

variable "cpu_machine_type" {
  description = "VM size of the system pool."
  type        = string
  default     = "Standard_D16s_v5"
}

variable "cpu_os_sku" {
  description = "Node OS of the system pool (Ubuntu or AzureLinux)."
  type        = string
  default     = "Ubuntu"
}

variable "cpu_node_pool_disk_size" {
  description = "OS disk of each system node in GB."
  type        = number
  default     = 128
}

variable "cpu_node_pool_count" {
  description = "System-pool size at creation."
  type        = number
  default     = 1
}

variable "cpu_node_pool_min_count" {
  description = "Autoscaler floor of the system pool."
  type        = number
  default     = 1
}

variable "cpu_node_pool_max_count" {
  description = "Autoscaler ceiling of the system pool."
  type        = number
  default     = 5
}

# --- MI355X pool ------------------------------------------------------------

variable "gpu_machine_type" {
  description = "VM size with 8 x AMD Instinct MI355X available to your subscription and region; plan stops until it is set."
  type        = string
  default     = ""
}

variable "gpu_os_sku" {
  description = "Node OS of the MI355X pool; must be Ubuntu because amdgpu-dkms builds against its kernel headers."
  type        = string
  default     = "Ubuntu"
  validation {
    condition     = var.gpu_os_sku == "Ubuntu"
    error_message = "The MI355X pool needs gpu_os_sku = \"Ubuntu\" (ROCm 7 amdgpu-dkms)."
  }
}

variable "gpu_node_pool_disk_size" {
  description = "OS disk of each MI355X node in GB (ROCm images are several GB)."
  type        = number
  default     = 1024
}

variable "gpu_node_pool_count" {
  description = "MI355X pool size at creation."
  type        = number
  default     = 1
}

variable "gpu_node_pool_min_count" {
  description = "Autoscaler floor of the MI355X pool."
  type        = number
  default     = 1
}

variable "gpu_node_pool_max_count" {
  description = "Autoscaler ceiling of the MI355X pool."
  type        = number
  default     = 5
}

variable "gpus_per_node" {
  description = "MI355X devices per node; the validation Job requests all of them."
  type        = number
  default     = 8
}

# --- AMD GPU stack and validation ---------------------------------------------

variable "gpu_stack_mode" {
  description = "\"operator\" (AMD GPU Operator + DeviceConfig) or \"daemonsets\" (amdgpu-dkms + rocm/k8s-device-plugin)."
  type        = string
  default     = "operator"
  validation {
    condition     = contains(["operator", "daemonsets"], var.gpu_stack_mode)
    error_message = "Either operator or daemonsets."
  }
}

variable "gpu_operator_version" {
  description = "AMD GPU Operator chart version."
  type        = string
  default     = "v1.3.0"
}

variable "gpu_operator_driver_version" {
  description = "amdgpu / ROCm release the stack installs; AKS images carry no amdgpu driver of their own."
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
