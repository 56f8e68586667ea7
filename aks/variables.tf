# Call surface of /root/reference/aks/variables.tf: all 18 names; required
# location + admin_group_object_ids unchanged. cpu_os_sku / gpu_os_sku were
# dead in the reference and are wired now.

/****************************
Azure Resource Group Variables
****************************/
variable "existing_resource_group_name" {
  description = "Existing resource group to deploy into; null = create <cluster_name>-rg."
  default     = null
  type        = string
}

variable "location" {
  type        = string
  description = "The region to create resources in"
}

/****************************
AKS Variables
****************************/
variable "cluster_name" {
  type        = string
  default     = "mi355x-cluster"
  description = "The name of the AKS Cluster to be created"
}

variable "kubernetes_version" {
  type        = string
  default     = "1.31"
  description = "Kubernetes version ('az aks get-versions --location <location> --output table' lists them)."
}

variable "cpu_node_pool_disk_size" {
  description = "OS disk size (GB) of the default (CPU) node pool"
  default     = 128
}

variable "cpu_node_pool_count" {
  description = "Initial node count of the default (CPU) pool"
  default     = 1
}

variable "cpu_node_pool_min_count" {
  description = "Min count of nodes in the default (CPU) pool"
  default     = 1
}

variable "cpu_node_pool_max_count" {
  description = "Max count of nodes in the default (CPU) pool"
  default     = 5
}

variable "cpu_machine_type" {
  default     = "Standard_D16s_v5"
  description = "VM size of the AKS CPU node pool"
}

variable "cpu_os_sku" {
  description = "OS SKU of the CPU pool (Ubuntu, AzureLinux)."
  default     = "Ubuntu"
}

/****************************
GPU Node Pool Variables
****************************/
variable "gpu_node_pool_disk_size" {
  description = "OS disk size (GB) of the MI355X GPU pool (ROCm images are multi-GB)"
  default     = 1024
}

variable "gpu_node_pool_count" {
  description = "Initial node count of the GPU pool"
  default     = 1
}

variable "gpu_node_pool_min_count" {
  description = "Min count of nodes in the GPU pool"
  default     = 1
}

variable "gpu_node_pool_max_count" {
  description = "Max count of nodes in the GPU pool"
  default     = 5
}

variable "gpu_machine_type" {
  type        = string
  default     = ""
  description = "VM size with 8x AMD Instinct MI355X (required for apply; set the ND-series MI355X size available in your region/quota)."
}

variable "gpu_os_sku" {
  description = "OS SKU of the GPU pool. Ubuntu: amdgpu-dkms needs the Ubuntu kernel headers."
  default     = "Ubuntu"

  validation {
    condition     = var.gpu_os_sku == "Ubuntu"
    error_message = "The MI355X GPU pool needs gpu_os_sku = \"Ubuntu\" (ROCm 7 amdgpu-dkms)."
  }
}

/****************************
GPU Operator Variables
****************************/
variable "gpu_operator_version" {
  type        = string
  default     = "v1.3.0"
  description = "AMD GPU Operator Helm chart version"
}

/****************************
Active Directory Variables
****************************/
variable "admin_group_object_ids" {
  type        = list(any)
  description = <<EOH
  (Required) A list of Object IDs (GUIDs) of Azure Active Directory Groups which should have Owner Role on the Cluster.
  This is not the email address of the group, the GUID can be found in the Azure panel by searching for the AD Group
  NOTE: You will need Azure "Owner" role (not "Contributor") to attach an AD role to the Kubernetes cluster.
  EOH
}

/****************************
New (not in the reference surface)
****************************/
variable "gpu_operator_driver_version" {
  type        = string
  default     = "7.0.2"
  description = "amdgpu driver / ROCm release for the GPU nodes. AKS node images ship no amdgpu driver, so the stack installs it (the reference's driver.enabled=false relied on a preinstalled NVIDIA driver)."
}

variable "gpu_operator_namespace" {
  type        = string
  default     = "kube-amd-gpu"
  description = "Namespace for the AMD GPU stack (the reference hard-coded its operator namespace)."
}

variable "gpu_stack_mode" {
  type        = string
  default     = "operator"
  description = "\"operator\" or \"daemonsets\"."
}

variable "gpus_per_node" {
  type        = number
  default     = 8
  description = "MI355X GPUs per GPU node (validation Job request)."
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
