# Call surface of the reference EKS module (/root/reference/eks/variables.tf),
# every name kept; defaults moved to MI355X values; previously dead variables
# (aws_profile, region, cpu_node_pool_additional_user_data,
# additional_user_data, enable_dns_support) are now wired.

/************************
  AWS Variables
*************************/

variable "aws_profile" {
  type        = string
  default     = ""
  description = "AWS CLI profile for the provider and the kube exec token (empty = default credential chain)."
}

variable "region" {
  type        = string
  default     = "us-west-2"
  description = "AWS region to provision the MI355X-ready Kubernetes cluster in."
}


/************************
  EKS Variables
*************************/

variable "cluster_name" {
  type        = string
  description = "Cluster name; the EKS control plane is named tf-<cluster_name>."
}

variable "cluster_version" {
  type        = string
  default     = "1.31"
  description = "EKS Kubernetes version (major.minor). Also selects the Ubuntu EKS AMI for GPU nodes."
}

/************************
  GPU Operator Variables (AMD GPU Operator)
*************************/
variable "gpu_operator_version" {
  type        = string
  default     = "v1.3.0"
  description = "AMD GPU Operator Helm chart version."
}

variable "gpu_operator_driver_version" {
  type        = string
  default     = "7.0.2"
  description = "amdgpu driver / ROCm release installed on GPU nodes (>= 7.0 for gfx950)."
}

variable "gpu_operator_namespace" {
  type        = string
  default     = "kube-amd-gpu"
  description = "Namespace for the AMD GPU stack and the validation Job."
}

/*****************************
  Managed Node Pool Variables
******************************/

/******************************
  GPU-only Node Pool Variables
*******************************/
variable "gpu_ami_id" {
  type        = string
  description = "AMI for the GPU nodes. Empty = look up the Canonical Ubuntu EKS image for cluster_version (ROCm 7 needs Ubuntu 22.04/24.04). A non-empty value is used as-is."
  default     = ""
}

variable "gpu_instance_type" {
  type        = string
  default     = ""
  description = "EC2 instance type with 8x AMD Instinct MI355X (gfx950, 288 GB HBM3E each). Required for apply: there is no public default, set the type of your capacity reservation."

  validation {
    condition     = var.gpu_instance_type == "" || can(regex("^[a-z0-9-]+\\.[a-z0-9]+$", var.gpu_instance_type))
    error_message = "gpu_instance_type must look like an EC2 instance type (family.size)."
  }
}

variable "max_gpu_nodes" {
  type        = string
  default     = "5"
  description = "Maximum number of GPU nodes in the Autoscaling Group"
}

variable "min_gpu_nodes" {
  type        = string
  default     = "1"
  description = "Minimum number of GPU nodes in the Autoscaling Group"
}

variable "desired_count_gpu_nodes" {
  type        = string
  default     = "1"
  description = "Desired number of GPU nodes in the Autoscaling Group"
}

variable "gpu_node_pool_root_disk_size_gb" {
  type        = number
  default     = 1024
  description = "Root disk size of GPU nodes (ROCm container images are multi-GB; 8-GPU nodes pull several)."

  validation {
    condition     = var.gpu_node_pool_root_disk_size_gb >= 256
    error_message = "GPU node root disks below 256 GB cannot hold ROCm images + DKMS build trees."
  }
}

variable "gpu_node_pool_root_volume_type" {
  type        = string
  default     = "gp3"
  description = "EBS volume type of the GPU node root disk."
}

variable "gpu_node_pool_delete_on_termination" {
  type        = bool
  default     = true
  description = "Delete the GPU nodes' root volumes on termination."
}

variable "gpu_node_pool_additional_user_data" {
  type        = string
  default     = ""
  description = "Shell appended after the EKS bootstrap (and after the MI355X host tuning) on GPU nodes."
}

/************************
  CPU-only Node Pool Variables
*************************/

variable "cpu_instance_type" {
  type        = string
  default     = "m7i.2xlarge"
  description = "CPU EC2 worker node instance type"
}

variable "cpu_node_pool_root_disk_size_gb" {
  type        = number
  default     = 512
  description = "Root disk size of CPU nodes."
}

variable "cpu_node_pool_root_volume_type" {
  type        = string
  default     = "gp3"
  description = "EBS volume type of the CPU node root disk."
}

variable "cpu_node_pool_delete_on_termination" {
  type        = bool
  default     = true
  description = "Delete the CPU nodes' root volumes on termination."
}

variable "cpu_node_pool_additional_user_data" {
  type        = string
  default     = ""
  description = "Shell appended after the EKS bootstrap on CPU nodes."
}

variable "max_cpu_nodes" {
  type        = string
  default     = "2"
  description = "Maximum number of CPU nodes in the Autoscaling Group"
}

variable "min_cpu_nodes" {
  type        = string
  default     = "0"
  description = "Minimum number of CPU nodes in the Autoscaling Group"
}

variable "desired_count_cpu_nodes" {
  type        = string
  default     = "1"
  description = "Desired number of CPU nodes in the Autoscaling Group"
}


/************************
  VPC Variables
*************************/

variable "existing_vpc_details" {
  type = object({
    vpc_id     = string
    subnet_ids = list(string)
  })
  default     = null
  description = "Re-use an existing VPC (vpc_id + private subnet_ids) instead of creating one."
}

variable "cidr_block" {
  type        = string
  default     = "10.0.0.0/16"
  description = "CIDR for VPC"
}

variable "additional_user_data" {
  type        = string
  default     = ""
  description = "Shell appended after the EKS bootstrap on ALL node pools (before the pool-specific additions)."
}

variable "private_subnets" {
  type        = list(any)
  description = "Private subnet ranges (one per AZ); GPU nodes live here."
  default     = ["10.0.0.0/19", "10.0.32.0/19", "10.0.64.0/19"]
}

variable "public_subnets" {
  type        = list(any)
  description = "Public subnet ranges (one per AZ)."
  default     = ["10.0.96.0/22", "10.0.100.0/22", "10.0.104.0/22"]
}

variable "ssh_key" {
  type        = string
  default     = ""
  description = "EC2 key pair name for node SSH access (empty = none)."
}

variable "enable_nat_gateway" {
  description = "Should be true if you want to provision NAT Gateways for each of your private networks"
  default     = true
  type        = bool
}

variable "single_nat_gateway" {
  type        = bool
  description = "Should be true if you want to provision a single shared NAT Gateway across all of your private networks"
  default     = false
}

variable "enable_dns_support" {
  type        = bool
  default     = true
  description = "Enable DNS support in the created VPC."
}

variable "enable_dns_hostnames" {
  description = "Whether or not the created VPC has DNS hostname support"
  default     = true
  type        = bool
}

variable "additional_security_group_ids" {
  type        = list(any)
  default     = []
  description = "Additional security groups attached to nodes (only when re-using a VPC)."
}

variable "additional_node_security_groups_rules" {
  description = "Additional rules merged into the node security group (CNPack hook)."
  type        = any
  default     = {}
}

/************************
  AMD GPU stack (new; not in the reference surface)
*************************/
variable "gpu_stack_mode" {
  type        = string
  default     = "operator"
  description = "\"operator\" (AMD GPU Operator + DeviceConfig) or \"daemonsets\" (amdgpu-dkms + rocm/k8s-device-plugin)."
}

variable "gpu_validation_enabled" {
  type        = bool
  default     = true
  description = "Run the MI355X validation Job (HIP GEMM + HBM + RCCL all-reduce) and make apply wait for it."
}

variable "gpu_validation_image" {
  type        = string
  default     = "ghcr.io/amd-instinct-terraform-modules/amdgpu-validate:0.1.0"
  description = "Image built from validation/image/Dockerfile."
}

variable "gpus_per_node" {
  type        = number
  default     = 8
  description = "MI355X GPUs per GPU node (the validation Job requests all of them)."
}

variable "gpu_validation_tflops_floor" {
  type        = number
  default     = 1000
  description = "Per-GPU bf16 GEMM TFLOP/s floor of the validation Job."
}
