# Inputs of the EKS root. Names and required-ness follow the reference module's
# call surface (pinned by tests/fixtures/reference_surface.json); descriptions,
# types, defaults and validation are this module's own. Sections:
#   1 identity   2 network   3 MI355X pool   4 CPU pool   5 node bootstrap
#   6 AMD GPU stack   7 validation Job

# --- 1 identity ------------------------------------------------------------

variable "cluster_name" {
  description = "Short name of the cluster. The control plane becomes tf-<name>; node groups, VPC and IAM roles derive their names from it."
  type        = string
  nullable    = false
  validation {
    condition     = can(regex("^[a-z][a-z0-9-]{0,30}$", var.cluster_name))
    error_message = "Use 1-31 lowercase letters, digits or dashes, starting with a letter."
  }
}

variable "region" {
  description = "Region for every AWS resource and for the token command of the kube providers."
  type        = string
  default     = "us-west-2"
}

variable "aws_profile" {
  description = "Named AWS CLI profile used by the provider and by `aws eks get-token`; leave empty for the default credential chain."
  type        = string
  default     = ""
}

variable "cluster_version" {
  description = "Kubernetes minor version of the control plane; it also picks the matching Ubuntu EKS image for MI355X nodes."
  type        = string
  default     = "1.31"
  validation {
    condition     = can(regex("^1\\.[0-9]{2}$", var.cluster_version))
    error_message = "Expected a Kubernetes minor version such as 1.31."
  }
}

# --- 2 network ---------------------------------------------------------------

variable "existing_vpc_details" {
  description = "Bring-your-own network: the VPC id and the private subnets the nodes go into. Null creates a fresh VPC."
  type = object({
    vpc_id     = string
    subnet_ids = list(string)
  })
  default = null
}

variable "cidr_block" {
  description = "Address space of the VPC this module creates."
  type        = string
  default     = "10.0.0.0/16"
  validation {
    condition     = can(cidrhost(var.cidr_block, 0))
    error_message = "cidr_block must be an IPv4 CIDR."
  }
}

variable "private_subnets" {
  description = "One private range per availability zone. MI355X nodes and the control-plane ENIs live here."
  type        = list(any)
  default     = ["10.0.0.0/19", "10.0.32.0/19", "10.0.64.0/19"]
}

variable "public_subnets" {
  description = "One public range per availability zone, for NAT gateways and load balancers."
  type        = list(any)
  default     = ["10.0.96.0/22", "10.0.100.0/22", "10.0.104.0/22"]
}

variable "enable_nat_gateway" {
  description = "Give the private subnets outbound internet through NAT (image pulls, driver downloads)."
  type        = bool
  default     = true
}

variable "single_nat_gateway" {
  description = "One shared NAT gateway instead of one per zone: cheaper, but a zone outage cuts egress for all."
  type        = bool
  default     = false
}

variable "enable_dns_support" {
  description = "Amazon-provided DNS resolution inside the new VPC."
  type        = bool
  default     = true
}

variable "enable_dns_hostnames" {
  description = "Public DNS hostnames for instances of the new VPC."
  type        = bool
  default     = true
}

variable "additional_security_group_ids" {
  description = "Extra security groups for every node when an existing VPC is reused."
  type        = list(any)
  default     = []
}

variable "additional_node_security_groups_rules" {
  description = "Rules merged into the node security group, e.g. the metrics-server / prometheus-adapter ports of the CNPack example."
  type        = any
  default     = {}
}

# --- 3 MI355X node group ---------------------------------------------------------

variable "gpu_instance_type" {
  description = "EC2 type that carries 8 x AMD Instinct MI355X (gfx950, 288 GB HBM3E per GPU). No public default exists: name the type of your capacity reservation; plan stops with a clear message while it is empty."
  type        = string
  default     = ""
  validation {
    condition     = var.gpu_instance_type == "" || can(regex("^[a-z0-9-]+\\.[a-z0-9]+$", var.gpu_instance_type))
    error_message = "Expected an EC2 type of the form family.size."
  }
}

variable "gpu_ami_id" {
  description = "Pin the MI355X node image. Empty: newest Canonical Ubuntu EKS image for cluster_version (ROCm 7 requires 22.04 or 24.04). Anything else is used verbatim."
  type        = string
  default     = ""
}

variable "min_gpu_nodes" {
  description = "Autoscaling floor of the MI355X group."
  type        = number
  default     = 1
  validation {
    condition     = var.min_gpu_nodes >= 0
    error_message = "Cannot be negative."
  }
}

variable "max_gpu_nodes" {
  description = "Autoscaling ceiling of the MI355X group."
  type        = number
  default     = 5
}

variable "desired_count_gpu_nodes" {
  description = "Initial size of the MI355X group (ignored by Terraform after creation, owned by the autoscaler)."
  type        = number
  default     = 1
}

variable "gpu_node_pool_root_disk_size_gb" {
  description = "Root volume of each MI355X node in GB: ROCm images are several GB each and DKMS keeps kernel build trees."
  type        = number
  default     = 1024
  validation {
    condition     = var.gpu_node_pool_root_disk_size_gb >= 256
    error_message = "Below 256 GB the ROCm images and DKMS trees do not fit."
  }
}

variable "gpu_node_pool_root_volume_type" {
  description = "EBS class of the MI355X root volumes."
  type        = string
  default     = "gp3"
}

variable "gpu_node_pool_delete_on_termination" {
  description = "Remove MI355X root volumes together with their instances."
  type        = bool
  default     = true
}

variable "gpu_node_pool_additional_user_data" {
  description = "Shell run on MI355X nodes after the EKS bootstrap and the built-in host tuning."
  type        = string
  default     = ""
}

# --- 4 CPU node group ------------------------------------------------------

variable "cpu_instance_type" {
  description = "EC2 type of the system pool (operator controllers, CoreDNS, monitoring)."
  type        = string
  default     = "m7i.2xlarge"
}

variable "min_cpu_nodes" {
  description = "Autoscaling floor of the system pool."
  type        = number
  default     = 0
}

variable "max_cpu_nodes" {
  description = "Autoscaling ceiling of the system pool."
  type        = number
  default     = 2
}

variable "desired_count_cpu_nodes" {
  description = "Initial size of the system pool."
  type        = number
  default     = 1
}

variable "cpu_node_pool_root_disk_size_gb" {
  description = "Root volume of each system node in GB."
  type        = number
  default     = 512
}

variable "cpu_node_pool_root_volume_type" {
  description = "EBS class of the system-node root volumes."
  type        = string
  default     = "gp3"
}

variable "cpu_node_pool_delete_on_termination" {
  description = "Remove system-node root volumes together with their instances."
  type        = bool
  default     = true
}

variable "cpu_node_pool_additional_user_data" {
  description = "Shell run on system nodes before the EKS bootstrap (EKS-optimized AMIs run only a pre-bootstrap hook)."
  type        = string
  default     = ""
}

# --- 5 node bootstrap ------------------------------------------------------

variable "additional_user_data" {
  description = "Shell run on every node, before the pool-specific snippets (MI355X nodes: after the EKS bootstrap; system nodes: before it)."
  type        = string
  default     = ""
}

variable "ssh_key" {
  description = "EC2 key pair for SSH to the nodes; empty disables remote access."
  type        = string
  default     = ""
}

# --- 6 AMD GPU stack ----------------------------------------------------------

variable "gpu_stack_mode" {
  description = "How the GPUs are enabled: \"operator\" = AMD GPU Operator with a DeviceConfig, \"daemonsets\" = amdgpu-dkms installer + rocm/k8s-device-plugin without an operator."
  type        = string
  default     = "operator"
  validation {
    condition     = contains(["operator", "daemonsets"], var.gpu_stack_mode)
    error_message = "Either operator or daemonsets."
  }
}

variable "gpu_operator_version" {
  description = "Chart version of the AMD GPU Operator."
  type        = string
  default     = "v1.3.0"
}

variable "gpu_operator_driver_version" {
  description = "amdgpu / ROCm release the operator (or the DKMS DaemonSet) installs; gfx950 needs 7.0 or newer."
  type        = string
  default     = "7.0.2"
}

variable "gpu_operator_namespace" {
  description = "Namespace holding the GPU stack, its exporter and the validation Job."
  type        = string
  default     = "kube-amd-gpu"
}

variable "gpus_per_node" {
  description = "MI355X devices per node; the validation Job asks for all of them."
  type        = number
  default     = 8
}

# --- 7 validation Job ---------------------------------------------------------

variable "gpu_validation_enabled" {
  description = "Gate apply on the MI355X validation Job (bf16 MFMA GEMM with ABFT, HBM stream, RCCL / xGMI all-reduce)."
  type        = bool
  default     = true
}

variable "gpu_node_iommu_passthrough" {
  description = "How MI355X nodes get iommu=pt (xGMI / PCIe peer DMA): \"reboot\" (add it, reboot once before joining), \"image\" (already in gpu_ami_id's kernel command line), or \"off\"."
  type        = string
  default     = "reboot"
  validation {
    condition     = contains(["reboot", "image", "off"], var.gpu_node_iommu_passthrough)
    error_message = "gpu_node_iommu_passthrough must be reboot, image or off."
  }
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
  description = "The MI355X node image (gpu_ami_id) already ships the amdgpu driver for gfx950: skip the driver install (operator: no KMM build/load; daemonsets: no DKMS DaemonSet) and run only the device plugin + labeller - the biggest in-cluster phase of time-to-GPU-ready (reference parity: driver.enabled=false, /root/reference/aks/main.tf:89-91). Requires gpu_ami_id; how to bake the driver: README \"Preinstalled driver\"."
  type        = bool
  default     = false
}

variable "gpu_node_prep_taint" {
  type        = bool
  default     = true
  description = "GPU nodes join with the startup taint startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep=pending:NoSchedule, which the node-prep DaemonSet removes once the MI355X host prep is verified on the node (NUMA balancing off, containerd running with LimitMEMLOCK=infinity). The GPU stack tolerates it, the validation Job does not, so the Job never races the prep. A cloud operation that re-applies the taint to a running node is undone by the prep pod's gate reconciler within 30 s, after the same verification."
}
