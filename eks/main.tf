/********************************************
  Network Config
********************************************/
module "vpc" {
  source  = "terraform-aws-modules/vpc/aws"
  version = "~> 5.16"
  count   = var.existing_vpc_details == null ? 1 : 0

  name                    = "tf-${var.cluster_name}-vpc"
  cidr                    = var.cidr_block
  azs                     = slice(data.aws_availability_zones.available.names, 0, length(var.private_subnets))
  private_subnets         = var.private_subnets
  public_subnets          = var.public_subnets
  enable_nat_gateway      = var.enable_nat_gateway
  single_nat_gateway      = var.single_nat_gateway
  enable_dns_support      = var.enable_dns_support
  enable_dns_hostnames    = var.enable_dns_hostnames
  map_public_ip_on_launch = true

  private_subnet_tags = {
    "kubernetes.io/role/internal-elb" = "1"
  }
  public_subnet_tags = {
    "kubernetes.io/role/elb" = "1"
  }
}


/********************************************
  Kubernetes Cluster Configuration
********************************************/

locals {
  vpc_id     = var.existing_vpc_details == null ? module.vpc[0].vpc_id : var.existing_vpc_details.vpc_id
  subnet_ids = var.existing_vpc_details == null ? module.vpc[0].private_subnets : var.existing_vpc_details.subnet_ids

  # node<->node all-protocol: RCCL falls back to TCP between nodes when no
  # RDMA fabric is attached (intra-node traffic rides xGMI and never leaves
  # the host). Same rule set as the reference (eks/main.tf:28-49).
  node_security_group_rules = {
    ingress_self_all = {
      description = "Node to node ingress, no external ingress"
      protocol    = "-1"
      from_port   = 0
      to_port     = 0
      type        = "ingress"
      self        = true
    }

    egress_all = {
      description      = "Node egress to open internet"
      protocol         = "-1"
      from_port        = 0
      to_port          = 0
      type             = "egress"
      cidr_blocks      = ["0.0.0.0/0"]
      ipv6_cidr_blocks = ["::/0"]
    }
  }

  gpu_node_labels = {
    "amd.com/gpu.present"     = "true"
    "amd.com/gpu.family"      = "mi355x"
    "amd.com/gpu.arch"        = "gfx950"
    "node.kubernetes.io/pool" = "gpu"
  }

  # MI355X host tuning appended after the EKS bootstrap on GPU nodes:
  # IOMMU passthrough for xGMI peer DMA, NUMA balancing off (pinned HBM
  # buffers), large locked-memory limit for RCCL, render/video group access.
  gpu_host_tuning = <<-EOT
    #!/bin/bash
    set -eux
    sysctl -w kernel.numa_balancing=0
    echo 'kernel.numa_balancing=0' > /etc/sysctl.d/99-amd-mi355x.conf
    if ! grep -q 'iommu=pt' /etc/default/grub; then
      sed -i 's/^GRUB_CMDLINE_LINUX="/GRUB_CMDLINE_LINUX="iommu=pt /' /etc/default/grub || true
      update-grub || true
    fi
    printf '* soft memlock unlimited\n* hard memlock unlimited\n' > /etc/security/limits.d/99-rccl.conf
  EOT

  common_user_data = var.additional_user_data
  gpu_user_data    = join("\n", compact([local.gpu_host_tuning, local.common_user_data, var.gpu_node_pool_additional_user_data]))
  cpu_user_data    = join("\n", compact([local.common_user_data, var.cpu_node_pool_additional_user_data]))
}

# apply-time guard: there is no public MI355X EC2 default to fall back on
resource "terraform_data" "gpu_instance_type_guard" {
  input = var.gpu_instance_type

  lifecycle {
    precondition {
      condition     = var.gpu_instance_type != ""
      error_message = "Set gpu_instance_type to an EC2 instance type with 8x AMD Instinct MI355X (gfx950)."
    }
  }
}

module "eks" {
  source  = "terraform-aws-modules/eks/aws"
  version = "~> 20.31"

  cluster_name                             = "tf-${var.cluster_name}"
  cluster_version                          = var.cluster_version
  cluster_endpoint_private_access          = true
  cluster_endpoint_public_access           = true
  create_cloudwatch_log_group              = false
  enable_irsa                              = true
  enable_cluster_creator_admin_permissions = true
  vpc_id                                   = local.vpc_id
  subnet_ids                               = local.subnet_ids
  control_plane_subnet_ids                 = local.subnet_ids

  # KMS envelope encryption of Kubernetes secrets
  create_kms_key                  = true
  enable_kms_key_rotation         = true
  kms_key_deletion_window_in_days = 7
  kms_key_enable_default_policy   = true
  cluster_encryption_config = {
    resources = ["secrets"]
  }

  cluster_security_group_additional_rules = {
    egress_nodes_ephemeral_ports_tcp = {
      description                = "Control plane egress to nodes on TCP Ports 1025-65535"
      protocol                   = "tcp"
      from_port                  = 1025
      to_port                    = 65535
      type                       = "egress"
      source_node_security_group = true
    }
  }
  node_security_group_additional_rules = merge(local.node_security_group_rules, var.additional_node_security_groups_rules)

  eks_managed_node_groups = {
    gpu_node_pool = {
      name                       = "tf-gpu"
      instance_types             = [var.gpu_instance_type]
      min_size                   = tonumber(var.min_gpu_nodes)
      max_size                   = tonumber(var.max_gpu_nodes)
      desired_size               = tonumber(var.desired_count_gpu_nodes)
      ami_id                     = local.gpu_ami_id
      ami_type                   = "CUSTOM"
      enable_bootstrap_user_data = true
      post_bootstrap_user_data   = local.gpu_user_data
      vpc_security_group_ids     = var.existing_vpc_details == null ? [] : var.additional_security_group_ids
      key_name                   = var.ssh_key == "" ? null : var.ssh_key
      labels                     = local.gpu_node_labels
      taints = {
        amd_gpu = {
          key    = "amd.com/gpu"
          value  = "present"
          effect = "NO_SCHEDULE"
        }
      }
      block_device_mappings = {
        root = {
          device_name = data.aws_ami.lookup.root_device_name
          ebs = {
            volume_size           = var.gpu_node_pool_root_disk_size_gb
            volume_type           = var.gpu_node_pool_root_volume_type
            delete_on_termination = var.gpu_node_pool_delete_on_termination
          }
        }
      }
      metadata_options = {
        http_endpoint               = "enabled"
        http_tokens                 = "required"
        http_put_response_hop_limit = 2
      }
    },
    cpu_node_pool = {
      name                     = "tf-cpu"
      instance_types           = [var.cpu_instance_type]
      min_size                 = tonumber(var.min_cpu_nodes)
      max_size                 = tonumber(var.max_cpu_nodes)
      desired_size             = tonumber(var.desired_count_cpu_nodes)
      vpc_security_group_ids   = var.existing_vpc_details == null ? [] : var.additional_security_group_ids
      key_name                 = var.ssh_key == "" ? null : var.ssh_key
      post_bootstrap_user_data = local.cpu_user_data
      labels                   = { "node.kubernetes.io/pool" = "cpu" }
      block_device_mappings = {
        root = {
          device_name = "/dev/xvda"
          ebs = {
            volume_size           = var.cpu_node_pool_root_disk_size_gb
            volume_type           = var.cpu_node_pool_root_volume_type
            delete_on_termination = var.cpu_node_pool_delete_on_termination
          }
        }
      }
    }
  }

  cluster_addons = {
    aws-ebs-csi-driver = {
      service_account_role_arn = module.ebs_csi_irsa_role.iam_role_arn
      most_recent              = true
    }
  }

  depends_on = [terraform_data.gpu_instance_type_guard]
}

/********************************************
  IRSA role for the EBS CSI driver
********************************************/
module "ebs_csi_irsa_role" {
  source  = "terraform-aws-modules/iam/aws//modules/iam-role-for-service-accounts-eks"
  version = "~> 5.48"

  role_name             = "${var.cluster_name}-ebs-csi"
  attach_ebs_csi_policy = true
  oidc_providers = {
    cluster = {
      provider_arn               = module.eks.oidc_provider_arn
      namespace_service_accounts = ["kube-system:ebs-csi-controller-sa"]
    }
  }
}

/********************************************
  GPU node AMI: Canonical Ubuntu EKS image (22.04 jammy: ROCm 7 supported)
  The reference computed local.ami_id and never used it, so a user-supplied
  gpu_ami_id fell through to an unfiltered most_recent lookup
  (/root/reference/eks/main.tf:160-180). Fixed: the override wins.
********************************************/
locals {
  ubuntu_ami_lookup = {
    owners = ["099720109477"] # Canonical
    filters = [
      {
        name   = "name"
        values = ["ubuntu-eks/k8s_${var.cluster_version}/images/hvm-ssd*/ubuntu-jammy-22.04-amd64-server-*"]
      },
      {
        name   = "virtualization-type"
        values = ["hvm"]
      }
    ]
  }
  explicit_ami_lookup = {
    owners = []
    filters = [
      {
        name   = "image-id"
        values = [var.gpu_ami_id]
      }
    ]
  }
  ami_lookup = var.gpu_ami_id == "" ? local.ubuntu_ami_lookup : local.explicit_ami_lookup
  gpu_ami_id = var.gpu_ami_id == "" ? data.aws_ami.lookup.id : var.gpu_ami_id
}

/********************************************
  AMD GPU stack: operator (or DKMS + device plugin) + metrics exporter +
  post-provision validation Job. Ordered explicitly after the GPU node group;
  the reference's count gate on data.aws_instances (eks/main.tf:186) never
  waited for anything.
********************************************/
module "amd_gpu_stack" {
  source = "../modules/amd-gpu-stack"

  cluster_name                = var.cluster_name
  gpu_stack_mode              = var.gpu_stack_mode
  gpu_operator_version        = var.gpu_operator_version
  gpu_operator_driver_version = var.gpu_operator_driver_version
  gpu_operator_namespace      = var.gpu_operator_namespace
  gpu_node_selector           = { "amd.com/gpu.present" = "true" }
  gpu_node_pool_ids           = [module.eks.eks_managed_node_groups["gpu_node_pool"].node_group_id]
  validation_enabled          = var.gpu_validation_enabled
  validation_image            = var.gpu_validation_image
  validation_gpu_count        = var.gpus_per_node
  validation_tflops_floor     = var.gpu_validation_tflops_floor

  depends_on = [module.eks]
}
