# EKS control plane + two managed node groups (MI355X and system), secrets
# encrypted with a rotating KMS key, IRSA for the EBS CSI add-on.

# Plan-time stop while no MI355X instance type is configured: there is no
# public default to fall back on, and an empty type would otherwise fail
# deep inside the node-group create.
resource "terraform_data" "gpu_instance_type_guard" {
  input = var.gpu_instance_type
  lifecycle {
    precondition {
      condition     = var.gpu_instance_type != ""
      error_message = "Set gpu_instance_type to an EC2 instance type with 8x AMD Instinct MI355X (gfx950)."
    }
  }
}

locals {
  node_sgs = local.byo_network ? var.additional_security_group_ids : []
  node_key = var.ssh_key == "" ? null : var.ssh_key

  # Host preparation for MI355X nodes, after the EKS bootstrap: IOMMU
  # pass-through for xGMI peer DMA, automatic NUMA balancing off (it
  # migrates pinned HBM staging buffers), unlimited locked memory for RCCL.
  mi355x_host_prep = <<-EOT
    #!/bin/bash
    set -eux
    printf 'kernel.numa_balancing = 0\n' > /etc/sysctl.d/60-mi355x.conf
    sysctl --system
    grep -q 'iommu=pt' /etc/default/grub || {
      sed -i 's/^GRUB_CMDLINE_LINUX="/&iommu=pt /' /etc/default/grub && update-grub || true
    }
    printf '%s\n' '* soft memlock unlimited' '* hard memlock unlimited' > /etc/security/limits.d/60-rccl.conf
  EOT

  pool_base = {
    vpc_security_group_ids = local.node_sgs
    key_name               = local.node_key
    metadata_options = {
      http_endpoint               = "enabled"
      http_tokens                 = "required"
      http_put_response_hop_limit = 2
    }
  }

  gpu_pool = merge(local.pool_base, {
    name                       = "tf-gpu"
    instance_types             = [var.gpu_instance_type]
    min_size                   = var.min_gpu_nodes
    max_size                   = var.max_gpu_nodes
    desired_size               = var.desired_count_gpu_nodes
    ami_type                   = "CUSTOM"
    ami_id                     = local.gpu_ami_id
    enable_bootstrap_user_data = true
    post_bootstrap_user_data = join("\n", compact([
      local.mi355x_host_prep, var.additional_user_data, var.gpu_node_pool_additional_user_data,
    ]))
    labels = {
      "amd.com/gpu.present"     = "true"
      "amd.com/gpu.family"      = "mi355x"
      "amd.com/gpu.arch"        = "gfx950"
      "node.kubernetes.io/pool" = "gpu"
    }
    taints = {
      amd_gpu = { key = "amd.com/gpu", value = "present", effect = "NO_SCHEDULE" }
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
  })

  cpu_pool = merge(local.pool_base, {
    name           = "tf-cpu"
    instance_types = [var.cpu_instance_type]
    min_size       = var.min_cpu_nodes
    max_size       = var.max_cpu_nodes
    desired_size   = var.desired_count_cpu_nodes
    post_bootstrap_user_data = join("\n", compact([
      var.additional_user_data, var.cpu_node_pool_additional_user_data,
    ]))
    labels = { "node.kubernetes.io/pool" = "cpu" }
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
  })
}

module "eks" {
  source  = "terraform-aws-modules/eks/aws"
  version = "~> 20.31"

  cluster_name    = "tf-${var.cluster_name}"
  cluster_version = var.cluster_version

  vpc_id                   = local.vpc_id
  subnet_ids               = local.node_subnets
  control_plane_subnet_ids = local.node_subnets

  cluster_endpoint_public_access           = true
  cluster_endpoint_private_access          = true
  enable_cluster_creator_admin_permissions = true
  enable_irsa                              = true
  create_cloudwatch_log_group              = false

  create_kms_key                  = true
  enable_kms_key_rotation         = true
  kms_key_enable_default_policy   = true
  kms_key_deletion_window_in_days = 7
  cluster_encryption_config       = { resources = ["secrets"] }

  cluster_security_group_additional_rules = {
    to_node_ephemeral = {
      type                       = "egress"
      description                = "API server to kubelets / webhooks on the nodes"
      protocol                   = "tcp"
      from_port                  = 1025
      to_port                    = 65535
      source_node_security_group = true
    }
  }
  node_security_group_additional_rules = merge(local.node_sg_rules, var.additional_node_security_groups_rules)

  eks_managed_node_groups = {
    gpu_node_pool = local.gpu_pool
    cpu_node_pool = local.cpu_pool
  }

  cluster_addons = {
    aws-ebs-csi-driver = {
      most_recent              = true
      service_account_role_arn = module.ebs_csi_irsa_role.iam_role_arn
    }
  }

  depends_on = [terraform_data.gpu_instance_type_guard]
}

# Web-identity role the EBS CSI controller assumes (kube-system SA).
module "ebs_csi_irsa_role" {
  source  = "terraform-aws-modules/iam/aws//modules/iam-role-for-service-accounts-eks"
  version = "~> 5.48"

  role_name             = "${var.cluster_name}-ebs-csi"
  attach_ebs_csi_policy = true
  oidc_providers = {
    this = {
      provider_arn               = module.eks.oidc_provider_arn
      namespace_service_accounts = ["kube-system:ebs-csi-controller-sa"]
    }
  }
}
