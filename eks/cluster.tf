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
  prep_taint_key = "startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep"
  node_sgs       = local.byo_network ? var.additional_security_group_ids : []
  node_key       = var.ssh_key == "" ? null : var.ssh_key

  # Host preparation for MI355X nodes, BEFORE the EKS bootstrap (kubelet and
  # every pod start with it in effect):
  #  * automatic NUMA balancing off - it migrates pinned HBM staging buffers;
  #  * containerd's systemd unit gets LimitMEMLOCK=infinity, so every pod
  #    (RCCL pins host memory) inherits an unlimited RLIMIT_MEMLOCK - a
  #    limits.d file only reaches PAM logins, never containers;
  #  * IOMMU pass-through (iommu=pt) for xGMI / PCIe peer DMA. A kernel
  #    argument only takes effect on a boot: "reboot" adds it and reboots once
  #    before the node joins (cloud-init runs user data once per instance, so a
  #    one-shot unit re-runs it after the reboot; the second pass sees iommu=pt
  #    in /proc/cmdline and proceeds to bootstrap). The reboot happens at most
  #    ONCE per instance: a sentinel is written before it, and a pass that
  #    finds the sentinel but still no iommu=pt (no GRUB_CMDLINE_LINUX line, a
  #    grub.d snippet overriding it, another boot loader) logs a warning and
  #    bootstraps without it instead of rebooting forever; the grub edit is
  #    non-fatal under the script's `set -e`. "image" expects it baked into
  #    gpu_ami_id and only records what the kernel booted with; "off" leaves
  #    it alone. The validation Job re-checks the result from inside the pod
  #    (amdgpu-validate --require-host-prep).
  # (Inlined into the node group's bootstrap script, which already runs
  # under `set -e`: no shebang, no shell options of its own.)
  mi355x_host_prep = <<-EOT
    mode="${var.gpu_node_iommu_passthrough}"
    sentinel=/var/lib/mi355x-iommu-rebooted
    if [ "$mode" = "reboot" ] && ! grep -qw 'iommu=pt' /proc/cmdline && [ -f "$sentinel" ]; then
      echo "mi355x: WARNING iommu=pt still absent after one reboot; bootstrapping without it" >&2
      mode="reboot-failed"
    fi
    if [ "$mode" = "reboot" ] && ! grep -qw 'iommu=pt' /proc/cmdline; then
      { grep -q 'iommu=pt' /etc/default/grub ||
          sed -i 's/^GRUB_CMDLINE_LINUX="/&iommu=pt /' /etc/default/grub; } || true
      update-grub || echo "mi355x: WARNING update-grub failed" >&2
      mkdir -p /var/lib && touch "$sentinel"
      cat > /etc/systemd/system/mi355x-userdata-rerun.service <<'UNIT'
    [Unit]
    Description=Re-run EC2 user data once after the iommu=pt reboot
    After=cloud-final.service
    [Service]
    Type=oneshot
    ExecStartPre=/bin/systemctl disable mi355x-userdata-rerun.service
    ExecStart=/usr/bin/cloud-init single --name scripts_user --frequency always
    [Install]
    WantedBy=multi-user.target
    UNIT
      systemctl enable mi355x-userdata-rerun.service
      systemctl reboot
      exit 0
    fi
    echo "mi355x: iommu mode=$mode cmdline: $(cat /proc/cmdline)" > /var/log/mi355x-host-prep.log
    printf 'kernel.numa_balancing = 0\n' > /etc/sysctl.d/60-mi355x.conf
    sysctl --system
    mkdir -p /etc/systemd/system/containerd.service.d
    printf '[Service]\nLimitMEMLOCK=infinity\n' > /etc/systemd/system/containerd.service.d/60-memlock.conf
    systemctl daemon-reload
    systemctl restart containerd
  EOT

  # Node groups live OUTSIDE module "eks" (the eks-managed-node-group
  # submodule): the GPU stack then depends on the control plane + system
  # pool only, and installs while the MI355X nodes boot. Inside module "eks"
  # every dependent of the module waited for the GPU node group too.
  node_group_common = {
    cluster_name                      = module.eks.cluster_name
    cluster_version                   = module.eks.cluster_version
    cluster_endpoint                  = module.eks.cluster_endpoint
    cluster_auth_base64               = module.eks.cluster_certificate_authority_data
    cluster_service_cidr              = module.eks.cluster_service_cidr
    cluster_primary_security_group_id = module.eks.cluster_primary_security_group_id
    subnet_ids                        = local.node_subnets
    vpc_security_group_ids            = concat([module.eks.node_security_group_id], local.node_sgs)
    key_name                          = local.node_key
    metadata_options = {
      http_endpoint               = "enabled"
      http_tokens                 = "required"
      http_put_response_hop_limit = 2
    }
  }
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

  depends_on = [terraform_data.gpu_instance_type_guard]
}

module "gpu_node_pool" {
  source  = "terraform-aws-modules/eks/aws//modules/eks-managed-node-group"
  version = "~> 20.31"

  name = "tf-gpu"

  cluster_name                      = local.node_group_common.cluster_name
  cluster_version                   = local.node_group_common.cluster_version
  cluster_endpoint                  = local.node_group_common.cluster_endpoint
  cluster_auth_base64               = local.node_group_common.cluster_auth_base64
  cluster_service_cidr              = local.node_group_common.cluster_service_cidr
  cluster_primary_security_group_id = local.node_group_common.cluster_primary_security_group_id
  subnet_ids                        = local.node_group_common.subnet_ids
  vpc_security_group_ids            = local.node_group_common.vpc_security_group_ids
  key_name                          = local.node_group_common.key_name
  metadata_options                  = local.node_group_common.metadata_options

  instance_types             = [var.gpu_instance_type]
  min_size                   = var.min_gpu_nodes
  max_size                   = var.max_gpu_nodes
  desired_size               = var.desired_count_gpu_nodes
  ami_type                   = "CUSTOM"
  ami_id                     = local.gpu_ami_id
  enable_bootstrap_user_data = true
  pre_bootstrap_user_data    = local.mi355x_host_prep
  post_bootstrap_user_data = join("\n", compact([
    var.additional_user_data, var.gpu_node_pool_additional_user_data,
  ]))

  labels = {
    "amd.com/gpu.present"     = "true"
    "amd.com/gpu.family"      = "mi355x"
    "amd.com/gpu.arch"        = "gfx950"
    "node.kubernetes.io/pool" = "gpu"
  }
  # + the startup taint the node-prep DaemonSet removes once the host prep is
  # verified on the node (the validation Job does not tolerate it)
  taints = merge({
    amd_gpu = { key = "amd.com/gpu", value = "present", effect = "NO_SCHEDULE" }
    }, var.gpu_node_prep_taint ? {
    mi355x_prep = { key = local.prep_taint_key, value = "pending", effect = "NO_SCHEDULE" }
  } : {})
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
}

module "cpu_node_pool" {
  source  = "terraform-aws-modules/eks/aws//modules/eks-managed-node-group"
  version = "~> 20.31"

  name = "tf-cpu"

  cluster_name                      = local.node_group_common.cluster_name
  cluster_version                   = local.node_group_common.cluster_version
  cluster_service_cidr              = local.node_group_common.cluster_service_cidr
  cluster_primary_security_group_id = local.node_group_common.cluster_primary_security_group_id
  subnet_ids                        = local.node_group_common.subnet_ids
  vpc_security_group_ids            = local.node_group_common.vpc_security_group_ids
  key_name                          = local.node_group_common.key_name
  metadata_options                  = local.node_group_common.metadata_options

  instance_types = [var.cpu_instance_type]
  min_size       = var.min_cpu_nodes
  max_size       = var.max_cpu_nodes
  desired_size   = var.desired_count_cpu_nodes
  # EKS-optimized AMI: the module merges only a pre-bootstrap hook into its
  # user data (post_bootstrap_user_data would be silently dropped).
  pre_bootstrap_user_data = join("\n", compact([
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
}

# EBS CSI add-on: a standalone resource after the system pool (its controller
# must schedule somewhere; inside module "eks" it would be created before any
# node exists now that the node groups live outside the module).
resource "aws_eks_addon" "ebs_csi" {
  cluster_name                = module.eks.cluster_name
  addon_name                  = "aws-ebs-csi-driver"
  service_account_role_arn    = module.ebs_csi_irsa_role.iam_role_arn
  resolve_conflicts_on_create = "OVERWRITE"
  resolve_conflicts_on_update = "OVERWRITE"

  depends_on = [module.cpu_node_pool]
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

# Deployments created before the node groups and the EBS CSI add-on left
# module "eks" (round 2) keep their objects with a one-time `terraform state
# mv` (eks/README.md "Upgrading"). A `moved` block cannot do it: module "eks"
# is a registry package, and Terraform rejects moves across module packages
# at plan time (tfcheck rule moved-cross-package).

# A preinstalled driver can only come from a pinned image: the default lookup
# (newest Canonical EKS Ubuntu) has no amdgpu, and the stack would then wait
# out validation_timeout for GPUs that never appear.
resource "terraform_data" "driver_preinstalled_guard" {
  input = var.gpu_driver_preinstalled
  lifecycle {
    precondition {
      condition     = !var.gpu_driver_preinstalled || var.gpu_ami_id != ""
      error_message = "gpu_driver_preinstalled = true needs gpu_ami_id: an AMI with the amdgpu driver for gfx950 baked in (README \"Preinstalled driver\")."
    }
  }
}
