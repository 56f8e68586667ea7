# The MI355X EKS cluster, plus the node security-group openings the
# in-cluster observability stack needs: the API server must reach the
# metrics-server (4443) and the prometheus-adapter (6443) on the nodes.

locals {
  api_to_node_ports = {
    metrics_server     = { enabled = var.metrics_server_enabled, port = 4443 }
    prometheus_adapter = { enabled = var.prom_adapter_enabled, port = 6443 }
  }
  api_to_node_rules = {
    for name, p in local.api_to_node_ports : "api_to_${name}" => {
      type                          = "ingress"
      description                   = "API server to ${replace(name, "_", "-")} on the nodes"
      protocol                      = "tcp"
      from_port                     = p.port
      to_port                       = p.port
      source_cluster_security_group = true
    } if p.enabled
  }

  # in-cluster identities the monitoring stack runs as
  monitoring_namespace      = "amd-monitoring"
  prometheus_serviceaccount = "amd-prometheus-prometheus"

  node_roles = {
    gpu = module.mi355x_eks.gpu_node_role_name
    cpu = module.mi355x_eks.cpu_node_role_name
  }
}

module "mi355x_eks" {
  source = "../.."

  cluster_name                          = var.cluster_name
  gpu_instance_type                     = var.gpu_instance_type
  additional_node_security_groups_rules = local.api_to_node_rules
}

data "aws_caller_identity" "current" {}
data "aws_partition" "current" {}
