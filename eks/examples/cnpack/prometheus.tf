# Amazon Managed Service for Prometheus: a workspace with its own log group,
# an ingest policy, and a web-identity role for the in-cluster Prometheus
# (remote_write of the AMD device-metrics-exporter series). The policy also
# goes on both node roles for agents that use the instance profile.

resource "random_string" "amp" {
  count   = var.amp_enabled ? 1 : 0
  length  = 3
  upper   = false
  special = false
}

locals {
  amp_suffix = var.amp_enabled ? random_string.amp[0].result : ""
}

resource "aws_cloudwatch_log_group" "amp" {
  count = var.amp_enabled ? 1 : 0
  name  = "cnpack-logs-${local.amp_suffix}"
}

resource "aws_prometheus_workspace" "amp" {
  count = var.amp_enabled ? 1 : 0
  alias = "cnpack-workspace-${local.amp_suffix}"
  tags  = { Environment = "non-production" }

  logging_configuration {
    log_group_arn = "${aws_cloudwatch_log_group.amp[0].arn}:*"
  }
}

data "aws_iam_policy_document" "amp_ingest" {
  statement {
    sid       = "RemoteWriteAndQuery"
    actions   = ["aps:RemoteWrite", "aps:GetSeries", "aps:GetLabels", "aps:GetMetricMetadata"]
    resources = ["*"]
  }
}

resource "aws_iam_policy" "amp_ingest" {
  count       = var.amp_enabled ? 1 : 0
  name        = "aws-amp-remote-write-ingest-policy-${local.amp_suffix}"
  description = "remote_write + read access to the CNPack AMP workspace"
  policy      = data.aws_iam_policy_document.amp_ingest.json
}

data "aws_iam_policy_document" "prometheus_trust" {
  statement {
    actions = ["sts:AssumeRoleWithWebIdentity"]
    principals {
      type        = "Federated"
      identifiers = ["arn:${data.aws_partition.current.partition}:iam::${data.aws_caller_identity.current.account_id}:oidc-provider/${module.mi355x_eks.oidc_endpoint}"]
    }
    condition {
      test     = "StringEquals"
      variable = "${module.mi355x_eks.oidc_endpoint}:sub"
      values   = ["system:serviceaccount:${local.monitoring_namespace}:${local.prometheus_serviceaccount}"]
    }
  }
}

resource "aws_iam_role" "amp_ingest" {
  count              = var.amp_enabled ? 1 : 0
  name               = "amp-ingest-role-${local.amp_suffix}"
  assume_role_policy = data.aws_iam_policy_document.prometheus_trust.json
  tags               = { managed-by = "terraform" }
}

resource "aws_iam_role_policy_attachment" "amp_ingest_role" {
  count      = var.amp_enabled ? 1 : 0
  role       = aws_iam_role.amp_ingest[0].name
  policy_arn = aws_iam_policy.amp_ingest[0].arn
}

resource "aws_iam_role_policy_attachment" "amp_ingest_nodes" {
  for_each   = var.amp_enabled ? local.node_roles : {}
  role       = each.value
  policy_arn = aws_iam_policy.amp_ingest[0].arn
}
