/*******************************************
AWS Managed Prometheus (AMP) for the AMD GPU metrics
(device-metrics-exporter -> in-cluster Prometheus -> remote_write to AMP)
*******************************************/
// Random suffix: running the example twice in one account must not collide
resource "random_string" "amp" {
  count   = var.amp_enabled ? 1 : 0
  length  = 3
  special = false
  upper   = false
}

resource "aws_cloudwatch_log_group" "cnpack-log-group" {
  count = var.amp_enabled ? 1 : 0
  name  = "cnpack-logs-${random_string.amp[count.index].result}"
}

resource "aws_prometheus_workspace" "cnpack-prom-workspace" {
  count = var.amp_enabled ? 1 : 0
  alias = "cnpack-workspace-${random_string.amp[count.index].result}"

  logging_configuration {
    log_group_arn = "${aws_cloudwatch_log_group.cnpack-log-group[count.index].arn}:*"
  }

  tags = {
    Environment = "non-production"
  }
}

output "amp_remotewrite_endpoint" {
  value = var.amp_enabled ? "${aws_prometheus_workspace.cnpack-prom-workspace[0].prometheus_endpoint}api/v1/remote_write" : null
}

output "amp_query_endpoint" {
  value = var.amp_enabled ? "${aws_prometheus_workspace.cnpack-prom-workspace[0].prometheus_endpoint}api/v1/query" : null
}

resource "aws_iam_policy" "amp-ingest-policy" {
  count       = var.amp_enabled ? 1 : 0
  name        = "aws-amp-remote-write-ingest-policy-${random_string.amp[count.index].result}"
  description = "Policy to connect K8s cluster to AWS AMP"
  policy = jsonencode({
    "Version" : "2012-10-17",
    "Statement" : [
      {
        "Effect" : "Allow",
        "Action" : [
          "aps:RemoteWrite",
          "aps:GetSeries",
          "aps:GetLabels",
          "aps:GetMetricMetadata"
        ],
        "Resource" : "*"
      }
    ]
  })
}

data "aws_caller_identity" "current" {}

// IRSA role for the in-cluster Prometheus service account
resource "aws_iam_role" "amp-ingest-role" {
  count = var.amp_enabled ? 1 : 0
  name  = "amp-ingest-role-${random_string.amp[count.index].result}"
  assume_role_policy = jsonencode({
    "Version" : "2012-10-17",
    "Statement" : [
      {
        "Effect" : "Allow",
        "Principal" : {
          "Federated" : "arn:aws:iam::${data.aws_caller_identity.current.account_id}:oidc-provider/${module.holoscan-eks-cluster.oidc_endpoint}"
        },
        "Action" : "sts:AssumeRoleWithWebIdentity",
        "Condition" : {
          "StringEquals" : {
            "${module.holoscan-eks-cluster.oidc_endpoint}:sub" : "system:serviceaccount:${local.monitoring_namespace}:${local.prometheus_serviceaccount}"
          }
        }
      }
    ]
  })
  tags = {
    managed-by = "terraform"
  }
}

resource "aws_iam_role_policy_attachment" "attach-amp-role-to-policy" {
  count      = var.amp_enabled ? 1 : 0
  role       = aws_iam_role.amp-ingest-role[count.index].name
  policy_arn = aws_iam_policy.amp-ingest-policy[count.index].arn
}

resource "aws_iam_role_policy_attachment" "attach-amp-policy-to-gpu-ng" {
  count      = var.amp_enabled ? 1 : 0
  role       = module.holoscan-eks-cluster.gpu_node_role_name
  policy_arn = aws_iam_policy.amp-ingest-policy[count.index].arn
}

resource "aws_iam_role_policy_attachment" "attach-amp-role-to-cpu-ng" {
  count      = var.amp_enabled ? 1 : 0
  role       = module.holoscan-eks-cluster.cpu_node_role_name
  policy_arn = aws_iam_policy.amp-ingest-policy[count.index].arn
}

// gated on amp_enabled (the reference gated it on pca_enabled: aws-amp.tf:110-112)
output "amp_ingest_role_arn" {
  value = var.amp_enabled ? aws_iam_role.amp-ingest-role[0].arn : null
}
