output "amp_remotewrite_endpoint" {
  description = "Prometheus remote_write URL of the AMP workspace (null with amp_enabled = false)."
  value       = var.amp_enabled ? "${aws_prometheus_workspace.amp[0].prometheus_endpoint}api/v1/remote_write" : null
}

output "amp_query_endpoint" {
  description = "PromQL query URL of the AMP workspace."
  value       = var.amp_enabled ? "${aws_prometheus_workspace.amp[0].prometheus_endpoint}api/v1/query" : null
}

output "amp_ingest_role_arn" {
  description = "Role the Prometheus service account assumes; null unless amp_enabled (upstream keyed this on pca_enabled)."
  value       = var.amp_enabled ? aws_iam_role.amp_ingest[0].arn : null
}

output "aws_pca_arn" {
  description = "ARN of the private root CA for the AWSPCAClusterIssuer."
  value       = var.pca_enabled ? aws_acmpca_certificate_authority.ca["root"].arn : null
}
