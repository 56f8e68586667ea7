# Fluent Bit ships container logs to CloudWatch with the node credentials:
# CloudWatchAgentServerPolicy on BOTH node roles (upstream attached the
# "cpu" copy to the GPU role a second time).

data "aws_iam_policy" "cloudwatch_agent" {
  count = var.fluentbit_enabled ? 1 : 0
  name  = "CloudWatchAgentServerPolicy"
}

resource "aws_iam_role_policy_attachment" "cloudwatch_agent_nodes" {
  for_each   = var.fluentbit_enabled ? local.node_roles : {}
  role       = each.value
  policy_arn = data.aws_iam_policy.cloudwatch_agent[0].arn
}
