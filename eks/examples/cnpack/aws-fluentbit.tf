/*******************************************
Fluent Bit -> CloudWatch: node roles need CloudWatchAgentServerPolicy
*******************************************/
data "aws_iam_policy" "cloudwatch-agent-server-policy" {
  count = var.fluentbit_enabled ? 1 : 0
  name  = "CloudWatchAgentServerPolicy"
}

resource "aws_iam_role_policy_attachment" "attach-cloudwatch-to-gpu-ng" {
  count      = var.fluentbit_enabled ? 1 : 0
  role       = module.holoscan-eks-cluster.gpu_node_role_name
  policy_arn = data.aws_iam_policy.cloudwatch-agent-server-policy[count.index].arn
}

// the reference attached this one to the GPU role again (aws-fluentbit.tf:22-25)
resource "aws_iam_role_policy_attachment" "attach-cloudwatch-to-cpu-ng" {
  count      = var.fluentbit_enabled ? 1 : 0
  role       = module.holoscan-eks-cluster.cpu_node_role_name
  policy_arn = data.aws_iam_policy.cloudwatch-agent-server-policy[count.index].arn
}
