# MI355X node image. By default the newest Canonical Ubuntu 22.04 EKS image
# for cluster_version (ROCm 7 supports jammy); a non-empty gpu_ami_id is
# honoured verbatim. (Upstream built an override and then never used it, so
# the override silently became an unfiltered "most recent" search.)

locals {
  canonical_owner = "099720109477"
  ami_search = (var.gpu_ami_id != ""
    ? { owners = [], filters = { "image-id" = [var.gpu_ami_id] } }
    : {
      owners = [local.canonical_owner]
      filters = {
        "name"                = ["ubuntu-eks/k8s_${var.cluster_version}/images/hvm-ssd*/ubuntu-jammy-22.04-amd64-server-*"]
        "virtualization-type" = ["hvm"]
      }
  })
}

data "aws_ami" "lookup" {
  most_recent = true
  owners      = local.ami_search.owners

  dynamic "filter" {
    for_each = local.ami_search.filters
    content {
      name   = filter.key
      values = filter.value
    }
  }
}

locals {
  gpu_ami_id = var.gpu_ami_id != "" ? var.gpu_ami_id : data.aws_ami.lookup.id
}
