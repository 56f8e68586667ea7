# Providers configured inside the root module, like the reference
# (/root/reference/eks/provider.tf:4-14), but with region/profile actually
# wired (the reference declared `region` and never used it) and the same
# exec api_version the kube_exec_* outputs advertise.

locals {
  kube_exec_api_version = "client.authentication.k8s.io/v1beta1"
  kube_exec_args = concat(
    var.aws_profile == "" ? [] : ["--profile", var.aws_profile],
    ["eks", "get-token", "--region", data.aws_region.current.name, "--cluster-name", module.eks.cluster_name]
  )
}

provider "aws" {
  region  = var.region
  profile = var.aws_profile == "" ? null : var.aws_profile
}

provider "kubernetes" {
  host                   = data.aws_eks_cluster.cluster.endpoint
  cluster_ca_certificate = base64decode(data.aws_eks_cluster.cluster.certificate_authority[0].data)
  exec {
    api_version = local.kube_exec_api_version
    command     = "aws"
    args        = local.kube_exec_args
  }
}

provider "helm" {
  kubernetes {
    host                   = data.aws_eks_cluster.cluster.endpoint
    cluster_ca_certificate = base64decode(data.aws_eks_cluster.cluster.certificate_authority[0].data)
    exec {
      api_version = local.kube_exec_api_version
      command     = "aws"
      args        = local.kube_exec_args
    }
  }
}
