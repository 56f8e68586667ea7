# Engine / provider requirements and provider wiring of the EKS root.
# helm is declared here too (the upstream module used it undeclared), and
# region / profile really reach the AWS provider and the token command.

terraform {
  required_version = ">= 1.5.0"

  required_providers {
    aws        = { source = "hashicorp/aws", version = ">= 5.79.0, < 6.0.0" }
    kubernetes = { source = "hashicorp/kubernetes", version = ">= 2.25.0, < 3.0.0" }
    helm       = { source = "hashicorp/helm", version = ">= 2.12.0, < 3.0.0" }
  }
}

provider "aws" {
  region  = var.region
  profile = var.aws_profile == "" ? null : var.aws_profile
}

data "aws_region" "current" {}

# endpoint + CA re-read from the API once the control plane exists
data "aws_eks_cluster" "cluster" {
  name = module.eks.cluster_name
}

locals {
  # one token recipe for both kube providers and for the kube_exec_* outputs
  kube_exec_api_version = "client.authentication.k8s.io/v1beta1"
  kube_exec_args = concat(
    ["eks", "get-token", "--cluster-name", module.eks.cluster_name, "--region", data.aws_region.current.name],
    var.aws_profile == "" ? [] : ["--profile", var.aws_profile],
  )
  kube_host = data.aws_eks_cluster.cluster.endpoint
  kube_ca   = base64decode(data.aws_eks_cluster.cluster.certificate_authority[0].data)
}

provider "kubernetes" {
  host                   = local.kube_host
  cluster_ca_certificate = local.kube_ca
  exec {
    api_version = local.kube_exec_api_version
    command     = "aws"
    args        = local.kube_exec_args
  }
}

provider "helm" {
  kubernetes {
    host                   = local.kube_host
    cluster_ca_certificate = local.kube_ca
    exec {
      api_version = local.kube_exec_api_version
      command     = "aws"
      args        = local.kube_exec_args
    }
  }
}
