# Provider pins for the EKS root module. Unlike the reference
# (/root/reference/eks/versions.tf:4-17) every provider the module uses is
# declared - helm was missing there.

terraform {
  required_providers {
    aws = {
      source  = "hashicorp/aws"
      version = ">= 5.79.0, < 6.0.0"
    }
    kubernetes = {
      source  = "hashicorp/kubernetes"
      version = ">= 2.25.0"
    }
    helm = {
      source  = "hashicorp/helm"
      version = ">= 2.12.0, < 3.0.0"
    }
  }

  required_version = ">= 1.5.0"
}
