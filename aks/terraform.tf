# Requirements and provider wiring of the AKS root. The kube providers get
# Entra ID tokens from `kubelogin get-token` (Azure CLI login) for the shared
# AKS AAD server application - no kubeconfig file is written or modified.

terraform {
  required_version = ">= 1.5.0"

  required_providers {
    azurerm    = { source = "hashicorp/azurerm", version = ">= 3.110.0, < 4.0.0" }
    kubernetes = { source = "hashicorp/kubernetes", version = ">= 2.25.0, < 3.0.0" }
    helm       = { source = "hashicorp/helm", version = ">= 2.12.0, < 3.0.0" }
  }
}

provider "azurerm" {
  features {}
}

locals {
  aks_aad_server_app = "6dae42f8-4368-4678-94ff-3960e28e3630"
  admin_kube         = azurerm_kubernetes_cluster.this.kube_config[0]
  token_cmd_args     = ["get-token", "--login", "azurecli", "--server-id", local.aks_aad_server_app]
}

provider "kubernetes" {
  host                   = local.admin_kube.host
  cluster_ca_certificate = base64decode(local.admin_kube.cluster_ca_certificate)
  exec {
    api_version = "client.authentication.k8s.io/v1beta1"
    command     = "kubelogin"
    args        = local.token_cmd_args
  }
}

provider "helm" {
  kubernetes {
    host                   = local.admin_kube.host
    cluster_ca_certificate = base64decode(local.admin_kube.cluster_ca_certificate)
    exec {
      api_version = "client.authentication.k8s.io/v1beta1"
      command     = "kubelogin"
      args        = local.token_cmd_args
    }
  }
}
