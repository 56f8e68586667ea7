# Providers of the AKS CNPack example. azapi creates the Azure Monitor
# workspace (an ARM type azurerm does not model in 3.x); kubernetes writes the
# Fluent Bit secret into the cluster with the same kubelogin exec tokens the
# root module uses - nothing depends on a local kubeconfig.

terraform {
  required_version = ">= 1.5.0"
  required_providers {
    azapi      = { source = "Azure/azapi", version = ">= 1.4.0, < 2.0.0" }
    azuread    = { source = "hashicorp/azuread", version = ">= 2.15.0, < 4.0.0" }
    azurerm    = { source = "hashicorp/azurerm", version = ">= 3.110.0, < 4.0.0" }
    kubernetes = { source = "hashicorp/kubernetes", version = ">= 2.25.0, < 3.0.0" }
  }
}

provider "azurerm" {
  features {}
}

provider "azapi" {}

provider "kubernetes" {
  host                   = local.kube.host
  cluster_ca_certificate = base64decode(local.kube.cluster_ca_certificate)
  exec {
    api_version = "client.authentication.k8s.io/v1beta1"
    command     = "kubelogin"
    args        = ["get-token", "--login", "azurecli", "--server-id", "6dae42f8-4368-4678-94ff-3960e28e3630"]
  }
}
