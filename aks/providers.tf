provider "azurerm" {
  features {}
}

# AAD-integrated cluster: exec kubelogin (azurecli login) for tokens; the
# server id is the AKS AAD server application shared by all AKS clusters.
locals {
  kube_host = azurerm_kubernetes_cluster.holoscan.kube_config[0].host
  kube_ca   = base64decode(azurerm_kubernetes_cluster.holoscan.kube_config[0].cluster_ca_certificate)
  kubelogin_args = [
    "get-token", "--login", "azurecli",
    "--server-id", "6dae42f8-4368-4678-94ff-3960e28e3630",
  ]
}

provider "kubernetes" {
  host                   = local.kube_host
  cluster_ca_certificate = local.kube_ca
  exec {
    api_version = "client.authentication.k8s.io/v1beta1"
    command     = "kubelogin"
    args        = local.kubelogin_args
  }
}

provider "helm" {
  kubernetes {
    host                   = local.kube_host
    cluster_ca_certificate = local.kube_ca
    exec {
      api_version = "client.authentication.k8s.io/v1beta1"
      command     = "kubelogin"
      args        = local.kubelogin_args
    }
  }
}
