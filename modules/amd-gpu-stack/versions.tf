# Cloud-agnostic AMD Instinct (MI355X / gfx950) Kubernetes GPU stack.
#
# Replaces the reference's per-cloud `helm_release "gpu_operator"` blocks
# (/root/reference/eks/main.tf:185-203, gke/main.tf:153-213, aks/main.tf:81-91)
# with ONE module used by eks/, gke/ and aks/. Providers are configured by the
# calling root module (this module declares requirements only).

terraform {
  required_version = ">= 1.5.0"

  required_providers {
    helm = {
      source  = "hashicorp/helm"
      version = ">= 2.12.0, < 3.0.0"
    }
    kubernetes = {
      source  = "hashicorp/kubernetes"
      version = ">= 2.25.0, < 3.0.0"
    }
  }
}
