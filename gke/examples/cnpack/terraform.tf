# Providers of the GKE CNPack example.
#  - kubernetes: reaches the cluster the root module builds, using the
#    caller's gcloud OAuth token (no kubeconfig file involved);
#  - google / google-beta: project + region defaults for everything here.

terraform {
  required_version = ">= 1.5.0"
  required_providers {
    kubernetes  = { source = "hashicorp/kubernetes", version = ">= 2.25.0, < 3.0.0" }
    google      = { source = "hashicorp/google", version = ">= 5.40.0, < 7.0.0" }
    google-beta = { source = "hashicorp/google-beta", version = ">= 5.40.0, < 7.0.0" }
    random      = { source = "hashicorp/random", version = ">= 3.5.1, < 4.0.0" }
  }
}

data "google_client_config" "caller" {}

provider "kubernetes" {
  token                  = data.google_client_config.caller.access_token
  host                   = "https://${module.mi355x_gke.kubernetes_cluster_endpoint_ip}"
  cluster_ca_certificate = base64decode(module.mi355x_gke.kubernetes_config_file)
}

provider "google" {
  region  = var.region
  project = var.project_id
}

provider "google-beta" {
  region  = var.region
  project = var.project_id
}
