# Requirements and provider wiring of the GKE root. kubernetes / helm are
# declared (upstream used them undeclared) and authenticate with the caller's
# gcloud access token against the cluster this root creates.

terraform {
  required_version = ">= 1.5.0"

  required_providers {
    google      = { source = "hashicorp/google", version = ">= 5.40.0, < 7.0.0" }
    google-beta = { source = "hashicorp/google-beta", version = ">= 5.40.0, < 7.0.0" }
    kubernetes  = { source = "hashicorp/kubernetes", version = ">= 2.25.0, < 3.0.0" }
    helm        = { source = "hashicorp/helm", version = ">= 2.12.0, < 3.0.0" }
  }
}

provider "google" {
  project = var.project_id
  region  = var.region
}

provider "google-beta" {
  project = var.project_id
  region  = var.region
}

data "google_client_config" "provider" {}

locals {
  api_server = "https://${google_container_cluster.this.endpoint}"
  api_ca     = base64decode(google_container_cluster.this.master_auth[0].cluster_ca_certificate)
  api_token  = data.google_client_config.provider.access_token
}

provider "kubernetes" {
  host                   = local.api_server
  cluster_ca_certificate = local.api_ca
  token                  = local.api_token
}

provider "helm" {
  kubernetes {
    host                   = local.api_server
    cluster_ca_certificate = local.api_ca
    token                  = local.api_token
  }
}
