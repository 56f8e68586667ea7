terraform {
  required_providers {
    google = {
      source  = "hashicorp/google"
      version = ">= 5.40.0, < 7.0.0"
    }
    google-beta = {
      source  = "hashicorp/google-beta"
      version = ">= 5.40.0, < 7.0.0"
    }
    random = {
      source  = "hashicorp/random"
      version = ">= 3.5.1"
    }
    kubernetes = {
      source  = "hashicorp/kubernetes"
      version = ">= 2.25.0"
    }
  }

  required_version = ">= 1.5.0"
}

provider "google" {
  project = var.project_id
  region  = var.region
}

provider "google-beta" {
  project = var.project_id
  region  = var.region
}

data "google_client_config" "gke" {}

provider "kubernetes" {
  host  = "https://${module.holoscan-ready-gke.kubernetes_cluster_endpoint_ip}"
  token = data.google_client_config.gke.access_token
  cluster_ca_certificate = base64decode(
    module.holoscan-ready-gke.kubernetes_config_file,
  )
}
