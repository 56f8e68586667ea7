# Inputs of the GKE CNPack example (upstream names, own wording).

variable "project_id" {
  description = "Project for the cluster and the Prometheus service account."
  type        = string
}

variable "region" {
  description = "Region of the cluster."
  type        = string
}

variable "node_zones" {
  description = "Node zones inside `region` (one zone gives a zonal cluster)."
  type        = list(string)
}

variable "cluster_name" {
  description = "Name handed to the GKE root module."
  type        = string
}

variable "gpu_instance_type" {
  description = "Machine type with AMD Instinct MI355X, handed to the root module."
  type        = string
  default     = ""
}

variable "gke_managed_prometheus_enabled" {
  description = "Create the Managed Prometheus writer identity for the in-cluster Prometheus."
  type        = bool
  default     = true
}
