/***************************
GCP Variables
***************************/
variable "project_id" {
  type        = string
  description = "GCP Project ID for the VPC and K8s Cluster. Shared VPC host projects are not supported."
}

variable "region" {
  type        = string
  description = "The Region resources (VPC, GKE, Compute Nodes) will be created in"
}

/***************************
GKE Variables
***************************/
variable "cluster_name" {
  description = "Name of the Kubernetes Cluster to provision"
  type        = string
}

variable "node_zones" {
  description = "Zones for the node pools (must be in the region above)"
  type        = list(string)
}

variable "gpu_instance_type" {
  type        = string
  default     = ""
  description = "Machine type with AMD Instinct MI355X attached."
}

/*******************************************
GCP Managed Prometheus Variables
*******************************************/
variable "gke_managed_prometheus_enabled" {
  type        = bool
  default     = true
  description = "Set to true to enable, false to disable"
}
