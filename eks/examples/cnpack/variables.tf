# Inputs of the EKS CNPack example: the upstream example's names, own wording.

variable "cluster_name" {
  description = "Name handed to the EKS root module."
  type        = string
}

variable "gpu_instance_type" {
  description = "EC2 type with 8 x AMD Instinct MI355X, handed to the root module."
  type        = string
  default     = ""
}

variable "amp_enabled" {
  description = "Create the Managed Prometheus workspace, its log group and ingest identities."
  type        = bool
  default     = true
}

variable "pca_enabled" {
  description = "Create the private root CA and the node policy cert-manager needs."
  type        = bool
  default     = true
}

variable "common_name" {
  description = "Subject CN of the private root CA."
  type        = string
  default     = "cluster.local"
}

variable "fluentbit_enabled" {
  description = "Grant the node roles CloudWatch agent permissions for Fluent Bit."
  type        = bool
  default     = true
}

variable "metrics_server_enabled" {
  description = "Open the API-server-to-node path of the metrics-server (TCP 4443)."
  type        = bool
  default     = true
}

variable "prom_adapter_enabled" {
  description = "Open the API-server-to-node path of the prometheus-adapter (TCP 6443)."
  type        = bool
  default     = true
}
