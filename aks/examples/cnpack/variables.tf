# Inputs of the AKS CNPack example (upstream names, own wording).

variable "cluster_name" {
  description = "Name handed to the AKS root module."
  type        = string
}

variable "location" {
  description = "Azure region of the cluster and its resource group."
  type        = string
}

variable "admin_group_object_ids" {
  description = "Object ids of the Entra ID groups that administer the cluster (GUIDs; requires the Owner role to assign)."
  type        = list(any)
}

variable "gpu_machine_type" {
  description = "VM size with 8 x AMD Instinct MI355X, handed to the root module."
  type        = string
  default     = ""
}

variable "prometheus-name" {
  description = "Name of the Azure Monitor (managed Prometheus) workspace."
  type        = string
}

variable "prometheus_resource_group_name" {
  description = "Resource group for the monitor workspace; empty uses the cluster's node resource group."
  type        = string
  default     = ""
}

variable "az_monitor-user-managed-id" {
  description = "Name of the user-assigned identity Prometheus uses for remote_write."
  type        = string
  default     = "tf-amd-monitor-identity"
}

variable "fluentbit_enabled" {
  description = "Create the Log Analytics workspace and the Fluent Bit secret."
  type        = bool
  default     = true
}

variable "fluentbit-workspace-name" {
  description = "Name of the Log Analytics workspace for Fluent Bit."
  type        = string
}

variable "azure_log_analytics_sku" {
  description = "Pricing tier of the Log Analytics workspace."
  type        = string
  default     = "PerGB2018"
}

variable "azure_log_analytics_retention_in_days" {
  description = "Days of log retention (7 on the Free tier, otherwise 30-730)."
  type        = number
  default     = 30
}
