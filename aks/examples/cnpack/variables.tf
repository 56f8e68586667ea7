/****************************
Azure Variables
****************************/
variable "location" {
  type        = string
  description = "The region to create resources in (can be set in terraform.tfvars)"
}

variable "az_monitor-user-managed-id" {
  type        = string
  default     = "tf-amd-monitor-identity"
  description = "Name of the user-assigned managed identity created for Azure Monitor remote-write (granted Monitoring Metrics Publisher on the workspace's data collection rule)."
}

/****************************
Active Directory Variables
****************************/
variable "admin_group_object_ids" {
  type        = list(any)
  description = <<EOH
  (Required) A list of Object IDs (GUIDs) of Azure Active Directory Groups which should have Owner Role on the Cluster.
  This is not the email address of the group, the GUID can be found in the Azure panel by searching for the AD Group
  NOTE: You will need Azure "Owner" role (not "Contributor") to attach an AD role to the Kubernetes cluster.
  EOH
}

/*******************************************
Cluster Variables
*******************************************/
variable "cluster_name" {
  type        = string
  description = "Name of the cluster"
}

variable "gpu_machine_type" {
  type        = string
  default     = ""
  description = "Azure VM size with 8x AMD Instinct MI355X."
}

/*******************************************
Fluentbit (Azure Logging) Variables
*******************************************/
variable "fluentbit_enabled" {
  type        = bool
  default     = true
  description = "Create the Log Analytics workspace and the fluentbit secret (was declared but ignored in the reference)"
}

variable "fluentbit-workspace-name" {
  description = "Name of the Azure Log Workspace for Fluentbit to be created"
  type        = string
}

variable "azure_log_analytics_sku" {
  description = "SKU of the Log Analytics Workspace (Free, PerNode, Premium, Standard, Standalone, Unlimited, CapacityReservation, PerGB2018)."
  default     = "PerGB2018"
}

variable "azure_log_analytics_retention_in_days" {
  default     = 30
  description = "Workspace data retention in days (7 on Free, else 30-730)"
}

/*******************************************
Prometheus (Azure Monitor) Variables
*******************************************/
variable "prometheus_resource_group_name" {
  type        = string
  default     = ""
  description = "Resource group for the Azure Monitor workspace (empty = the cluster's node resource group)."
}

variable "prometheus-name" {
  type        = string
  description = "The name of the Azure Monitor Workspace for Prometheus"
}
