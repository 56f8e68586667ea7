# Resource group: the caller's (existing_resource_group_name) or a new
# "<cluster_name>-rg" in `location`.

data "azurerm_resource_group" "existing" {
  count = var.existing_resource_group_name == null ? 0 : 1
  name  = var.existing_resource_group_name
}

resource "azurerm_resource_group" "this" {
  count    = var.existing_resource_group_name == null ? 1 : 0
  name     = "${var.cluster_name}-rg"
  location = var.location
  tags     = local.tags
}

locals {
  tags           = { group = "amd-instinct", managed_by = "Terraform" }
  prep_taint_key = "startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep"
  rg             = var.existing_resource_group_name == null ? azurerm_resource_group.this[0] : data.azurerm_resource_group.existing[0]
}
