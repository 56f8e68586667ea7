# cluster_name           = "amd-mi355x-aks-cluster"
# admin_group_object_ids = []
# location               = "West US 2"
# gpu_machine_type       = "<Azure VM size with 8x MI355X>"
