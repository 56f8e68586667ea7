# location, admin_group_object_ids and gpu_machine_type have no usable
# defaults.
#
# location               = "westus3"
# admin_group_object_ids = ["<Entra ID group object id>"]
# gpu_machine_type       = "<VM size with 8 x MI355X>"
# cluster_name           = "mi355x"
