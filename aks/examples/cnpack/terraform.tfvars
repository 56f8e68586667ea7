# Required before apply:
# cluster_name             = "cnpack-mi355x"
# location                 = "westus3"
# admin_group_object_ids   = ["<Entra ID group object id>"]
# gpu_machine_type         = "<VM size with 8 x MI355X>"
# prometheus-name          = "cnpack-prometheus"
# fluentbit-workspace-name = "cnpack-fluentbit"
