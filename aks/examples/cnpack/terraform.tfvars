// Cluster Variables
# cluster_name           = "cnpack-mi355x"
# location               = "West US 2"
# admin_group_object_ids = []
# gpu_machine_type       = "<Azure VM size with 8x MI355X>"

// Fluentbit/Azure Log Configuration Variables
# fluentbit-workspace-name = "fluentbit-test"

// Prometheus/Azure Monitor Configuration Variables
# prometheus-name = "cnpack-prometheus"
