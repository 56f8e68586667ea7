# Only the cluster name is required; the MI355X type is needed for apply.
# cluster_name      = "cnpack-mi355x"
# gpu_instance_type = "<EC2 type with 8 x MI355X>"
