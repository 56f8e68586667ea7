# Required inputs of the GKE root; keep real project ids out of git.
#
# project_id        = "<project>"
# cluster_name      = "mi355x"
# region            = "us-central1"
# node_zones        = ["us-central1-a"]       # one zone -> zonal cluster
# gpu_instance_type = "<machine type with 8 x MI355X>"
