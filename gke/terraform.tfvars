# Do not commit this file to Git if you add sensitive values
# project_id        = ""
# cluster_name      = ""
# region            = "us-west1"
# node_zones        = ["us-west1-b"]
# gpu_instance_type = "<machine type with 8x MI355X>"
