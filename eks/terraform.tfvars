# Sample tfvars file. Uncomment out values to use
# cluster_name      = "mi355x-cluster"
# region            = "us-west-2"
# gpu_instance_type = "<EC2 type with 8x MI355X>"

# Optional: If deploying into an existing VPC, use the following variable
# existing_vpc_details = {vpc_id = "", subnet_ids = ["", ""]}
