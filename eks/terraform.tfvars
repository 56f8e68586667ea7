# Values for a first apply. cluster_name and gpu_instance_type have no
# usable defaults; everything else is optional.
#
# cluster_name      = "mi355x"
# region            = "us-west-2"
# gpu_instance_type = "<EC2 type with 8 x MI355X>"
#
# Reuse a VPC instead of creating one:
# existing_vpc_details = { vpc_id = "vpc-...", subnet_ids = ["subnet-...", "subnet-..."] }
