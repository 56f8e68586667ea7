# cluster_name = "cnpack-mi355x-cluster"
