cluster_name                   = ""
gke_managed_prometheus_enabled = true
node_zones                     = ["us-west1-b"]
project_id                     = ""
region                         = "us-west1"
