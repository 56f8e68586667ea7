# Fill in before applying (project_id and cluster_name have no defaults).
project_id   = ""
cluster_name = ""
region       = "us-central1"
node_zones   = ["us-central1-a"]

gke_managed_prometheus_enabled = true
