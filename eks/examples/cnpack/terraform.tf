# Providers this example itself uses (the upstream example declared none and
# relied on implicit hashicorp/* resolution). aws / kubernetes / helm for the
# cluster come from the root module it calls.

terraform {
  required_version = ">= 1.5.0"

  required_providers {
    aws    = { source = "hashicorp/aws", version = ">= 5.79.0, < 6.0.0" }
    random = { source = "hashicorp/random", version = ">= 3.5.1, < 4.0.0" }
  }
}
