# The reference example declared no providers at all (implicit hashicorp/*).
terraform {
  required_providers {
    aws = {
      source  = "hashicorp/aws"
      version = ">= 5.79.0, < 6.0.0"
    }
    random = {
      source  = "hashicorp/random"
      version = ">= 3.5.1"
    }
  }

  required_version = ">= 1.5.0"
}
