# Network: either a fresh VPC (one private + one public subnet per zone, NAT
# for image pulls) or the caller's VPC from existing_vpc_details.

data "aws_availability_zones" "available" {
  state = "available"
}

module "vpc" {
  count   = var.existing_vpc_details == null ? 1 : 0
  source  = "terraform-aws-modules/vpc/aws"
  version = "~> 5.16"

  name = "tf-${var.cluster_name}-vpc"
  cidr = var.cidr_block
  azs  = slice(data.aws_availability_zones.available.names, 0, length(var.private_subnets))

  private_subnets = var.private_subnets
  public_subnets  = var.public_subnets

  enable_nat_gateway   = var.enable_nat_gateway
  single_nat_gateway   = var.single_nat_gateway
  enable_dns_support   = var.enable_dns_support
  enable_dns_hostnames = var.enable_dns_hostnames

  map_public_ip_on_launch = true
  public_subnet_tags      = { "kubernetes.io/role/elb" = "1" }
  private_subnet_tags     = { "kubernetes.io/role/internal-elb" = "1" }
}

locals {
  byo_network  = var.existing_vpc_details != null
  vpc_id       = local.byo_network ? var.existing_vpc_details.vpc_id : module.vpc[0].vpc_id
  node_subnets = local.byo_network ? var.existing_vpc_details.subnet_ids : module.vpc[0].private_subnets

  # Nodes talk to each other on every protocol (RCCL's socket transport
  # between nodes when no RDMA fabric is attached; within one node the
  # collectives ride xGMI) and reach anything outbound.
  node_sg_rules = {
    mesh_ingress = {
      type        = "ingress"
      description = "any protocol from other nodes of this cluster"
      protocol    = "-1"
      from_port   = 0
      to_port     = 0
      self        = true
    }
    open_egress = {
      type             = "egress"
      description      = "outbound to anywhere"
      protocol         = "-1"
      from_port        = 0
      to_port          = 0
      cidr_blocks      = ["0.0.0.0/0"]
      ipv6_cidr_blocks = ["::/0"]
    }
  }
}
