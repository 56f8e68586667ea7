# AWS Private CA behind cert-manager's AWSPCAClusterIssuer. Everything here is
# keyed by local.ca_instances ({} when pca_enabled = false, else one "root"
# entry), so the whole set appears or disappears together.

locals {
  ca = {
    common_name    = var.common_name
    key            = "RSA_4096"
    signature      = "SHA512WITHRSA"
    valid_for_yrs  = 1
    delete_after_d = 7
    root_template  = "arn:${data.aws_partition.current.partition}:acm-pca:::template/RootCACertificate/V1"
  }
  ca_instances = var.pca_enabled ? { root = local.ca } : {}
}

resource "random_string" "pca" {
  for_each = local.ca_instances
  length   = 3
  upper    = false
  special  = false
}

resource "aws_acmpca_certificate_authority" "ca" {
  for_each                        = local.ca_instances
  type                            = "ROOT"
  permanent_deletion_time_in_days = each.value.delete_after_d

  certificate_authority_configuration {
    key_algorithm     = each.value.key
    signing_algorithm = each.value.signature
    subject {
      common_name = each.value.common_name
    }
  }
}

# a root CA issues nothing until its own self-signed certificate is installed
resource "aws_acmpca_certificate" "self_signed" {
  for_each                    = local.ca_instances
  certificate_authority_arn   = aws_acmpca_certificate_authority.ca[each.key].arn
  certificate_signing_request = aws_acmpca_certificate_authority.ca[each.key].certificate_signing_request
  signing_algorithm           = each.value.signature
  template_arn                = each.value.root_template
  validity {
    type  = "YEARS"
    value = each.value.valid_for_yrs
  }
}

resource "aws_acmpca_certificate_authority_certificate" "installed" {
  for_each                  = local.ca_instances
  certificate_authority_arn = aws_acmpca_certificate_authority.ca[each.key].arn
  certificate               = aws_acmpca_certificate.self_signed[each.key].certificate
  certificate_chain         = aws_acmpca_certificate.self_signed[each.key].certificate_chain
}

# ACM may renew certificates it issued from this CA
resource "aws_acmpca_permission" "acm_renewal" {
  for_each                  = local.ca_instances
  certificate_authority_arn = aws_acmpca_certificate_authority.ca[each.key].arn
  principal                 = "acm.amazonaws.com"
  actions                   = ["IssueCertificate", "GetCertificate", "ListPermissions"]
}

# nodes (cert-manager's issuer plugin uses the instance role) may request
data "aws_iam_policy_document" "request_certs" {
  for_each = local.ca_instances
  statement {
    sid       = "RequestFromPrivateCA"
    resources = [aws_acmpca_certificate_authority.ca[each.key].arn]
    actions = [
      "acm-pca:DescribeCertificateAuthority",
      "acm-pca:GetCertificate",
      "acm-pca:IssueCertificate",
    ]
  }
}

resource "aws_iam_policy" "request_certs" {
  for_each    = local.ca_instances
  name        = "aws-pca-node-role-policy-${random_string.pca[each.key].result}"
  description = "cert-manager on the nodes may request certificates from the CNPack private CA"
  policy      = data.aws_iam_policy_document.request_certs[each.key].json
}

resource "aws_iam_role_policy_attachment" "request_certs" {
  for_each   = var.pca_enabled ? local.node_roles : {}
  role       = each.value
  policy_arn = aws_iam_policy.request_certs["root"].arn
}
