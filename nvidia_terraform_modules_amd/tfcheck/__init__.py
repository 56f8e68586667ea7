"""Offline HCL2 parser + static checker for the Terraform modules (no terraform binary)."""
