"""Workload models: the validation Job (flagship) and the cluster
time-to-GPU-ready phase model."""
from .validation_job import GemmWorkload, ValidationConfig, ValidationReport, run_validation  # noqa: F401
