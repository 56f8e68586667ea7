"""amd-instinct-terraform-modules: MI355X-native GPU-cluster modules + validation.

Python side of the framework (the Terraform modules live in ``eks/``, ``gke/``,
``aks/`` and ``modules/`` at the repo root):

* ``ops``       - gfx950 HIP kernels (bf16 MFMA GEMM, HBM stream, fill/verify).
* ``parallel``  - RCCL-over-xGMI collectives harness + hand-written P2P all-reduce.
* ``models``    - the validation-Job workload and the time-to-GPU-ready model.
* ``tfcheck``   - offline HCL2 parser / static checker / call-surface contract.
* ``gpu_ready`` - time-to-GPU-ready phase stamping and critical-path analysis.
* ``utils``     - timing, JSON reporting, environment helpers.

The package name is the importable spelling of ``nvidia-terraform-modules_amd``.
"""
__version__ = "0.1.0"
