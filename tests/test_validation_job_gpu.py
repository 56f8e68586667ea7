"""End-to-end validation Job on one MI355X, including fault injection."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _env():
    from nvidia_terraform_modules_amd.parallel.dist import init

    return init()


def test_validation_job_passes():
    from nvidia_terraform_modules_amd.models.validation_job import ValidationConfig, run_validation

    cfg = ValidationConfig(size=1024, gemm_iters=5, hbm_bytes=64 << 20, hbm_iters=2,
                           min_hbm_capacity_gb=100.0, fault_inject="")
    rep = run_validation(_env(), cfg)
    assert rep.passed, rep.failures
    assert rep.gemm["verify"]["ok"]
    assert rep.gemm["tflops"] > 10
    assert rep.hbm["copy_ok"] and rep.hbm["capacity_total_gb"] > 250  # 288 GB HBM3E
    ph = rep.phases["elapsed_s"]
    assert ph["hip_init"] <= ph["first_kernel"] <= ph["gemm_verified"] <= ph["done"]


def test_validation_job_detects_injected_gemm_fault():
    from nvidia_terraform_modules_amd.models.validation_job import ValidationConfig, run_validation

    cfg = ValidationConfig(size=512, gemm_iters=2, hbm_bytes=16 << 20, hbm_iters=1,
                           fault_inject="corrupt_gemm")
    rep = run_validation(_env(), cfg)
    assert not rep.passed
    assert any("gemm verification" in f for f in rep.failures)


def test_validation_job_tflops_floor():
    from nvidia_terraform_modules_amd.models.validation_job import ValidationConfig, run_validation

    cfg = ValidationConfig(size=512, gemm_iters=2, hbm_bytes=16 << 20, hbm_iters=1,
                           tflops_floor=1e9, fault_inject="")
    rep = run_validation(_env(), cfg, with_hbm=False)
    assert not rep.passed and "below floor" in rep.failures[0]
    torch.cuda.synchronize()


def test_validation_job_abft_detects_injected_fault():
    from nvidia_terraform_modules_amd.models.validation_job import ValidationConfig, run_validation

    cfg = ValidationConfig(size=1024, gemm_iters=2, check=False, abft_iters=2,
                           fault_inject="corrupt_abft")
    rep = run_validation(_env(), cfg, with_hbm=False)
    assert not rep.passed
    assert any("ABFT" in f for f in rep.failures)
    assert rep.gemm["abft"]["bad_store"] == 1


def test_validation_job_reports_abft_clean():
    from nvidia_terraform_modules_amd.models.validation_job import ValidationConfig, run_validation

    cfg = ValidationConfig(size=2048, gemm_iters=3, abft_iters=3, fault_inject="")
    rep = run_validation(_env(), cfg, with_hbm=False)
    assert rep.passed, rep.failures
    assert rep.gemm["abft"]["ok"] and rep.gemm["abft_tflops"] > 10
