"""Per-rank power / thermal / throttle telemetry (ops/smi.py over libntm_smi.so,
host-only C++ on the AMD SMI library): the window arithmetic on CPU, a real
sample on the GPU box."""
import pytest

from nvidia_terraform_modules_amd.ops import smi


def _s(**kw):
    base = {"host_ns": 0, "energy_uj": 0, "accumulation_counter": 0, "ppt_residency_acc": 0,
            "socket_thm_residency_acc": 0, "prochot_residency_acc": 0, "hbm_thm_residency_acc": 0,
            "vr_thm_residency_acc": 0, "socket_power_w": 900.0, "temp_hotspot_c": 60.0,
            "temp_mem_c": 50.0, "gfxclk_mhz": 2100.0, "gfxclk_min_mhz": 2000.0,
            "indep_throttle_status": 0, "throttle_status": None}
    base.update(kw)
    return base


def test_window_power_and_residencies():
    a = _s()
    b = _s(host_ns=2_000_000_000, energy_uj=2_800_000_000, accumulation_counter=2000,
           ppt_residency_acc=1500, socket_thm_residency_acc=20, socket_power_w=1400.0)
    w = smi.window(a, b)
    assert w["seconds"] == 2.0
    assert w["avg_power_W"] == 1400.0            # 2800 J over 2 s
    assert w["ppt_pct"] == 75.0                  # PVIOL: 1500 of 2000 firmware iterations
    assert w["thermal_pct"] == 1.0               # TVIOL
    assert w["prochot_pct"] == 0.0
    assert w["socket_power_w"] == [900.0, 1400.0]
    assert w["throttle_status"] == [0, 0]         # independent status preferred, 0 kept
    assert "error" not in w


def test_window_unsupported_fields_are_none():
    a = _s(energy_uj=None, accumulation_counter=None)
    b = _s(host_ns=10**9, energy_uj=None, accumulation_counter=None)
    w = smi.window(a, b)
    assert w["avg_power_W"] is None and w["ppt_pct"] is None and w["thermal_pct"] is None
    # counters that went backwards (firmware reset) are not turned into a percentage
    w = smi.window(_s(accumulation_counter=100, ppt_residency_acc=50),
                   _s(host_ns=1, accumulation_counter=200, ppt_residency_acc=10))
    assert w["ppt_pct"] is None


def test_window_carries_sampling_errors():
    w = smi.window({"error": "AMD SMI did not initialise", "host_ns": 1}, _s(host_ns=2))
    assert w["error"] == "AMD SMI did not initialise"


def test_sample_without_gpu_never_raises():
    s = smi.sample_at(0, 0, 0, 0)
    assert "host_ns" in s or "error" in s
    if smi.SMI_LIB_PATH.exists():
        # this container has no GPU: the library loads and reports why
        assert s.get("error")


@pytest.mark.gpu
def test_sample_on_mi355x():
    """The bench's own device: power, temperature, clock and the residency
    counters the PVIOL / TVIOL percentages come from."""
    import torch

    s = smi.sample(torch.device("cuda", 0))
    assert "error" not in s, s
    assert s["socket_power_w"] and 50 < s["socket_power_w"] < 2000, s
    assert s["temp_hotspot_c"] and 10 < s["temp_hotspot_c"] < 120, s
    assert s["gfxclk_mhz"] and 100 < s["gfxclk_mhz"] < 3000, s
    assert s["energy_uj"] is not None and s["accumulation_counter"] is not None, s
