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


def test_window_shorter_than_the_metrics_refresh_is_stale_not_zero():
    """BENCH r5: a 20-step timed loop (13 ms) read the same energy counter at both
    ends; that is no data, not 0 W."""
    a = _s(energy_uj=5_000_000, accumulation_counter=700, ppt_residency_acc=600)
    b = _s(host_ns=16_000_000, energy_uj=5_000_000, accumulation_counter=700,
           ppt_residency_acc=600)
    w = smi.window(a, b)
    assert w["stale"] is True and w["avg_power_W"] is None and w["ppt_pct"] is None
    w = smi.window(a, _s(host_ns=10**9, energy_uj=6_400_000_000, accumulation_counter=1700,
                         ppt_residency_acc=1600))
    assert w["stale"] is False and w["avg_power_W"] == 6395.0 and w["ppt_pct"] == 100.0


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


def test_clock_summary_groups_by_real_xcc_and_finds_the_bounding_xcd():
    """ops.clock_summary (host side of gemm_clock_ghz) on a synthetic record:
    8 XCDs, XCD 3 the slowest; the dispatcher's round robin intact, then broken."""
    import torch

    from nvidia_terraform_modules_amd.ops.kernels import clock_summary

    steps, grid = 4, 64
    st = torch.zeros((steps, grid, 6), dtype=torch.int64)
    ghz = {x: 1.70 - (0.10 if x == 3 else 0.01 * x) for x in range(8)}
    for i in range(steps):
        for b in range(grid):
            x = b & 7
            win_ticks = 65000                          # 650 us at 100 MHz
            st[i, b, 0] = 10_000 + i * 1_000_000       # start cycles
            st[i, b, 1] = 500 + i * 100_000 + (b >> 3)  # start ticks (ramp)
            st[i, b, 3] = st[i, b, 1] + win_ticks
            st[i, b, 2] = st[i, b, 0] + int(ghz[x] * 1e9 * win_ticks / 1e8)
            st[i, b, 4] = x                            # XCC_ID
    r = clock_summary(st, 0.68)
    assert r["xcc_ids"] == list(range(8)) and r["blockidx_mod_8_is_xcc"] is True
    assert abs(r["per_xcc_median_GHz"]["3"] - 1.60) < 1e-3
    assert abs(r["bound_GHz"] - 1.60) < 1e-3            # the slowest XCD bounds the launch
    assert r["xcc_clock_spread_pct"] > 6
    assert r["launches"] == steps and r["ms_per_launch"] == 0.68
    assert r["xcc_finish_spread_us"] >= 0
    # an XCD layout the round robin does not explain: flagged, and grouped by the register
    st[:, :, 4] = (torch.arange(grid) // 8) % 8
    r = clock_summary(st, 0.68)
    assert r["blockidx_mod_8_is_xcc"] is False


def test_sample_gives_up_on_a_stuck_library(monkeypatch):
    """A sample that never returns (a cross-process AMD SMI lock held by a dead
    process) costs the caller at most the timeout, and later samples return at
    once without calling the library again."""
    import threading
    import time

    release = threading.Event()
    calls = []

    def stuck(*a):
        calls.append(a)
        release.wait(30)
        return {}

    monkeypatch.setattr(smi, "sample_at", stuck)
    monkeypatch.setattr(smi, "pci_address", lambda d: (0, 0, 0, 0))
    monkeypatch.setattr(smi, "_stuck", False)
    t0 = time.monotonic()
    s = smi.sample("dev", timeout_s=0.2)
    assert "did not return" in s["error"] and time.monotonic() - t0 < 5
    s = smi.sample("dev", timeout_s=0.2)
    assert "earlier" in s["error"] and len(calls) == 1
    release.set()
