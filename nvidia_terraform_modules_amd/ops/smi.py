"""Per-GPU power / thermal / throttle telemetry over a timed region.

ctypes binding to ``libntm_smi.so`` (validation/src/ntm_smi.cpp, host-only C++
on the AMD SMI library). ``sample(device)`` reads one GPU, matched to the
PyTorch device by PCI address; ``window(before, after)`` turns two samples
into what happened between them:

* ``avg_power_W`` from the energy counter over the host clock,
* ``ppt_pct`` / ``thermal_pct`` / ``prochot_pct`` / ``hbm_thermal_pct``: the
  share of firmware iterations spent in power (PVIOL) or thermal (TVIOL)
  throttling, from the accumulated residency counters,
* power, temperatures and clocks at both ends.

bench.py records this per rank around the timed loop, so that on a multi-GPU
run a power-capped rank reads differently from a slow one.
The reference leaves GPU telemetry to the NVIDIA chart's DCGM exporter
(``/root/reference/eks/main.tf:185-203``). Nothing here raises on a missing
library or an unsupported field: telemetry is context, not a verdict.
"""
from __future__ import annotations

import ctypes
from pathlib import Path

SMI_LIB_PATH = Path(__file__).resolve().parent / "libntm_smi.so"
_NA = (1 << 64) - 1


class _Sample(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "socket_power_w", "temp_hotspot_c", "temp_mem_c", "gfxclk_mhz", "gfxclk_min_mhz",
        "uclk_mhz")] + [(n, ctypes.c_uint64) for n in (
        "throttle_status", "indep_throttle_status", "accumulation_counter",
        "prochot_residency_acc", "ppt_residency_acc", "socket_thm_residency_acc",
        "vr_thm_residency_acc", "hbm_thm_residency_acc", "energy_uj", "host_ns")]


_smi: ctypes.CDLL | None = None
_ERR = {1: "AMD SMI did not initialise", 2: "no GPU at that PCI address",
        3: "metrics table not readable"}


def _lib() -> ctypes.CDLL | None:
    global _smi
    if _smi is None and SMI_LIB_PATH.exists():
        try:
            lib = ctypes.CDLL(str(SMI_LIB_PATH))
        except OSError:
            return None
        lib.ntm_smi_sample.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.POINTER(_Sample)]
        lib.ntm_smi_sample.restype = ctypes.c_int
        lib.ntm_smi_sample_bytes.restype = ctypes.c_int
        if lib.ntm_smi_sample_bytes() != ctypes.sizeof(_Sample):
            raise RuntimeError("libntm_smi.so sample layout differs from ops/smi.py")
        _smi = lib
    return _smi


def pci_address(device) -> tuple[int, int, int, int]:
    """(domain, bus, device, function) of a PyTorch GPU device."""
    import torch

    p = torch.cuda.get_device_properties(device)
    return int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id), 0


def sample_at(domain: int, bus: int, dev: int, fn: int = 0) -> dict:
    """One raw sample of the GPU at that PCI address (``error`` set on failure)."""
    lib = _lib()
    if lib is None:
        return {"error": f"{SMI_LIB_PATH.name} not built"}
    s = _Sample()
    rc = lib.ntm_smi_sample(domain, bus, dev, fn, ctypes.byref(s))
    out = {k: getattr(s, k) for k, _ in _Sample._fields_}
    for k, _ in _Sample._fields_:
        if isinstance(out[k], float) and out[k] < 0:
            out[k] = None
        elif isinstance(out[k], int) and out[k] == _NA:
            out[k] = None
    if rc:
        out["error"] = _ERR.get(rc, f"rc {rc}")
    return out


_stuck = False   # a sample that never returned: AMD SMI is not called again in this process


def sample(device, timeout_s: float = 10.0) -> dict:
    """One sample of a PyTorch GPU device (never raises, never blocks for more
    than ``timeout_s``). The library call runs on a daemon thread: AMD SMI takes
    a cross-process lock at init, and a bench rank must not hang on telemetry if
    another process died holding it. After a timeout the process stops calling
    AMD SMI (the stuck thread is abandoned at exit)."""
    global _stuck
    if _stuck:
        return {"error": "AMD SMI did not return earlier in this process"}
    import threading

    box: dict = {}

    def run():
        try:
            box["s"] = sample_at(*pci_address(device))
        except Exception as e:  # noqa: BLE001 - telemetry is context only
            box["s"] = {"error": f"{type(e).__name__}: {e}"[:200]}

    t = threading.Thread(target=run, name="ntm-smi-sample", daemon=True)
    t.start()
    t.join(timeout_s)
    if t.is_alive():
        _stuck = True
        return {"error": f"AMD SMI sample did not return within {timeout_s} s"}
    return box["s"]


def _pct(num_a, num_b, den_a, den_b):
    if None in (num_a, num_b, den_a, den_b) or den_b <= den_a or num_b < num_a:
        return None
    return round(100.0 * (num_b - num_a) / (den_b - den_a), 2)


def window(before: dict, after: dict) -> dict:
    """What happened between two samples of one GPU: average power from the
    energy counter, throttle residencies in percent of firmware iterations,
    and power / temperature / clock at both ends (None where unsupported)."""
    res: dict = {}
    err = before.get("error") or after.get("error")
    if err:
        res["error"] = err
    dt = ((after.get("host_ns") or 0) - (before.get("host_ns") or 0)) / 1e9
    res["seconds"] = round(dt, 4) if dt > 0 else None
    ea, eb = before.get("energy_uj"), after.get("energy_uj")
    # the firmware metrics table refreshes every few tens of ms: a window shorter
    # than that reads the same energy / accumulation counters at both ends, which
    # is "no data", not 0 W (BENCH at 20 x 0.67 ms read 0.0 W at 1388 W socket power)
    res["stale"] = ea is not None and ea == eb
    res["avg_power_W"] = (round((eb - ea) / 1e6 / dt, 1)
                          if None not in (ea, eb) and eb > ea and dt > 0 else None)
    acc = (before.get("accumulation_counter"), after.get("accumulation_counter"))
    for key, field in (("ppt_pct", "ppt_residency_acc"), ("thermal_pct", "socket_thm_residency_acc"),
                       ("prochot_pct", "prochot_residency_acc"),
                       ("hbm_thermal_pct", "hbm_thm_residency_acc"),
                       ("vr_thermal_pct", "vr_thm_residency_acc")):
        res[key] = _pct(before.get(field), after.get(field), *acc)
    for key in ("socket_power_w", "temp_hotspot_c", "temp_mem_c", "gfxclk_mhz", "gfxclk_min_mhz"):
        res[key] = [before.get(key), after.get(key)]
    def _status(s: dict):
        v = s.get("indep_throttle_status")
        return v if v is not None else s.get("throttle_status")

    res["throttle_status"] = [_status(before), _status(after)]
    return res
