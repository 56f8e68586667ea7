"""Phase stamping for the time-to-GPU-ready metric.

BASELINE.md defines ``time_to_gpu_ready_s = t(validation Job Succeeded) -
t(terraform apply start)`` split into six phases:

    1 network  2 control_plane  3 gpu_nodes_ready  4 operator_deployed
    5 gpu_allocatable  6 validation_done

The reference has no such instrumentation; its only number is the ~5 min gap
between "apply returned" and "GPU operator Running" (/root/reference/gke/
README.md:50). Phases 1-5 are cloud/Kubernetes side and are stamped by
:mod:`.apply_timeline` from ``terraform apply -json`` + ``kubectl`` watch
events; phase 6 is split further *inside the validation container* by
:class:`PhaseClock` (container start -> HIP init -> K1/K2/C1 done), which is
what this repo can measure on a real MI355X through ``gpurun``.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass, field

CLUSTER_PHASES = (
    "network",
    "control_plane",
    "gpu_nodes_ready",
    "operator_deployed",
    "gpu_allocatable",
    "validation_done",
)

IN_NODE_PHASES = (
    "process_start",
    "runtime_import",
    "hip_init",
    "buffers_ready",
    "first_kernel",
    "gemm_verified",
    "hbm_checked",
    "collectives_checked",
    "done",
)


def process_start_time() -> float:
    """Wall-clock (epoch seconds) at which this process was started.

    Uses /proc (Linux) so the Python interpreter's own start-up is included;
    falls back to "now" elsewhere.
    """
    try:
        with open("/proc/self/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        start_ticks = int(fields[19])  # field 22 overall, 0-based after comm
        hz = os.sysconf(os.sysconf_names["SC_CLK_TCK"])
        with open("/proc/uptime") as f:
            uptime = float(f.read().split()[0])
        return time.time() - uptime + start_ticks / hz
    except (OSError, ValueError, IndexError, KeyError):
        return time.time()


@dataclass
class PhaseClock:
    """Monotone phase stamps relative to an origin (default: process start)."""

    origin: float = field(default_factory=process_start_time)
    stamps: dict[str, float] = field(default_factory=dict)

    def mark(self, name: str, t: float | None = None) -> float:
        t = time.time() if t is None else t
        if self.stamps:
            last = max(self.stamps.values())
            t = max(t, last)  # monotone even across clock steps
        self.stamps[name] = t
        return t - self.origin

    def elapsed(self, name: str) -> float:
        return self.stamps[name] - self.origin

    def durations(self) -> dict[str, float]:
        """Per-phase durations in stamp order (first phase measured from origin)."""
        out, prev = {}, self.origin
        for name, t in sorted(self.stamps.items(), key=lambda kv: kv[1]):
            out[name] = t - prev
            prev = t
        return out

    def as_dict(self) -> dict:
        return {
            "origin_epoch_s": self.origin,
            "elapsed_s": {k: v - self.origin for k, v in self.stamps.items()},
            "phase_s": self.durations(),
            "total_s": (max(self.stamps.values()) - self.origin) if self.stamps else 0.0,
        }

    def to_json(self) -> str:
        return json.dumps(self.as_dict(), sort_keys=True)
