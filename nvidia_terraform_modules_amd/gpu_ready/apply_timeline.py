"""Stamp the six time-to-GPU-ready phases from real provisioning logs.

Inputs (all produced by standard tooling, no cloud SDK needed here):

* ``terraform apply -json`` machine-readable UI log (one JSON object per line;
  ``type`` in {"apply_start", "apply_progress", "apply_complete",
  "apply_errored"}, ``hook.resource.addr``, ``hook.elapsed_seconds``,
  ``@timestamp``),
* optionally ``kubectl get events -A -o json`` / ``--watch -o json`` output
  and the validation Job's JSON report (``kubectl logs job/...``).

Output: per-resource durations (feeding :func:`critical_path.durations_from_
timeline`) and the phase table of BASELINE.md:

    network -> control_plane -> gpu_nodes_ready -> operator_deployed
            -> gpu_allocatable -> validation_done

The reference (NVIDIA modules) has no such instrumentation; its only figure
is "~5 minutes after apply for the operator to be running"
(/root/reference/gke/README.md:50).
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from datetime import datetime

from .critical_path import phase_of
from .phases import CLUSTER_PHASES


def parse_ts(s: str) -> float:
    """RFC3339 timestamp (terraform uses microseconds + offset) -> epoch seconds."""
    s = s.strip()
    if s.endswith("Z"):
        s = s[:-1] + "+00:00"
    # python < 3.11 cannot parse >6 fractional digits
    if "." in s:
        head, rest = s.split(".", 1)
        frac = ""
        i = 0
        while i < len(rest) and rest[i].isdigit():
            frac += rest[i]
            i += 1
        s = f"{head}.{frac[:6].ljust(6, '0')}{rest[i:]}"
    return datetime.fromisoformat(s).timestamp()


@dataclass
class ResourceEvent:
    address: str
    action: str
    start: float | None = None
    end: float | None = None
    elapsed_s: float | None = None
    errored: bool = False

    def as_dict(self) -> dict:
        return {"address": self.address, "action": self.action, "start": self.start,
                "end": self.end, "elapsed_s": self.elapsed_s, "errored": self.errored}


def parse_apply_json(lines) -> list[dict]:
    """Resource create/modify events from a ``terraform apply -json`` log."""
    events: dict[str, ResourceEvent] = {}
    for raw in lines:
        raw = raw.strip()
        if not raw or not raw.startswith("{"):
            continue
        try:
            msg = json.loads(raw)
        except json.JSONDecodeError:
            continue
        typ = msg.get("type", "")
        if not typ.startswith("apply_"):
            continue
        hook = msg.get("hook", {})
        addr = hook.get("resource", {}).get("addr")
        if not addr:
            continue
        ts = parse_ts(msg["@timestamp"]) if "@timestamp" in msg else None
        ev = events.setdefault(addr, ResourceEvent(addr, hook.get("action", "")))
        if typ == "apply_start":
            ev.start = ts
            ev.action = hook.get("action", ev.action)
        elif typ == "apply_complete":
            ev.end = ts
            if "elapsed_seconds" in hook:
                ev.elapsed_s = float(hook["elapsed_seconds"])
            elif ev.start is not None and ts is not None:
                ev.elapsed_s = ts - ev.start
        elif typ == "apply_errored":
            ev.end = ts
            ev.errored = True
    return [e.as_dict() for e in sorted(events.values(), key=lambda e: (e.start or 0.0, e.address))]


def gpu_allocatable_time(k8s_events: dict | list) -> float | None:
    """Earliest time a node reported ``amd.com/gpu`` allocatable, from
    ``kubectl get events -o json`` (the device plugin's registration shows up
    as a Node event / condition update); None if never seen."""
    items = k8s_events.get("items", []) if isinstance(k8s_events, dict) else k8s_events
    best = None
    for it in items:
        text = json.dumps(it)
        if "amd.com/gpu" not in text:
            continue
        ts = it.get("lastTimestamp") or it.get("eventTime") or it.get("firstTimestamp")
        if not ts:
            continue
        t = parse_ts(ts)
        best = t if best is None or t < best else best
    return best


@dataclass
class Timeline:
    apply_start: float
    phases: dict              # phase -> end time (epoch s)
    resources: list

    @property
    def time_to_gpu_ready_s(self) -> float | None:
        end = self.phases.get("validation_done")
        return None if end is None else end - self.apply_start

    def phase_durations(self) -> dict:
        out, prev = {}, self.apply_start
        for ph in CLUSTER_PHASES:
            if ph in self.phases and self.phases[ph] is not None:
                out[ph] = max(0.0, self.phases[ph] - prev)
                prev = max(prev, self.phases[ph])
        return out

    def as_dict(self) -> dict:
        return {"apply_start": self.apply_start, "phase_end": self.phases,
                "phase_s": self.phase_durations(), "time_to_gpu_ready_s": self.time_to_gpu_ready_s,
                "resources": self.resources}


def build_timeline(apply_log_lines, k8s_events=None, validation_report: dict | None = None) -> Timeline:
    """Combine the apply log (+ optional k8s events / Job report) into phases.

    A phase ends when the LAST resource attributed to it (critical_path.
    phase_of) completes; gpu_allocatable comes from k8s events when given
    (else it coincides with the device-plugin DaemonSets / DeviceConfig
    completing); validation_done is the validation Job resource completing
    (apply waits for it) or the Job report's own end stamp.
    """
    res = parse_apply_json(apply_log_lines)
    starts = [r["start"] for r in res if r["start"] is not None]
    if not starts:
        raise ValueError("no apply_start events in the log")
    t0 = min(starts)
    phases: dict = {}
    for r in res:
        if r["end"] is None or r["errored"]:
            continue
        ph = phase_of(r["address"])
        if ph in CLUSTER_PHASES:
            phases[ph] = max(phases.get(ph, r["end"]), r["end"])
    if k8s_events is not None:
        t = gpu_allocatable_time(k8s_events)
        if t is not None:
            phases["gpu_allocatable"] = t
    if validation_report and validation_report.get("end_epoch_s"):
        phases["validation_done"] = float(validation_report["end_epoch_s"])
    return Timeline(apply_start=t0, phases=phases, resources=res)
