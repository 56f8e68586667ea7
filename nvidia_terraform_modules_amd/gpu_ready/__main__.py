"""Time-to-GPU-ready CLI.

    python -m nvidia_terraform_modules_amd.gpu_ready record --out runs/eks1 \\
        [--kubectl "kubectl --kubeconfig kc"] [--namespace kube-amd-gpu] \\
        -- terraform apply -json -auto-approve
    python -m nvidia_terraform_modules_amd.gpu_ready timeline runs/eks1/apply.jsonl \\
        [--k8s-events runs/eks1/k8s_events.json] [--validation-report runs/eks1/validation.json]
    python -m nvidia_terraform_modules_amd.gpu_ready critical-path eks \\
        [--stack-mode operator|daemonsets] [--apply-log runs/eks1/apply.jsonl]

``record`` runs the apply as a CHILD process (output passed through and saved
line by line), and meanwhile polls the cluster with kubectl: the first time
any node reports ``amd.com/gpu`` allocatable becomes the ``gpu_allocatable``
stamp, and the validation Job pods' termination messages (amdgpu-validate's
one-line verdicts, one pod per GPU node: ``--validation-pods``) give
``validation_done``, the last pod's finish. kubectl failures before the
cluster exists are expected and ignored. ``critical-path`` is the offline
model over the plan graph (prior durations, or measured ones from a log).
The reference has none of this (its only figure is "~5 minutes" after apply,
/root/reference/gke/README.md:50).
"""
from __future__ import annotations

import argparse
import json
import shlex
import subprocess
import sys
import threading
import time
from datetime import datetime, timezone
from pathlib import Path

from .apply_timeline import build_timeline, parse_apply_json
from .critical_path import critical_path, durations_from_timeline


def _iso(t: float) -> str:
    return datetime.fromtimestamp(t, tz=timezone.utc).isoformat()


def _kubectl_json(kubectl: list[str], args: list[str], timeout: float = 20.0):
    try:
        p = subprocess.run(kubectl + args + ["-o", "json"], capture_output=True, text=True,
                           timeout=timeout)
    except (OSError, subprocess.TimeoutExpired):
        return None
    if p.returncode != 0:
        return None
    try:
        return json.loads(p.stdout)
    except json.JSONDecodeError:
        return None


class ClusterWatcher(threading.Thread):
    """Polls nodes for amd.com/gpu allocatable and the validation pods for
    their termination messages until stopped.

    The Job runs one pod per GPU node (the module's validation_node_count):
    ``expected_pods`` of them, and as many GPU nodes are watched for their
    first ``amd.com/gpu`` (one GPUAllocatable event each; the timeline's
    gpu_allocatable stamp is the earliest). ``report`` is set once they have all reported:
    the verdict of the pod that finished LAST (its ``end_epoch_s`` is the
    validation_done stamp), with ``per_node`` listing every pod's node, finish
    time and verdict. If apply returns first, ``finish`` builds it from the
    pods seen so far, with ``nodes_validated`` < ``nodes_expected``."""

    def __init__(self, kubectl: list[str], namespace: str, poll_s: float,
                 expected_pods: int = 1):
        super().__init__(daemon=True)
        self.kubectl, self.ns, self.poll_s = kubectl, namespace, poll_s
        self.expected_pods = max(1, expected_pods)
        self.events: list[dict] = []          # k8s-event-shaped records
        self.reports: dict[str, dict] = {}    # pod name -> its verdict
        self.report: dict | None = None
        self._stop_evt = threading.Event()

    def _merge(self) -> dict | None:
        if not self.reports:
            return None
        last = max(self.reports.values(), key=lambda r: r["end_epoch_s"])
        out = {k: v for k, v in last.items() if not k.startswith("_")}
        out["per_node"] = [
            {"pod": pod, "node": r.get("_node"), "end_epoch_s": r["end_epoch_s"],
             "passed": r.get("passed", r.get("ok"))}
            for pod, r in sorted(self.reports.items(), key=lambda kv: kv[1]["end_epoch_s"])]
        out["nodes_validated"] = len(self.reports)
        out["nodes_expected"] = self.expected_pods
        return out

    def finish(self) -> None:
        """Apply has returned: one last poll, then the report from what was seen."""
        self.poll_once()
        if self.report is None:
            self.report = self._merge()

    def _gpu_nodes(self) -> set:
        return {e["involvedObject"]["name"] for e in self.events}

    def poll_once(self) -> None:
        now = time.time()
        # one GPUAllocatable event per node, the first poll that sees its
        # amd.com/gpu; polled until every expected GPU node has reported
        if len(self._gpu_nodes()) < self.expected_pods:
            seen = self._gpu_nodes()
            nodes = _kubectl_json(self.kubectl, ["get", "nodes"])
            for it in (nodes or {}).get("items", []):
                alloc = it.get("status", {}).get("allocatable", {})
                n = alloc.get("amd.com/gpu")
                name = it["metadata"]["name"]
                if n not in (None, "0", 0) and name not in seen:
                    self.events.append({
                        "lastTimestamp": _iso(now),
                        "involvedObject": {"kind": "Node", "name": name},
                        "reason": "GPUAllocatable",
                        "message": f"amd.com/gpu allocatable {n}"})
        if self.report is None:
            pods = _kubectl_json(self.kubectl, ["-n", self.ns, "get", "pods", "-l",
                                                "app.kubernetes.io/name=amd-gpu-validation"])
            for it in (pods or {}).get("items", []):
                name = it.get("metadata", {}).get("name", "?")
                if name in self.reports:
                    continue
                for cs in it.get("status", {}).get("containerStatuses", []):
                    term = cs.get("state", {}).get("terminated")
                    if not term or not term.get("message"):
                        continue
                    try:
                        rep = json.loads(term["message"])
                    except json.JSONDecodeError:
                        continue
                    if not isinstance(rep, dict):
                        continue
                    fin = term.get("finishedAt")
                    if fin:
                        from .apply_timeline import parse_ts
                        rep.setdefault("end_epoch_s", parse_ts(fin))
                    else:
                        rep.setdefault("end_epoch_s", now)
                    rep["_node"] = it.get("spec", {}).get("nodeName")
                    self.reports[name] = rep
            if len(self.reports) >= self.expected_pods:
                self.report = self._merge()

    def run(self) -> None:
        while not self._stop_evt.is_set():
            self.poll_once()
            if len(self._gpu_nodes()) >= self.expected_pods and self.report is not None:
                return
            self._stop_evt.wait(self.poll_s)

    def stop(self) -> None:
        self._stop_evt.set()


def cmd_record(a) -> int:
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    if not a.command:
        print("record: missing command after --", file=sys.stderr)
        return 2
    watcher = None
    if a.kubectl:
        watcher = ClusterWatcher(shlex.split(a.kubectl), a.namespace, a.poll, a.validation_pods)
        watcher.start()
    t0 = time.time()
    with open(out / "apply.jsonl", "w") as log:
        proc = subprocess.Popen(a.command, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                text=True, bufsize=1)
        for line in proc.stdout:
            sys.stdout.write(line)
            log.write(line)
            log.flush()
        rc = proc.wait()
    if watcher is not None:
        watcher.stop()
        watcher.join(timeout=a.poll + 30)
        watcher.finish()                 # apply returned after the Job: catch up
        (out / "k8s_events.json").write_text(json.dumps({"items": watcher.events}, indent=1))
        if watcher.report is not None:
            (out / "validation.json").write_text(json.dumps(watcher.report, indent=1))
    meta = {"command": a.command, "rc": rc, "wall_start": t0, "wall_end": time.time()}
    (out / "record.json").write_text(json.dumps(meta, indent=1))
    lines = (out / "apply.jsonl").read_text().splitlines()
    try:
        tl = build_timeline(lines, watcher.events if watcher else None,
                            watcher.report if watcher else None)
        (out / "timeline.json").write_text(json.dumps(tl.as_dict(), indent=1))
        _print_timeline(tl.as_dict())
    except ValueError as e:
        print(f"record: no timeline ({e})", file=sys.stderr)
    return rc


def _print_timeline(d: dict) -> None:
    print("phase                      seconds")
    for ph, s in d["phase_s"].items():
        print(f"  {ph:<24} {s:8.1f}")
    ttr = d["time_to_gpu_ready_s"]
    print(f"time_to_gpu_ready_s        {ttr:8.1f}" if ttr is not None
          else "time_to_gpu_ready_s        (validation not observed)")


def cmd_timeline(a) -> int:
    lines = Path(a.apply_log).read_text().splitlines()
    ev = json.loads(Path(a.k8s_events).read_text()) if a.k8s_events else None
    rep = json.loads(Path(a.validation_report).read_text()) if a.validation_report else None
    d = build_timeline(lines, ev, rep).as_dict()
    if a.json:
        print(json.dumps(d, indent=1))
    else:
        _print_timeline(d)
    return 0


def cmd_critical_path(a) -> int:
    from ..tfcheck.graph import build_graph

    g = build_graph(a.root)
    durations = None
    if a.apply_log:
        durations = durations_from_timeline(parse_apply_json(Path(a.apply_log).read_text().splitlines()))
    cp = critical_path(g, durations, stack_mode=a.stack_mode,
                       driver_preinstalled=a.driver_preinstalled)
    if a.json:
        print(json.dumps(cp.as_dict(), indent=1))
        return 0
    drv = ", driver preinstalled" if a.driver_preinstalled else ""
    print(f"critical path of {a.root} ({a.stack_mode}{drv}): {cp.total_s:.0f} s")
    for addr, s in cp.path:
        print(f"  {s:7.0f} s  {addr}")
    print("by phase: " + ", ".join(f"{k} {v:.0f}s" for k, v in cp.phases.items()))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gpu_ready", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("record", help="run terraform apply -json and stamp the phases")
    r.add_argument("--out", required=True)
    r.add_argument("--kubectl", default="", help='e.g. "kubectl --kubeconfig ./kubeconfig"')
    r.add_argument("--namespace", default="kube-amd-gpu")
    r.add_argument("--poll", type=float, default=10.0)
    r.add_argument("--validation-pods", type=int, default=1,
                   help="validation pods to wait for: the module's validation_node_count (one "
                        "per GPU node); validation_done = the last one's finish")
    r.add_argument("command", nargs=argparse.REMAINDER)
    t = sub.add_parser("timeline", help="phase table from saved logs")
    t.add_argument("apply_log")
    t.add_argument("--k8s-events")
    t.add_argument("--validation-report")
    t.add_argument("--json", action="store_true")
    c = sub.add_parser("critical-path", help="offline critical path over the plan graph")
    c.add_argument("root")
    c.add_argument("--stack-mode", default="operator", choices=["operator", "daemonsets"])
    c.add_argument("--apply-log", help="measured durations from an apply -json log")
    c.add_argument("--driver-preinstalled", action="store_true",
                   help="the root's gpu_driver_preinstalled = true (no driver install phase)")
    c.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    if a.cmd == "record":
        if a.command and a.command[0] == "--":
            a.command = a.command[1:]
        return cmd_record(a)
    if a.cmd == "timeline":
        return cmd_timeline(a)
    return cmd_critical_path(a)


if __name__ == "__main__":
    sys.exit(main())
