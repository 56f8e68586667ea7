"""amdgpu-exporter (validation/src/amdgpu_exporter.cpp): Prometheus text
format, no-GPU behaviour on CPU, real metrics + HTTP serving on MI355X."""
import re
import signal
import socket
import subprocess
import time
import urllib.request
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "validation" / "build" / "amdgpu-exporter"
SAMPLE = re.compile(r'^[a-zA-Z_:][a-zA-Z0-9_:]*(\{[a-zA-Z_][a-zA-Z0-9_]*="[^"]*"'
                    r'(,[a-zA-Z_][a-zA-Z0-9_]*="[^"]*")*\})? -?[0-9.eE+-]+$')


def _have():
    if not BIN.exists():
        pytest.skip("amdgpu-exporter not built")


def parse(text):
    """Strict-enough Prometheus text parser: every family has HELP + TYPE,
    every sample line is well formed. Returns {name: [(labels, value)]}."""
    out, typed = {}, set()
    for ln in text.splitlines():
        if ln.startswith("# TYPE "):
            typed.add(ln.split()[2])
            continue
        if ln.startswith("#") or not ln:
            continue
        assert SAMPLE.match(ln), ln
        name = ln.split("{")[0].split(" ")[0]
        assert name in typed, f"sample before TYPE: {ln}"
        labels = dict(re.findall(r'([a-zA-Z_]+)="([^"]*)"', ln.split(" ")[0]))
        out.setdefault(name, []).append((labels, float(ln.rsplit(" ", 1)[1])))
    return out


def test_once_without_gpu_reports_down():
    _have()
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    p = subprocess.run([str(BIN), "--once"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 2
    m = parse(p.stdout)
    assert m["amdgpu_exporter_up"][0][1] == 0 and m["amdgpu_gpu_count"][0][1] == 0


def test_bad_arguments():
    _have()
    p = subprocess.run([str(BIN), "--port"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 2 and "usage" in p.stderr


@pytest.mark.gpu
def test_once_on_mi355x():
    _have()
    p = subprocess.run([str(BIN), "--once"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stdout + p.stderr
    m = parse(p.stdout)
    assert m["amdgpu_exporter_up"][0][1] == 1
    assert m["amdgpu_gpu_count"][0][1] >= 1
    total = m["amdgpu_vram_total_bytes"][0][1]
    assert total > 250e9                              # 288 GB HBM3E class
    assert 0 <= m["amdgpu_vram_used_bytes"][0][1] <= total
    assert any(k.startswith("amdgpu_temperature") or k.startswith("amdgpu_socket_power")
               for k in m), sorted(m)


@pytest.mark.gpu
def test_http_serving_and_sigterm():
    _have()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.Popen([str(BIN), "--port", str(port)], stderr=subprocess.PIPE, text=True)
    try:
        body = None
        for _ in range(50):
            try:
                body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read()
                break
            except OSError:
                time.sleep(0.1)
        assert body is not None
        assert parse(body.decode())["amdgpu_exporter_up"][0][1] == 1
        assert urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5).read() == b"ok\n"
    finally:
        p.send_signal(signal.SIGTERM)   # must interrupt the blocked accept()
        rc = p.wait(timeout=10)
    assert rc == 0
