"""The node-prep startup-taint gate: the reconciler
script the module ships, run for real with sh against a fake /proc and a stub
kubectl that keeps the node's taints in a file; the DaemonSet / RBAC /
precondition wiring through tfcheck's evaluator and plan."""
import os
import stat
import subprocess
import time
from pathlib import Path

import pytest

from nvidia_terraform_modules_amd.tfcheck.config import load_module
from nvidia_terraform_modules_amd.tfcheck.docs import render
from nvidia_terraform_modules_amd.tfcheck.plan import plan

ROOT = Path(__file__).resolve().parents[1]
STACK_DIR = ROOT / "modules" / "amd-gpu-stack"
KEY = "startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep"

STUB_KUBECTL = r"""#!/bin/sh
# stub: node taints live in $TAINTS (one key per line); every call is logged
echo "$*" >> "$KUBECTL_LOG"
if [ "$1" = get ] && [ "$2" = node ]; then
  [ -f "$TAINTS" ] && cat "$TAINTS"
  exit 0
fi
if [ "$1" = taint ] && [ "$2" = node ]; then
  spec="$4"
  case "$spec" in
    *-) key="${spec%%:*}"
        grep -qxF "$key" "$TAINTS" 2>/dev/null || { echo "taint $key not found" >&2; exit 1; }
        grep -vxF "$key" "$TAINTS" > "$TAINTS.new"; mv "$TAINTS.new" "$TAINTS"; exit 0 ;;
  esac
fi
echo "stub kubectl: unsupported $*" >&2
exit 2
"""


def _script(name: str, strict: bool = True) -> str:
    e = load_module(STACK_DIR).locals[name][0]
    if strict:
        assert all(isinstance(p, str) for p in e.parts), "gate script must not interpolate HCL"
    return "".join(p for p in e.parts if isinstance(p, str))


@pytest.fixture
def node(tmp_path):
    proc = tmp_path / "proc"
    (proc / "sys" / "kernel").mkdir(parents=True)
    (proc / "sys" / "kernel" / "numa_balancing").write_text("0\n")
    for pid, comm, memlock in ((1, "systemd", "65536"), (812, "containerd", "unlimited"),
                               (900, "kubelet", "65536")):
        d = proc / str(pid)
        d.mkdir()
        (d / "comm").write_text(comm + "\n")
        (d / "limits").write_text(
            "Limit                     Soft Limit           Hard Limit           Units\n"
            f"Max locked memory         {memlock:<20} {memlock:<20} bytes\n")
    bindir = tmp_path / "bin"
    bindir.mkdir()
    k = bindir / "kubectl"
    k.write_text(STUB_KUBECTL)
    k.chmod(k.stat().st_mode | stat.S_IEXEC)
    taints = tmp_path / "taints"
    taints.write_text(f"amd.com/gpu\n{KEY}\n")
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", PROC_ROOT=str(proc),
               NODE_NAME="gpu-node-0", TAINT_KEY=KEY, GATE_INTERVAL_S="0.2",
               TAINTS=str(taints), KUBECTL_LOG=str(tmp_path / "kubectl.log"))
    return {"proc": proc, "taints": taints, "env": env, "log": tmp_path / "kubectl.log"}


def _once(node):
    env = dict(node["env"], GATE_ONCE="1")
    return subprocess.run(["sh", "-c", _script("node_prep_gate_script")], env=env,
                          capture_output=True, text=True, timeout=30)


def _keys(node):
    return node["taints"].read_text().split()


def test_gate_removes_the_taint_after_verifying(node):
    p = _once(node)
    assert p.returncode == 0, p.stderr
    assert _keys(node) == ["amd.com/gpu"]                      # only the prep taint goes
    assert f"taint node gpu-node-0 {KEY}:NoSchedule-" in node["log"].read_text()
    assert "host prep verified" in p.stdout
    # nothing to do on the next pass: no taint call at all
    before = node["log"].read_text().count("taint node")
    assert _once(node).returncode == 0
    assert node["log"].read_text().count("taint node") == before


@pytest.mark.parametrize("breakage,reason", [
    ("numa", "kernel.numa_balancing=1"),
    ("memlock", "not yet running with LimitMEMLOCK=infinity"),
    ("no-containerd", "no containerd process visible"),
])
def test_gate_keeps_the_taint_until_the_prep_holds(node, breakage, reason):
    if breakage == "numa":
        (node["proc"] / "sys" / "kernel" / "numa_balancing").write_text("1\n")
    elif breakage == "memlock":
        (node["proc"] / "812" / "limits").write_text("Max locked memory 65536 65536 bytes\n")
    else:
        (node["proc"] / "812" / "comm").write_text("containerd-shim\n")
    p = _once(node)
    assert p.returncode == 0 and reason in p.stdout
    assert KEY in _keys(node)
    assert "taint node" not in node["log"].read_text()


def test_reapplied_taint_is_removed_again(node):
    """The reconciler loop: a cloud re-applies the pool taint after the first
    removal (node-group update); the gate re-verifies and removes it again
    within its interval - and leaves it while the prep does not hold."""
    proc = subprocess.Popen(["sh", "-c", _script("node_prep_gate_script")], env=node["env"],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)

    def wait_for(cond, timeout=10.0):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if cond():
                return True
            time.sleep(0.05)
        return False

    try:
        assert wait_for(lambda: KEY not in _keys(node))
        node["taints"].write_text(f"amd.com/gpu\n{KEY}\n")          # re-applied
        assert wait_for(lambda: KEY not in _keys(node))
        # a containerd restarted WITHOUT the limit: the re-applied taint stays
        (node["proc"] / "812" / "limits").write_text("Max locked memory 65536 65536 bytes\n")
        node["taints"].write_text(f"amd.com/gpu\n{KEY}\n")
        time.sleep(1.0)
        assert KEY in _keys(node)
        (node["proc"] / "812" / "limits").write_text("Max locked memory unlimited unlimited bytes\n")
        assert wait_for(lambda: KEY not in _keys(node))
        assert proc.poll() is None                                   # still reconciling
    finally:
        proc.kill()
        proc.wait(timeout=10)
    assert node["log"].read_text().count(f"{KEY}:NoSchedule-") == 3


def test_gate_survives_an_api_error(node):
    env = dict(node["env"], GATE_ONCE="1", PATH="/usr/bin:/bin")   # no kubectl at all
    p = subprocess.run(["sh", "-c", _script("node_prep_gate_script")], env=env,
                       capture_output=True, text=True, timeout=30)
    assert p.returncode == 0 and "cannot read node" in p.stdout


def test_prep_restarts_containerd_from_the_running_limit():
    """the restart is decided from the running containerd's limits, so a
    run that wrote the drop-in and lost its restart still restarts it next time."""
    s = _script("node_prep_script", strict=False)
    i_file = s.index('"$dropin"')
    i_proc = s.index("Max locked memory *unlimited")
    i_restart = s.index("systemctl --no-block restart containerd")
    assert i_file < i_proc < i_restart
    block = s[s.index("restart=0"):s.index("# 3. iommu=pt")]
    assert "/limits" in block and "restart=1" in block and "$dropin" not in block


def _blocks(body, btype):
    return [b for b in body.blocks if b.type == btype]


def _pod_spec(res):
    spec = _blocks(res.block.body, "spec")[0]
    tmpl = _blocks(spec.body, "template")[0]
    return _blocks(tmpl.body, "spec")[0].body


def test_daemonset_runs_the_reconciler_and_scopes_the_token():
    from test_host_prep_and_driver import _eval

    stack = load_module(STACK_DIR)
    spec = _pod_spec(stack.resources["kubernetes_daemon_set_v1.node_prep"])
    assert render(spec.attr("automount_service_account_token")) == "false"
    inits = _blocks(spec, "init_container")
    assert [render(b.body.attr("name")) for b in inits] == ['"prep"']
    assert not [b for b in _blocks(spec, "dynamic") if b.labels == ["init_container"]]
    conts = {b.labels[0]: b for b in _blocks(spec, "dynamic") if b.labels == ["container"]}
    dyn = [b for b in _blocks(spec, "dynamic") if b.labels == ["container"]]
    assert len(dyn) == 2 and not conts.get("x")
    fe = [_eval(STACK_DIR, b.body.attr("for_each"), node_prep_startup_taint=True) for b in dyn]
    assert fe == [["gate"], []]
    fe_off = [_eval(STACK_DIR, b.body.attr("for_each")) for b in dyn]
    assert fe_off == [[], ["hold"]]
    gate = _blocks(dyn[0].body, "content")[0].body
    assert render(gate.attr("image")) == "var.node_prep_gate_image"
    assert render(gate.attr("command")) == '["sh", "-c", local.node_prep_gate_script]'
    envs = {render(e.body.attr("name")) for e in _blocks(gate, "env")}
    assert {'"NODE_NAME"', '"TAINT_KEY"', '"GATE_INTERVAL_S"'} <= envs
    mounts = [render(m.body.attr("mount_path")) for m in _blocks(gate, "volume_mount")]
    assert '"/var/run/secrets/kubernetes.io/serviceaccount"' in mounts
    sc = _blocks(gate, "security_context")[0].body
    assert render(sc.attr("run_as_non_root")) == "true"
    # the privileged prep container gets no token mount
    prep = inits[0].body
    assert not _blocks(prep, "volume_mount")
    role = stack.resources["kubernetes_cluster_role_v1.node_prep"].block.body
    assert render(_blocks(role, "rule")[0].body.attr("verbs")) == '["get", "patch"]'


def _stack_plan(tmp_path, **kv):
    """Plan a throwaway root that calls the module with these inputs."""
    args = "\n".join(f"  {k} = {str(v).lower() if isinstance(v, bool) else repr(v)}"
                     for k, v in kv.items())
    src = os.path.relpath(STACK_DIR, tmp_path)                     # a LOCAL module path
    (tmp_path / "main.tf").write_text(
        f'module "stack" {{\n  source = "{src}"\n  cluster_name = "c"\n'
        f'  validation_enabled = false\n{args}\n}}\n')
    r = plan(tmp_path)
    assert not r.registry_modules, r.registry_modules
    return r


def test_startup_taint_without_prep_is_refused(tmp_path):
    bad = _stack_plan(tmp_path, node_prep_enabled=False, node_prep_startup_taint=True)
    assert any("node_prep_startup_taint needs node_prep_enabled" in e for e in bad.errors), bad.errors
    good = _stack_plan(tmp_path, node_prep_enabled=True, node_prep_startup_taint=True)
    assert not [e for e in good.errors if "precondition" in e], good.errors
    assert "module.stack.kubernetes_daemon_set_v1.node_prep[0]" in good.resources
    off = _stack_plan(tmp_path, node_prep_enabled=False, node_prep_startup_taint=False)
    assert not [e for e in off.errors if "precondition" in e], off.errors
