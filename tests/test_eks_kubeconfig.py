"""eks/setup-kube-config.sh builds a kubeconfig from the module outputs only
(no aws CLI call, no ~/.kube/config edit). A stub `terraform` serves the
outputs."""
import os
import stat
import subprocess
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[1]

STUB = r'''#!/usr/bin/env bash
case "$*" in
  "output -raw cluster_endpoint") printf 'https://ABC.gr7.us-west-2.eks.amazonaws.com' ;;
  "output -raw cluster_ca_certificate") printf 'LS0tLS1CRUdJTg==' ;;
  "output -raw kube_exec_api_version") printf 'client.authentication.k8s.io/v1beta1' ;;
  "output -raw kube_exec_command") printf 'aws' ;;
  "output -json kube_exec_args") printf '[\n  "eks",\n  "get-token",\n  "--cluster-name",\n  "tf-mi355x",\n  "--region",\n  "us-west-2"\n]\n' ;;
  *) echo "unexpected: $*" >&2; exit 3 ;;
esac
'''


def test_kubeconfig_from_outputs(tmp_path):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    tf = bindir / "terraform"
    tf.write_text(STUB)
    tf.chmod(tf.stat().st_mode | stat.S_IEXEC)
    out = tmp_path / "kc"
    home = tmp_path / "home"
    home.mkdir()
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", HOME=str(home))
    subprocess.run(["bash", str(ROOT / "eks" / "setup-kube-config.sh"), str(out)], check=True,
                   env=env, cwd=tmp_path, capture_output=True, timeout=60)
    cfg = yaml.safe_load(out.read_text())
    assert cfg["clusters"][0]["cluster"]["server"].startswith("https://")
    assert cfg["clusters"][0]["cluster"]["certificate-authority-data"] == "LS0tLS1CRUdJTg=="
    ex = cfg["users"][0]["user"]["exec"]
    assert ex["command"] == "aws" and ex["apiVersion"].endswith("v1beta1")
    assert ex["args"] == ["eks", "get-token", "--cluster-name", "tf-mi355x", "--region", "us-west-2"]
    assert cfg["current-context"] == "amd-eks"
    assert oct(out.stat().st_mode & 0o777) == "0o600"       # credentials file
    assert not (home / ".kube").exists()                    # never touches ~/.kube
