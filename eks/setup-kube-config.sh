#!/usr/bin/env bash
# Write a standalone kubeconfig for the cluster this root module created,
# built only from its outputs (cluster_endpoint, cluster_ca_certificate,
# kube_exec_api_version / _command / _args) - the same exec credential the
# kubernetes/helm providers use. Unlike `aws eks update-kubeconfig` it never
# edits ~/.kube/config (the reference's AKS local-exec did exactly that);
# point KUBECONFIG at the file instead.
#
# usage: ./setup-kube-config.sh [OUTPUT_FILE]      (run after terraform apply, in eks/)
set -euo pipefail
out=${1:-./kubeconfig}
tf() { terraform output -raw "$1"; }

endpoint=$(tf cluster_endpoint)
ca=$(tf cluster_ca_certificate)
api=$(tf kube_exec_api_version)
cmd=$(tf kube_exec_command)
# kube_exec_args is a list: render it as a YAML flow sequence of quoted strings
args=$(terraform output -json kube_exec_args | tr -d '\n' | sed -e 's/^\[//' -e 's/\]$//')

umask 077
cat > "$out" <<KCFG
apiVersion: v1
kind: Config
clusters:
- name: amd-eks
  cluster:
    server: ${endpoint}
    certificate-authority-data: ${ca}
users:
- name: amd-eks
  user:
    exec:
      apiVersion: ${api}
      command: ${cmd}
      args: [${args}]
      interactiveMode: Never
contexts:
- name: amd-eks
  context:
    cluster: amd-eks
    user: amd-eks
current-context: amd-eks
KCFG
echo "wrote ${out}; use: KUBECONFIG=${out} kubectl get nodes"
