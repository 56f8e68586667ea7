/********************************************
  MI355X host preparation, every cloud
  ------------------------------------
  The same three host settings EKS applies in its pre-bootstrap user data
  (eks/cluster.tf local.mi355x_host_prep), as a privileged DaemonSet on the
  GPU nodes, so GKE and AKS - whose managed node images take no bootstrap
  script, and whose linux_node_config / linux_os_config sysctl allow-lists do
  not include kernel.numa_balancing - get them too:
   * automatic NUMA balancing off (it migrates pinned HBM staging buffers);
   * containerd's systemd unit gets LimitMEMLOCK=infinity, so every pod
     inherits an unlimited RLIMIT_MEMLOCK (RCCL pins host memory); the
     restart is queued (--no-block) and happens once per node;
   * iommu=pt: "check" records whether the kernel booted with it; "reboot"
     adds it to GRUB and reboots the node at most ONCE (sentinel; a second
     miss logs a warning and proceeds); "off" leaves it alone. A kernel
     argument is a boot-time setting: the cloud-neutral way is a node image
     that already has it (EKS gpu_ami_id); GKE / AKS managed images cannot be
     changed, so "reboot" is the only in-cluster lever there.
  The reference's per-pool bootstrap hook is /root/reference/eks/main.tf:95-97
  (post_bootstrap_user_data); it had nothing for GKE / AKS.
  The validation Job re-checks the result from inside its pod
  (amdgpu-validate --require-host-prep), so a node whose prep has not taken
  effect fails the readiness gate instead of passing it.

  Gate (node_prep_startup_taint): the GPU pools join with the startup taint
  node_prep_taint_key=pending:NoSchedule. The prep pod runs
    prep    the script below (init container, host namespaces);
    gate    a reconciler (main container, node_prep_gate_image: sh + kubectl)
            that checks the node every node_prep_gate_interval_s seconds. When
            the node carries the startup taint it verifies the prep - this
            pod sees the host PIDs: NUMA balancing is 0 and the RUNNING
            containerd has "Max locked memory unlimited", i.e. its restart
            with the drop-in has happened, so every pod created from now on
            inherits the limit - and only then removes the taint. A taint that
            comes back (an EKS node-group update, AKS / GKE pool-taint
            reconciliation) is removed again at the next check, after the same
            verification: no human has to delete the pod.
  Only the GPU stack's own DaemonSets tolerate the startup taint, so the
  validation Job lands on a node only after a verified prep: no race with the
  containerd restart or the iommu reboot, no fail-and-retry. In "reboot" mode
  the prep step waits for the reboot it requested instead of exiting, so the
  gate never starts before the reboot.
  API access: the gate container alone mounts a (projected, short-lived)
  service-account token - get + patch on nodes; the privileged prep container
  gets none (automount is off for the pod).
********************************************/
locals {
  node_prep_script = <<-EOT
    set -eu
    mode="${var.node_prep_iommu_mode}"
    log=/var/log/mi355x-host-prep.log
    # 1. automatic NUMA balancing off, now and on every boot
    printf 'kernel.numa_balancing = 0\n' > /etc/sysctl.d/60-mi355x.conf
    if [ -w /proc/sys/kernel/numa_balancing ]; then echo 0 > /proc/sys/kernel/numa_balancing; fi
    # 2. containerd LimitMEMLOCK=infinity (inherited by every container)
    dropin=/etc/systemd/system/containerd.service.d/60-memlock.conf
    want="$(printf '[Service]\nLimitMEMLOCK=infinity')"
    if [ "$(cat "$dropin" 2>/dev/null || true)" != "$want" ]; then
      mkdir -p "$(dirname "$dropin")"
      printf '%s\n' "$want" > "$dropin"
    fi
    # restart decided from the RUNNING containerd (what the gate checks), not
    # from the file: a run that wrote the drop-in and lost its queued restart
    # (killed pod, failed reload) must not leave the node gated forever
    restart=0
    for c in /proc/[0-9]*/comm; do
      [ "$(cat "$c" 2>/dev/null)" = containerd ] || continue
      grep -q '^Max locked memory *unlimited' "$${c%/comm}/limits" 2>/dev/null || restart=1
    done
    if [ "$restart" = 1 ]; then systemctl daemon-reload; fi
    # 3. iommu=pt (boot-time kernel argument)
    sentinel=/var/lib/mi355x-iommu-rebooted
    if grep -qw 'iommu=pt' /proc/cmdline; then
      iommu=on
    elif [ "$mode" = "reboot" ] && [ ! -f "$sentinel" ]; then
      { grep -q 'iommu=pt' /etc/default/grub ||
          sed -i 's/^GRUB_CMDLINE_LINUX="/&iommu=pt /' /etc/default/grub; } || true
      update-grub || echo "WARNING update-grub failed" >> "$log"
      mkdir -p /var/lib && touch "$sentinel"
      echo "mi355x: adding iommu=pt, rebooting once" >> "$log"
      systemctl --no-block reboot
      # wait for the reboot: the gate must not start (and untaint the
      # node) before it; a reboot that never comes fails this step (retried)
      sleep 600
      exit 1
    elif [ "$mode" = "reboot" ]; then
      iommu="absent-after-reboot"
      echo "WARNING iommu=pt still absent after one reboot; continuing without it" >> "$log"
    else
      iommu=absent
    fi
    echo "mi355x node prep: numa_balancing=$(cat /proc/sys/kernel/numa_balancing) memlock-dropin=ok iommu=$iommu mode=$mode" | tee -a "$log"
    # last: containerd restarts after this container has exited (running
    # containers keep running across a containerd restart)
    if [ "$restart" = 1 ]; then systemctl --no-block restart containerd; fi
  EOT

  # gate reconciler (the prep pod's main container, hostPID, sh + kubectl):
  # what the Job's --require-host-prep checks, read from the host - NUMA
  # balancing, and the memlock limit of the containerd that creates the next
  # pods - gates the removal of the startup taint, re-checked every
  # GATE_INTERVAL_S. PROC_ROOT / GATE_ONCE exist for the offline test
  # (tests/test_node_prep_gate.py: fake /proc, stub kubectl).
  node_prep_gate_script = <<-EOT
    set -u
    proc="$${PROC_ROOT:-/proc}"
    verify() {
      nb="$(cat "$proc/sys/kernel/numa_balancing" 2>/dev/null || echo missing)"
      if [ "$nb" != 0 ]; then echo "mi355x gate: kernel.numa_balancing=$nb, waiting"; return 1; fi
      found=0
      for c in "$proc"/[0-9]*/comm; do
        [ "$(cat "$c" 2>/dev/null)" = containerd ] || continue
        found=1
        d="$${c%/comm}"
        if ! grep -q '^Max locked memory *unlimited' "$d/limits" 2>/dev/null; then
          echo "mi355x gate: containerd ($d) not yet running with LimitMEMLOCK=infinity, waiting"
          return 1
        fi
      done
      if [ "$found" = 0 ]; then echo "mi355x gate: no containerd process visible, waiting"; return 1; fi
      return 0
    }
    while :; do
      if keys="$(kubectl get node "$NODE_NAME" -o jsonpath='{range .spec.taints[*]}{.key}{"\n"}{end}')"; then
        if printf '%s\n' "$keys" | grep -qxF "$TAINT_KEY"; then
          if verify; then
            kubectl taint node "$NODE_NAME" "$TAINT_KEY:NoSchedule-" &&
              echo "mi355x gate: host prep verified, $TAINT_KEY removed from $NODE_NAME"
          fi
        fi
      else
        echo "mi355x gate: cannot read node $NODE_NAME, retrying"
      fi
      [ -n "$${GATE_ONCE:-}" ] && exit 0
      sleep "$GATE_INTERVAL_S"
    done
  EOT
  prep_gate             = var.node_prep_enabled && var.node_prep_startup_taint
}

# The gate's API access: get + patch on Node objects, nothing else.
resource "kubernetes_service_account_v1" "node_prep" {
  count = local.prep_gate ? 1 : 0
  metadata {
    name      = "mi355x-node-prep"
    namespace = local.namespace
    labels    = local.common_labels
  }
}

resource "kubernetes_cluster_role_v1" "node_prep" {
  count = local.prep_gate ? 1 : 0
  metadata {
    name   = "${var.cluster_name}-mi355x-node-prep"
    labels = local.common_labels
  }
  rule {
    api_groups = [""]
    resources  = ["nodes"]
    verbs      = ["get", "patch"]
  }
}

resource "kubernetes_cluster_role_binding_v1" "node_prep" {
  count = local.prep_gate ? 1 : 0
  metadata {
    name   = "${var.cluster_name}-mi355x-node-prep"
    labels = local.common_labels
  }
  role_ref {
    api_group = "rbac.authorization.k8s.io"
    kind      = "ClusterRole"
    name      = kubernetes_cluster_role_v1.node_prep[0].metadata[0].name
  }
  subject {
    kind      = "ServiceAccount"
    name      = kubernetes_service_account_v1.node_prep[0].metadata[0].name
    namespace = local.namespace
  }
}

resource "kubernetes_daemon_set_v1" "node_prep" {
  count = var.node_prep_enabled ? 1 : 0

  metadata {
    name      = "mi355x-node-prep"
    namespace = local.namespace
    labels    = merge(local.common_labels, { "app.kubernetes.io/name" = "mi355x-node-prep" })
  }

  # GPU nodes may still be booting when this is created (the stack installs
  # beside them); the Job's in-pod check is the gate, not this rollout
  wait_for_rollout = false

  spec {
    selector {
      match_labels = { "app.kubernetes.io/name" = "mi355x-node-prep" }
    }
    template {
      metadata {
        labels = merge(local.common_labels, { "app.kubernetes.io/name" = "mi355x-node-prep" })
      }
      spec {
        host_pid                        = true
        priority_class_name             = "system-node-critical"
        node_selector                   = var.gpu_node_selector
        service_account_name            = local.prep_gate ? kubernetes_service_account_v1.node_prep[0].metadata[0].name : "default"
        automount_service_account_token = false
        toleration {
          key      = var.gpu_node_taint_key
          operator = "Exists"
          effect   = "NoSchedule"
        }
        dynamic "toleration" {
          for_each = local.prep_tolerations
          content {
            key      = toleration.value.key
            operator = toleration.value.operator
            effect   = toleration.value.effect
          }
        }
        init_container {
          name    = "prep"
          image   = var.node_prep_image
          command = ["nsenter", "--target", "1", "--mount", "--uts", "--ipc", "--net", "--pid", "--", "sh", "-c", local.node_prep_script]
          security_context {
            privileged = true
          }
        }
        dynamic "container" {
          for_each = local.prep_gate ? ["gate"] : []
          content {
            name    = "gate"
            image   = var.node_prep_gate_image
            command = ["sh", "-c", local.node_prep_gate_script]
            env {
              name = "NODE_NAME"
              value_from {
                field_ref {
                  field_path = "spec.nodeName"
                }
              }
            }
            env {
              name  = "TAINT_KEY"
              value = var.node_prep_taint_key
            }
            env {
              name  = "GATE_INTERVAL_S"
              value = tostring(var.node_prep_gate_interval_s)
            }
            env {
              # kubectl's discovery cache: the root filesystem is read-only
              name  = "HOME"
              value = "/tmp"
            }
            volume_mount {
              name       = "gate-token"
              mount_path = "/var/run/secrets/kubernetes.io/serviceaccount"
              read_only  = true
            }
            volume_mount {
              name       = "gate-tmp"
              mount_path = "/tmp"
            }
            resources {
              requests = { cpu = "5m", memory = "32Mi" }
              limits   = { memory = "128Mi" }
            }
            security_context {
              allow_privilege_escalation = false
              read_only_root_filesystem  = true
              run_as_non_root            = true
              run_as_user                = 65532
              capabilities {
                drop = ["ALL"]
              }
            }
          }
        }
        dynamic "container" {
          for_each = local.prep_gate ? [] : ["hold"]
          content {
            name  = "hold"
            image = var.pause_image
            resources {
              requests = { cpu = "1m", memory = "8Mi" }
              limits   = { memory = "16Mi" }
            }
            security_context {
              allow_privilege_escalation = false
              read_only_root_filesystem  = true
              capabilities {
                drop = ["ALL"]
              }
            }
          }
        }
        dynamic "volume" {
          for_each = local.prep_gate ? ["gate-tmp"] : []
          content {
            name = volume.value
            empty_dir {
              size_limit = "16Mi"
            }
          }
        }
        # the gate's API token, for the gate container only (what automount
        # would give every container: token, cluster CA, namespace)
        dynamic "volume" {
          for_each = local.prep_gate ? ["gate-token"] : []
          content {
            name = volume.value
            projected {
              default_mode = "0444"
              sources {
                service_account_token {
                  path               = "token"
                  expiration_seconds = 3607
                }
              }
              sources {
                config_map {
                  name = "kube-root-ca.crt"
                  items {
                    key  = "ca.crt"
                    path = "ca.crt"
                  }
                }
              }
              sources {
                downward_api {
                  items {
                    path = "namespace"
                    field_ref {
                      field_path = "metadata.namespace"
                    }
                  }
                }
              }
            }
          }
        }
      }
    }
  }
}
