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
  node_prep_taint_key=pending:NoSchedule. The prep pod's init chain is
    prep    the script below (host namespaces);
    verify  this pod sees the host PIDs: NUMA balancing is 0 and the RUNNING
            containerd has "Max locked memory unlimited" - i.e. its queued
            restart with the drop-in has happened, so every pod created from
            now on inherits the limit. Fails (kubelet retries it with backoff)
            until then;
    taint   kubectl taint ... --overwrite (idempotent: makes the removal below
            valid on a pod restart, when the taint is already gone);
    untaint kubectl taint ... - (removes it).
  Only the GPU stack's own DaemonSets tolerate the startup taint, so the
  validation Job lands on a node only after a verified prep: no race with the
  containerd restart or the iommu reboot, no fail-and-retry. In "reboot" mode
  the prep step waits for the reboot it requested instead of exiting, so the
  chain never reaches untaint before the reboot.
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
    restart=0
    if [ "$(cat "$dropin" 2>/dev/null || true)" != "$want" ]; then
      mkdir -p "$(dirname "$dropin")"
      printf '%s\n' "$want" > "$dropin"
      systemctl daemon-reload
      restart=1
    fi
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
      # wait for the reboot: the init chain must not go on (and untaint the
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

  # verify step (in the prep pod, hostPID): what the Job's --require-host-prep
  # checks, read from the host - NUMA balancing, and the memlock limit of the
  # containerd that creates the next pods
  node_prep_verify_script = <<-EOT
    set -u
    nb="$(cat /proc/sys/kernel/numa_balancing 2>/dev/null || echo missing)"
    if [ "$nb" != 0 ]; then echo "mi355x gate: kernel.numa_balancing=$nb, waiting"; exit 1; fi
    found=0
    for c in /proc/[0-9]*/comm; do
      [ "$(cat "$c" 2>/dev/null)" = containerd ] || continue
      found=1
      d=$${c%/comm}
      if ! grep -q '^Max locked memory *unlimited' "$d/limits" 2>/dev/null; then
        echo "mi355x gate: containerd ($d) not yet running with LimitMEMLOCK=infinity, waiting"
        exit 1
      fi
    done
    if [ "$found" = 0 ]; then echo "mi355x gate: no containerd process visible, waiting"; exit 1; fi
    echo "mi355x gate: host prep verified"
  EOT
  prep_gate = var.node_prep_enabled && var.node_prep_startup_taint
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
        automount_service_account_token = local.prep_gate
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
        dynamic "init_container" {
          for_each = local.prep_gate ? ["verify"] : []
          content {
            name    = "verify"
            image   = var.node_prep_image
            command = ["sh", "-c", local.node_prep_verify_script]
            security_context {
              allow_privilege_escalation = false
              read_only_root_filesystem  = true
            }
          }
        }
        # ensure, then remove: both single kubectl calls (no shell in the
        # image); "kubectl taint ... -" fails on an absent taint, the ensure
        # step makes it present on every run
        dynamic "init_container" {
          for_each = local.prep_gate ? {
            taint   = "${var.node_prep_taint_key}=pending:NoSchedule"
            untaint = "${var.node_prep_taint_key}=pending:NoSchedule-"
          } : {}
          content {
            name    = init_container.key
            image   = var.kubectl_image
            command = concat(["kubectl", "taint", "node", "$(NODE_NAME)", init_container.value],
            init_container.key == "taint" ? ["--overwrite"] : [])
            env {
              name = "NODE_NAME"
              value_from {
                field_ref {
                  field_path = "spec.nodeName"
                }
              }
            }
            security_context {
              allow_privilege_escalation = false
              run_as_non_root            = true
              run_as_user                = 65532
            }
          }
        }
        container {
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
    }
  }
}
