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
      exit 0
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
        host_pid            = true
        priority_class_name = "system-node-critical"
        node_selector       = var.gpu_node_selector
        toleration {
          key      = var.gpu_node_taint_key
          operator = "Exists"
          effect   = "NoSchedule"
        }
        init_container {
          name    = "prep"
          image   = var.node_prep_image
          command = ["nsenter", "--target", "1", "--mount", "--uts", "--ipc", "--net", "--pid", "--", "sh", "-c", local.node_prep_script]
          security_context {
            privileged = true
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
