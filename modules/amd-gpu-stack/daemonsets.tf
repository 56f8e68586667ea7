/********************************************
  daemonsets mode: explicit amdgpu-dkms + rocm/k8s-device-plugin
  (no operator; AMD only - there is no vendor switch anywhere)
********************************************/
locals {
  ds_mode = var.gpu_stack_mode == "daemonsets"

  # Host preparation, run on the node through nsenter into PID 1's
  # namespaces: install amdgpu-dkms for the running kernel from
  # repo.radeon.com (package name layout: amdgpu-install_<M>.<m>.<M><mm><pp>-1,
  # e.g. 7.0.2 -> 7.0.70002-1), then load the module. Idempotent; the sentinel
  # makes restarts cheap (seconds, no DKMS rebuild).
  dkms_script = <<-EOT
    set -euo pipefail
    want="${var.gpu_operator_driver_version}"
    sentinel="/var/lib/amdgpu-dkms/installed-$want-$(uname -r)"
    if [ ! -f "$sentinel" ]; then
      . /etc/os-release
      IFS=. read -r M m p <<<"$want.0"
      pkg=$(printf 'amdgpu-install_%s.%s.%d%02d%02d-1_all.deb' "$M" "$m" "$M" "$m" "$${p:-0}")
      url="${var.amdgpu_repo_base_url}/$want/ubuntu/$VERSION_CODENAME/$pkg"
      export DEBIAN_FRONTEND=noninteractive
      curl -fsSL -o /tmp/amdgpu-install.deb "$url"
      apt-get update -y
      apt-get install -y "linux-headers-$(uname -r)" "linux-modules-extra-$(uname -r)" || true
      apt-get install -y /tmp/amdgpu-install.deb
      amdgpu-install -y --usecase=dkms --no-32
      mkdir -p /var/lib/amdgpu-dkms && touch "$sentinel"
    fi
    modprobe amdgpu
    test -e /dev/kfd
    echo "amdgpu ready: $(cat /sys/module/amdgpu/version 2>/dev/null || echo loaded)"
  EOT
}

resource "kubernetes_daemon_set_v1" "amdgpu_dkms" {
  count = local.ds_mode && var.driver_enabled ? 1 : 0

  metadata {
    name      = "amdgpu-dkms-installer"
    namespace = local.namespace
    labels    = merge(local.common_labels, { "app.kubernetes.io/name" = "amdgpu-dkms-installer" })
  }

  spec {
    selector {
      match_labels = { "app.kubernetes.io/name" = "amdgpu-dkms-installer" }
    }
    template {
      metadata {
        labels = merge(local.common_labels, { "app.kubernetes.io/name" = "amdgpu-dkms-installer" })
      }
      spec {
        host_pid             = true
        priority_class_name  = "system-node-critical"
        node_selector        = var.gpu_node_selector
        service_account_name = "default"
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
          name    = "install"
          image   = var.amdgpu_dkms_image
          command = ["nsenter", "--target", "1", "--mount", "--uts", "--ipc", "--net", "--pid", "--", "bash", "-c", local.dkms_script]
          security_context {
            privileged = true
          }
        }
        container {
          name    = "hold"
          image   = var.amdgpu_dkms_image
          command = ["sleep", "infinity"]
          resources {
            requests = { cpu = "10m", memory = "16Mi" }
            limits   = { memory = "64Mi" }
          }
        }
      }
    }
  }
}

resource "kubernetes_daemon_set_v1" "rocm_device_plugin" {
  count = local.ds_mode ? 1 : 0

  metadata {
    name      = "amdgpu-device-plugin"
    namespace = local.namespace
    labels    = merge(local.common_labels, { "app.kubernetes.io/name" = "amdgpu-device-plugin" })
  }

  spec {
    selector {
      match_labels = { "app.kubernetes.io/name" = "amdgpu-device-plugin" }
    }
    template {
      metadata {
        labels = merge(local.common_labels, { "app.kubernetes.io/name" = "amdgpu-device-plugin" })
      }
      spec {
        priority_class_name = "system-node-critical"
        node_selector       = var.gpu_node_selector
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
        container {
          name  = "device-plugin"
          image = var.device_plugin_image
          args  = ["-pulse", "30"]
          security_context {
            privileged = true
          }
          volume_mount {
            name       = "device-plugins"
            mount_path = "/var/lib/kubelet/device-plugins"
          }
          volume_mount {
            name       = "sys"
            mount_path = "/sys"
          }
          resources {
            requests = { cpu = "10m", memory = "32Mi" }
            limits   = { memory = "128Mi" }
          }
        }
        volume {
          name = "device-plugins"
          host_path {
            path = "/var/lib/kubelet/device-plugins"
          }
        }
        volume {
          name = "sys"
          host_path {
            path = "/sys"
          }
        }
      }
    }
  }

  depends_on = [kubernetes_daemon_set_v1.amdgpu_dkms]
}

resource "kubernetes_service_account_v1" "node_labeller" {
  count = local.ds_mode ? 1 : 0
  metadata {
    name      = "amdgpu-node-labeller"
    namespace = local.namespace
    labels    = local.common_labels
  }
}

resource "kubernetes_cluster_role_v1" "node_labeller" {
  count = local.ds_mode ? 1 : 0
  metadata {
    name   = "${var.cluster_name}-amdgpu-node-labeller"
    labels = local.common_labels
  }
  rule {
    api_groups = [""]
    resources  = ["nodes"]
    verbs      = ["get", "list", "watch", "patch", "update"]
  }
}

resource "kubernetes_cluster_role_binding_v1" "node_labeller" {
  count = local.ds_mode ? 1 : 0
  metadata {
    name   = "${var.cluster_name}-amdgpu-node-labeller"
    labels = local.common_labels
  }
  role_ref {
    api_group = "rbac.authorization.k8s.io"
    kind      = "ClusterRole"
    name      = kubernetes_cluster_role_v1.node_labeller[0].metadata[0].name
  }
  subject {
    kind      = "ServiceAccount"
    name      = kubernetes_service_account_v1.node_labeller[0].metadata[0].name
    namespace = local.namespace
  }
}

resource "kubernetes_daemon_set_v1" "node_labeller" {
  count = local.ds_mode ? 1 : 0

  metadata {
    name      = "amdgpu-node-labeller"
    namespace = local.namespace
    labels    = merge(local.common_labels, { "app.kubernetes.io/name" = "amdgpu-node-labeller" })
  }

  spec {
    selector {
      match_labels = { "app.kubernetes.io/name" = "amdgpu-node-labeller" }
    }
    template {
      metadata {
        labels = merge(local.common_labels, { "app.kubernetes.io/name" = "amdgpu-node-labeller" })
      }
      spec {
        service_account_name = kubernetes_service_account_v1.node_labeller[0].metadata[0].name
        node_selector        = var.gpu_node_selector
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
        container {
          name  = "labeller"
          image = var.node_labeller_image
          args  = ["-vram", "-cu-count", "-simd-count", "-device-id", "-family", "-product-name", "-driver-version"]
          env {
            name = "DS_NODE_NAME"
            value_from {
              field_ref {
                field_path = "spec.nodeName"
              }
            }
          }
          security_context {
            privileged = true
          }
          volume_mount {
            name       = "sys"
            mount_path = "/sys"
          }
          volume_mount {
            name       = "dev"
            mount_path = "/dev"
          }
        }
        volume {
          name = "sys"
          host_path {
            path = "/sys"
          }
        }
        volume {
          name = "dev"
          host_path {
            path = "/dev"
          }
        }
      }
    }
  }

  depends_on = [kubernetes_daemon_set_v1.amdgpu_dkms]
}

/********************************************
  Metrics exporter (daemonsets mode; the operator deploys its own)
********************************************/
resource "kubernetes_daemon_set_v1" "metrics_exporter" {
  count = local.ds_mode && var.metrics_exporter_enabled ? 1 : 0

  metadata {
    name      = "amd-device-metrics-exporter"
    namespace = local.namespace
    labels    = merge(local.common_labels, { "app.kubernetes.io/name" = "amd-device-metrics-exporter" })
  }

  spec {
    selector {
      match_labels = { "app.kubernetes.io/name" = "amd-device-metrics-exporter" }
    }
    template {
      metadata {
        labels = merge(local.common_labels, { "app.kubernetes.io/name" = "amd-device-metrics-exporter" })
        annotations = {
          "prometheus.io/scrape" = "true"
          "prometheus.io/port"   = tostring(var.metrics_exporter_port)
        }
      }
      spec {
        node_selector = var.gpu_node_selector
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
        container {
          name  = "exporter"
          image = var.metrics_exporter_native ? var.validation_image : var.metrics_exporter_image
          # native exporter: validation/src/amdgpu_exporter.cpp (AMD SMI, /metrics + /healthz)
          command = var.metrics_exporter_native ? ["/opt/ntm/bin/amdgpu-exporter", "--port", tostring(var.metrics_exporter_port)] : null
          port {
            name           = "metrics"
            container_port = var.metrics_exporter_port
          }
          security_context {
            privileged = true
          }
          volume_mount {
            name       = "dev"
            mount_path = "/dev"
          }
          volume_mount {
            name       = "pod-resources"
            mount_path = "/var/lib/kubelet/pod-resources"
          }
          readiness_probe {
            http_get {
              path = "/metrics"
              port = var.metrics_exporter_port
            }
            period_seconds = 15
          }
        }
        volume {
          name = "dev"
          host_path {
            path = "/dev"
          }
        }
        volume {
          name = "pod-resources"
          host_path {
            path = "/var/lib/kubelet/pod-resources"
          }
        }
      }
    }
  }

  lifecycle {
    precondition {
      condition     = !var.metrics_exporter_native || var.validation_image != ""
      error_message = "metrics_exporter_native runs amdgpu-exporter from validation_image: set validation_image."
    }
  }

  depends_on = [kubernetes_daemon_set_v1.amdgpu_dkms]
}

resource "kubernetes_service_v1" "metrics_exporter" {
  count = local.ds_mode && var.metrics_exporter_enabled ? 1 : 0

  metadata {
    name      = "amd-device-metrics-exporter"
    namespace = local.namespace
    labels    = merge(local.common_labels, { "app.kubernetes.io/name" = "amd-device-metrics-exporter" })
  }
  spec {
    selector = { "app.kubernetes.io/name" = "amd-device-metrics-exporter" }
    port {
      name        = "metrics"
      port        = var.metrics_exporter_port
      target_port = var.metrics_exporter_port
    }
  }
}

# ServiceMonitor in daemonsets mode goes through the same local chart.
resource "helm_release" "service_monitor" {
  count = local.ds_mode && var.metrics_exporter_enabled && var.service_monitor_enabled ? 1 : 0

  name      = "amd-gpu-servicemonitor"
  chart     = "${path.module}/charts/amd-gpu-extras"
  namespace = local.namespace
  values    = [yamlencode(merge(local.device_config_values, { mode = "daemonsets" }))]

  depends_on = [kubernetes_service_v1.metrics_exporter]
}
