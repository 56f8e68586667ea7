/********************************************
  Post-provision validation Job
  -----------------------------
  The reference has no readiness gate: `apply` returns before the NVIDIA
  operator has even loaded a driver (~5 min later per gke/README.md:50) and
  its helm_release count-gate on data.aws_instances never actually waits
  (eks/main.tf:186). Here `apply` blocks on a Job that requests amd.com/gpu
  (so it only schedules once the device plugin has registered GPUs) and runs
  the hand-written HIP bf16 / fp8 MFMA GEMMs + HBM stream + RCCL all-reduce
  over xGMI + a per-link xGMI pull matrix. Job completion timestamp == end of
  time-to-GPU-ready.
  One pod per GPU node (validation_node_count, from the pools' size at
  creation): all pods run at once, a required anti-affinity on the hostname
  puts each on its own node, and the Job completes when every node passed.
  (The reference's GPU group starts with 2 nodes, /root/reference/eks/
  variables.tf:86-90, and nothing checks either of them.)
********************************************/
locals {
  validation_multi_gpu  = var.validation_gpu_count > 1
  validation_multi_node = var.validation_node_count > 1
  validation_labels     = merge(local.common_labels, { "app.kubernetes.io/name" = "amd-gpu-validation" })
  validation_args = concat(
    [
      "--gpus", tostring(var.validation_gpu_count),
      "--size", tostring(var.validation_gemm_size),
      "--tflops-floor", tostring(var.validation_tflops_floor),
      "--min-hbm-gb", tostring(var.validation_min_hbm_gb),
      "--allreduce-max-mib", tostring(var.validation_allreduce_max_mib),
      "--json",
    ],
    var.validation_fp8 ? [
      "--fp8-tflops-floor", tostring(var.validation_fp8_tflops_floor),
    ] : ["--no-fp8"],
    var.validation_p2p_floor_gbps > 0 ? [
      "--p2p-floor-gbps", tostring(var.validation_p2p_floor_gbps),
    ] : [],
    local.validation_multi_gpu && var.validation_rccl_busbw_floor_gbps > 0 ? [
      "--rccl-busbw-floor-gbps", tostring(var.validation_rccl_busbw_floor_gbps),
    ] : [],
    local.validation_multi_gpu && var.validation_xgmi_busbw_floor_gbps > 0 ? [
      "--xgmi-busbw-floor-gbps", tostring(var.validation_xgmi_busbw_floor_gbps),
    ] : [],
    # the hand-written all-reduce runs in the configuration a mini-sweep picks
    # (blocks per rank x one-shot cutoff, well under 2 s at 8 GPUs)
    local.validation_multi_gpu ? ["--xgmi-tune"] : [],
    var.node_prep_enabled && var.validation_require_host_prep ? ["--require-host-prep"] : [],
    var.validation_require_iommu_pt ? ["--require-iommu-pt"] : [],
    # one-line verdict surfaced as the pod's termination message
    ["--termination-log", "/dev/termination-log"],
  )
  validation_env = merge({
    # RCCL over the xGMI mesh inside one node; no host network transport needed
    NCCL_IB_DISABLE        = "1"
    NCCL_SOCKET_IFNAME     = "lo"
    HSA_NO_SCRATCH_RECLAIM = "1"
  }, var.validation_env)
}

resource "kubernetes_job_v1" "gpu_validation" {
  count = var.validation_enabled ? 1 : 0

  metadata {
    name      = "amd-gpu-validation"
    namespace = local.namespace
    labels    = local.validation_labels
    annotations = {
      "amd-gpu-stack/gpu-node-pools" = local.node_pool_hash
      "amd-gpu-stack/stack-mode"     = var.gpu_stack_mode
    }
  }

  spec {
    # one pod per node: a retry could land on a node that already passed and
    # hide the node that failed, so several nodes get no retry
    backoff_limit              = local.validation_multi_node ? 0 : var.validation_backoff_limit
    active_deadline_seconds    = var.validation_active_deadline_seconds
    ttl_seconds_after_finished = 86400
    completions                = var.validation_node_count
    parallelism                = var.validation_node_count

    template {
      metadata {
        labels = local.validation_labels
      }
      spec {
        restart_policy = "Never"
        host_ipc       = true # RCCL peer-to-peer IPC between the ranks' GPU buffers
        node_selector  = var.gpu_node_selector

        # every pod on its own GPU node (the pods run at once: parallelism =
        # completions), also when validation_gpu_count leaves room for two
        affinity {
          pod_anti_affinity {
            required_during_scheduling_ignored_during_execution {
              label_selector {
                match_labels = { "app.kubernetes.io/name" = "amd-gpu-validation" }
              }
              topology_key = "kubernetes.io/hostname"
            }
          }
        }

        # The GPU taint only: NOT the node-prep startup taint
        # (node_prep_startup_taint), so the Job schedules on a node only after
        # the prep has been verified there and containerd restarted with
        # LimitMEMLOCK=infinity - no race with the prep, no fail-and-retry.
        toleration {
          key      = var.gpu_node_taint_key
          operator = "Exists"
          effect   = "NoSchedule"
        }

        container {
          name    = "amdgpu-validate"
          image   = var.validation_image
          command = ["/opt/ntm/bin/amdgpu-validate"]
          args    = local.validation_args

          termination_message_path   = "/dev/termination-log"
          termination_message_policy = "FallbackToLogsOnError"

          security_context {
            allow_privilege_escalation = false
            read_only_root_filesystem  = true
            capabilities {
              drop = ["ALL"]
            }
          }

          dynamic "env" {
            for_each = local.validation_env
            content {
              name  = env.key
              value = env.value
            }
          }
          # the node's name in the verdict, the metrics and the termination message
          # (one pod per GPU node)
          env {
            name = "NODE_NAME"
            value_from {
              field_ref {
                field_path = "spec.nodeName"
              }
            }
          }

          resources {
            limits = {
              (local.gpu_resource) = tostring(var.validation_gpu_count)
              memory               = "64Gi"
            }
            requests = {
              (local.gpu_resource) = tostring(var.validation_gpu_count)
              cpu                  = tostring(var.validation_gpu_count * 2)
              memory               = "32Gi"
            }
          }

          volume_mount {
            name       = "dshm"
            mount_path = "/dev/shm"
          }
        }

        volume {
          name = "dshm"
          empty_dir {
            medium     = "Memory"
            size_limit = "16Gi"
          }
        }
      }
    }
  }

  wait_for_completion = var.wait_for_validation

  lifecycle {
    precondition {
      condition     = var.validation_image != ""
      error_message = "validation_enabled needs validation_image: build validation/image/Dockerfile, push it to a registry the GPU nodes can pull from, and pass its reference (or set validation_enabled = false)."
    }
  }

  timeouts {
    create = var.validation_timeout
    update = var.validation_timeout
  }

  depends_on = [
    helm_release.device_config,
    kubernetes_daemon_set_v1.rocm_device_plugin,
    kubernetes_daemon_set_v1.amdgpu_dkms,
    kubernetes_daemon_set_v1.node_prep,
  ]
}

/********************************************
  Validation image pre-pull
  -------------------------
  The Job can only schedule once amd.com/gpu is allocatable, i.e. after the
  amdgpu driver is loaded on a GPU node (minutes: KMM/DKMS). Without help its
  image pull starts only then and sits on the critical path. This DaemonSet
  depends on nothing but the namespace, so it lands on every GPU node as the
  node joins and pulls the image while the driver installs; its init
  container runs `amdgpu-validate --help`, which also proves the image's
  runtime-library closure links on the node before any GPU is up.
  apply does not wait for its rollout (nodes may still be booting).
********************************************/
resource "kubernetes_daemon_set_v1" "validation_prepull" {
  count = var.validation_enabled && var.prepull_validation_image ? 1 : 0

  metadata {
    name      = "amd-gpu-validation-prepull"
    namespace = local.namespace
    labels    = merge(local.common_labels, { "app.kubernetes.io/name" = "amd-gpu-validation-prepull" })
  }

  wait_for_rollout = false

  spec {
    selector {
      match_labels = { "app.kubernetes.io/name" = "amd-gpu-validation-prepull" }
    }
    template {
      metadata {
        labels = merge(local.common_labels, { "app.kubernetes.io/name" = "amd-gpu-validation-prepull" })
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
        init_container {
          name    = "pull-and-link-check"
          image   = var.validation_image
          command = ["/opt/ntm/bin/amdgpu-validate", "--help"]
          security_context {
            allow_privilege_escalation = false
            read_only_root_filesystem  = true
            capabilities {
              drop = ["ALL"]
            }
          }
        }
        container {
          name  = "hold"
          image = var.pause_image
          resources {
            requests = {
              cpu    = "1m"
              memory = "8Mi"
            }
            limits = {
              memory = "16Mi"
            }
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
