/********************************************
  Shared locals
********************************************/
locals {
  common_labels = merge({
    "app.kubernetes.io/part-of"    = "amd-gpu-stack"
    "app.kubernetes.io/managed-by" = "terraform"
    "cluster"                      = var.cluster_name
  }, var.labels)

  namespace      = var.create_namespace ? kubernetes_namespace_v1.gpu_stack[0].metadata[0].name : var.gpu_operator_namespace
  operator_mode  = var.gpu_stack_mode == "operator"
  gpu_resource   = "amd.com/gpu"
  node_pool_hash = sha1(join(",", var.gpu_node_pool_ids))

  # CRDs the destroy-time janitor may delete: the KMM CRDs only when this
  # release installs KMM (driver_enabled), the NFD ones only when it installs
  # NFD. Otherwise they belong to a separate cluster-wide install, and deleting
  # a CRD cascades to every CR of that kind in the cluster.
  crd_cleanup_list = [
    for crd in var.gpu_operator_crds : crd
    if alltrue([
      var.driver_enabled || !endswith(crd, ".kmm.sigs.x-k8s.io"),
      var.install_node_feature_discovery || !endswith(crd, ".nfd.k8s-sigs.io"),
    ])
  ]

  # the startup taint of not-yet-prepared GPU nodes (node-prep.tf): tolerated
  # by the GPU stack's own components (they install beside the prep), never by
  # the validation Job
  prep_tolerations = var.node_prep_enabled && var.node_prep_startup_taint ? [
    { key = var.node_prep_taint_key, operator = "Exists", effect = "NoSchedule" },
  ] : []
  gpu_tolerations = concat([
    { key = var.gpu_node_taint_key, operator = "Exists", effect = "NoSchedule" },
  ], local.prep_tolerations)

  # One typed map, one code path, AMD only: rendered once with yamlencode.
  operator_values = {
    "node-feature-discovery" = {
      enabled = var.install_node_feature_discovery
      worker = {
        tolerations = local.gpu_tolerations
      }
    }
    controllerManager = {
      manager = {
        env = [{ name = "CLUSTER_NAME", value = var.cluster_name }]
      }
    }
    kmm = {
      enabled = var.driver_enabled
    }
    installdefaultNFDRule = true
    crds = {
      defaultCR = {
        install = false # the DeviceConfig below is ours
      }
    }
  }

  device_config_values = {
    name      = "${var.cluster_name}-mi355x"
    namespace = local.namespace
    spec = {
      # Every component the operator places on the (tainted) GPU nodes carries
      # the GPU toleration - the KMM driver build/load pods included: without
      # it amd.com/gpu never becomes allocatable and apply waits out
      # validation_timeout. tfcheck rule gpu-toleration enforces this.
      driver = merge({
        enable      = var.driver_enabled
        blacklist   = true
        version     = var.gpu_operator_driver_version
        tolerations = local.gpu_tolerations
      }, var.driver_image_repository == "" ? {} : { image = var.driver_image_repository })
      devicePlugin = {
        devicePluginImage       = var.device_plugin_image
        nodeLabellerImage       = var.node_labeller_image
        enableNodeLabeller      = true
        devicePluginTolerations = local.gpu_tolerations
        nodeLabellerTolerations = local.gpu_tolerations
      }
      metricsExporter = {
        enable      = var.metrics_exporter_enabled
        image       = var.metrics_exporter_image
        port        = var.metrics_exporter_port
        serviceType = "ClusterIP"
        tolerations = local.gpu_tolerations
      }
      selector = var.gpu_node_selector
    }
    serviceMonitor = {
      enabled   = var.service_monitor_enabled
      port      = var.metrics_exporter_port
      selector  = { "app.kubernetes.io/name" = "amd-device-metrics-exporter" }
      namespace = local.namespace
    }
  }
}

/********************************************
  Namespace (+ critical-priority quota, GKE)
********************************************/
resource "kubernetes_namespace_v1" "gpu_stack" {
  count = var.create_namespace ? 1 : 0

  metadata {
    name   = var.gpu_operator_namespace
    labels = merge(local.common_labels, { "pod-security.kubernetes.io/enforce" = "privileged" })
  }
}

# GKE only admits system-*-critical pods outside kube-system when a quota
# scoped to those PriorityClasses exists (reference gke/main.tf:173-191).
resource "kubernetes_resource_quota_v1" "critical_pods" {
  count = var.critical_pod_quota ? 1 : 0

  metadata {
    name      = "amd-gpu-critical-pods"
    namespace = local.namespace
    labels    = local.common_labels
  }
  spec {
    hard = {
      pods = 200
    }
    scope_selector {
      match_expression {
        operator   = "In"
        scope_name = "PriorityClass"
        values     = ["system-node-critical", "system-cluster-critical"]
      }
    }
  }
}

/********************************************
  AMD GPU Operator (operator mode)
********************************************/
# CRD cleanup on destroy. `helm uninstall` of the operator leaves its CRDs
# (DeviceConfig, KMM, NFD) behind; the reference removed them through the
# NVIDIA chart's operator.cleanupCRD value (/root/reference/aks/main.tf:89-91).
# The AMD chart's equivalent cannot be pinned offline, so the module owns it:
# this release is created BEFORE the operator (which depends on it), hence
# destroyed AFTER it, and its pre-delete hook Job deletes the CRDs.
resource "helm_release" "crd_janitor" {
  count = local.operator_mode && var.gpu_operator_crd_cleanup ? 1 : 0

  name      = "amd-gpu-crd-janitor"
  chart     = "${path.module}/charts/amd-gpu-crd-janitor"
  namespace = local.namespace
  atomic    = true
  timeout   = var.helm_timeout_seconds
  values = [yamlencode({
    name   = "amd-gpu-crd-janitor"
    image  = var.kubectl_image
    crds   = local.crd_cleanup_list
    labels = local.common_labels
  })]

  depends_on = [kubernetes_resource_quota_v1.critical_pods]
}

resource "helm_release" "amd_gpu_operator" {
  count = local.operator_mode ? 1 : 0

  name             = "amd-gpu-operator"
  repository       = var.gpu_operator_chart_repository
  chart            = var.gpu_operator_chart_name
  version          = var.gpu_operator_version
  namespace        = local.namespace
  create_namespace = false
  atomic           = true
  cleanup_on_fail  = true
  reset_values     = true # reference eks/main.tf:193-196: no values carried over on upgrade
  wait             = true
  timeout          = var.helm_timeout_seconds
  values           = [yamlencode(local.operator_values)]

  depends_on = [kubernetes_resource_quota_v1.critical_pods, helm_release.crd_janitor]
}

# The DeviceConfig CR is rendered by a module-local chart instead of
# kubernetes_manifest: kubernetes_manifest needs the CRD at PLAN time, which
# does not exist on a cluster created in the same apply. Destroy order is
# the reverse: CR first (operator finalizers run), then the operator - the
# reason the reference needed `terraform state rm` (gke/README.md:59).
resource "helm_release" "device_config" {
  count = local.operator_mode ? 1 : 0

  name      = "amd-gpu-deviceconfig"
  chart     = "${path.module}/charts/amd-gpu-extras"
  namespace = local.namespace
  atomic    = true
  wait      = true
  timeout   = var.helm_timeout_seconds
  values    = [yamlencode(merge(local.device_config_values, { mode = "operator" }))]

  depends_on = [helm_release.amd_gpu_operator]
}
