/************************
  Identity
*************************/
variable "cluster_name" {
  type        = string
  description = "Name of the Kubernetes cluster (used for labels and object names)."
}

variable "labels" {
  type        = map(string)
  default     = {}
  description = "Extra labels applied to every Kubernetes object this module creates."
}

/************************
  Deployment mode
*************************/
variable "gpu_stack_mode" {
  type        = string
  default     = "operator"
  description = "How the amdgpu driver and the amd.com/gpu device plugin get onto GPU nodes: \"operator\" (AMD GPU Operator Helm chart + DeviceConfig CR) or \"daemonsets\" (explicit amdgpu-dkms installer + rocm/k8s-device-plugin + node labeller DaemonSets, no operator)."

  validation {
    condition     = contains(["operator", "daemonsets"], var.gpu_stack_mode)
    error_message = "gpu_stack_mode must be \"operator\" or \"daemonsets\"."
  }
}

/************************
  AMD GPU Operator (names kept from the reference's gpu_operator_* variables)
*************************/
variable "gpu_operator_version" {
  type        = string
  default     = "v1.3.0"
  description = "AMD GPU Operator Helm chart version (chart gpu-operator-charts). Pin a release that lists gfx950 / MI355X support."
}

variable "gpu_operator_driver_version" {
  type        = string
  default     = "7.0.2"
  description = "amdgpu kernel driver version (ROCm release) the operator / DKMS installer puts on GPU nodes. ROCm 7.x is required for gfx950."

  validation {
    condition     = can(regex("^[0-9]+\\.[0-9]+(\\.[0-9]+)?$", var.gpu_operator_driver_version)) && tonumber(split(".", var.gpu_operator_driver_version)[0]) >= 7
    error_message = "gpu_operator_driver_version must be a ROCm release >= 7.0 (MI355X / gfx950 needs ROCm 7)."
  }
}

variable "gpu_operator_namespace" {
  type        = string
  default     = "kube-amd-gpu"
  description = "Namespace for the AMD GPU Operator / device plugin / exporter / validation Job."
}

variable "gpu_operator_chart_repository" {
  type        = string
  default     = "https://rocm.github.io/gpu-operator"
  description = "Helm repository of the AMD GPU Operator chart."
}

variable "gpu_operator_chart_name" {
  type        = string
  default     = "gpu-operator-charts"
  description = "Chart name inside gpu_operator_chart_repository."
}

variable "gpu_operator_crd_cleanup" {
  type        = bool
  default     = true
  description = "Delete the operator's CRDs on destroy, after the operator release is gone (pre-delete hook of a module-local chart running kubectl_image). Only the CRDs this release installs are deleted: the KMM ones only with driver_enabled, the NFD ones only with install_node_feature_discovery. Parity with the reference's operator.cleanupCRD=true (aks/main.tf:89-91). Escape hatch: false skips the hook (e.g. when kubectl_image cannot be pulled, which would block destroy)."
}

variable "gpu_operator_crds" {
  type = list(string)
  default = [
    "deviceconfigs.amd.com",
    "modules.kmm.sigs.x-k8s.io",
    "nodemodulesconfigs.kmm.sigs.x-k8s.io",
    "preflightvalidations.kmm.sigs.x-k8s.io",
    "nodefeatures.nfd.k8s-sigs.io",
    "nodefeaturerules.nfd.k8s-sigs.io",
    "nodefeaturegroups.nfd.k8s-sigs.io",
  ]
  description = "CRDs the AMD GPU Operator chart (with its KMM and NFD subcharts) registers; deleted on destroy when gpu_operator_crd_cleanup."
}

variable "kubectl_image" {
  type        = string
  default     = "registry.k8s.io/kubectl:v1.31.4"
  description = "Image with kubectl for the destroy-time CRD cleanup Job (the Kubernetes project's own registry; Bitnami stopped publishing versioned tags on docker.io). It is pulled only at destroy time: if the GPU nodes' cluster cannot pull it (air-gapped, registry allow-list), mirror it and set this, or set gpu_operator_crd_cleanup = false - a hook whose image cannot be pulled fails after its 300 s deadline and blocks `terraform destroy` of the operator."
}

variable "create_namespace" {
  type        = bool
  default     = true
  description = "Create gpu_operator_namespace (set false when it already exists)."
}

variable "critical_pod_quota" {
  type        = bool
  default     = false
  description = "Create a ResourceQuota admitting system-node-critical / system-cluster-critical pods in the namespace (required on GKE for critical-priority DaemonSets outside kube-system; reference gke/main.tf:173-191)."
}

variable "install_node_feature_discovery" {
  type        = bool
  default     = true
  description = "Let the operator chart install Node Feature Discovery (labels feature.node.kubernetes.io/amd-gpu)."
}

variable "helm_timeout_seconds" {
  type        = number
  default     = 900
  description = "Helm wait timeout for the operator release."
}

/************************
  Driver / device plugin / labeller / exporter
*************************/
variable "driver_enabled" {
  type        = bool
  default     = true
  description = "Install the amdgpu driver on GPU nodes (false only for node images that ship amdgpu for gfx950 already)."
}

variable "driver_image_repository" {
  type        = string
  default     = ""
  description = "Optional registry for operator-built driver images (DeviceConfig spec.driver.image). Empty = operator default."
}

variable "amdgpu_dkms_image" {
  type        = string
  default     = "docker.io/library/ubuntu:22.04"
  description = "daemonsets mode: image of the privileged, hostPID installer pod; it only needs nsenter (util-linux) because the install runs in the host's namespaces."
}

variable "amdgpu_repo_base_url" {
  type        = string
  default     = "https://repo.radeon.com/amdgpu-install"
  description = "daemonsets mode: base URL of the amdgpu-install packages (mirror it for air-gapped node pools)."
}

variable "device_plugin_image" {
  type        = string
  default     = "docker.io/rocm/k8s-device-plugin:1.31.0.7"
  description = "rocm/k8s-device-plugin image (registers amd.com/gpu with the kubelet)."
}

variable "node_labeller_image" {
  type        = string
  default     = "docker.io/rocm/k8s-device-plugin:labeller-1.31.0.7"
  description = "rocm/k8s-device-plugin node labeller image (amd.com/gpu.family, .device-id, .vram ...)."
}

variable "metrics_exporter_enabled" {
  type        = bool
  default     = true
  description = "Deploy the AMD device-metrics-exporter (GPU utilisation, HBM, power, xGMI counters) on GPU nodes."
}

variable "metrics_exporter_image" {
  type        = string
  default     = "docker.io/rocm/device-metrics-exporter:v1.3.0"
  description = "AMD device-metrics-exporter image."
}

variable "metrics_exporter_native" {
  type        = bool
  default     = false
  description = "Run the native amdgpu-exporter (AMD SMI, shipped in validation_image) instead of metrics_exporter_image in daemonsets mode."
}

variable "metrics_exporter_port" {
  type        = number
  default     = 5000
  description = "Port the metrics exporter serves Prometheus metrics on."
}

variable "service_monitor_enabled" {
  type        = bool
  default     = false
  description = "Create a Prometheus-operator ServiceMonitor for the exporter (needs the monitoring.coreos.com CRDs, e.g. from the CNPack Prometheus stack)."
}

variable "gpu_node_selector" {
  type        = map(string)
  default     = { "amd.com/gpu.present" = "true" }
  description = "Node labels that identify MI355X GPU nodes (set by the node pools of the root modules)."
}

variable "gpu_node_taint_key" {
  type        = string
  default     = "amd.com/gpu"
  description = "Taint key placed on GPU node pools; every GPU DaemonSet / Job tolerates it."
}

variable "gpu_node_pool_ids" {
  type        = list(string)
  default     = []
  description = "IDs of the GPU node pools. Only the validation Job depends on them, so the namespace / operator / DeviceConfig install overlaps with GPU node boot (the operator controller runs on CPU nodes)."
}

/************************
  Post-provision validation Job
*************************/
variable "validation_enabled" {
  type        = bool
  default     = true
  description = "Run the MI355X validation Job (HIP bf16 MFMA GEMM + HBM stream + RCCL all-reduce over xGMI) after the stack is up."
}

variable "validation_image" {
  type        = string
  default     = ""
  description = "Image built from validation/image/Dockerfile and pushed to a registry the nodes can pull from (contains only the amdgpu-validate binary + ROCm runtime + RCCL). Required when validation_enabled (or metrics_exporter_native): there is no public default, and a wrong one would sit in ImagePullBackOff until validation_timeout."
}

variable "prepull_validation_image" {
  type        = bool
  default     = true
  description = "Pull the validation image on GPU nodes as they join (DaemonSet), in parallel with the driver install, so the Job starts the moment amd.com/gpu is allocatable."
}

variable "pause_image" {
  type        = string
  default     = "registry.k8s.io/pause:3.10"
  description = "Image of the pre-pull DaemonSet's idle container."
}

variable "validation_gpu_count" {
  type        = number
  default     = 8
  description = "amd.com/gpu requested by the validation Job (1, 2, 4 or 8 MI355X on one node)."

  validation {
    condition     = contains([1, 2, 4, 8], var.validation_gpu_count)
    error_message = "validation_gpu_count must be 1, 2, 4 or 8 (GPUs of one MI355X node)."
  }
}

variable "validation_node_count" {
  type        = number
  default     = 1
  description = "GPU nodes the validation Job covers: one pod per node, all at once (completions = parallelism = this, required pod anti-affinity on the hostname). The roots pass the GPU pools' size at creation, so apply returns only once every GPU node has passed. Above 1 the Job's backoffLimit is 0: a retry could land on a node that already passed and hide the one that failed."

  validation {
    condition     = var.validation_node_count >= 1 && floor(var.validation_node_count) == var.validation_node_count
    error_message = "validation_node_count must be a whole number >= 1."
  }
}

variable "validation_gemm_size" {
  type        = number
  default     = 8192
  description = "M = N = K of the per-GPU validation GEMM (multiple of 256)."

  validation {
    condition     = var.validation_gemm_size >= 256 && var.validation_gemm_size % 256 == 0
    error_message = "validation_gemm_size must be a positive multiple of 256."
  }
}

variable "validation_tflops_floor" {
  type        = number
  default     = 1000
  description = "Per-GPU bf16 GEMM TFLOP/s below which the Job fails (MI355X dense bf16 peak ~2500; the hand-written kernel measures ~1600 at 8192^3)."
}

variable "validation_fp8" {
  type        = bool
  default     = true
  description = "Also run and verify the OCP e4m3 GEMM on the MX-scaled matrix cores (K1-fp8)."
}

variable "validation_fp8_tflops_floor" {
  type        = number
  default     = 2000
  description = "Per-GPU e4m3 GEMM TFLOP/s below which the Job fails (the hand-written kernel measures ~3100 at 8192^3; 0 disables the floor)."

  validation {
    condition     = var.validation_fp8_tflops_floor >= 0
    error_message = "validation_fp8_tflops_floor must be >= 0."
  }
}

variable "validation_p2p_floor_gbps" {
  type        = number
  default     = 0
  description = "Per-link xGMI pull bandwidth (GB/s, dst <- src, one pair at a time) below which the Job fails; 0 reports the matrix without a floor."

  validation {
    condition     = var.validation_p2p_floor_gbps >= 0
    error_message = "validation_p2p_floor_gbps must be >= 0."
  }
}

variable "validation_min_hbm_gb" {
  type        = number
  default     = 250
  description = "Per-GPU HBM capacity floor in GB (MI355X: 288 GB HBM3E)."
}

variable "validation_allreduce_max_mib" {
  type        = number
  default     = 1024
  description = "Largest RCCL all-reduce message in the busbw sweep."
}

variable "validation_backoff_limit" {
  type        = number
  default     = 1
  description = "Job backoffLimit."
}

variable "validation_active_deadline_seconds" {
  type        = number
  default     = 900
  description = "Job activeDeadlineSeconds (hard stop for a hung GPU)."
}

variable "validation_timeout" {
  type        = string
  default     = "20m"
  description = "How long terraform waits for the Job to complete (wait_for_completion)."
}

variable "wait_for_validation" {
  type        = bool
  default     = true
  description = "Make terraform apply block until the validation Job succeeded: apply returning == GPUs proven usable."
}

variable "validation_env" {
  type        = map(string)
  default     = {}
  description = "Extra environment for the validation container (e.g. NCCL_DEBUG=INFO)."
}

/************************
  MI355X host preparation (node-prep.tf)
*************************/
variable "node_prep_enabled" {
  type        = bool
  default     = true
  description = "Run the privileged mi355x-node-prep DaemonSet on the GPU nodes: automatic NUMA balancing off, containerd LimitMEMLOCK=infinity, iommu=pt per node_prep_iommu_mode. Idempotent (EKS user data applies the same settings before the join; here it then only verifies)."
}

variable "node_prep_startup_taint" {
  type        = bool
  default     = false
  description = "The GPU node pools carry the startup taint node_prep_taint_key=pending:NoSchedule (the eks / gke / aks roots set it with gpu_node_prep_taint). The node-prep DaemonSet removes it from a node once the host prep is verified there (NUMA balancing off, containerd running with LimitMEMLOCK=infinity, so every pod created afterwards inherits it); only the GPU-stack DaemonSets tolerate it, never the validation Job, which therefore lands on prepared nodes only. Needs kubectl_image at node-join time and a ClusterRole that may get / patch nodes."
}

variable "node_prep_taint_key" {
  type        = string
  default     = "startup-taint.cluster-autoscaler.kubernetes.io/amd-mi355x-prep"
  description = "Key of the GPU node pools' startup taint (node_prep_startup_taint). The cluster-autoscaler prefix marks it as a startup taint: the autoscaler ignores it when it simulates whether a pending pod (the validation Job) fits a new node, so the gate never blocks a scale-up."
}

variable "node_prep_iommu_mode" {
  type        = string
  default     = "check"
  description = "iommu=pt handling on the GPU nodes: \"check\" records whether the kernel booted with it, \"reboot\" adds it to GRUB and reboots each node at most once, \"off\" skips it. A kernel argument needs a boot: prefer a node image that has it (EKS gpu_ami_id). WARNING: applying \"reboot\" to nodes that already run workloads reboots all of them at once (no cordon / drain); nodes that join behind the node_prep_startup_taint carry no workloads yet, so for them it is safe."

  validation {
    condition     = contains(["off", "check", "reboot"], var.node_prep_iommu_mode)
    error_message = "node_prep_iommu_mode must be \"off\", \"check\" or \"reboot\"."
  }
}

variable "node_prep_gate_image" {
  type        = string
  default     = "docker.io/alpine/k8s:1.31.4"
  description = "Image of the node-prep startup-taint gate (node_prep_startup_taint): a long-running reconciler loop, so it needs a POSIX shell and kubectl in one image (registry.k8s.io/kubectl has no shell). Pulled when a GPU node joins: mirror it for air-gapped clusters."
}

variable "node_prep_gate_interval_s" {
  type        = number
  default     = 30
  description = "Seconds between the gate's checks of its node: a startup taint that a cloud reconciler re-applies (node-group update, pool-taint reconciliation) is removed again, after re-verifying the host prep, within this interval."

  validation {
    condition     = var.node_prep_gate_interval_s >= 5 && var.node_prep_gate_interval_s <= 600
    error_message = "node_prep_gate_interval_s must be between 5 and 600 seconds."
  }
}

variable "node_prep_image" {
  type        = string
  default     = "docker.io/library/ubuntu:22.04"
  description = "Image of the node-prep init container; it only needs nsenter (util-linux): the script runs in the host's namespaces."
}

variable "validation_require_host_prep" {
  type        = bool
  default     = true
  description = "The validation Job fails (amdgpu-validate --require-host-prep) unless its pod sees kernel.numa_balancing = 0 and an unlimited RLIMIT_MEMLOCK. Only passed while node_prep_enabled."
}

variable "validation_require_iommu_pt" {
  type        = bool
  default     = false
  description = "The validation Job also fails unless the node kernel booted with iommu=pt (amdgpu-validate --require-iommu-pt)."
}

/************************
  Interconnect gates of the validation Job
*************************/
variable "validation_rccl_busbw_floor_gbps" {
  type        = number
  default     = 0
  description = "Peak bf16 RCCL all-reduce busbw (GB/s) below which the Job fails; applied when validation_gpu_count > 1. 0 = report only. Set it from the first 8-GPU measurement of the node type (no such number exists yet: BASELINE has none, and the single-GPU development boxes cannot produce one)."

  validation {
    condition     = var.validation_rccl_busbw_floor_gbps >= 0
    error_message = "validation_rccl_busbw_floor_gbps must be >= 0."
  }
}

variable "validation_xgmi_busbw_floor_gbps" {
  type        = number
  default     = 0
  description = "The same floor for the hand-written xGMI all-reduce (C2); applied when validation_gpu_count > 1. 0 = report only."

  validation {
    condition     = var.validation_xgmi_busbw_floor_gbps >= 0
    error_message = "validation_xgmi_busbw_floor_gbps must be >= 0."
  }
}
