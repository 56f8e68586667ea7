# round-4 fp8 store-path study + GEMM clock check (one gpurun call)
bash tools/gpu_run.sh r4_clock clock && \
PMC_DTYPE=fp8 bash tools/gpu_run.sh r4_fp8pmc_8192 pmc && \
PMC_DTYPE=fp8 PMC_SHAPE=8192x8192x4096 bash tools/gpu_run.sh r4_fp8pmc_8k8k4k pmc && \
PMC_DTYPE=fp8 PMC_SHAPE=4096x4096x4096 bash tools/gpu_run.sh r4_fp8pmc_4096 pmc
