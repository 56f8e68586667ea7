# round-4: race screens of the new K1 builds, the GEMM clock check, and the
# fp8 store-path PMC (K1-fp8 vs hipBLASLt fp8 at the Job's three shapes)
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8_persistent" -m gpu > gpurun_out/r4_fp8pp6_test.log 2>&1 && \
PYARGS="--variants pingpong8om,pingpong8ol,pingpong8ols,pingpong8od --repeats 100" bash tools/gpu_run.sh r4_race py:tools/race_screen.py && \
bash tools/gpu_run.sh r4_clock clock && \
PMC_DTYPE=fp8 bash tools/gpu_run.sh r4_fp8pmc_8192 pmc && \
PMC_DTYPE=fp8 PMC_SHAPE=8192x8192x4096 bash tools/gpu_run.sh r4_fp8pmc_8k8k4k pmc && \
PMC_DTYPE=fp8 PMC_SHAPE=4096x4096x4096 bash tools/gpu_run.sh r4_fp8pmc_4096 pmc && \
PYARGS="--sizes 4096,8192,8192x8192x4096 --variants tile256x128,tile128x256 --knobs 30 --no-bf16 --rounds 7 --iters 30" bash tools/gpu_run.sh r4_fp8tiles py:tools/gemm_fp8_check.py
