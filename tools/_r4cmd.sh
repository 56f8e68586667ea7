export PMC_ARGS="--variant pingpong8o --versus pingpong8ols"
PYARGS="--sizes 8192,5120,8192x8192x4096 --variants pingpong8o,pingpong8ols,pingpong8od --rounds 9 --iters 30" bash tools/gpu_run.sh r4_stg "tests:persistent or xgmi_tune or missing_rank or dma4 or clock" py:tools/gemm_check.py pmc && \
PYARGS="--sizes 4472x5688x5832,4472x5688x5888,5000x4104x4096,6000x7000x3000,3000x9000x4096 --variants pingpong8cm,pingpong8om --rounds 7 --iters 30" bash tools/gpu_run.sh r4_om py:tools/gemm_check.py && \
PYARGS="--size 8192 --k 8192" bash tools/gpu_run.sh r4_stamps py:tools/pp6_stamps.py
