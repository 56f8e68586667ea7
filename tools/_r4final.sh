# round-4 final standing on one box (run once per box; tools/k1_boxes.py takes
# the median over boxes): the shipping default plans, bf16 and fp8, vs hipBLASLt
TAG=${1:?tag}
PYARGS="--sizes 8192,5120,4096,8192x8192x4096,8192x8192x6144,4472x5688x5832 --variants default --rounds 7 --iters 30" bash tools/gpu_run.sh ${TAG}_bf16 py:tools/gemm_check.py && \
PYARGS="--sizes 4096,8192,8192x8192x4096,6144 --no-bf16 --rounds 7 --iters 30" bash tools/gpu_run.sh ${TAG}_fp8 py:tools/gemm_fp8_check.py
