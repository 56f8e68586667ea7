# round-4 A/B on one box (run once per box; tools/k1_boxes.py takes the median over boxes):
# bf16 pingpong8o vs the spread / LDS-staged-line builds, fp8 default vs the
# persistent overlap build on VGPR accumulators (fp8 knob 30)
TAG=${1:?tag}
PYARGS="--sizes 8192,5120,8192x8192x4096,8192x8192x6144,6144x6144x8192,4096x8192x8192 --variants pingpong8o,pingpong8od --rounds 7 --iters 30" bash tools/gpu_run.sh ${TAG}_bf16 py:tools/gemm_check.py && \
PYARGS="--sizes 4096,8192,8192x8192x4096,6144,8192x4096x8192,4096x8192x8192 --knobs 30 --no-bf16 --rounds 7 --iters 30" bash tools/gpu_run.sh ${TAG}_fp8 py:tools/gemm_fp8_check.py
