# round-4 A/B #2 on one box: K1-fp8 persistent build with spread boundary stores
# (fp8 knob 31) vs the plain persistent build (knob 30) vs hipBLASLt fp8
TAG=${1:?tag}
PYARGS="--sizes 4096,8192,8192x8192x4096,8192x4096x8192,4096x8192x8192,6144x6144x4096 --knobs 30,31 --no-bf16 --rounds 7 --iters 30" bash tools/gpu_run.sh ${TAG}_fp8 py:tools/gemm_fp8_check.py
