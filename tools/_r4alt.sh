# round-4: alternating K direction per tile (pingpong8oa / fp8 knob 32) vs the shipping builds
PYARGS="--variants pingpong8oa --repeats 40" bash tools/gpu_run.sh r4_alt_race py:tools/race_screen.py && \
PYARGS="--sizes 8192,8192x8192x4096,5120,8192x8192x6144,4096x8192x8192 --variants pingpong8o,pingpong8oa --rounds 9 --iters 30" bash tools/gpu_run.sh r4_alt_bf16 py:tools/gemm_check.py && \
PYARGS="--sizes 4096,8192,8192x8192x4096,8192x4096x8192,4096x8192x8192 --knobs 32 --no-bf16 --rounds 7 --iters 30" bash tools/gpu_run.sh r4_alt_fp8 py:tools/gemm_fp8_check.py
