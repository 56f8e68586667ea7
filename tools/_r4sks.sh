# round-4: stream-K split mode (at most half a round of 256x256 tiles) - tests, race screen, timing
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stream_k" -m gpu > gpurun_out/r4_sks_test.log 2>&1 && \
PYARGS="--variants pingpong8s --repeats 30" bash tools/gpu_run.sh r4_sks_race py:tools/race_screen.py && \
PYARGS="--sizes 4672x1472x6696,5624x752x5880,2048x2048x4096,280x6352x7568,2048x1024x8192,3072x2048x6144,4096x2048x8192,1024x8192x8192,2560x2560x8192,1000x1000x8000,1000x4096x16384,2048x4096x16384,333x4096x16384 --variants default,pingpong8s --rounds 7 --iters 20" bash tools/gpu_run.sh r4_sks_time py:tools/gemm_check.py
