# round-4: stream-K (pingpong8s) - GPU tests, race screen, timing vs the data-parallel kernels
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stream_k" -m gpu > gpurun_out/r4_sk_test.log 2>&1 && \
PYARGS="--variants pingpong8s,pingpong8s_rev --repeats 30" bash tools/gpu_run.sh r4_sk_race py:tools/race_screen.py && \
PYARGS="--sizes 4472x5688x5832,4472x5688x5888,5000x4104x4096,6000x7000x3000,3000x9000x4096,6144,4608x4608x1024,4672x5888x4096 --variants default,pingpong8cm,pingpong8s --rounds 7 --iters 20" bash tools/gpu_run.sh r4_sk_time py:tools/gemm_check.py
