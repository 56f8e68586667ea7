#!/bin/bash
# pingpong8w (32-MFMA segments) + widened epilogue: numerics, race screen, timing vs pp3 / hipBLASLt.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/epi
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "variants" --timeout 120 --timeout-method thread > gpurun_out/epi/tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/epi/tests.log; exit 1; }
tail -2 gpurun_out/epi/tests.log
timeout -k 10 300 python -u tools/gemm_check.py --sizes 8192,4096 --iters 50 --variants pingpong8c,pingpong8cw,pingpong8cwe,pingpong8cwn,pingpong8cwne,pingpong8pw --rounds 9 > gpurun_out/epi/check.log 2>&1 || { echo CHECK_FAIL; tail -30 gpurun_out/epi/check.log; exit 1; }
cat gpurun_out/epi/check.log
timeout -k 10 300 python -u tools/race_screen.py --variants pingpong8cwe,pingpong8pw --repeats 60 > gpurun_out/epi/race.log 2>&1 || { echo RACE_FAIL; tail -30 gpurun_out/epi/race.log; exit 1; }
tail -1 gpurun_out/epi/race.log
