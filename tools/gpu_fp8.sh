#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/fp8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fp8 or stream_copy" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/gemm_fp8_check.py --sizes 8192,4096 > $O/check.log 2>&1 || { echo CHECK_FAIL; tail -20 $O/check.log; exit 1; }
cat $O/check.log | grep size
