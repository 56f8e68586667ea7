#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/fp8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fp8 or e4m3 or fill or ref_gemm" --timeout 120 --timeout-method thread > $O/tests2.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
