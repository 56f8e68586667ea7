#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/fp8c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_validate_binary.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/gemm_fp8_check.py --sizes 8192,4096 --iters 30 --rounds 11 > $O/check.log 2>&1; grep -v amdgpu.ids $O/check.log
