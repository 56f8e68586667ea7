#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/t256
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k tile > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u tools/gemm_policy.py --shapes 2048x2048x2048,2048x2048x8192,2560x2560x2560,4096x2048x4096,2048x4096x4096,3072x3072x3072,4096x4096x4096,6144x6144x6144,3584x3584x3584,8192x8192x8192 > $O/policy.log 2>&1; grep -v amdgpu.ids $O/policy.log
