#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/t128
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_all.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
timeout -k 10 400 python -u tools/gemm_policy.py --shapes 1024x1024x1024,2048x2048x2048,2048x2048x8192,2560x2560x2560,4096x2048x4096,3072x3072x3072,4096x4096x4096,1536x1536x1536 > $O/policy.log 2>&1; grep -v amdgpu.ids $O/policy.log
