#!/bin/bash
# Plan with 160-wide tiles: full GPU suite, then default vs alternatives on the shapes it changed.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/t160b
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_all.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
timeout -k 10 600 python -u tools/gemm_policy.py --rounds 7 --shapes 2560x2560x2560,3200x3200x3200,4096x2560x4096,5120x5120x5120,8192x5120x4096,2560x2560x1280,1280x800x384,2560x1600x2560,4352x4352x4352 > $O/policy.log 2>&1 || { echo POLICY_FAIL; tail -20 $O/policy.log; exit 1; }
grep -v amdgpu.ids $O/policy.log
