#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/t256b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_all.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
timeout -k 10 500 python -u tools/race_screen.py --variants tile128,tile256x128 --repeats 200 > $O/race.log 2>&1 || { echo RACE_FAIL; grep -v amdgpu.ids $O/race.log | tail; exit 1; }
tail -1 $O/race.log
timeout -k 10 500 python -u tools/gemm_policy.py --shapes 1024x1024x1024,1536x1536x1536,2048x2048x2048,2560x2560x2560,4096x2048x4096,3072x3072x3072,3584x3584x3584,4096x4096x4096,6144x6144x6144,8192x8192x8192 > $O/policy.log 2>&1; grep -v amdgpu.ids $O/policy.log
