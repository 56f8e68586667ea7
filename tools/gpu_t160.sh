#!/bin/bash
# 160-wide tiles (tile160 / tile256x160): GPU suite, race screen, policy timing.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/t160
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "tile160 or split or tile128" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/race_screen.py --variants tile160,tile256x160 --repeats 100 > $O/race.log 2>&1 || { echo RACE_FAIL; grep -v amdgpu.ids $O/race.log | tail; exit 1; }
tail -1 $O/race.log
timeout -k 10 500 python -u tools/gemm_policy.py --rounds 5 --shapes 1920x1920x1920,2560x2560x2560,2560x2560x8192,3200x3200x3200,3840x3840x3840,4096x2560x4096,5120x5120x5120,8192x5120x4096,2560x2560x1280 > $O/policy.log 2>&1 || { echo POLICY_FAIL; tail -20 $O/policy.log; exit 1; }
grep -v amdgpu.ids $O/policy.log
