#!/bin/bash
# Split-plan check on non-square shapes + kernel trace of the split dispatch at 4352^3.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/split2
mkdir -p $O
timeout -k 10 600 python -u tools/gemm_policy.py --rounds 5 --shapes 8192x4096x8192,6144x4096x4096,3840x3840x3840,5120x5120x5120,4608x8192x4096,12288x4096x4096,2304x8192x8192,1792x8192x4096,10240x10240x4096,5376x5376x5376,2816x2816x2816 > $O/policy.log 2>&1 || { echo POLICY_FAIL; tail -20 $O/policy.log; exit 1; }
grep -v amdgpu.ids $O/policy.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/gemm_policy.py --rounds 1 --iters 20 --shapes 4352x4352x4352 > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -3
