#!/bin/bash
# Split-plan pass: full GPU suite (incl. the split-dispatch numerics), policy timing
# on the shapes whose default plan splits C by rows, smoke and bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/split
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_all.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
timeout -k 10 500 python -u tools/gemm_policy.py --shapes 4352x4352x4352,4608x4608x4608,4864x4864x4864,5888x5888x5888,6144x6144x6144,6400x6400x6400,7168x7168x7168,7424x7424x7424,8192x8192x8192 > $O/policy.log 2>&1 || { echo POLICY_FAIL; tail -20 $O/policy.log; exit 1; }
grep -v amdgpu.ids $O/policy.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
tail -c 800 $O/bench.log
