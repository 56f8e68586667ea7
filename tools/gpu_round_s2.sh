#!/bin/bash
# Session-2 confirm round: GPU tests, smoke, bench, rocprofv3 kernel stats (tree built on the CPU host).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s2/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/s2/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s2/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/s2/smoke.log; exit 1; }
tail -1 gpurun_out/s2/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/s2/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/s2/bench.log; exit 1; }
tail -1 gpurun_out/s2/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s2/prof -o run -- python3 bench.py --steps 50 --warmup 5 --no-extras > gpurun_out/s2/prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/s2/prof.log; exit 1; }
find gpurun_out/s2/prof -name '*stats*' | head -5
