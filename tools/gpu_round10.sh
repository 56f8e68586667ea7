#!/bin/bash
# Round-9 GPU pass: full GPU suite, smoke, validate binary, bench, kernel stats of the bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 ./validation/build/amdgpu-validate --gpus 1 --size 8192 --iters 30 --out $O/validate_1gpu.json > $O/validate.log 2>&1 || { echo VAL_FAIL; tail -20 $O/validate.log; exit 1; }
timeout -k 10 300 python -u bench.py --out $O/bench.json > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 5 > $O/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/bench_prof.log; exit 1; }
echo DONE
