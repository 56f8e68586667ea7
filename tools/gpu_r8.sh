#!/bin/bash
# Round-8 GPU pass: full GPU test suite (fp8 additions included), bench, fp8 validate report
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 ./validation/build/amdgpu-validate --gpus 1 --size 8192 --iters 30 --out $O/validate.json > $O/validate.log 2>&1 || { echo VAL_FAIL; tail -20 $O/validate.log; exit 1; }
tail -c 1500 $O/validate.json
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
