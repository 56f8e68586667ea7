#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -m nvidia_terraform_modules_amd.ops.build -q --asan > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 validation/build/amdgpu-validate --size 8192 --iters 30 --min-hbm-gb 250 --tflops-floor 1000 --out gpurun_out/validate_1gpu.json > gpurun_out/validate.log 2>&1; rc=$?; echo "validate rc=$rc"; cat gpurun_out/validate.log | head -c 3000; echo
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench2.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench2.log; exit 1; }
tail -1 gpurun_out/bench2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
