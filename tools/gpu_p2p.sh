#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/p2p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_validate_binary.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 ./validation/build/amdgpu-validate --size 4096 --iters 5 --p2p-loopback --out $O/loopback.json > $O/loopback.log 2>&1; tail -c 700 $O/loopback.json
