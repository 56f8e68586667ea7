#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/t128
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k tile128 > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/gemm_check.py --sizes 1024,2048,3072,4096 --iters 100 --rounds 7 --variants pingpong8c,tile128 > $O/check.log 2>&1; grep -v amdgpu.ids $O/check.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if 'size' in d: print(d['size'], {k:round(v,1) for k,v in d.items() if k.endswith('tflops_med')}, {k:v['bad'] for k,v in d.items() if k.startswith('verify')})
"
