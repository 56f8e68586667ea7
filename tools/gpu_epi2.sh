#!/bin/bash
# Epilogue round 2: LDS-staged full-row stores, persistent + wide/NT, GROUP_M 4; K1 tests.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/epi2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/race_screen.py --variants knob21 --repeats 40 > $O/race.log 2>&1 || { echo RACE_FAIL; tail -20 $O/race.log; exit 1; }
tail -1 $O/race.log
timeout -k 10 400 python -u tools/gemm_check.py --sizes 8192,4096 --iters 50 --rounds 11 --variants default,knob16,knob21,knob22,pingpong8pw > $O/check.log 2>&1 || { echo CHECK_FAIL; tail -20 $O/check.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/epi2/check.log"):
    if l.startswith('{"size"'):
        d=json.loads(l); print(d["size"], {k[:-len("_tflops_med")]: round(v) for k,v in d.items() if k.endswith("_tflops_med")})
PY
