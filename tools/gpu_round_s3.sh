#!/bin/bash
# Confirm round for the wide + nontemporal epilogue default: all GPU tests, race screen,
# GROUP_M re-check, bench, smoke, validate binary, rocprofv3 kernel stats (csv).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/race_screen.py --variants default --repeats 100 > $O/race_default.log 2>&1 || { echo RACE_FAIL; tail -20 $O/race_default.log; exit 1; }
tail -1 $O/race_default.log
timeout -k 10 300 python -u tools/gemm_check.py --sizes 8192,4096 --iters 50 --rounds 9 --variants default,knob5,knob12,knob14 > $O/groupm_check.log 2>&1 || { echo CHECK_FAIL; tail -20 $O/groupm_check.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/s4/groupm_check.log"):
    if l.startswith('{"size"'):
        d=json.loads(l); print(d["size"], {k[:-12]: round(v) for k,v in d.items() if k.endswith("_tflops_med")})
PY
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 validation/build/amdgpu-validate --size 8192 --iters 30 --min-hbm-gb 250 --tflops-floor 1000 --out $O/validate_1gpu.json > $O/validate.log 2>&1; rc=$?; echo "validate rc=$rc"; [ $rc -le 1 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 5 --no-extras > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec head -6 {} \;
