#!/bin/bash
# Default-candidate shoot-out (15 interleaved rounds) + write/fetch bytes of the LDS-staged epilogue.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/epi3
mkdir -p $O
timeout -k 10 500 python -u tools/gemm_check.py --sizes 8192,4096 --iters 50 --rounds 15 --variants default,knob16,knob21,knob23 > $O/check.log 2>&1 || { echo CHECK_FAIL; tail -20 $O/check.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/epi3/check.log"):
    if l.startswith('{"size"'):
        d=json.loads(l); print(d["size"], {k[:-len("_tflops_med")]: round(v) for k,v in d.items() if k.endswith("_tflops_med")})
PY
for cnt in WRITE_SIZE FETCH_SIZE; do
timeout -k 10 240 rocprofv3 --pmc $cnt --kernel-trace --output-format csv -d $O/$cnt -o run -- python3 tools/gemm_pair.py --size 8192 --iters 5 --which ours --variant knob21 > $O/$cnt.log 2>&1 || { echo "FAIL $cnt"; tail -5 $O/$cnt.log; exit 1; }
done
python tools/pmc_summary.py $O
