#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/bench_job
mkdir -p $O
timeout -k 10 400 python -u bench.py --out $O/bench.json > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], json.dumps(d['validation_job']))"
