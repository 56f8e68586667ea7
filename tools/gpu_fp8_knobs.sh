#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/fp8_knobs
mkdir -p $O
timeout -k 10 400 python -u tools/gemm_fp8_check.py --sizes 8192,4096,6144 --iters 30 --rounds 15 --knobs 5 > $O/knobs.log 2>&1
cat $O/knobs.log | grep -v amdgpu.ids
