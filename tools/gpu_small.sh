#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/small
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_check.py --sizes 1024,2048,3072,4096 --iters 100 --rounds 7 --variants pingpong8c > $O/check.log 2>&1; grep -v amdgpu.ids $O/check.log | tail -12
