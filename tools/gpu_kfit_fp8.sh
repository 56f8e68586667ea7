#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/kfit_fp8
mkdir -p $O
timeout -k 10 240 python -u tools/gemm_kfit.py --dtype fp8 --mn 8192 --ks 1024,2048,4096,8192,16384 --rounds 5 > $O/kfit_8192.log 2>&1 && \
timeout -k 10 240 python -u tools/gemm_kfit.py --dtype bf16 --mn 8192 --ks 1024,2048,4096,8192 --rounds 5 > $O/kfit_bf16_8192.log 2>&1
cat $O/*.log | grep fit
