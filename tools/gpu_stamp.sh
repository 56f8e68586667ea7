#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/stamp
mkdir -p $O
timeout -k 10 200 python -u tools/gemm_stamp.py --size 8192 > $O/stamp8192.log 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamp8192.log; exit 1; }
tail -1 $O/stamp8192.log
timeout -k 10 200 python -u tools/gemm_stamp.py --size 4096 --rounds 1 > $O/stamp4096.log 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamp4096.log; exit 1; }
tail -1 $O/stamp4096.log
