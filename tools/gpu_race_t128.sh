#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/t128
mkdir -p $O
timeout -k 10 500 python -u tools/race_screen.py --variants tile128 --repeats 200 > $O/race.log 2>&1; rc=$?
grep -v amdgpu.ids $O/race.log; exit $rc
