#!/bin/bash
# GPU-box check of validation/image/strip-fatbin.py (developer tool): builds the
# validation image's runtime closure twice in /tmp - stock, and with librccl's
# fat binary cut to gfx950 - then runs amdgpu-validate's RCCL phase from each,
# alternating, and records the JSON reports (phases_s: hbm_done -> rccl_done is
# RCCL's set-up, code-object load and the verified all-reduce sweep).
#   bash tools/fatbin_strip_check.sh <tag> [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:?tag}
R=${2:-3}
mkdir -p "$O"
C=/tmp/ntm_clos_stock
S=/tmp/ntm_clos_gfx950
rm -rf "$C" "$S"
NTM_KEEP_FATBIN=1 bash validation/image/collect-runtime.sh validation/build/amdgpu-validate "$C" > "$O/collect.log" 2>&1 \
  || { tail "$O/collect.log"; exit 1; }
cp -a "$C" "$S"
python3 validation/image/strip-fatbin.py "$S/lib/librccl.so.1" > "$O/strip.json" || exit 1
cat "$O/strip.json"
LD_LIBRARY_PATH="$S/lib" ldd "$S/bin/amdgpu-validate" | grep -E "rccl|amdhip" > "$O/ldd_gfx950.txt"
cat "$O/ldd_gfx950.txt"
du -sb "$C" "$S" > "$O/closure_bytes.txt"
(cd "$C" && tar cf - . | gzip -1 | wc -c) > "$O/stock_gzip1_bytes.txt"
(cd "$S" && tar cf - . | gzip -1 | wc -c) > "$O/gfx950_gzip1_bytes.txt"
for i in $(seq 1 "$R"); do
  for v in ${ORDER:-stock gfx950}; do
    d=$C
    [ "$v" = gfx950 ] && d=$S
    LD_LIBRARY_PATH="$d/lib" timeout -k 10 120 "$d/bin/amdgpu-validate" --gpus 1 --size 2048 --iters 3 \
      --rccl --allreduce-max-mib 64 --no-fp8 --no-p2p --json > "$O/run_${v}_$i.json" 2> "$O/run_${v}_$i.err" \
      || { echo "FAIL $v $i"; tail -20 "$O/run_${v}_$i.err"; exit 1; }
    python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=r['phases_s']; a=r.get('rccl_allreduce') or []; print(sys.argv[2], 'passed', r.get('passed'), 'rccl_s', round(p['rccl_done']-p['hbm_done'],3), 'end', round(p['end'],3), 'sizes', len(a), 'wrong', sum(x.get('wrong') or 0 for x in a))" "$O/run_${v}_$i.json" "$v$i"
  done
done
rm -rf "$C" "$S"
echo DONE
