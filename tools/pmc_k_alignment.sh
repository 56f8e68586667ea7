set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for shp in 5024x2568x8320 5024x2568x8328; do
  P=gpurun_out/r6_k8pmc/$shp
  mkdir -p $P
  pair="tools/gemm_pair.py --shape $shp --iters 10 --variant pingpong8cm"
  for pass in "tcp:TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
              "ta:TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
              "tcc:TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
              "sq:SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES"; do
    name=${pass%%:*}
    timeout -s KILL 120 rocprofv3 --pmc ${pass#*:} --kernel-trace --output-format csv -d "$P/$name" -o run -- python3 $pair > "$P/$name.log" 2>&1 || { echo "FAIL $shp $name"; tail -20 "$P/$name.log"; exit 1; }
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/trace" -o run -- python3 $pair > "$P/trace.log" 2>&1 || { echo FAIL trace; exit 1; }
  python3 tools/pmc_summary.py "$P" > "$P/summary.json" || exit 1
done
echo DONE
