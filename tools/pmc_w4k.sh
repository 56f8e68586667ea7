# PMC of the 4-wave dma4k_d3 vs the 8-wave default vs hipBLASLt at bf16 8192^3
# (profiles/r6_w4kh): two SQ counter passes + a kernel trace per pair, each pass
# its own rocprofv3 run, summarised by tools/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in dma4k_d3 default; do
  P=gpurun_out/r6_w4kpmc/$v
  mkdir -p $P
  pair="tools/gemm_pair.py --size 8192 --iters 10 --warm-iters 30 --variant $v"
  for pass in "sq1:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
              "sq2:SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    name=${pass%%:*}
    timeout -s KILL 120 rocprofv3 --pmc ${pass#*:} --kernel-trace --output-format csv -d "$P/$name" -o run -- python3 $pair > "$P/$name.log" 2>&1 || { echo "FAIL $v $name"; tail -20 "$P/$name.log"; exit 1; }
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/trace" -o run -- python3 $pair > "$P/trace.log" 2>&1 || { echo FAIL trace; exit 1; }
  python3 tools/pmc_summary.py "$P" > "$P/summary.json" || exit 1
done
echo DONE
