#!/bin/bash
# PMC profile of K1-fp8 vs hipBLASLt fp8 (torch._scaled_mm), counters in their own runs.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmc_fp8
mkdir -p $OUT
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 tools/gemm_pair.py --dtype fp8 --size 8192 --iters 10 > $OUT/$name.log 2>&1 || { echo "FAIL $name"; tail -20 $OUT/$name.log; return 1; }
}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/gemm_pair.py --dtype fp8 --size 8192 --iters 20 > $OUT/trace.log 2>&1 && \
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE && \
run sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS && \
run sq3 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE && \
run tcc TCC_HIT_sum TCC_MISS_sum && \
run fetch FETCH_SIZE && \
echo PMC_DONE
