#!/bin/bash
# One parameterised GPU pass for `gpurun` (replaces the per-round tools/gpu_*.sh
# scratch scripts). Every GPU step has its own time limit and the first failure
# ends the pass (no retries); logs land under gpurun_out/<tag>/.
#
#   tools/gpu_run.sh <tag> [steps...]
#
# steps (run in the order given; default: tests smoke validate bench prof):
#   tests      pytest -m gpu (one process, per-test 120 s thread timeout)
#   tests:<k>  pytest -m gpu -k <k>
#   smoke      __graft_entry__.smoke()
#   validate   amdgpu-validate on 1 GPU (JSON report)
#   bench      bench.py exactly as the driver runs it (--steps 20 --warmup 5)
#   bench200   bench.py --steps 200 --warmup 20
#   prof       rocprofv3 --kernel-trace --stats of a short bench
#   pmc        PMC passes (counters in their own runs, --kernel-trace only) of K1 vs
#              hipBLASLt at 8192^3 (PMC_DTYPE=fp8: K1-fp8 vs hipBLASLt fp8; PMC_ARGS: extra
#              tools/gemm_pair.py arguments, e.g. "--variant A --versus B"; PMC_SHAPE:
#              MxNxK instead of 8192^3) +
#              tools/pmc_summary.py -> <tag>/pmc/summary.json
#   clock      the GEMM's in-kernel clock (stamped pingpong8o) vs GRBM_GUI_ACTIVE of the
#              same dispatches (one rocprofv3 --pmc pass)
#   fp8        K1-fp8 vs hipBLASLt fp8: square sizes (gemm_fp8_check) + the 41-shape sweep
#   standing   where the shipping default plans stand vs hipBLASLt on this box: named bf16
#              shapes (gemm_check), fp8 (gemm_fp8_check), a seeded ragged one-round set
#              (k1_ab.py ragged) and 48 seeded random shapes (gemm_policy); STAND_SEED picks
#              the fresh sets. Run on >= 3 boxes; tools/k1_boxes.py takes the median.
#   py:<file>  python -u <file> (a tool script; its own args via PYARGS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${1:?usage: gpu_run.sh <tag> [steps...]}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
STEPS=("$@")
[ ${#STEPS[@]} -eq 0 ] && STEPS=(tests smoke validate bench prof)

fail() { echo "FAIL $1 (rc $2)"; tail -40 "$3"; exit 1; }

for s in "${STEPS[@]}"; do
  echo "== $s $(date +%T)"
  case "$s" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1 || fail tests $? "$O/pytest_gpu.log"
      tail -1 "$O/pytest_gpu.log" ;;
    tests:*)
      k=${s#tests:}
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$k" \
        > "$O/pytest_gpu_k.log" 2>&1 || fail "$s" $? "$O/pytest_gpu_k.log"
      tail -1 "$O/pytest_gpu_k.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || fail smoke $? "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    validate)
      timeout -k 10 300 ./validation/build/amdgpu-validate --gpus 1 --size 8192 --iters 30 \
        --out "$O/validate_1gpu.json" > "$O/validate.log" 2>&1 || fail validate $? "$O/validate.log"
      tail -3 "$O/validate.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out "$O/bench.json" \
        > "$O/bench.log" 2>&1 || fail bench $? "$O/bench.log"
      tail -c 1500 "$O/bench.json" ;;
    bench200)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 --out "$O/bench200.json" \
        > "$O/bench200.log" 2>&1 || fail bench200 $? "$O/bench200.log"
      tail -c 600 "$O/bench200.json" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
        -- python3 bench.py --steps 50 --warmup 5 --no-job > "$O/bench_prof.log" 2>&1 \
        || fail prof $? "$O/bench_prof.log"
      find "$O/prof" -name '*kernel_stats.csv' -exec head -12 {} \; ;;
    pmc)
      P="$O/pmc"
      mkdir -p "$P"
      pair="tools/gemm_pair.py --size 8192 --iters 10 --dtype ${PMC_DTYPE:-bf16} ${PMC_ARGS:-}"
      [ -n "${PMC_SHAPE:-}" ] && pair="$pair --shape $PMC_SHAPE"
      for pass in "sq1:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
                  "sq2:SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
                  "sq3:SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE" \
                  "tcc:TCC_HIT_sum TCC_MISS_sum" "fetch:FETCH_SIZE" "write:WRITE_SIZE" \
                  "wrreq:TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
        name=${pass%%:*}
        timeout -s KILL 120 rocprofv3 --pmc ${pass#*:} --kernel-trace --output-format csv \
          -d "$P/$name" -o run -- python3 $pair > "$P/$name.log" 2>&1 || fail "pmc $name" $? "$P/$name.log"
      done
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/trace" -o run \
        -- python3 $pair > "$P/trace.log" 2>&1 || fail "pmc trace" $? "$P/trace.log"
      python3 tools/pmc_summary.py "$P" > "$P/summary.json" && head -c 3000 "$P/summary.json" ;;
    clock)
      # the GEMM's own clock (stamped build) vs its PMC clock, same dispatches
      timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
        -d "$O/clock_pmc" -o run -- python3 tools/clock_check.py --out "$O/clock_inkernel.json" \
        > "$O/clock.log" 2>&1 || fail clock $? "$O/clock.log"
      python3 tools/clock_check.py --compare "$O/clock_pmc" --inkernel "$O/clock_inkernel.json" \
        | tee "$O/clock_compare.json" ;;
    fp8)
      timeout -k 10 600 python -u tools/gemm_fp8_check.py --sizes 1024,2048,2560,3072,4096,4608,6144,8192 \
        --iters 30 --rounds 5 > "$O/fp8_check.log" 2>&1 || fail fp8 $? "$O/fp8_check.log"
      timeout -k 10 900 python -u tools/gemm_policy.py --dtype fp8 --only-default --shapes 8192x8192x8192 \
        --random 40 --rounds 5 --iters 20 > "$O/fp8_policy_random.log" 2>&1 \
        || fail "fp8 policy" $? "$O/fp8_policy_random.log"
      python3 -c "import json,statistics,sys; r=[json.loads(l)['default_over_hipblaslt'] for l in open(sys.argv[1]) if l.startswith('{')]; print(f'fp8 default ahead of hipBLASLt on {sum(x > 1 for x in r)} of {len(r)}, median {statistics.median(r):.3f}')" "$O/fp8_policy_random.log" ;;
    standing)
      sd=${STAND_SEED:-23}
      timeout -k 10 600 python -u tools/gemm_check.py --variants default --rounds 7 --iters 30 \
        --sizes 8192,5120,4096,8192x8192x4096,8192x8192x6144,4472x5688x5832,4152x1096x16056,2840x1768x8904 \
        > "$O/standing_bf16.log" 2>&1 || fail "standing bf16" $? "$O/standing_bf16.log"
      timeout -k 10 600 python -u tools/gemm_fp8_check.py --sizes 4096,8192,8192x8192x4096,6144 --no-bf16 \
        --rounds 7 --iters 30 > "$O/standing_fp8.log" 2>&1 || fail "standing fp8" $? "$O/standing_fp8.log"
      timeout -k 10 600 python -u tools/k1_ab.py ragged --n 24 --seed "$sd" --rounds 5 --iters 10 \
        > "$O/standing_ragged_seed$sd.log" 2>&1 || fail "standing ragged" $? "$O/standing_ragged_seed$sd.log"
      timeout -k 10 900 python -u tools/gemm_policy.py --only-default --shapes "" --random 48 --seed "$sd" \
        --rounds 5 --iters 20 > "$O/standing_random48_seed$sd.log" 2>&1 \
        || fail "standing random" $? "$O/standing_random48_seed$sd.log"
      tail -1 "$O/standing_ragged_seed$sd.log"
      python3 -c "import json,statistics,sys; r=[(lambda d: d['default_tflops'] / d['torch_tflops'])(json.loads(l)) for l in open(sys.argv[1]) if l.startswith('{')]; print(f'random48 seed $sd: ahead on {sum(x > 1 for x in r)} of {len(r)}, below 0.97 {sum(x < 0.97 for x in r)}, min {min(r):.3f}, median {statistics.median(r):.3f}')" "$O/standing_random48_seed$sd.log" ;;
    py:*)
      f=${s#py:}
      timeout -k 10 600 python -u "$f" $PYARGS > "$O/$(basename "$f" .py).log" 2>&1 \
        || fail "$s" $? "$O/$(basename "$f" .py).log"
      tail -30 "$O/$(basename "$f" .py).log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo DONE
