set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_pf; mkdir -p $O
bash tools/gpu_run.sh r5_pf "tests:l2_touch or persistent_overlap" || exit 1
timeout -k 10 300 python -u tools/race_screen.py --variants pingpong8op,pingpong8od --repeats 100 > $O/race.log 2>&1 || { tail -20 $O/race.log; exit 1; }
tail -3 $O/race.log
timeout -k 10 300 python -u tools/pp6_stamps.py --grids 256 --modes 2,3,0,4 > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep modes $O/stamps.log
timeout -k 10 600 python -u tools/gemm_check.py --sizes 8192,8192x8192x4096,5120,8192x8192x6144 --variants pingpong8od,pingpong8op --rounds 9 --iters 30 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log | cut -c1-400
