set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_s2; mkdir -p $O
bash tools/gpu_run.sh r5_s2 "tests:stream_k" || exit 1
timeout -k 10 300 python -u tools/race_screen.py --variants pingpong8s --repeats 100 > $O/race.log 2>&1 || { tail -20 $O/race.log; exit 1; }
tail -2 $O/race.log
timeout -k 10 600 python -u tools/gemm_policy.py --shapes 2840x1768x8904,4672x1472x6696,4216x1576x12816,3040x2512x16160,4096x2048x8192,8000x1000x4432,1224x2880x9000,3000x1000x12000 --variants pingpong8s,pingpong8s_nopair --rounds 9 --iters 20 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
