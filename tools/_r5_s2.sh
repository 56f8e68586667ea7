set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r5_s2; mkdir -p $O gpurun_out/r5_s2cal
bash tools/gpu_run.sh r5_s2 "tests:stream_k" || exit 1
timeout -k 10 300 python -u tools/race_screen.py --variants pingpong8s --repeats 100 > $O/race.log 2>&1 || { tail -20 $O/race.log; exit 1; }
tail -2 $O/race.log
timeout -k 10 600 python -u tools/gemm_policy.py --shapes 2840x1768x8904,4672x1472x6696,4216x1576x12816,3040x2512x16160,4096x2048x8192,8000x1000x4432,1224x2880x9000,3000x1000x12000 --variants pingpong8s,pingpong8s_nopair --rounds 9 --iters 20 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 900 python -u tools/gemm_check.py --sizes 5680x840x12408,2104x2368x14568,2168x2480x9712,2320x3040x11120,1384x3776x15440,3416x1528x6648,6264x904x11192,2592x2000x9912,3888x1504x8968,2120x2816x16360,960x5872x15000,624x7224x8744,6168x1024x8552,5392x840x12432,5200x1360x9792,2896x2256x14632,952x8120x5784,1992x3320x4848,2984x1664x5792,912x8088x5768,976x5872x4392,5776x1168x2592,1544x4032x3976,7824x864x4360,568x6864x1232,4464x1032x4344,2752x2216x2552,2888x2224x3512 --variants default,pingpong8s,pingpong8s_nopair --rounds 5 --iters 20 > gpurun_out/r5_s2cal/gemm_check.log 2>&1 || { tail -20 gpurun_out/r5_s2cal/gemm_check.log; exit 1; }
tail -c 300 gpurun_out/r5_s2cal/gemm_check.log
