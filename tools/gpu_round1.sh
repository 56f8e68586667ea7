set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench1.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench1.log; exit 1; }
tail -2 gpurun_out/bench1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-extras > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof_bench -name "*stats*" | head
