set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --events 10000000 --keys 100000 --steps 3 --warmup 1 --cpu-sample 0 --check > gpurun_out/bench_check.log 2>&1 || { echo "bench check failed rc=$?"; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench full failed rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
grep -h '"metric"' gpurun_out/bench_check.log gpurun_out/bench_full.log | cut -c1-400
head -4 gpurun_out/prof/run_kernel_stats.csv | cut -c1-160
echo ALL_OK
