set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_gpu.log | head -40; tail -3 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/ablate_groupby.py --variants 0,1,2,4 > gpurun_out/ablate1.log 2>&1 || { echo "ablate1 failed"; tail gpurun_out/ablate1.log; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --keys 1000 --variants 0,1,2,4 > gpurun_out/ablate3.log 2>&1 || { echo "ablate3 failed"; exit 1; }
grep -h '{' gpurun_out/ablate*.log
timeout -k 10 300 python bench.py --events 10000000 --keys 100000 --steps 3 --warmup 1 --cpu-sample 0 --check > gpurun_out/bench_check.log 2>&1 || { echo "bench check failed rc=$?"; tail gpurun_out/bench_check.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench full failed rc=$?"; tail gpurun_out/bench_full.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_check.log gpurun_out/bench_full.log | cut -c1-600
echo ALL_OK
