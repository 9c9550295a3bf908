set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groupby.py tests/test_gpu_parity.py tests/test_gpu_gadgets.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gb.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_gb.log | head -30; tail -3 gpurun_out/pytest_gb.log; exit 1; }
tail -1 gpurun_out/pytest_gb.log
timeout -k 10 300 python tools/ablate_groupby.py --variants 0 > gpurun_out/ablate1.log 2>&1 || { echo "ablate1 failed"; tail gpurun_out/ablate1.log; exit 1; }
grep -h '{' gpurun_out/ablate1.log | cut -c1-80
timeout -k 10 300 python tools/ablate_groupby.py --keys 10000 --variants 0 > gpurun_out/ablate2.log 2>&1 || { echo "ablate2 failed"; exit 1; }
grep -h '{' gpurun_out/ablate2.log | cut -c1-80
timeout -k 10 300 python tools/bench_configs.py --only c4,c5 > gpurun_out/c45.log 2>&1 || { echo "c45 failed"; tail gpurun_out/c45.log; exit 1; }
grep -h '{' gpurun_out/c45.log | cut -c1-200
