# igx_take parity + the filter/sort/gadget/dist paths that now gather through it, then C1 timing.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_gpu.log | head -40; tail -3 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 tools/bench_configs.py --only c1 > gpurun_out/c1.log 2>&1 || { echo "c1 failed rc=$?"; tail gpurun_out/c1.log; exit 1; }
grep '{' gpurun_out/c1.log | cut -c1-400
echo ALL_OK
