# GPU check: parity tests, smoke, per-config bench, default bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_gpu.log | head -40; tail -3 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || { echo "configs failed rc=$?"; tail -20 gpurun_out/configs.log; exit 1; }
grep '{' gpurun_out/configs.log | cut -c1-400
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed rc=$?"; tail gpurun_out/bench_full.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_full.log | cut -c1-700
echo ALL_OK
