set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_gpu.log | head -40; tail -3 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || { echo "configs failed rc=$?"; tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log | grep '{'
echo ALL_OK
