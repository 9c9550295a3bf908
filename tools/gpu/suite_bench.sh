# The whole -m gpu suite, then a short bench of the given configs: bash tools/gpu/suite_bench.sh [configs] [env sets]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_gpu.log | head -40; tail -3 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/gpu/ab_modes.sh ${1:-c5} "${2:-IGX_GB_MODE=0}"
