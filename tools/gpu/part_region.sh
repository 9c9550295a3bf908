set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groupby.py tests/test_gpu_fullsize.py -x -q -m gpu -k "partitioned or direct or c4 or c5" --timeout 200 --timeout-method thread > gpurun_out/pytest_part.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_part.log | head -30; tail -3 gpurun_out/pytest_part.log; exit 1; }
tail -2 gpurun_out/pytest_part.log
bash tools/gpu/ab_modes.sh c4 "IGX_GBP_EXACT=1;IGX_GB_MODE=0" && bash tools/gpu/ktrace.sh reg c4
