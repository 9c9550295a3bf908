set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groupby.py -x -q -m gpu -k "partitioned or prober or direct" --timeout 200 --timeout-method thread > gpurun_out/part_tests.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/part_tests.log | head -20; tail -3 gpurun_out/part_tests.log; exit 1; }
tail -1 gpurun_out/part_tests.log
DBGS="0 1 6 8 16" CFG=${CFG:-c4} bash tools/gpu/part_phases.sh
