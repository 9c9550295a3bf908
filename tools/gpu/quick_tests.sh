# Run a subset of GPU tests: bash tools/gpu/quick_tests.sh tests/test_x.py [...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_quick.log | head -40; tail -3 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
