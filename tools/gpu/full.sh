# Round checkpoint: the whole -m gpu suite, smoke, then tools/gpu/profile.sh <round>.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pytest_gpu.log | head -40; tail -3 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
bash tools/gpu/profile.sh ${1:-r03}
