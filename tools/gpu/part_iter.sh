# Partitioned form iteration: parity tests, then the per-pass ablation on C4 / C5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_groupby.py -x -q -m gpu -k "${TK:-partitioned}" --timeout 120 --timeout-method thread > gpurun_out/part_tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/part_tests.log | head -30; tail -3 gpurun_out/part_tests.log; exit 1; }
tail -1 gpurun_out/part_tests.log
timeout -k 10 300 python -u tools/ablate_part.py --configs ${CFG:-c4,c5} --dbg ${DBG:-0,257,256,512,516,8,32,64,16} > gpurun_out/ablate_part.log 2>&1 || { echo "ablate failed"; tail gpurun_out/ablate_part.log; exit 1; }
grep config gpurun_out/ablate_part.log
