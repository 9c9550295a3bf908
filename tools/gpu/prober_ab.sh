# groupby tests under the batch prober (0) and the state-machine prober (1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  IGX_GB_PROBER=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_groupby.py -x -q -m gpu --timeout 60 --timeout-method thread > gpurun_out/prober_$v.log 2>&1 || { echo "PROBER=$v failed"; grep -E "^(FAILED|ERROR)|^E  |Timeout|test_gpu" gpurun_out/prober_$v.log | head -20; exit 1; }
  echo "PROBER=$v $(tail -1 gpurun_out/prober_$v.log)"
done
