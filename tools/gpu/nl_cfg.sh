# configs C4/C5 and the C2 bench under IGX_GB_LOADERS values
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=${2:-IGX_GB_LOADERS}
for v in $1; do
  env $VAR=$v timeout -k 10 300 python tools/bench_configs.py --only c4,c5 --reps 3 > gpurun_out/nl_$v.log 2>&1 || { echo "nl=$v failed"; tail -3 gpurun_out/nl_$v.log; exit 1; }
  env $VAR=$v timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/nlb_$v.log 2>&1 || { echo "bench nl=$v failed"; tail -3 gpurun_out/nlb_$v.log; exit 1; }
  echo "nl=$v"; grep '^{' gpurun_out/nl_$v.log | cut -c1-110; grep -o '"ms_per_step": [0-9.]*' gpurun_out/nlb_$v.log
done
