# pass-C wave pre-combine rounds (IGX_GBP_COMBINE) on the partitioned form (C4, C5)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cb
for cb in 0 1 4; do
  IGX_GBP_COMBINE=$cb timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cb/t$cb -o run --output-format csv -- python3 tools/ablate_forms.py --configs c4,c5 --forms part --reps 2 > gpurun_out/cb/cb$cb.log 2>&1 || { echo "cb=$cb failed"; tail -5 gpurun_out/cb/cb$cb.log; exit 1; }
  echo "cb=$cb"; grep -h '{' gpurun_out/cb/cb$cb.log | cut -c1-100
done
