# C4 / C5 under both probers
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  IGX_GB_PROBER=$v timeout -k 10 300 python tools/bench_configs.py --only c4,c5 --reps 3 > gpurun_out/pcfg_$v.log 2>&1 || { echo "PROBER=$v failed"; tail -3 gpurun_out/pcfg_$v.log; exit 1; }
  echo "PROBER=$v"; grep '^{' gpurun_out/pcfg_$v.log | cut -c1-120
done
