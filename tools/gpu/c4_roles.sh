set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for nl in 2 4 6 8 10; do
  IGX_GB_LOADERS=$nl timeout -k 10 300 python tools/bench_configs.py --only c4,c5 --reps 3 > gpurun_out/c4_$nl.log 2>&1 || { echo "nl=$nl failed"; tail -3 gpurun_out/c4_$nl.log; exit 1; }
  echo "nl=$nl"; grep '^{' gpurun_out/c4_$nl.log | cut -c1-110
done
