set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for nl in 8 9 10 11 12; do
  IGX_GB_LOADERS=$nl timeout -k 10 200 python tools/ablate_groupby.py --variants 0 --rounds 3 > gpurun_out/roles_$nl.log 2>&1 || { echo "nl=$nl failed"; tail -3 gpurun_out/roles_$nl.log; exit 1; }
  IGX_GB_LOADERS=$nl timeout -k 10 200 python tools/ablate_groupby.py --variants 0 --rounds 3 --keys 10000 >> gpurun_out/roles_$nl.log 2>&1 || { echo "nl=$nl failed"; exit 1; }
  echo "nl=$nl"; grep '{' gpurun_out/roles_$nl.log | cut -c1-60
done
