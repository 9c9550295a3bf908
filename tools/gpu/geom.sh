# table geometry sweep for C2 (slot factor x KR rounding), full k_groupby only
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "8 0" "5 0" "8 1" "5 1"; do
  set -- $cfg
  IGX_GB_SLOTF=$1 IGX_GB_KR16=$2 timeout -k 10 200 python tools/ablate_groupby.py --variants 0,8 --rounds 3 > gpurun_out/geom_$1_$2.log 2>&1 || { echo "geom $cfg failed"; tail gpurun_out/geom_$1_$2.log; exit 1; }
  echo "slotf=$1 kr16=$2 $(grep -h '{' gpurun_out/geom_$1_$2.log)"
done
