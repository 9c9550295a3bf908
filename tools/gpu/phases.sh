# Pass phases of the partitioned form (IGX_GBP_DEBUG values) for one library build:
#   bash tools/gpu/phases.sh TAG LIB.so [configs] [dbg values...]
set -o pipefail
export TMPDIR=/tmp
T=$1; L=$2; CFG=${3:-c4}; shift 3 2>/dev/null || shift $#
DBG=("$@"); [ ${#DBG[@]} -eq 0 ] && DBG=(0 8 16 32)
O=gpurun_out/ph_$T
rm -rf $O; mkdir -p $O
for d in "${DBG[@]}"; do
  IGX_LIB=$PWD/inspektor-gadget_amd/$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/t$d -o run -- python3 tools/ablate_part.py --configs $CFG --dbg $d --reps 4 > $O/t$d.log 2>&1 || { echo "trace $d failed"; tail $O/t$d.log; exit 1; }
  f=$(find $O/t$d -name '*kernel_trace.csv' | head -1)
  echo "dbg $d: $(python3 tools/kavg.py $f 'k_gbp_a<' 'k_gbp_b<' 'k_gbp_c<')"
done | tee $O/phases.txt
