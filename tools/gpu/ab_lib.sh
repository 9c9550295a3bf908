# Interleaved A/B of library builds on the partitioned form's passes (C4 by default):
#   bash tools/gpu/ab_lib.sh TAG "libA.so libB.so:ENV=V" [configs] [kernel patterns...]
# Each rep runs tools/ablate_part.py under a rocprofv3 kernel trace with IGX_LIB set to each
# build in turn, and prints the average duration of every kernel pattern.
set -o pipefail
export TMPDIR=/tmp
T=$1; LIBS=$2; CFG=${3:-c4}; shift 3 2>/dev/null || shift $#
PATS=("$@"); [ ${#PATS[@]} -eq 0 ] && PATS=('k_gbp_a<' 'k_gbp_b<' 'k_gbp_c<')
O=gpurun_out/ab_$T
rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for LE in $LIBS; do
    L=${LE%%:*}; EV=; [ "$LE" != "$L" ] && EV=${LE#*:}
    d=$O/$(echo "$LE" | tr ':=' '__')_$rep
    env $EV IGX_LIB=$PWD/inspektor-gadget_amd/$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/ablate_part.py --configs $CFG --dbg 0 --reps 4 > $d.log 2>&1 || { echo "$L rep $rep failed"; tail $d.log; exit 1; }
    f=$(find $d -name '*kernel_trace.csv' | head -1)
    echo "$LE rep $rep: $(grep -h '"config"' $d.log | tr -d '\n') :: $(python3 tools/kavg.py $f "${PATS[@]}")"
  done
done | tee $O/ab.txt
