# the memory-side atomics of the cached group-by, counted two ways on the
# same launches -- the debug kernel's per-kind counters (IGX_GB_DEBUG bit 18, libigx_dbg.so
# built with -DIGX_GB_DEBUG_FILE: make -C inspektor-gadget_amd/csrc OUT=../libigx_dbg.so OBJDIR=../.build_dbg
# EXTRA=-DIGX_GB_DEBUG_FILE) and rocprofv3's TCC_EA0_ATOMIC -- for C5 (top file) and C2.
# Three launches per layout over one batch: the first starts a generation (claims), the next two
# keep its keys.   bash tools/gpu/r06_atomics.sh -> gpurun_out/atom/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/atom
rm -rf $O; mkdir -p $O
export IGX_LIB=inspektor-gadget_amd/libigx_dbg.so
R5="python3 tools/ablate_groupby.py --layout file --events 125000000 --keys 10000000 --zipf 1.05 --variants 262144 --rounds 3"
R2="python3 tools/ablate_groupby.py --layout tcp --events 100000000 --keys 1000000 --zipf 1.1 --variants 262144 --rounds 3"
timeout -k 10 300 $R5 > $O/c5_counts.json 2> $O/c5_counts.err || { echo "c5 counts failed"; tail $O/c5_counts.err; exit 1; }
timeout -k 10 300 $R2 > $O/c2_counts.json 2> $O/c2_counts.err || { echo "c2 counts failed"; tail $O/c2_counts.err; exit 1; }
i=0
for g in "TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $O/p5_$i -o p -- $R5 > $O/p5_$i.log 2>&1 || { echo "c5 pass $i failed"; tail -5 $O/p5_$i.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $O/p2_$i -o p -- $R2 > $O/p2_$i.log 2>&1 || { echo "c2 pass $i failed"; tail -5 $O/p2_$i.log; exit 1; }
done
echo "C5 counters:"; cat $O/c5_counts.json
echo "C5 PMC per launch:"; python3 tools/pmc_summary.py --per-dispatch --kernel 'StaticLayout<8, 4, 4, 4>, true' $O/p5_1 $O/p5_2
echo "C2 counters:"; cat $O/c2_counts.json
echo "C2 PMC per launch:"; python3 tools/pmc_summary.py --per-dispatch --kernel 'StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>, true' $O/p2_1 $O/p2_2
echo ATOM_OK
