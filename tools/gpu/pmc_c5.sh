# Memory-side request counters of the C5 cached group-by (k_groupby<file_id>): reads, writes,
# atomics, L2 hits / misses per launch, plus the same for C2 for comparison.  One PMC pass per
# counter group (rocprofv3 does not split passes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc5${PMC_TAG}
rm -rf $O; mkdir -p $O
R="python3 tools/ablate_forms.py --configs c5,c2 --forms cached --reps 2"
i=0
for g in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $O/p$i -o p -- $R > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo "C5:"; python3 tools/pmc_summary.py --kernel 'StaticLayout<8, 4, 4, 4>, false' $O/p1 $O/p2 $O/p3 $O/p4
echo "C2:"; python3 tools/pmc_summary.py --kernel 'StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>, false' $O/p1 $O/p2 $O/p3 $O/p4
grep -h "ms" $O/p1.log | tail -4
