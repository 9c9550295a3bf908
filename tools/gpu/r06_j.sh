# Round 6, pass j: where C4's pass C spends its time -- kernel traces of the partitioned form
# with phases skipped (IGX_GBP_DEBUG: 8 no record loop, 16 no flush, 32 decode + hash only),
# then the SQ counters of the C4 bench config.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j
rm -rf $O; mkdir -p $O
for d in 0 8 16 32; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/t$d -o run -- python3 tools/ablate_part.py --configs c4 --dbg $d --reps 4 > $O/t$d.log 2>&1 || { echo "trace $d failed"; tail $O/t$d.log; exit 1; }
  f=$(find $O/t$d -name '*kernel_trace.csv' | head -1)
  echo "dbg $d: $(python3 tools/kavg.py $f 'k_gbp_a<' 'k_gbp_b<' 'k_gbp_c<')"
done | tee $O/ablate.txt || exit 1
bash tools/gpu/pmc_sq.sh c4j c4 > $O/sq.txt 2>&1 || { echo "sq failed"; tail $O/sq.txt; exit 1; }
grep -E "k_gbp_(a|b|c)" $O/sq.txt
echo R06J_OK
