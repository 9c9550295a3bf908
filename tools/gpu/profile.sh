# Per-round profile (bash tools/gpu/profile.sh r03): rocprofv3 kernel trace + stats of the bench (all configs), separate
# FETCH_SIZE / WRITE_SIZE PMC passes -> per-config dominant-kernel traffic, and the L2
# hit/miss + memory-side request counters of the C2 group-by.  Outputs under gpurun_out/<round>/
# (copy to profiles/<round>/ afterwards).
set -o pipefail
export TMPDIR=/tmp
R=${1:-r03}
O=gpurun_out/$R
rm -rf $O; mkdir -p $O
B="python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --config-steps 3 --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; tail $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o p -- $B > $O/fetch.log 2>&1 || { echo "fetch failed rc=$?"; tail $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o p -- $B > $O/write.log 2>&1 || { echo "write failed rc=$?"; tail $O/write.log; exit 1; }
C2="python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-check --configs="
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/tcc1 -o p -- $C2 > $O/tcc1.log 2>&1 || { echo "tcc1 failed rc=$?"; tail $O/tcc1.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d $O/tcc2 -o p -- $C2 > $O/tcc2.log 2>&1 || { echo "tcc2 failed rc=$?"; tail $O/tcc2.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum --kernel-trace --output-format csv -d $O/tcc3 -o p -- $C2 > $O/tcc3.log 2>&1 || echo "tcc3 failed rc=$? (optional)"
timeout -k 10 200 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum --kernel-trace --output-format csv -d $O/tcc4 -o p -- $C2 > $O/tcc4.log 2>&1 || echo "tcc4 failed rc=$? (optional)"
T=tools/pmc_traffic.py
python3 $T --fetch $O/fetch --write $O/write --kernel 'StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>, false' --config '{"events": 100000000, "keys": 1000000, "zipf": 1.1}' --out $O/traffic_c2.json &&
python3 $T --fetch $O/fetch --write $O/write --kernel 'k_hist<' --config '{"events": 125000000}' --out $O/traffic_c3.json &&
python3 $T --fetch $O/fetch --write $O/write --kernel 'k_gb' --anchor 'k_gbp_a<' --extra k_np_mark --config '{"events": 125000000}' --out $O/traffic_c4.json &&
python3 $T --fetch $O/fetch --write $O/write --kernel 'StaticLayout<8, 4, 4, 4>, false' --config '{"events": 125000000, "keys": 10000000}' --out $O/traffic_c5.json || { echo "traffic parse failed"; exit 1; }
python3 tools/pmc_summary.py --kernel 'StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>, false' $O/tcc1 $O/tcc2 $O/tcc3 $O/tcc4 > $O/tcc_c2.txt 2>&1 || echo "tcc summary failed"
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log > $O/bench.json
cat $O/tcc_c2.txt
head -12 $O/kernel_stats.csv | cut -c1-160
echo ALL_OK
