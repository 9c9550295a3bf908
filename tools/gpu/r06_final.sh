# Round 6, final profile (bash tools/gpu/r06_final.sh): rocprofv3 kernel trace + stats of the
# bench (all configs), FETCH_SIZE / WRITE_SIZE PMC passes -> per-config dominant-kernel traffic
# (the group-by's SAMPLE instance, the seeded cache's first pass, excluded), and the default bench.
# Outputs under gpurun_out/r06final/ (copy to profiles/r06/ afterwards).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06final
rm -rf $O; mkdir -p $O
B="python3 bench.py --cpu-sample 0 --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; tail $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o p -- $B > $O/fetch.log 2>&1 || { echo "fetch failed rc=$?"; tail $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o p -- $B > $O/write.log 2>&1 || { echo "write failed rc=$?"; tail $O/write.log; exit 1; }
T=tools/pmc_traffic.py
python3 $T --fetch $O/fetch --write $O/write --kernel 'StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>, false' --exclude ', true>' --config '{"events": 100000000, "keys": 1000000, "zipf": 1.1}' --out $O/traffic_c2.json &&
python3 $T --fetch $O/fetch --write $O/write --kernel 'k_hist<' --config '{"events": 125000000}' --out $O/traffic_c3.json &&
python3 $T --fetch $O/fetch --write $O/write --kernel 'k_gb' --exclude 'k_gb_seeds' --anchor 'k_gbp_a<' --extra k_np_mark --config '{"events": 125000000}' --out $O/traffic_c4.json &&
python3 $T --fetch $O/fetch --write $O/write --kernel 'StaticLayout<8, 4, 4, 4>, false' --exclude ', true>' --config '{"events": 125000000, "keys": 10000000}' --out $O/traffic_c5.json || { echo "traffic parse failed"; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
cp $O/traffic_c*.json profiles/r06/ 2>/dev/null
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log > $O/bench.json
cut -d, -f1-4 $O/kernel_stats.csv | head -30
echo ALL_OK
