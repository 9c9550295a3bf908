# Round 6, pass d: the fused compose + AND/OR of the table top-K (tail tests), the filter's
# compaction at 1M / 4M / 16M rows, the atomics accounting by lane groups, and a
# bench with a kernel trace.   bash tools/gpu/r06_d.sh -> gpurun_out/r06d/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tail.py \
    tests/test_gpu_parity.py tests/test_gpu_filter_golden.py tests/test_gpu_owner_exchange.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/filter_scale.py > $O/filter_scale.json 2> $O/filter_scale.err || { echo "filter scale failed"; tail $O/filter_scale.err; exit 1; }
cat $O/filter_scale.json
bash tools/gpu/r06_atomics.sh > $O/atomics.txt 2>&1 || { echo "atomics failed"; tail -20 $O/atomics.txt; exit 1; }
grep -A1 "counters:" $O/atomics.txt | grep -v "^--" | cut -c1-2000
grep -A1 "PMC per launch" $O/atomics.txt | grep -v "^--"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --configs c5 > $O/bench.log 2>&1 || { echo "bench failed"; tail $O/bench.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
python3 - $O/bench.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f tail %.3f | exact %s" % (j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"], c["ms_per_step"] - c["roofline"]["kernel_ms"], j["check"]["all_bit_exact"]))
PY
echo R06D_OK
