# Round 6, pass e: parity at the bench's sizes with kept keys + seeds (full-size, soak,
# persist, group-by suites), the filter's per-kernel trace at 1M/4M/16M rows, and an
# interleaved A/B of the seeds.   bash tools/gpu/r06_e.sh -> gpurun_out/r06e/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_persist.py \
    tests/test_gpu_fullsize.py tests/test_gpu_soak.py tests/test_gpu_groupby.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ftrace -o f --output-format csv -- python3 tools/filter_scale.py --reps 5 > $O/filter_scale.json 2> $O/filter_scale.err || { echo "filter trace failed"; tail $O/filter_scale.err; exit 1; }
cat $O/filter_scale.json
find $O/ftrace -name '*kernel_stats.csv' -exec cp {} $O/filter_kernel_stats.csv \;
cut -d, -f1-4 $O/filter_kernel_stats.csv | head -16
for rep in 1 2; do
  for v in seed noseed; do
    if [ $v = noseed ]; then S=0; else S=1; fi
    IGX_GB_SEED=$S timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --configs c5 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("%-6s C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f tail %.3f | exact %s" % (sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"], c["ms_per_step"] - c["roofline"]["kernel_ms"], j["check"]["all_bit_exact"]))
PY
  done
done | tee $O/ab_seed.txt || exit 1
echo R06E_OK
