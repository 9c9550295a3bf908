# Round 6, pass g: the hinted top-K (k_tk_*) -- its parity tests, the table suites that sort,
# and the bench's C2 / C5 tails with the hint on and off (IGX_TOPK_HINT=0), interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk_hint.py \
    tests/test_gpu_tail.py tests/test_gpu_persist.py tests/test_gpu_gadgets.py tests/test_gpu_dist.py tests/test_gpu_owner_exchange.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export IGX_TOPK_HINT=0; else unset IGX_TOPK_HINT; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --configs c5 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("%-4s C2 ms/step %.3f kernel %.3f tail %.3f | C5 ms/step %.3f kernel %.3f tail %.3f | exact %s" % (
            sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], j["ms_per_step"] - j["roofline"]["kernel_ms"],
            c["ms_per_step"], c["roofline"]["kernel_ms"], c["ms_per_step"] - c["roofline"]["kernel_ms"], j["check"]["all_bit_exact"]))
PY
  done
done | tee $O/ab_topk.txt || exit 1
unset IGX_TOPK_HINT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-4 $O/kernel_stats.csv | head -40
echo R06G_OK
