# Round 6, pass h: the reset's slot-list loads batched (k_reset_clear) -- the kept-key suites,
# then the C2 / C5 bench and a C5 kernel trace (the reset's duration in the step tail).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_persist.py \
    tests/test_gpu_topk_hint.py tests/test_gpu_tail.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --configs c5 > $O/bench_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_$rep.log; exit 1; }
  python3 - $O/bench_$rep.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("C2 ms/step %.3f kernel %.3f tail %.3f | C5 ms/step %.3f kernel %.3f tail %.3f | exact %s" % (
            j["ms_per_step"], j["roofline"]["kernel_ms"], j["ms_per_step"] - j["roofline"]["kernel_ms"],
            c["ms_per_step"], c["roofline"]["kernel_ms"], c["ms_per_step"] - c["roofline"]["kernel_ms"], j["check"]["all_bit_exact"]))
PY
done | tee $O/bench.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
python3 tools/trace_tail.py $O/trace/run_kernel_trace.csv 'StaticLayout<8, 4, 4, 4>, false, 4, false' --which -2
echo R06H_OK
