# Round 6, first pass: the new parity tests (kept keys, owner exchange, the N>1 bench rehearsal),
# the group-by suites, the A/B of kept keys on/off on the bench, and the emulated rank of 8.
# bash tools/gpu/r06_round1.sh -> gpurun_out/r06a/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_persist.py \
    tests/test_gpu_owner_exchange.py tests/test_gpu_bench_dist.py tests/test_gpu_groupby.py tests/test_gpu_tail.py \
    tests/test_gpu_dist.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then P=0; else P=1; fi
    IGX_GB_PERSIST=$P timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --configs c5 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("%-4s C2 ms/step %.3f kernel %.3f claims %s batches %s | C5 ms/step %.3f kernel %.3f claims %s batches %s | exact %s" % (
            sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], j["config"].get("claims_per_interval"), j["config"].get("batches"),
            c["ms_per_step"], c["roofline"]["kernel_ms"], c.get("claims_per_interval"), c.get("batches"), j["check"]["all_bit_exact"]))
PY
  done
done | tee $O/ab.txt || exit 1
timeout -k 10 300 python3 tools/emulate_rank8.py --out $O/emulated_rank8.json > $O/emul.log 2>&1 || { echo "emulate failed"; tail $O/emul.log; exit 1; }
cat $O/emul.log

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-4 $O/kernel_stats.csv | head -40
echo TRACE_OK
