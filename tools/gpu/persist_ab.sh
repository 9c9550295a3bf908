# Keys kept across intervals (generations): the parity tests, then an interleaved A/B of the
# bench (C2 headline + C5, rotating batches) with persistence on and off (IGX_GB_PERSIST=0).
# bash tools/gpu/persist_ab.sh [tests...] -> gpurun_out/persist/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/persist
rm -rf $O; mkdir -p $O
T=${@:-tests/test_gpu_persist.py tests/test_gpu_groupby.py tests/test_gpu_tail.py}
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread $T > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in on off; do
    if [ $v = off ]; then P=0; else P=1; fi
    IGX_GB_PERSIST=$P timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --configs c5 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("%-4s C2 ms/step %.3f kernel %.3f claims %s | C5 ms/step %.3f kernel %.3f claims %s | exact %s" % (
            sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], j["config"].get("claims_per_interval"),
            c["ms_per_step"], c["roofline"]["kernel_ms"], c.get("claims_per_interval"), j["check"]["all_bit_exact"]))
PY
  done
done | tee $O/ab.txt || exit 1
echo PERSIST_OK
