# Round 6, pass b: kept keys + the sample-seeded LDS cache (parity, soak), the owner exchange
# and the emulated rank of 8 after the faster table partition, an interleaved A/B of the seeds,
# and the atomics accounting.   bash tools/gpu/r06_b.sh -> gpurun_out/r06b/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_persist.py \
    tests/test_gpu_owner_exchange.py tests/test_gpu_soak.py tests/test_gpu_groupby.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/emulate_rank8.py --out $O/emulated_rank8.json > $O/emul.log 2>&1 || { echo "emulate failed"; tail $O/emul.log; exit 1; }
cat $O/emul.log
for rep in 1 2; do
  for v in seed noseed; do
    if [ $v = noseed ]; then S=0; else S=1; fi
    IGX_GB_SEED=$S timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --configs c5 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("%-6s C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f | exact %s" % (sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"], j["check"]["all_bit_exact"]))
PY
  done
done | tee $O/ab_seed.txt || exit 1
bash tools/gpu/r06_atomics.sh || exit 1
echo R06B_OK
