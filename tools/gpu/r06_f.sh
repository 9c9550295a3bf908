# Round 6, pass f: 8-lane-aligned update runs in the server ring (IGX_RING_ALIGN) -- parity,
# the atomics accounting with the aligned debug build, and an interleaved A/B against the
# unaligned build (IGX_LIB=inspektor-gadget_amd/libigx_noalign.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_groupby.py \
    tests/test_gpu_persist.py tests/test_gpu_soak.py tests/test_gpu_gadgets.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/r06_atomics.sh > $O/atomics.txt 2>&1 || { echo "atomics failed"; tail -20 $O/atomics.txt; exit 1; }
grep -A1 "PMC per launch" $O/atomics.txt | grep -v "^--"
for rep in 1 2 3; do
  for v in align noalign; do
    if [ $v = noalign ]; then export IGX_LIB=inspektor-gadget_amd/libigx_noalign.so; else unset IGX_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-check --configs c5 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("%-8s C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f" % (sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"]))
PY
  done
done | tee $O/ab_align.txt || exit 1
unset IGX_LIB
echo R06F_OK
