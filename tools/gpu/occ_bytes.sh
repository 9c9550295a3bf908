# Occupancy byte map for the cached form's claims (a plain byte store instead of a bitmap atomic):
# group-by parity, then an interleaved A/B of the bench (C2 headline + C5) against the previous
# build (IGX_LIB=inspektor-gadget_amd/.build_ab/libigx.so), then a kernel trace.
# bash tools/gpu/occ_bytes.sh -> gpurun_out/occ_bytes/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/occ_bytes
B=inspektor-gadget_amd/.build_ab/libigx.so
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groupby.py \
    tests/test_gpu_fullsize.py tests/test_gpu_tail.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then L=$B; else L=; fi
    IGX_LIB=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("%-4s C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f" % (sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"]))
PY
  done
done | tee $O/ab.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-4 $O/kernel_stats.csv | head -30 | grep -E "k_groupby<|slots|reset" || true
echo OCCB_OK
