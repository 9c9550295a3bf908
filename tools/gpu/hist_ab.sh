# k_hist A/B: histogram parity tests, then an interleaved bench of C3 against the previous build
# (IGX_LIB=inspektor-gadget_amd/.build_ab/libigx.so).  bash tools/gpu/hist_ab.sh -> gpurun_out/hist_ab/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hist_ab
B=inspektor-gadget_amd/.build_ab/libigx.so
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py::test_c3_full_size_histogram \
    tests/test_gpu_parity.py -k "hist or c3" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then L=$B; else L=; fi
    IGX_LIB=$L timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-check --configs c3 > $O/bench_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_${v}_$rep.log; exit 1; }
    python3 - $O/bench_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c3"]
        print("%-4s C3 ms/step %.4f kernel %.4f frac %.3f" % (sys.argv[2], c["ms_per_step"], c["roofline"]["kernel_ms"], c["roofline"]["frac"]))
PY
  done
done | tee $O/ab.txt || exit 1
echo HIST_OK
