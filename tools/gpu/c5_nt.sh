# C5 with plain stream loads in the cached top-file kernel: group-by parity (top file) and two
# bench runs (C2 headline + C5).  bash tools/gpu/c5_nt.sh -> gpurun_out/c5_nt/
set -o pipefail
O=gpurun_out/c5_nt
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groupby.py::test_top_file_layout \
    tests/test_gpu_fullsize.py::test_c5_full_size_table_and_topk tests/test_gpu_fullsize.py::test_bench_c5_async_intervals_match_oracle \
    > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/bench_$rep.log 2>&1 || { echo "bench failed"; tail $O/bench_$rep.log; exit 1; }
  python3 - $O/bench_$rep.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f" % (j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"]))
PY
done
echo C5_OK
