# Round 6: a long bench (100 timed steps, every config) and the whole -m gpu suite on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06long
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u bench.py --steps 100 --warmup 10 --config-steps 100 > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log > $O/bench.json
python3 - $O/bench.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read())
print("C2 %.3f/%.3f frac %.3f" % (j["ms_per_step"], j["roofline"]["kernel_ms"], j["roofline"]["frac"]),
      " ".join("%s %.3f/%s" % (k, c["ms_per_step"], (c.get("roofline") or {}).get("kernel_ms") and round(c["roofline"]["kernel_ms"], 3)) for k, c in j["configs"].items()),
      "exact", j["check"]["all_bit_exact"])
PY
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo R06LONG_OK
