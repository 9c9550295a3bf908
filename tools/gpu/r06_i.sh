# Round 6, pass i (re-entry check): the whole -m gpu suite, smoke, and the default bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log > $O/bench.json
python3 - $O/bench.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read())
print("C2", j["value"], j["ms_per_step"], j["roofline"]["frac"], j["roofline"].get("kernel_ms"), j["check"]["all_bit_exact"])
for k, c in j.get("configs", {}).items():
    print(k, c.get("ms_per_step"), c.get("roofline", {}).get("frac"), c.get("roofline", {}).get("kernel_ms"))
PY
echo R06I_OK
