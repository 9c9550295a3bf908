# Round 6: the default bench on one more fresh box (box-to-box spread): bash tools/gpu/r06_box.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06box_$1
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log > $O/bench.json
python3 - $O/bench.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read())
print("C2 %.3f/%.3f frac %.3f" % (j["ms_per_step"], j["roofline"]["kernel_ms"], j["roofline"]["frac"]),
      " ".join("%s %.3f/%s" % (k, c["ms_per_step"], (c.get("roofline") or {}).get("kernel_ms") and round(c["roofline"]["kernel_ms"], 3)) for k, c in j["configs"].items()),
      "exact", j["check"]["all_bit_exact"])
PY
