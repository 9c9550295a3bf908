# Quick bench of the headline plus the given configs (default c4,c5): one line per config with
# ms/step, dominant-kernel ms and roofline frac.  Extra env vars pass through.
#   bash tools/gpu/bench_cfg.sh [configs] [tests...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${1:-c4,c5}
shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 400 --timeout-method thread > gpurun_out/bc_tests.log 2>&1 || { echo "tests failed"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/bc_tests.log | head -30; tail -3 gpurun_out/bc_tests.log; exit 1; }
  tail -1 gpurun_out/bc_tests.log
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --configs "$CFG" > gpurun_out/bc.json 2>&1 || { echo "bench failed"; tail gpurun_out/bc.json; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bc.json") if l.startswith("{")][-1])
r = d["roofline"]
print("c2", round(d["ms_per_step"], 3), round(r["kernel_ms"], 3), round(r["frac"], 4))
for k, v in d["configs"].items():
    r = v.get("roofline") or {}
    print(k, round(v["ms_per_step"], 3), round(r.get("kernel_ms", 0), 3), round(r.get("frac", 0), 4))
PY
