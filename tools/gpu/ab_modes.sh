# A/B of the group-by forms on the bench configs: bash tools/gpu/ab_modes.sh "<configs>" "<mode env sets ;-separated>"
# e.g. bash tools/gpu/ab_modes.sh c4,c5 "IGX_GB_MODE=0;IGX_GB_MODE=4;IGX_GB_MODE=4 IGX_GBH_NOCACHE=1"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
CFG=${1:-c4,c5}
IFS=';' read -ra SETS <<< "${2:-IGX_GB_MODE=0;IGX_GB_MODE=4}"
i=0
for S in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 env $S python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --config-steps 5 --configs=$CFG > gpurun_out/ab/run$i.log 2>&1 || { echo "run $i ($S) failed rc=$?"; tail -5 gpurun_out/ab/run$i.log; exit 1; }
  python3 - "$S" gpurun_out/ab/run$i.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
out = [f"c2 {d['ms_per_step']:.3f}/{d['roofline']['kernel_ms']:.3f}"]
for k, v in d["configs"].items():
    r = v.get("roofline") or {}
    out.append(f"{k} {v['ms_per_step']:.3f}/{r.get('kernel_ms', float('nan')):.3f}")
print(sys.argv[1], "|", "  ".join(out))
PY
done
