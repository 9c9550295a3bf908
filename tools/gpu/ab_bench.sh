# Interleaved A/B of env settings on the default bench (C2 headline + the given configs):
#   bash tools/gpu/ab_bench.sh TAG "ENV=V ENV2=V;ENV=W" [configs] [reps]
set -o pipefail
export TMPDIR=/tmp
T=$1; CFG=${3:-c5}; REPS=${4:-2}
IFS=';' read -ra SETS <<< "$2"
O=gpurun_out/abb_$T
rm -rf $O; mkdir -p $O
for rep in $(seq 1 $REPS); do
  i=0
  for S in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 300 env $S python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --configs $CFG > $O/run${i}_$rep.log 2>&1 || { echo "run $i ($S) failed rc=$?"; tail -5 $O/run${i}_$rep.log; exit 1; }
    python3 - "$S" $O/run${i}_$rep.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
out = [f"c2 {d['ms_per_step']:.3f}/{d['roofline']['kernel_ms']:.3f}"]
for k, v in d["configs"].items():
    r = v.get("roofline") or {}
    out.append(f"{k} {v['ms_per_step']:.3f}/{r.get('kernel_ms', float('nan')):.3f}")
print(f"{sys.argv[1]:40s}", "|", "  ".join(out), "| exact", d["check"]["all_bit_exact"])
PY
  done
done | tee $O/ab.txt
