set -o pipefail
O=gpurun_out/slotf; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for v in 8 6 5; do
    IGX_GB_SLOTF=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/b_${v}_$rep.log 2>&1 || { echo "bench failed"; tail $O/b_${v}_$rep.log; exit 1; }
    python3 - $O/b_${v}_$rep.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("slotf=%s C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f" % (sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"]))
PY
  done
done | tee $O/ab.txt
