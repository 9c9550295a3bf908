# Per-kernel times of one bench config under an env setting:
#   bash tools/gpu/ktrace.sh <tag> <configs> [ENV=V ...]
set -o pipefail
export TMPDIR=/tmp
T=$1; CFG=$2; shift 2
O=gpurun_out/kt_$T
rm -rf $O; mkdir -p $O
timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --config-steps 3 --configs=$CFG > $O/log 2>&1 || { echo "trace failed rc=$?"; tail -5 $O/log; exit 1; }
f=$(find $O -name '*kernel_stats.csv' | head -1)
python3 - "$f" "$T" <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
print("==", sys.argv[2])
for r in rows[:int(__import__("os").environ.get("KT_ROWS","14"))]:
    n = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
    n = re.sub(r"\((GbArgs|PartArgs|\(anonymous).*", "", n)[:70]
    print(f"{n:70s} {int(r['Calls']):4d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
