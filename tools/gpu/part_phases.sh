# phase ablation of the partitioned form (IGX_GBP_DEBUG bits; results invalid under them)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 4 6 8 16 24}; do
  IGX_GBP_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ph_$d -o run --output-format csv -- python3 tools/ablate_forms.py --configs ${CFG:-c4} --forms part --reps 2 > gpurun_out/ph_$d.log 2>&1 || { echo "failed $d"; tail -3 gpurun_out/ph_$d.log; exit 1; }
  python3 - $d <<'PY'
import csv, glob, sys
d = sys.argv[1]
f = glob.glob(f'gpurun_out/ph_{d}/**/*kernel_stats.csv', recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if 'k_gbp' in r['Name']:
        n = r['Name'].split('::')[1].split('(')[0].split('<')[0]
        out.append(f"{n} {float(r['AverageNs'])/1e6:.3f}")
print(f"dbg={d}: " + ", ".join(sorted(out)))
PY
done
