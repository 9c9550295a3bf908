# partitioned-form parity tests + pass timings (C4, C5), then the admission sweep
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/part_c.sh || exit 1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/pc2/t/run_kernel_stats.csv')))
print(' '.join(sorted(f"{r['Name'].split('::')[1].split('(')[0][:22]}:{float(r['AverageNs'])/1e6:.3f}" for r in rows if 'k_gbp' in r['Name'])))
PY
bash tools/gpu/sweep_admit.sh
