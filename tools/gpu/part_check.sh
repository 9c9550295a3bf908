# Partitioned form: parity tests, then the forms ablation and a per-kernel trace on C4/C5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_groupby.py -x -q -m gpu -k "partitioned" --timeout 120 --timeout-method thread > gpurun_out/part_tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/part_tests.log | head -30; tail -3 gpurun_out/part_tests.log; exit 1; }
tail -2 gpurun_out/part_tests.log
timeout -k 10 300 python -u tools/ablate_forms.py --configs ${CFG:-c4,c5} --forms ${FORMS:-part} --reps 3 > gpurun_out/forms.log 2>&1 || { echo "forms failed"; tail gpurun_out/forms.log; exit 1; }
grep config gpurun_out/forms.log | tail -${NL:-2}
CFG=${CFG:-c4,c5} bash tools/gpu/prof_part.sh > gpurun_out/prof_part.log 2>&1 || { echo "prof failed"; tail gpurun_out/prof_part.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_part/trace/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    if 'gbp' in r['Name'] or 'groupby' in r['Name']:
        print(f"{float(r['AverageNs'])/1e6:8.3f} ms x{r['Calls']:>4}  {r['Name'][:100]}")
PY
