# SQ counters of the partitioned form's kernels on C4 (one --pmc pass).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_c; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU --kernel-trace --output-format csv -d $O -o p -- python3 tools/ablate_part.py --configs ${CFG:-c4} --dbg 0 --reps 1 > $O/run.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 $O/run.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_c/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'][:60]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    if 'gbp' in k:
        print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
