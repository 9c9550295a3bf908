# PMC counters of the partitioned form's kernels on C4 (separate passes, kernel trace only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_part
rm -rf $O; mkdir -p $O
B="python3 tools/ablate_forms.py --configs ${CFG:-c4} --forms part --reps 1"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_FLAT SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o p -- $B > $O/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 $O/p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(int)
for f in glob.glob('gpurun_out/pmc_part/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'k_gbp' not in k: continue
        k = k.split('(')[0].split('::')[-1] + ('<' + k.split('<', 1)[1].split('>')[0] + '>' if '<' in k else '')
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    print(k[:40], {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
