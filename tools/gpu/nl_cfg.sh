# the bench (C2 headline + C4/C5 in the same line) under values of a tuning knob:
#   bash tools/gpu/nl_cfg.sh "7 8 9" [IGX_GB_LOADERS]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=${2:-IGX_GB_LOADERS}
for v in $1; do
  env $VAR=$v timeout -k 10 300 python bench.py --cpu-sample 0 --configs c4,c5 > gpurun_out/nlb_$v.log 2>&1 || { echo "bench $VAR=$v failed"; tail -3 gpurun_out/nlb_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/nlb_$v.log') if l.startswith('{')][-1]); print('$VAR=$v', 'c2', round(d['ms_per_step'],3), ' '.join(k + ' ' + str(round(c['ms_per_step'],3)) for k, c in d['configs'].items()))"
done
