# A/B of a variant libigx.so (tools/variants/<name>.so) against the in-tree one on C2 and C5:
#   bash tools/gpu/variant_ab.sh libigx_nt0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
cp inspektor-gadget_amd/libigx.so gpurun_out/ab/base.so
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --configs c5 --config-steps 3"
for r in 1 2; do
  for v in base $1; do
    if [ $v = base ]; then cp gpurun_out/ab/base.so inspektor-gadget_amd/libigx.so; else cp tools/variants/$v.so inspektor-gadget_amd/libigx.so; fi
    timeout -k 10 200 $B > gpurun_out/ab/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab/$v.log; cp gpurun_out/ab/base.so inspektor-gadget_amd/libigx.so; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab/$v.log') if l.startswith('{')][-1]); c=d['configs']['c5']; print('$v', 'c2', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), 'c5', round(c['ms_per_step'],3), round(c['roofline']['kernel_ms'],3))"
  done
done
cp gpurun_out/ab/base.so inspektor-gadget_amd/libigx.so
rm -f gpurun_out/ab/base.so
