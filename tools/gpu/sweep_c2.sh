set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sw
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --configs="
run() { name=$1; shift; env "$@" timeout -k 10 120 $B > gpurun_out/sw/$name.log 2>&1 || { echo "$name failed"; return 1; }; python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sw/$name.log') if l.startswith('{')][-1]); print('$name', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"; }
run base A=1 && run slotf5 IGX_GB_SLOTF=5 && run kr16 IGX_GB_KR16=1 && run both IGX_GB_SLOTF=5 IGX_GB_KR16=1 && run sm IGX_GB_PROBER=1 && run nl7 IGX_GB_LOADERS=7 && run nl9 IGX_GB_LOADERS=9 && run base2 A=1
