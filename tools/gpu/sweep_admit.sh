# LDS admission threshold sweep (IGX_GB_ADMIT: admit on the (k+1)-th miss) on C2 (bench) and C5 (cached form)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ad
B="python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --configs="
for k in 1 2 3 1; do
  IGX_GB_ADMIT=$k timeout -k 10 120 $B > gpurun_out/ad/c2_$k.log 2>&1 || { echo "c2 k=$k failed"; tail -5 gpurun_out/ad/c2_$k.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ad/c2_$k.log') if l.startswith('{')][-1]); print('c2 admit=$k', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"
done
for k in 1 2 3; do
  IGX_GB_ADMIT=$k timeout -k 10 200 python3 tools/ablate_forms.py --configs c5 --forms cached --reps 3 > gpurun_out/ad/c5_$k.log 2>&1 || { echo "c5 k=$k failed"; tail -5 gpurun_out/ad/c5_$k.log; exit 1; }
  echo "c5 admit=$k $(grep -h '{' gpurun_out/ad/c5_$k.log | cut -c1-90)"
done
