# C5 (cached form) under the batch and state-machine probers and loader counts
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c5p
for cfg in "IGX_GB_PROBER=0" "IGX_GB_PROBER=1" "IGX_GB_PROBER=1 IGX_GB_LOADERS=6" "IGX_GB_PROBER=0 IGX_GB_LOADERS=6" "IGX_GB_PROBER=0"; do
  env $cfg timeout -k 10 200 python3 tools/ablate_forms.py --configs c5 --forms cached --reps 3 > gpurun_out/c5p/run.log 2>&1 || { echo "$cfg failed"; tail -5 gpurun_out/c5p/run.log; exit 1; }
  echo "$cfg $(grep -h '{' gpurun_out/c5p/run.log | grep -o '"cached_ms": [0-9.]*')"
done
