# who waits on whom inside k_groupby (IGX_GB_DEBUG bit 16 sleep counters; diagnostics)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "--keys 1000000 --zipf 1.1" "--keys 5000000 --zipf 0.0001" "--keys 10000 --zipf 1.1"; do
  timeout -k 10 200 python tools/ablate_groupby.py $cfg --rounds 2 --variants 0,65536 > gpurun_out/waits.log 2>&1 || { echo "failed"; tail gpurun_out/waits.log; exit 1; }
  grep -h '{' gpurun_out/waits.log
done
