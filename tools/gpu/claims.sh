# cost of first-touch claims: launches on a table that already holds every key (diagnostics)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "--keys 1000000 --zipf 1.1" "--keys 5000000 --zipf 0.0001"; do
  timeout -k 10 200 python tools/ablate_groupby.py $cfg --rounds 3 --variants 0,4 > gpurun_out/claims_a.log 2>&1 || { echo "failed"; tail gpurun_out/claims_a.log; exit 1; }
  timeout -k 10 200 python tools/ablate_groupby.py $cfg --rounds 3 --variants 0,4 --noreset > gpurun_out/claims_b.log 2>&1 || { echo "failed"; tail gpurun_out/claims_b.log; exit 1; }
  echo "reset   $(grep -h '{' gpurun_out/claims_a.log)"
  echo "noreset $(grep -h '{' gpurun_out/claims_b.log)"
done
