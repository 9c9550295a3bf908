# LDS admission filter on/off (IGX_GB_ADMIT=0: admit on the first miss)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/admit.log
for k in 0 1; do
  for cfg in "--keys 1000000 --zipf 1.1" "--keys 10000 --zipf 1.1" "--keys 100000 --zipf 0.9" "--keys 1000000 --zipf 0.0001"; do
    IGX_GB_ADMIT=$k timeout -k 10 120 python tools/ablate_groupby.py $cfg --rounds 2 --variants 0,8 > gpurun_out/admit_one.log 2>&1 || { echo "failed k=$k $cfg"; tail gpurun_out/admit_one.log; exit 1; }
    echo "k=$k $(grep -h '{' gpurun_out/admit_one.log)" | tee -a gpurun_out/admit.log
  done
done
