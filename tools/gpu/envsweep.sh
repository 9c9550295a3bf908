# k_groupby under an environment knob: bash tools/gpu/envsweep.sh VAR "v1 v2 ..." (diagnostics)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=$1; VALS=$2
: > gpurun_out/envsweep.log
for v in $VALS; do
  for cfg in "--keys 1000000 --zipf 1.1" "--keys 10000 --zipf 1.1" "--keys 5000000 --zipf 0.0001"; do
    env $VAR=$v timeout -k 10 120 python tools/ablate_groupby.py $cfg --rounds 3 --variants 0 > gpurun_out/envsweep_one.log 2>&1 || { echo "failed $VAR=$v $cfg"; tail gpurun_out/envsweep_one.log; exit 1; }
    echo "$VAR=$v $(grep -h '{' gpurun_out/envsweep_one.log)" | tee -a gpurun_out/envsweep.log
  done
done
