set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ablate_groupby.py --variants 0,4,16,20,32,36,96,100,112,116 > gpurun_out/ablate1.log 2>&1 || { echo "ablate1 failed"; tail gpurun_out/ablate1.log; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --keys 10000 --variants 0,4,16,20,32,36,96,100,112,116 > gpurun_out/ablate2.log 2>&1 || { echo "ablate2 failed"; exit 1; }
grep -h '{' gpurun_out/ablate*.log
