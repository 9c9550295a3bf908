# hit/miss counts and load-only time of k_groupby at 1M and 10K keys (diagnostics)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ablate_groupby.py --variants 0,1,2,8 > gpurun_out/hit1.log 2>&1 || { echo "hit1 failed"; tail gpurun_out/hit1.log; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --keys 10000 --variants 0,8 > gpurun_out/hit2.log 2>&1 || { echo "hit2 failed"; tail gpurun_out/hit2.log; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --zipf 0.0001 --keys 1000000 --variants 0,8 > gpurun_out/hit3.log 2>&1 || { echo "hit3 failed"; tail gpurun_out/hit3.log; exit 1; }
grep -h '{' gpurun_out/hit*.log
