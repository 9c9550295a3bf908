# where the miss path's time goes: 0 full, 4 no HBM atomics, 256 no HBM probe, 260 neither, 2 misses dropped
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
true
timeout -k 10 300 python tools/ablate_groupby.py --keys 5000000 --zipf 0.0001 --events 100000000 --variants 0,4,256,260,2 --rounds 2 > gpurun_out/ablate_miss2.log 2>&1 || { echo "failed2"; tail gpurun_out/ablate_miss2.log; exit 1; }
grep -h '{' gpurun_out/ablate_miss*.log
