# where the miss path's time goes: 0 full, 4 no HBM atomics, 256 no HBM probe, 260 neither, 2 misses dropped, 1 load+hash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ablate_groupby.py --variants 0,256,260,2,1 --rounds 3 > gpurun_out/ablate_miss.log 2>&1 || { echo "failed"; tail gpurun_out/ablate_miss.log; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --variants 0,4 --rounds 3 --noreset > gpurun_out/ablate_miss2.log 2>&1 || { echo "failed2"; tail gpurun_out/ablate_miss2.log; exit 1; }
grep -h '{' gpurun_out/ablate_miss*.log
