set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || echo "list failed"
timeout -k 10 300 python tools/ablate_groupby.py > gpurun_out/ablate1.log 2>&1 || { echo "ablate1 failed"; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --zipf 0.0 > gpurun_out/ablate2.log 2>&1 || { echo "ablate2 failed"; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --keys 1000 > gpurun_out/ablate3.log 2>&1 || { echo "ablate3 failed"; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --keys 10000000 --zipf 1.05 > gpurun_out/ablate4.log 2>&1 || { echo "ablate4 failed"; exit 1; }
grep -h '{' gpurun_out/ablate*.log
echo ALL_OK
