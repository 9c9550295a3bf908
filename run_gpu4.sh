set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --variants 0,1,2,4 > gpurun_out/ablate1.log 2>&1 || { echo "ablate1 failed"; exit 1; }
IGX_GB_GENERIC=1 timeout -k 10 300 python tools/ablate_groupby.py --variants 0,1 > gpurun_out/ablate1g.log 2>&1 || { echo "ablate1g failed"; exit 1; }
timeout -k 10 300 python tools/ablate_groupby.py --keys 1000 --variants 0,1,2,4 > gpurun_out/ablate3.log 2>&1 || { echo "ablate3 failed"; exit 1; }
grep -h '{' gpurun_out/ablate*.log
echo ALL_OK
