set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || { echo "configs failed rc=$?"; tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log | grep '{'
echo ALL_OK
