# partitioned-form parity tests, then pass timings of C4 / C5 in the partitioned form
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pc2
timeout -k 10 400 python -u -m pytest tests/test_gpu_groupby.py -k "partitioned or direct or netpolicy or prober" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pc2/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/pc2/pytest.log | head -30; tail -3 gpurun_out/pc2/pytest.log; exit 1; }
tail -1 gpurun_out/pc2/pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pc2/t -o run --output-format csv -- python3 tools/ablate_forms.py --configs c4,c5 --forms part --reps 2 > gpurun_out/pc2/forms.log 2>&1 || { echo "forms failed"; tail -5 gpurun_out/pc2/forms.log; exit 1; }
grep -h '{' gpurun_out/pc2/forms.log | cut -c1-110
