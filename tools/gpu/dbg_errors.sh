set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_regex.py tests/test_gpu_parity.py::test_topk_matches_go_sort -q -m gpu --timeout 120 --timeout-method thread -x > gpurun_out/dbg.log 2>&1; echo "rc=$?"
grep -n ":1:\|rocvirtual\|hip_\|Error\|error" gpurun_out/dbg.log | head -30
