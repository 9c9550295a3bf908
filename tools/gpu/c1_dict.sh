# String-dictionary sort (k_dict_*) on the GPU: the sort parity tests, then C1's step with and
# without the dictionary (IGX_SORT_DICT=0), then a kernel trace of the dictionary step.
# bash tools/gpu/c1_dict.sh -> gpurun_out/c1_dict/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c1_dict
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py \
    -k "sort or filter or c1 or topk or ties" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  IGX_SORT_DICT=0 timeout -k 10 120 python3 tools/c1_step.py 50 >> $O/step.log 2>&1 || { echo "step failed"; tail $O/step.log; exit 1; }
  echo "^ dict off" >> $O/step.log
  timeout -k 10 120 python3 tools/c1_step.py 50 >> $O/step.log 2>&1 || { echo "step failed"; tail $O/step.log; exit 1; }
  echo "^ dict on" >> $O/step.log
done
cat $O/step.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/c1_step.py 20 > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-8 $O/kernel_stats.csv | head -20
echo ALL_OK
