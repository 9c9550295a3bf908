# Round 6, pass k: the C5 step tail on the current build -- a kernel trace of the C5 bench
# config and the kernels between one interval's group-by and the next one's.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-check --configs c5 > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
grep -h '"metric"' $O/trace.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); c=j['configs']['c5']; print('C5 ms/step %.3f kernel %.3f' % (c['ms_per_step'], c['roofline']['kernel_ms']))"
python3 tools/trace_tail.py $O/trace/run_kernel_trace.csv 'StaticLayout<8, 4, 4, 4>, false, 4, false' --which -2 --before 6 --after 24
echo R06K_OK
