# A/B of bench.py --tables (interval tables in flight), each with --check, then a kernel trace
# of --tables 3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 1 2 3 1 3 4; do
  timeout -k 10 300 python3 bench.py --tables $t --check --cpu-sample 0 > gpurun_out/pipe_$t.log 2>&1 || { echo "bench t=$t failed rc=$?"; tail gpurun_out/pipe_$t.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/pipe_$t.log') if l.startswith('{')][-1]);print('tables=$t', round(d['value']/1e9,3),'G/s', round(d['ms_per_step'],4),'ms', 'gb', round(d['roofline']['kernel_ms'],4), d.get('check'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe -o run --output-format csv -- python3 bench.py --tables 3 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof_pipe.log 2>&1 || { echo "rocprof failed rc=$?"; tail gpurun_out/prof_pipe.log; exit 1; }
head -4 gpurun_out/prof_pipe/run_kernel_stats.csv | cut -c1-200
echo ALL_OK
