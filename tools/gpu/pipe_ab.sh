# A/B of the double-buffered interval loop in bench.py (pipeline 1 vs 0), both with --check,
# then a kernel trace of the pipelined form.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 0 1 0 1; do
  timeout -k 10 300 python3 bench.py --pipeline $p --check --cpu-sample 0 > gpurun_out/pipe_$p.log 2>&1 || { echo "bench p=$p failed rc=$?"; tail gpurun_out/pipe_$p.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/pipe_$p.log') if l.startswith('{')][-1]);print('pipeline=$p', round(d['value']/1e9,3),'G/s', round(d['ms_per_step'],4),'ms', 'gb', round(d['roofline']['kernel_ms'],4), d.get('check'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe -o run --output-format csv -- python3 bench.py --pipeline 1 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof_pipe.log 2>&1 || { echo "rocprof failed rc=$?"; tail gpurun_out/prof_pipe.log; exit 1; }
head -4 gpurun_out/prof_pipe/run_kernel_stats.csv | cut -c1-200
echo ALL_OK
