# k_hist iteration: histogram parity tests, then C3 timing (kernel stats) through the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hi
timeout -k 10 400 python -u -m pytest tests -k "hist or block_io or profile" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/hi/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/hi/pytest.log | head -30; tail -3 gpurun_out/hi/pytest.log; exit 1; }
tail -1 gpurun_out/hi/pytest.log
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --configs c3 --config-steps 10 > gpurun_out/hi/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/hi/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/hi/bench.log') if l.startswith('{')][-1]); c=d['configs']['c3']; print('c3', c['ms_per_step'], c['roofline']['kernel_ms'], c['roofline']['frac'])"
