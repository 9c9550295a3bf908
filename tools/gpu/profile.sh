# Round profile: rocprofv3 kernel trace + stats of the bench command, the HBM-traffic PMC
# passes (FETCH_SIZE and WRITE_SIZE in separate runs), the default bench line, and the
# per-config bench under rocprofv3 --stats.  Results are copied to profiles/$1/.
set -o pipefail
export TMPDIR=/tmp
R=${1:-r01}
mkdir -p gpurun_out profiles/$R
B="python3 bench.py --steps 5 --warmup 2 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $B > gpurun_out/prof.log 2>&1 || { echo "rocprof trace failed rc=$?"; tail gpurun_out/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o p -- $B > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed rc=$?"; tail gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o p -- $B > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed rc=$?"; tail gpurun_out/pmc_write.log; exit 1; }
python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --kernel k_groupby \
  --config '{"events": 100000000, "keys": 1000000, "zipf": 1.1}' --out gpurun_out/traffic.json || { echo "traffic parse failed"; exit 1; }
# (files under profiles/ do not travel back: copy them from gpurun_out/ afterwards)
cp gpurun_out/traffic.json profiles/$R/traffic.json
cp gpurun_out/prof/run_kernel_stats.csv profiles/$R/kernel_stats.csv
timeout -k 10 600 python3 bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench full failed rc=$?"; tail gpurun_out/bench_full.log; exit 1; }
grep -h '"metric"' gpurun_out/bench_full.log > profiles/$R/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profc -o run --output-format csv -- python3 tools/bench_configs.py > gpurun_out/configs.log 2>&1 || { echo "configs failed rc=$?"; tail gpurun_out/configs.log; exit 1; }
grep -h '{' gpurun_out/configs.log > profiles/$R/configs.jsonl
cp gpurun_out/profc/run_kernel_stats.csv profiles/$R/configs_kernel_stats.csv
cat profiles/$R/bench.json | cut -c1-1500
head -6 profiles/$R/kernel_stats.csv | cut -c1-220
echo ALL_OK
# gpurun merges back gpurun_out/ only; locally, after the call:
#   cp gpurun_out/traffic.json profiles/R/; cp gpurun_out/prof/run_kernel_stats.csv profiles/R/kernel_stats.csv
#   grep '"metric"' gpurun_out/bench_full.log > profiles/R/bench.json; grep '^{' gpurun_out/configs.log > profiles/R/configs.jsonl
#   cp gpurun_out/profc/run_kernel_stats.csv profiles/R/configs_kernel_stats.csv
