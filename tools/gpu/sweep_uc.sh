# pass-C round size sweep of the partitioned form (C4, C5): IGX_GBP_UC records per thread per round
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/uc
for uc in 1 2 3 4; do
  IGX_GBP_UC=$uc timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/uc/t$uc -o run --output-format csv -- python3 tools/ablate_forms.py --configs c4,c5 --forms part --reps 2 > gpurun_out/uc/uc$uc.log 2>&1 || { echo "uc=$uc failed"; tail -5 gpurun_out/uc/uc$uc.log; exit 1; }
  echo "uc=$uc"; grep -h '{' gpurun_out/uc/uc$uc.log
  grep -h 'k_gbp_c\|k_gbp_a\|k_gbp_b\|k_gbp_count' gpurun_out/uc/t$uc/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
done
