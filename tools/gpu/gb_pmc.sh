# SQ / LDS / L2 counters of k_groupby for two variants (full, hits-only) at 10K and 1M keys
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for keys in 10000 1000000; do
for v in 0 2; do
  P="python3 tools/ablate_groupby.py --events 50000000 --rounds 1 --keys $keys --variants $v"
  i=0
  for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum" ; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/pmc_${keys}_${v}_$i -o p -- $P > gpurun_out/pmc_${keys}_${v}_$i.log 2>&1 || { echo "pmc $keys $v $i failed"; tail -5 gpurun_out/pmc_${keys}_${v}_$i.log; exit 1; }
  done
  echo "keys=$keys variant=$v"
  python3 tools/pmc_summary.py --kernel k_groupby gpurun_out/pmc_${keys}_${v}_* || exit 1
done
done
