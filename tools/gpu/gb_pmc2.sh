set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-1 772 0}; do
  P="python3 tools/ablate_groupby.py --events 50000000 --rounds 1 --keys 1000000 --variants $v"
  i=0
  for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_LDS_ADDR_CONFLICT" ; do
    i=$((i+1))
    rm -rf gpurun_out/pmc2_${v}_$i
    timeout -k 10 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/pmc2_${v}_$i -o p -- $P > gpurun_out/pmc2_${v}_$i.log 2>&1 || { echo "pmc $v $i failed"; tail -5 gpurun_out/pmc2_${v}_$i.log; }
  done
  echo "variant=$v"
  python3 tools/pmc_summary.py --kernel k_groupby gpurun_out/pmc2_${v}_* || exit 1
done
