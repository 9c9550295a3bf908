set -o pipefail
export TMPDIR=/tmp
P="python3 tools/ablate_groupby.py --events 50000000 --rounds 1"
for v in 1 0; do
  for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE TCC_EA0_ATOMIC_sum" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    tag=$(echo $pmc | cut -d' ' -f1)
    timeout -k 10 200 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/pmc_v${v}_${tag} -o p -- $P --variants $v > gpurun_out/pmc_v${v}_${tag}.log 2>&1 || { echo "pmc $v $tag failed"; tail -5 gpurun_out/pmc_v${v}_${tag}.log; }
  done
done
echo ALL_OK
