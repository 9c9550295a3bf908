# SQ instruction / wait counters of the partitioned form's passes (C4, C5): VALU-, LDS- or memory-bound?
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pc/p1 -o p -- python3 tools/ablate_forms.py --configs c4,c5 --forms part --reps 1 > gpurun_out/pc/p1.log 2>&1 || { echo "p1 failed"; tail -5 gpurun_out/pc/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pc/p2 -o p -- python3 tools/ablate_forms.py --configs c4,c5 --forms part --reps 1 > gpurun_out/pc/p2.log 2>&1 || { echo "p2 failed"; tail -5 gpurun_out/pc/p2.log; exit 1; }
find gpurun_out/pc -name '*counter_collection.csv'
