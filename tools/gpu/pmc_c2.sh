# SQ instruction / wait counters of the C2 cached group-by (is the kernel issue-bound anywhere?)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pq
C2="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --configs="
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pq/p1 -o p -- $C2 > gpurun_out/pq/p1.log 2>&1 || { echo "p1 failed"; tail -5 gpurun_out/pq/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pq/p2 -o p -- $C2 > gpurun_out/pq/p2.log 2>&1 || { echo "p2 failed"; tail -5 gpurun_out/pq/p2.log; exit 1; }
echo ok
