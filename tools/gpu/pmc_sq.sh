# SQ counters per kernel of one bench config: bash tools/gpu/pmc_sq.sh <tag> <configs> [ENV=V ...]
set -o pipefail
export TMPDIR=/tmp
T=$1; CFG=$2; shift 2
O=gpurun_out/pmc_$T
rm -rf $O; mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --config-steps 2 --configs=$CFG"
timeout -s KILL 120 env "$@" rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/p1 -o p -- $B > $O/p1.log 2>&1 || { echo "pmc1 failed rc=$?"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 env "$@" rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/p2 -o p -- $B > $O/p2.log 2>&1 || echo "pmc2 failed rc=$? (optional)"
python3 tools/pmc_sq.py $O
