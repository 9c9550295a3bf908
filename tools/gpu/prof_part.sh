# Kernel-trace of the partitioned form alone on C4 and C5 (per-pass durations).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_part
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/ablate_forms.py --configs ${CFG:-c4,c5} --forms part --reps 2 > $O/run.log 2>&1 || { echo "failed rc=$?"; tail $O/run.log; exit 1; }
tail -3 $O/run.log
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -30
