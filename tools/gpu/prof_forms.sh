# kernel times of the partitioned form on C4 / C5 (rocprofv3 kernel trace + stats)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_part
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 tools/ablate_forms.py --configs ${CFG:-c4,c5} --forms part --reps 2 > $O/log.txt 2>&1 || { echo "prof failed rc=$?"; tail -5 $O/log.txt; exit 1; }
grep -v amdgpu.ids $O/log.txt
f=$(find $O -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -20
