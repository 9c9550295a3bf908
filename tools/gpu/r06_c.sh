# Round 6, pass c: the atomics accounting on kept keys, the owner-merge form for the emulated
# rank of 8, and a loader-wave sweep of the kept-key + seeded kernels.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
rm -rf $O; mkdir -p $O
bash tools/gpu/r06_atomics.sh > $O/atomics.txt 2>&1 || { echo "atomics failed"; tail -20 $O/atomics.txt; exit 1; }
cat $O/atomics.txt
for m in direct cached part; do
  timeout -k 10 300 python3 tools/emulate_rank8.py --merge-mode $m --reps 6 --out $O/emul_$m.json > $O/emul_$m.log 2>&1 || { echo "emulate $m failed"; tail $O/emul_$m.log; exit 1; }
  echo "merge $m"; grep -E "^c[45] " $O/emul_$m.log
done
for L in 8 9 7 def; do
  if [ $L = def ]; then unset IGX_GB_LOADERS; else export IGX_GB_LOADERS=$L; fi
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-check --configs c5 > $O/bench_L$L.log 2>&1 || { echo "bench failed"; tail $O/bench_L$L.log; exit 1; }
  python3 - $O/bench_L$L.log $L <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        j = json.loads(l); c = j["configs"]["c5"]
        print("loaders %-3s C2 ms/step %.3f kernel %.3f | C5 ms/step %.3f kernel %.3f" % (sys.argv[2], j["ms_per_step"], j["roofline"]["kernel_ms"], c["ms_per_step"], c["roofline"]["kernel_ms"]))
PY
done | tee $O/loaders.txt || exit 1
echo R06C_OK
