# Round 6, pass l: the owner merge unpacks the exchanged rows in one igx_ingest_aos pass --
# its tests, the partitioned-form suite (dense flush), then rank 0 of 8 emulated (merge time).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_owner_exchange.py \
    tests/test_gpu_groupby.py tests/test_gpu_dist.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "^(FAILED|ERROR)|^E  " $O/tests.log | head -40; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 tools/emulate_rank8.py --reps 6 --out $O/emulated_rank8.json > $O/emu.log 2>&1 || { echo "emulate failed"; tail $O/emu.log; exit 1; }
python3 -c "
import json; j=json.load(open('$O/emulated_rank8.json'))
for k in ('c5','c4'):
    print(k, {kk: (round(vv,3) if isinstance(vv,float) else vv) for kk,vv in j[k]['ms'].items()})"
echo R06L_OK
