# Round 6, final build: memory-side atomics and write requests of the product group-by kernels
# on the bench's own C5 / C2 streams (kept keys, seeded cache), per launch in dispatch order.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/atomf
rm -rf $O; mkdir -p $O
B="python3 bench.py --steps 8 --warmup 3 --cpu-sample 0 --no-check --configs c5"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum --kernel-trace --output-format csv -d $O/p1 -o p -- $B > $O/p1.log 2>&1 || { echo "pass 1 failed"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d $O/p2 -o p -- $B > $O/p2.log 2>&1 || { echo "pass 2 failed"; tail -5 $O/p2.log; exit 1; }
echo "C5 k_groupby<file_id> per launch:"; python3 tools/pmc_summary.py --per-dispatch --kernel 'StaticLayout<8, 4, 4, 4>, false' $O/p1 $O/p2
echo "C2 k_groupby<ip_key_t> per launch:"; python3 tools/pmc_summary.py --per-dispatch --kernel 'StaticLayout<16, 16, 8, 4, 16, 2, 2, 2>, false' $O/p1 $O/p2
echo ATOMF_OK
