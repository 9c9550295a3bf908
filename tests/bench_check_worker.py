"""world_size-2 gloo worker for tests/test_bench_check.py: bench.py's N>1 post-run check
(gather_checks over the process group, merge_rank_topk, sum_rank_hists) against the oracle
run over the union of both ranks' events.  Exits non-zero on a mismatch."""
import os
import sys

import numpy as np
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402

N, G, K = 150_000, 4_000, 20


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx = {"rank": rank, "world": world, "dist": dist}
    cdf = O.zipf_cdf(G, 1.1)
    # C2: each rank's own key universe and global event indices rank*N.., as bench.run_c2
    h = O.gen_tcp(0xC2, rank, G, cdf, rank * N, N)
    Gr, sent, recv, first = O.top_tcp_mt(h, K, base_idx=rank * N, threads=2)
    recs = bench.gather_checks(ctx, {"groups": int(Gr), "sent": sent, "recv": recv, "first": first})
    # C3: each rank's slice of one stream, histograms summed as the device all-reduce does
    q = O.lognormal_quantiles(np.log(2e5), 1.5)
    hb = O.gen_bio(0xC3, q, rank * N, N)
    hists = bench.gather_checks(ctx, O.hist_log2_mt(hb["dev"], hb["cont"], hb["delta"], bench.C3_DEVS,
                                                    bench.C3_NCONT, threads=2))
    if rank == 0:
        assert len(recs) == world and len(hists) == world
        S, R, F = bench.merge_rank_topk(O, recs, K)
        parts = [O.gen_tcp(0xC2, r, G, cdf, r * N, N) for r in range(world)]
        union = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
        Gu, _, us, ur, uf = O.top_tcp(union, K)
        assert Gu == sum(r["groups"] for r in recs), (Gu, [r["groups"] for r in recs])
        assert np.array_equal(F, uf) and np.array_equal(S, us) and np.array_equal(R, ur)
        bu = O.gen_bio(0xC3, q, 0, world * N)
        ref = O.hist_log2(bu["dev"], bu["cont"], bu["delta"], bench.C3_DEVS, bench.C3_NCONT)
        assert np.array_equal(bench.sum_rank_hists(hists), ref)
        print("BENCH_CHECK_OK", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
