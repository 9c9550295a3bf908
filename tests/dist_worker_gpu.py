"""world_size-2 worker for tests/test_gpu_dist.py: both ranks on cuda:0, gloo carrying
host-staged tensors (RCCL refuses two ranks on one GPU), so the exchanges are torch's but
everything else is the product's libigx.so path:

  C3  each rank histograms its slice of the global stream (igx_hist_log2) ->
      dist.allreduce_hist                                    == oracle on the union
  C4  each rank marks + dedups its slice (igx_np_mark, igx_groupby) -> partial rows
      (igx_groupby_gather) -> dist.exchange_rows (igx_partition_rows + all-to-all) ->
      dist.merge_partials (igx_groupby_update_ex, SUM / MIN first) on the owner
                                                             == oracle on the union, each key
                                                                on exactly one rank
  C5  top file: per-rank group-by of a slice of ONE global key universe -> exchange ->
      owner merge -> per-owner top-20 by -wbytes -> dist.merge_topk (all-gather + igx_topk)
                                                             == oracle group-by + Go sort
  C2  rank-disjoint top tcp (ingest-partitioned) -> dist.merge_topk
                                                             == oracle top_tcp on the union
Rank 0 checks every result and exits non-zero on a mismatch.
"""
import importlib
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

igx = importlib.import_module("inspektor-gadget_amd")
D, E, H, A = igx.dist, igx.engine, igx.columns, igx._abi

N = 400_000


def check(ok, what):
    if not ok:
        print(f"MISMATCH: {what}", flush=True)
        sys.exit(3)


def table_rows(tab):
    """every group of a finalized table as packed rows (key | aggs | first)."""
    fin = tab.finalize()
    G = fin["n_groups"]
    slots = torch.empty(max(1, G), dtype=torch.int32, device="cuda")[:G]
    if G:
        tab.ctx.check(tab.ctx.L.igx_memcpy_d2d(tab.ctx.h, slots.data_ptr(), fin["groups_ptr"], G * 4))
    return tab.gather(slots), fin


def c3(rank, ws):
    q = E.lognormal_quantiles(np.log(2e5), 1.5)
    devs = [(8 << 20) | (16 * k) for k in range(16)]
    ev = E.gen_bio(0xC3, H.to_device(q), rank * N, N)
    hist = E.hist_log2(ev["dev"], ev["cont"], ev["delta"].view(torch.int64), devs, 256)
    D.allreduce_hist(hist)
    if rank == 0:
        a = O.gen_bio(0xC3, q, 0, ws * N)
        ref = O.hist_log2(a["dev"], a["cont"], a["delta"], devs, 256)
        check(np.array_equal(H.host(hist), ref), "C3 all-reduced histogram")


def c4(rank, ws):
    names = ("src", "pkt", "peer", "port")
    widths = [4, 1, 4, 2]
    ev = E.gen_np(0xC4, 2_000, 20_000, rank * N, N)
    keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
    tab = E.Table(widths, [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], N)
    tab.update([ev[k] for k in names], [0, 1, 2, 3], N, rank * N, valid=keep)
    rows, fin = table_rows(tab)
    kb = fin["key_bytes"]
    mine = D.exchange_rows(rows, kb)
    merged = D.merge_partials(mine, widths, [8], max(1, mine.shape[0]))
    out, _ = table_rows(merged)
    check(bool((O.key_owner(H.host(out)[:, :kb], ws) == rank).all()), "C4 ownership after the exchange")
    allrows = H.host(D.allgather_rows(out))
    if rank == 0:
        a = O.gen_np(0xC4, 2_000, 20_000, 0, ws * N)
        rk, ra, rf = O.groupby(O.pad_keys(a, names), [{"kind": "count"}], valid=O.np_mark(a))
        ref = {bytes(k): (int(c), int(f)) for k, c, f in zip(rk, ra[0], rf)}
        got = {}
        for r in allrows:
            k = bytes(r[:kb])
            check(k not in got, "C4 key owned by two ranks")
            got[k] = (int(r[kb:kb + 8].copy().view(np.uint64)[0]), int(r[kb + 8:kb + 16].copy().view(np.uint64)[0]))
        check(got == ref, "C4 distinct tuples (count, first) after exchange + merge")


def c5(rank, ws):
    G, K = 200_000, 20
    names = ("inode", "dev", "pid", "tid", "op", "count")
    widths = [8, 4, 4, 4]
    cdf = E.zipf_cdf(G, 1.05)
    ev = E.gen_file(0xC5, 0, G, H.to_device(cdf), rank * N, N)   # one global key universe
    aggs = [A.Agg(A.AGG_COUNT, 0, 4, 8, 0), A.Agg(A.AGG_SUM, 5, 4, 8, 0),
            A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 8, 1)]
    tab = E.Table(widths, aggs, G + G // 4)
    tab.update([ev[k] for k in names], [0, 1, 2, 3], N, rank * N)
    rows, fin = table_rows(tab)
    kb = fin["key_bytes"]
    mine = D.exchange_rows(rows, kb)
    own = D.merge_partials(mine, widths, [8, 8, 8, 8], G + G // 4)
    slots = own.sort([(A.TSRC_AGG, 3, True)], K)      # ["-wbytes"] on the owner's groups
    cand = own.gather(slots)
    top = H.host(D.merge_topk(cand, kb, 4, [(3, True)], K))
    if rank == 0:
        a = O.gen_file(0xC5, 0, G, cdf, 0, ws * N)
        op, cnt = a["op"], a["count"]
        ok_, oa, of = O.groupby(O.pad_keys(a, ("inode", "dev", "pid", "tid")),
                                [{"kind": "count", "cond": op, "cond_val": 0},
                                 {"kind": "sum", "val": cnt, "cond": op, "cond_val": 0},
                                 {"kind": "count", "cond": op, "cond_val": 1},
                                 {"kind": "sum", "val": cnt, "cond": op, "cond_val": 1}])
        perm = O.go_sort_entries([(oa[3], "uint64", True)], len(of))[:K].astype(np.int64)
        got_first = top[:, kb + 32:kb + 40].copy().view(np.uint64).ravel()
        got_wb = top[:, kb + 24:kb + 32].copy().view(np.uint64).ravel()
        check(np.array_equal(got_first, of[perm]) and np.array_equal(got_wb, oa[3][perm]),
              "C5 top-20 by -wbytes after exchange + owner merge + all-gather")
        check(np.array_equal(top[:, :kb], ok_[perm]), "C5 top-20 keys")


def c2(rank, ws):
    G, K = 20_000, 20
    cdf = E.zipf_cdf(G, 1.1)
    ev = E.gen_tcp(0xC2, rank, G, H.to_device(cdf), rank * N, N)   # ingest-partitioned universes
    cols = [ev[k] for k in ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family", "size", "dir")]
    tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2], [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)],
                  G + G // 4)
    tab.update(cols, list(range(8)), N, rank * N)
    tab.finalize()
    cand = tab.gather(tab.sort([(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, True)], K))
    top = H.host(D.merge_topk(cand, 72, 2, [(0, True), (1, True)], K))
    if rank == 0:
        evs = [O.gen_tcp(0xC2, r, G, cdf, r * N, N) for r in range(ws)]
        allev = {k: np.concatenate([e[k] for e in evs]) for k in evs[0]}
        _, keys, sent, recv, first = O.top_tcp(allev, K)
        check(np.array_equal(top[:, 88:96].copy().view(np.uint64).ravel(), first), "C2 merged top-20 first")
        check(np.array_equal(top[:, 72:80].copy().view(np.uint64).ravel(), sent), "C2 merged top-20 sent")
        check(np.array_equal(top[:, 80:88].copy().view(np.uint64).ravel(), recv), "C2 merged top-20 recv")


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, ws = dist.get_rank(), dist.get_world_size()
    check(D.comm().name == "torch", "gloo group -> torch transport")
    c3(rank, ws)
    c4(rank, ws)
    c5(rank, ws)
    c2(rank, ws)
    dist.barrier()
    if rank == 0:
        print("DIST_GPU_OK", flush=True)
    D.shutdown()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
