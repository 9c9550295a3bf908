"""world_size-2 worker for tests/test_dist_cpu.py (gloo, CPU tensors).

Runs the torch.distributed transport of inspektor-gadget_amd/dist.py (TorchComm) for C3
(all-reduce), C4 (all-to-all by key owner) and the top-K all-gather.  There is no GPU in
this container, so the per-rank aggregation and the owner-side merges that libigx.so does
are stood in for by the oracle here; tests/test_gpu_dist.py runs the same exchanges with the
product's aggregation, partition and merges on the GPU (two ranks sharing cuda:0).  Rank 0 checks every result against
the oracle run over the union of all ranks' events and exits non-zero on a mismatch.
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

D = importlib.import_module("inspektor-gadget_amd.dist")

N = 60_000


def rows_of(keys_padded, aggs, first):
    """packed group rows: padded key | u64 aggregates | u64 first (igx_groupby_gather)."""
    parts = [keys_padded] + [np.ascontiguousarray(a, np.uint64).view(np.uint8).reshape(-1, 8) for a in aggs]
    parts.append(np.ascontiguousarray(first, np.uint64).view(np.uint8).reshape(-1, 8))
    return np.ascontiguousarray(np.concatenate(parts, axis=1))


def merge_owner(rows, kb, naggs):
    """oracle stand-in for the owner's igx_groupby_update_ex merge: SUM partials, MIN first."""
    acc = {}
    for r in rows:
        k = bytes(r[:kb])
        a = r[kb:kb + 8 * naggs].copy().view(np.uint64)
        f = int(r[kb + 8 * naggs:].copy().view(np.uint64)[0])
        if k in acc:
            s, f0 = acc[k]
            acc[k] = (s + a, min(f0, f))
        else:
            acc[k] = (a.copy(), f)
    return acc


def check(ok, what):
    if not ok:
        print(f"MISMATCH: {what}", flush=True)
        sys.exit(3)


def c3_allreduce(rank, ws):
    q = O.lognormal_quantiles(np.log(2e5), 1.5)
    devs = [(8 << 20) | (16 * k) for k in range(4)]
    ev = O.gen_bio(0xC3, q, rank * N, N)
    h = torch.from_numpy(O.hist_log2(ev["dev"], ev["cont"], ev["delta"], devs, 256).astype(np.uint32).view(np.int32))
    D.allreduce_hist(h)
    if rank == 0:
        allev = O.gen_bio(0xC3, q, 0, ws * N)
        ref = O.hist_log2(allev["dev"], allev["cont"], allev["delta"], devs, 256)
        check(np.array_equal(h.numpy().view(np.uint32), ref), "C3 all-reduce histogram")


def c4_exchange(rank, ws):
    names = ("src", "pkt", "peer", "port")
    ev = O.gen_np(0xC4, 500, 5_000, rank * N, N)
    keep = O.np_mark(ev)
    okeys, oaggs, ofirst = O.groupby(O.pad_keys(ev, names), [{"kind": "count"}], valid=keep,
                                     base_idx=rank * N)
    rows = torch.from_numpy(rows_of(okeys, oaggs, ofirst))
    kb = okeys.shape[1]
    # the device partition (igx_partition_rows) runs in tests/dist_worker_gpu.py; here the
    # oracle's grouping (same owner function) feeds the product's exchange
    part, counts = O.partition_rows(rows.numpy(), kb, ws)
    mine = D.exchange_partitioned(torch.from_numpy(part), counts)
    # every received key is owned by this rank
    check(bool((O.key_owner(mine.numpy()[:, :kb], ws) == rank).all()), "C4 ownership after all-to-all")
    merged = merge_owner(mine.numpy(), kb, 1)
    out = np.array([np.concatenate([np.frombuffer(k, np.uint8), s.view(np.uint8),
                                    np.array([f], np.uint64).view(np.uint8)])
                    for k, (s, f) in merged.items()], dtype=np.uint8).reshape(-1, kb + 16)
    allrows = D.allgather_rows(torch.from_numpy(out)).numpy()
    if rank == 0:
        allev = O.gen_np(0xC4, 500, 5_000, 0, ws * N)
        rk, ra, rf = O.groupby(O.pad_keys(allev, names), [{"kind": "count"}], valid=O.np_mark(allev))
        ref = {bytes(k): (int(a), int(f)) for k, a, f in zip(rk, ra[0], rf)}
        got = {}
        for r in allrows:
            k = bytes(r[:kb])
            check(k not in got, "C4 key owned by two ranks")
            got[k] = (int(r[kb:kb + 8].copy().view(np.uint64)[0]), int(r[kb + 8:].copy().view(np.uint64)[0]))
        check(got == ref, "C4 distinct tuples (count, first) after exchange + merge")


def topk_allgather(rank, ws):
    G, K = 3000, 20
    cdf = O.zipf_cdf(G, 1.1)
    ev = O.gen_tcp(0xC2, rank, G, cdf, rank * N, N)
    Gr, keys, sent, recv, first = O.top_tcp(ev, K, base_idx=rank * N)
    cand = torch.from_numpy(rows_of(keys, [sent, recv], first))
    allc = D.allgather_rows(cand).numpy()
    if rank == 0:
        s = allc[:, 72:80].copy().view(np.uint64).ravel()
        r = allc[:, 80:88].copy().view(np.uint64).ravel()
        f = allc[:, 88:96].copy().view(np.uint64).ravel()
        order = np.argsort(f, kind="stable")     # merge position = global first index
        perm = O.go_sort_entries([(s[order], "uint64", True), (r[order], "uint64", True)], len(f))
        got = f[order][perm.astype(np.int64)][:K]
        evs = [O.gen_tcp(0xC2, rr, G, cdf, rr * N, N) for rr in range(ws)]
        allev = {k: np.concatenate([e[k] for e in evs]) for k in evs[0]}
        _, _, _, _, ref_first = O.top_tcp(allev, K)
        check(np.array_equal(got, ref_first), "top-K all-gather merge")


def main():
    dist.init_process_group("gloo")
    rank, ws = dist.get_rank(), dist.get_world_size()
    c3_allreduce(rank, ws)
    c4_exchange(rank, ws)
    topk_allgather(rank, ws)
    dist.barrier()
    if rank == 0:
        print("DIST_OK", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
