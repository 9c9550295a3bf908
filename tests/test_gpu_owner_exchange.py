"""The N > 1 step of C4 / C5 without its host round trips (bench.py run_c4 / run_c5):
partial table finalized asynchronously -> igx_partition_groups straight from the table (the
device group count sizes the passes) -> exchange -> owner merge finalized asynchronously ->
device-count top-K.

test_partition_groups_matches_partition_rows: the table-view partition equals
igx_partition_rows over the gathered rows, after a synchronous and an asynchronous finalize,
for the top-file layout (4 aggregates) and the distinct-only network-policy tuple.

test_emulated_rank_of_8_owner_merge: one GPU plays rank 0 of 8.  Eight slices of one global
stream are aggregated into partial tables; each is partitioned by owner and owner 0's rows are
kept (what the all-to-all would deliver, the transfer itself left out); rank 0 merges them into
a table sized from its share (dist.owner_capacity).  The owner table must be exactly the
oracle's group-by of all eight slices restricted to the keys owner 0 owns
(pkg/snapshotcombiner/snapshotcombiner.go:79-106 concatenates nodes; the exact merge here is
stricter), and its top-20 must be the oracle's top-20 of those groups.

test_bench_transport_check_single_rank: bench.transport_check's comparison through a one-rank
"nccl" group (torch's collectives vs the igx_dist_* C ABI; the only RCCL shape a one-GPU box
allows) on the C2 / C3 / C5 exchanges.
"""
import importlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C5_NAMES = ("inode", "dev", "pid", "tid", "op", "count")


def _rows_sorted(rows):
    rows = np.ascontiguousarray(rows)
    return np.sort(rows.view(np.dtype((np.void, rows.shape[1]))).ravel())


def test_partition_groups_matches_partition_rows(igx, torch):
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    cdf = H.to_device(E.zipf_cdf(200_000, 1.05))
    ev = E.gen_file(0xC5, 0, 200_000, cdf, 0, 4_000_000)
    cols = [ev[k] for k in C5_NAMES]
    tab = E.Table(bench.C5_WIDTHS, bench.c5_aggs(A), 250_000)
    for sync in (True, False):
        for ws in (1, 3, 8):
            tab.reset()
            tab.update(cols, [0, 1, 2, 3], 4_000_000, 77)
            tab.finalize(sync=sync)
            prow, cnt = tab.partition(ws)
            counts = cnt.cpu().tolist()
            G = tab.wait()
            assert sum(counts) == G
            ref, rcnt = E.partition_rows(bench.table_rows(E, torch, tab, tab.fin), tab.fin["key_bytes"], ws)
            assert counts == rcnt
            # same rows per owner (table_rows lists slots in ascending order, so does the slot list)
            assert torch.equal(prow[:G], ref)
    ev = E.gen_np(*bench.C4_GEN, 0, 2_000_000)
    cols = [ev[k] for k in bench.C4_NAMES]
    tab4 = E.Table(bench.C4_WIDTHS, [], 2_000_000)
    keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
    tab4.update(cols, [0, 1, 2, 3], 2_000_000, 0, valid=keep)
    tab4.finalize(sync=False)
    prow, cnt = tab4.partition(8)
    counts = cnt.cpu().tolist()
    G = tab4.wait()
    ref, rcnt = E.partition_rows(bench.table_rows(E, torch, tab4, tab4.fin), tab4.fin["key_bytes"], 8)
    assert counts == rcnt and torch.equal(prow[:G], ref)
    tab.destroy()
    tab4.destroy()


def test_emulated_rank_of_8_owner_merge(igx, torch, oracle):
    E, H, A, D = igx.engine, igx.columns, igx._abi, igx.dist
    bench = importlib.import_module("bench")
    WS, n, G, K = 8, 1_500_000, 300_000, 20
    cap = G + G // 4
    cdf_h = E.zipf_cdf(G, 1.05)
    cdf = H.to_device(cdf_h)
    tab = E.Table(bench.C5_WIDTHS, bench.c5_aggs(A), cap)
    recv = []
    for r in range(WS):
        ev = E.gen_file(0xC5, 0, G, cdf, r * n, n)     # rank r's slice of one global stream
        tab.reset()
        tab.update([ev[k] for k in C5_NAMES], [0, 1, 2, 3], n, r * n)
        tab.finalize(sync=False)
        rows, cnt = tab.partition(WS)
        counts = cnt.cpu().tolist()
        recv.append(rows[:counts[0]].clone())           # what rank r sends to owner 0
    mine = torch.cat(recv)
    own_cap = D.owner_capacity(cap, WS)
    assert own_cap < cap // 4
    own = D.merge_partials(mine, bench.C5_WIDTHS, [8, 8, 8, 8], own_cap, sync=False)
    top = H.host(own.gather(own.sort([(A.TSRC_AGG, 3, True)], K)))
    Gown = own.wait()
    rows = H.host(bench.table_rows(E, torch, own, own.fin))
    # the oracle: every slice's events, grouped, restricted to owner 0's keys
    h = oracle.gen_file(0xC5, 0, G, cdf_h, 0, WS * n)
    keys = oracle.pad_keys(h, ("inode", "dev", "pid", "tid"))
    k, aggs, first = oracle.groupby(keys, bench.c5_oracle_aggs(h))
    mask = oracle.key_owner(k, WS) == 0
    k, aggs, first = k[mask], aggs[:, mask], first[mask]
    ref = np.concatenate([k] + [aggs[x].copy().view(np.uint8).reshape(-1, 8) for x in range(4)]
                         + [first.copy().view(np.uint8).reshape(-1, 8)], axis=1)
    assert Gown == rows.shape[0] == ref.shape[0]
    assert np.array_equal(_rows_sorted(rows), _rows_sorted(ref))
    # the owner's top-20 by -wbytes: Go SliceStable with the global first index as the position
    order = np.argsort(first, kind="stable")
    perm = oracle.go_sort_entries([(aggs[3][order], "uint64", True)], len(first))
    sel = order[perm[:K].astype(np.int64)]
    u64 = lambda a, o: a[:, o:o + 8].copy().view(np.uint64).ravel()   # noqa: E731
    assert np.array_equal(u64(top, 52), first[sel]) and np.array_equal(u64(top, 44), aggs[3][sel])
    tab.destroy()
    own.destroy()


def test_bench_transport_check_single_rank(igx, torch):
    import socket
    import torch.distributed as dist
    bench = importlib.import_module("bench")
    if not dist.is_initialized():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        ctx = bench.make_ctx(torch, dist, igx, 0, 2, torch.device("cuda", 0), False)   # world 2: run the check
        ctx["world"] = 2
        D = igx.dist
        rows = torch.randint(0, 256, (1000, 60), dtype=torch.uint8, device="cuda")
        r = bench.transport_check(ctx, "all-gather", lambda c: D.allgather_rows(rows, c).flatten())
        assert r["transport_igx_equal"] is True, r
        hist = torch.randint(0, 1 << 30, (4096, 27), dtype=torch.int32, device="cuda").view(torch.uint32)
        r = bench.transport_check(ctx, "all-reduce",
                                  lambda c: D.allreduce_hist(hist.clone(), c).flatten().view(torch.uint8))
        assert r["transport_igx_equal"] is True, r
        part, counts = igx.engine.partition_rows(rows, 20, 1)
        r = bench.transport_check(ctx, "all-to-all", lambda c: D.exchange_partitioned(part, counts, c).flatten())
        assert r["transport_igx_equal"] is True, r
        # a transport that returns other bytes is a mismatch
        r = bench.transport_check(ctx, "mismatch", lambda c: rows.flatten() if c.name == "torch" else rows.flatten() ^ 1)
        assert r["transport_igx_equal"] is False
        ctx["igx_comm"].close()
    finally:
        dist.destroy_process_group()



@pytest.mark.parametrize("layout", ["c5", "c2", "c4"])
def test_unpack_rows_matches_slicing(igx, torch, layout):
    """dist.unpack_rows (the owner merge's exchanged rows -> the SoA columns the update reads,
    one igx_ingest_aos pass) equals slicing every field out of the rows on the host -- key
    columns padded to 4 bytes, then the u64 aggregates and first index -- for C5's, C2's and C4's
    rows, including zero rows."""
    D = importlib.import_module("inspektor-gadget_amd.dist")
    widths, naggs = {"c5": ([8, 4, 4, 4], 4), "c2": ([16, 16, 8, 4, 16, 2, 2, 2], 2), "c4": ([4, 1, 4, 2], 0)}[layout]
    offs, o = [], 0
    for w in widths:
        offs.append(o)
        o += (w + 3) // 4 * 4
    rb = o + 8 * (naggs + 1)
    rng = np.random.default_rng(rb)
    for n in (0, 1, 1000, 300_001):
        h = rng.integers(0, 256, size=(n, rb), dtype=np.uint8)
        kcols, aggs, first = D.unpack_rows(igx.columns.to_device(h), widths, naggs)
        got = [(t, ko, w) for t, ko, w in zip(kcols, offs, widths)]
        got += [(t, o + 8 * x, 8) for x, t in enumerate(aggs + [first])]
        for t, fo, w in got:
            b = t.view(torch.uint8).cpu().numpy().reshape(n, w)
            assert np.array_equal(b, h[:, fo:fo + w]), (layout, n, fo, w)
