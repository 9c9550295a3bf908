"""The planning step of the igx_dist_* row exchanges (igx_dist_plan_alltoallv / _allgather,
csrc/igx_dist.cpp), which decides for every rank alike -- proceed, IGX_ENOSPC or IGX_EINVAL --
and gives the row offsets the RCCL send/recv loops use.  It is a host function of the
all-gathered metadata, so it runs here without a GPU or a communicator:

  * unit cases for 1..8 ranks: uneven and zero counts, a capacity overflow on one rank, an
    argument error on one rank, a size query, ranks that disagree on the query;
  * the exchange it plans, emulated for every rank, equals torch.distributed's gloo
    all_to_all_single / all_gather on the same rows, for world sizes 2, 3 and 8.

Reference merge this replaces: pkg/snapshotcombiner/snapshotcombiner.go:79-106 (per-node
arrays concatenated on the client, fed by pkg/runtime/grpc/grpc-runtime.go:221-237).
"""
import ctypes as C
import importlib
import os
import socket

import numpy as np
import pytest

A = importlib.import_module("inspektor-gadget_amd._abi")


def _meta_a2a(counts, caps, flags):
    """rank rows: send_counts | cap | flags"""
    nr = len(caps)
    m = np.zeros((nr, nr + 2), np.uint64)
    m[:, :nr] = counts
    m[:, nr] = caps
    m[:, nr + 1] = flags
    return np.ascontiguousarray(m)


def _plan_a2a(meta, rank):
    nr = meta.shape[0]
    p = A.DistPlan()
    assert A.lib().igx_dist_plan_alltoallv(nr, rank, meta.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(p)) == 0
    return p


def _plan_ag(meta, rank):
    nr = meta.shape[0]
    p = A.DistPlan()
    assert A.lib().igx_dist_plan_allgather(nr, rank, meta.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(p)) == 0
    return p


def _emulate_a2a(counts, rows_of):
    """rows each rank receives, by the plans: from src q, q's rows [send_off_q[r], +counts[q][r])
    at recv_off_r[q]"""
    nr = counts.shape[0]
    meta = _meta_a2a(counts, [1 << 40] * nr, [0] * nr)
    plans = [_plan_a2a(meta, r) for r in range(nr)]
    out = []
    for r in range(nr):
        p = plans[r]
        assert p.status == 0 and p.culprit == -1
        buf = np.full((p.total_rows, rows_of(0).shape[1]), -1, np.int64)
        for q in range(nr):
            c = int(counts[q][r])
            assert p.recv_counts[q] == c
            so = plans[q].send_off[r]
            buf[p.recv_off[q]:p.recv_off[q] + c] = rows_of(q)[so:so + c]
        out.append(buf)
    return out


def _send_rows(counts, q):
    """rank q's send buffer: rows grouped by destination, each row (src, dst, i)"""
    parts = [np.stack([np.full(c, q), np.full(c, d), np.arange(c)], axis=1) for d, c in enumerate(counts[q])]
    return np.concatenate(parts).astype(np.int64) if parts else np.zeros((0, 3), np.int64)


@pytest.mark.parametrize("nr", [1, 2, 3, 5, 8])
def test_alltoallv_plan_offsets(nr):
    rng = np.random.default_rng(nr)
    counts = rng.integers(0, 50, size=(nr, nr)).astype(np.uint64)
    counts[rng.random((nr, nr)) < 0.3] = 0            # zero counts, some whole rows / columns
    if nr > 2:
        counts[1, :] = 0
        counts[:, 2] = 0
    recv = _emulate_a2a(counts, lambda q: _send_rows(counts, q))
    for r in range(nr):
        want = np.concatenate([_send_rows(counts, q)[_send_rows(counts, q)[:, 1] == r] for q in range(nr)])
        assert np.array_equal(recv[r], want.reshape(-1, 3))


@pytest.mark.parametrize("nr", [2, 4, 8])
def test_alltoallv_plan_decisions(nr):
    rng = np.random.default_rng(100 + nr)
    counts = rng.integers(0, 20, size=(nr, nr)).astype(np.uint64)
    need = counts.sum(axis=0)
    caps = need.copy()
    # exact capacities: everyone proceeds
    for r in range(nr):
        p = _plan_a2a(_meta_a2a(counts, caps, [0] * nr), r)
        assert (p.status, p.culprit, p.total_rows) == (0, -1, int(need[r]))
    # one rank one row short: every rank returns ENOSPC naming it
    bad = nr - 1
    caps2 = caps.copy()
    caps2[bad] = need[bad] - 1 if need[bad] else 0
    if need[bad] == 0:
        counts[0, bad] = 1
    for r in range(nr):
        p = _plan_a2a(_meta_a2a(counts, caps2, [0] * nr), r)
        assert (p.status, p.culprit) == (A.IGX_ENOSPC, bad)
    # an argument error on one rank beats a capacity error on another, on every rank
    fl = [0] * nr
    fl[1] = A.DIST_F_BADARG
    for r in range(nr):
        p = _plan_a2a(_meta_a2a(counts, caps2, fl), r)
        assert (p.status, p.culprit) == (A.IGX_EINVAL, 1)
    # a size query on every rank proceeds whatever the capacities, with the counts
    for r in range(nr):
        p = _plan_a2a(_meta_a2a(counts, [0] * nr, [A.DIST_F_QUERY] * nr), r)
        assert p.status == 0 and [p.recv_counts[q] for q in range(nr)] == [int(counts[q][r]) for q in range(nr)]
    # ranks that disagree on query vs data: every rank fails
    fl = [A.DIST_F_QUERY] * nr
    fl[nr // 2] = 0
    culprits = {_plan_a2a(_meta_a2a(counts, caps, fl), r).culprit for r in range(nr)}
    statuses = {_plan_a2a(_meta_a2a(counts, caps, fl), r).status for r in range(nr)}
    assert statuses == {A.IGX_EINVAL} and len(culprits) == 1


@pytest.mark.parametrize("nr", [1, 3, 8])
def test_allgather_plan(nr):
    rng = np.random.default_rng(7 + nr)
    n = rng.integers(0, 30, size=nr).astype(np.uint64)
    n[0] = 0
    tot = int(n.sum())
    meta = np.ascontiguousarray(np.stack([n, np.full(nr, tot, np.uint64), np.zeros(nr, np.uint64)], axis=1))
    for r in range(nr):
        p = _plan_ag(meta, r)
        assert (p.status, p.total_rows) == (0, tot)
        assert [p.recv_off[q] for q in range(nr)] == np.concatenate([[0], np.cumsum(n)[:-1]]).tolist()
    meta[nr - 1, 1] = tot - 1 if tot else 0
    if tot == 0:
        meta[0, 0] = 1
    for r in range(nr):
        assert (_plan_ag(meta, r).status, _plan_ag(meta, r).culprit) == (A.IGX_ENOSPC, nr - 1)
    meta[0, 2] = A.DIST_F_BADARG
    assert _plan_ag(meta, nr - 1).status == A.IGX_EINVAL


def test_plan_rejects_bad_shapes():
    m = np.zeros((2, 4), np.uint64)
    p = A.DistPlan()
    ptr = m.ctypes.data_as(C.POINTER(C.c_uint64))
    assert A.lib().igx_dist_plan_alltoallv(0, 0, ptr, C.byref(p)) == A.IGX_EINVAL
    assert A.lib().igx_dist_plan_alltoallv(2, 2, ptr, C.byref(p)) == A.IGX_EINVAL
    assert A.lib().igx_dist_plan_alltoallv(65, 0, ptr, C.byref(p)) == A.IGX_EINVAL
    assert A.lib().igx_dist_plan_allgather(2, -1, ptr, C.byref(p)) == A.IGX_EINVAL


# ---- the same exchanges through gloo, world sizes 2 / 3 / 8 ---------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _counts(nr, seed):
    rng = np.random.default_rng(seed)
    c = rng.integers(0, 40, size=(nr, nr)).astype(np.uint64)
    c[rng.random((nr, nr)) < 0.25] = 0
    return c


def _worker(rank, nr, port, seed, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=nr)
    try:
        counts = _counts(nr, seed)
        send = torch.from_numpy(_send_rows(counts, rank))
        rc = [int(counts[s][rank]) for s in range(nr)]
        out = torch.empty((sum(rc), 3), dtype=torch.int64)
        dist.all_to_all_single(out, send, rc, [int(x) for x in counts[rank]])
        mine = torch.from_numpy(_send_rows(counts, rank)[: int(counts[rank].sum()) // 2])
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(nr)]
        dist.all_gather(sizes, torch.tensor([mine.shape[0]]))
        m = max(int(s) for s in sizes)
        pad = torch.zeros((max(1, m), 3), dtype=torch.int64)
        pad[: mine.shape[0]] = mine
        outs = [torch.empty_like(pad) for _ in range(nr)]
        dist.all_gather(outs, pad)
        ag = torch.cat([o[: int(s)] for o, s in zip(outs, sizes)])
        q.put((rank, out.numpy(), ag.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nr", [2, 3, 8])
def test_plan_matches_gloo_exchanges(nr):
    import torch.multiprocessing as mp
    seed = 1000 + nr
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, nr, port, seed, q)) for r in range(nr)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(nr):
        r, a2a, ag = q.get(timeout=300)
        got[r] = (a2a, ag)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    counts = _counts(nr, seed)
    plan_a2a = _emulate_a2a(counts, lambda s: _send_rows(counts, s))
    # all-gather of each rank's first half of its send rows, by the allgather plan
    halves = [_send_rows(counts, s)[: int(counts[s].sum()) // 2] for s in range(nr)]
    meta = np.ascontiguousarray(np.stack([np.array([h.shape[0] for h in halves], np.uint64),
                                          np.full(nr, 1 << 40, np.uint64), np.zeros(nr, np.uint64)], axis=1))
    for r in range(nr):
        assert np.array_equal(plan_a2a[r], got[r][0].reshape(-1, 3)), r
        p = _plan_ag(meta, r)
        buf = np.zeros((p.total_rows, 3), np.int64)
        for s in range(nr):
            buf[p.recv_off[s]:p.recv_off[s] + p.recv_counts[s]] = halves[s]
        assert np.array_equal(buf, got[r][1].reshape(-1, 3)), r
