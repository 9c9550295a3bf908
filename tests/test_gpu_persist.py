"""Keys kept across intervals (igx_groupby_reset's generations, k_groupby.hip header): every
interval's table must still be exactly the reference's per-interval map drain
(pkg/gadgets/top/file/tracer/tracer.go:148-220, tcp/tracer/tracer.go:147-226) -- the
interval's own groups, sums and first indices -- while the keys themselves stay in the table.

Streams whose key sets change between intervals (a sliding window over a key universe: keys
appear, recur and disappear), event indices that repeat (the bench's rotating batches) or
grow, an age-out rebuild (the generation's keys plus a full interval's capacity passing 4/5 of
the slots), a failed interval (capacity exceeded), form switches (partitioned and direct
intervals start their own generation) and an unfinalized interval -- each interval against the
oracle's or_groupby of that interval's rows, and the claims each interval reports (keys
inserted, the others found) against a host model of the generation.
"""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAMES = ("inode", "dev", "pid", "tid", "op", "count")
WIDTHS = [8, 4, 4, 4]


def _universe(n):
    """key id -> (inode, dev, pid, tid), distinct per id"""
    i = np.arange(n, dtype=np.uint64)
    return {"inode": i * np.uint64(0x9E3779B1) + np.uint64(12345),
            "dev": (i % np.uint64(7) + np.uint64(8 << 20)).astype(np.uint32),
            "pid": (i // np.uint64(3) + np.uint64(1000)).astype(np.uint32),
            "tid": (i * np.uint64(2654435761) >> np.uint64(7)).astype(np.uint32)}


HOT = 500


def _batch(rng, U, lo, width, n):
    """n events: half over the window of key ids [lo, lo + width) (every key of it appears at
    these sizes), half over HOT fixed ids spread over the universe (Zipf-like), which recur in
    every interval"""
    hot = (np.arange(HOT, dtype=np.int64) * 7919) % len(U["pid"])
    pick = np.minimum((rng.pareto(1.2, n // 2) * 20).astype(np.int64), HOT - 1)
    ids = np.concatenate([lo + rng.integers(0, width, n - n // 2), hot[pick]])
    rng.shuffle(ids)
    h = {k: U[k][ids] for k in ("inode", "dev", "pid", "tid")}
    h["op"] = rng.integers(0, 3, n).astype(np.uint8)
    h["count"] = rng.integers(0, 1 << 20, n).astype(np.uint32)
    return h, np.unique(ids)


def _dev_rows(bench, E, H, torch, tab, fin):
    rows = H.host(bench.table_rows(E, torch, tab, fin))
    return np.sort(rows.view(np.dtype((np.void, rows.shape[1]))).ravel())


def _ref_rows(oracle, bench, h, base):
    keys = oracle.pad_keys(h, ("inode", "dev", "pid", "tid"))
    k, aggs, first = oracle.groupby(keys, bench.c5_oracle_aggs(h), base_idx=base)
    rows = np.concatenate([k] + [aggs[x].copy().view(np.uint8).reshape(-1, 8) for x in range(4)]
                          + [first.copy().view(np.uint8).reshape(-1, 8)], axis=1)
    return np.sort(np.ascontiguousarray(rows).view(np.dtype((np.void, rows.shape[1]))).ravel())


class Run:
    def __init__(self, igx, torch, oracle, cap, mode=None):
        self.E, self.H, self.A = igx.engine, igx.columns, igx._abi
        self.bench = importlib.import_module("bench")
        self.torch, self.oracle = torch, oracle
        self.tab = self.E.Table(WIDTHS, self.bench.c5_aggs(self.A), cap)
        if mode is not None:
            self.tab.set_mode(mode)
        self.gen = set()          # host model of the generation's keys
        self.cap = cap

    def limit(self):
        ns = 1024
        while ns * 4 < 8 * self.cap:
            ns <<= 1
        return ns // 5 * 4 - self.cap

    def interval(self, h, ids, base, fresh=False, finalize=True):
        """one interval; returns (claims reported, claims the model expects)"""
        n = len(h["op"])
        cols = [self.H.to_device(np.ascontiguousarray(h[k])) for k in NAMES]
        self.tab.reset()
        self.tab.update(cols, [0, 1, 2, 3], n, base)
        if not finalize:
            return None
        fin = self.tab.finalize()
        got = _dev_rows(self.bench, self.E, self.H, self.torch, self.tab, fin)
        want = _ref_rows(self.oracle, self.bench, h, base)
        assert got.shape == want.shape and np.array_equal(got, want)
        if fresh or len(self.gen) > self.limit():
            self.gen = set()
        keys = set(ids.tolist())
        expect = len(keys - self.gen)
        self.gen |= keys
        return self.tab.info()["claims"], expect


def test_sliding_key_sets_exact_and_kept(igx, torch, oracle):
    rng = np.random.default_rng(0x6E6)
    U = _universe(200_000)
    r = Run(igx, torch, oracle, 100_000, igx._abi.GB_CACHED)
    claims = []
    for k in range(10):
        h, ids = _batch(rng, U, 6_000 * k, 40_000, 600_000)
        base = 0 if k % 2 else k * 600_000      # repeating and growing event indices
        claims.append(r.interval(h, ids, base, fresh=(k == 0)))
    assert all(g == w for g, w in claims), claims
    # keys were kept: after the first interval only the window's new keys are inserted
    assert all(g < 0.5 * len(r.gen) for g, _ in claims[1:]), claims
    assert r.tab.info()["persist"] == 1
    r.tab.destroy()


def test_age_out_rebuild_and_recovery(igx, torch, oracle):
    """a small table: the generation's keys pass the limit every few intervals and the next
    interval starts an empty table (claims == its groups); a capacity overflow fails its
    interval and the next one is exact again"""
    rng = np.random.default_rng(0xA6E)
    U = _universe(300_000)
    r = Run(igx, torch, oracle, 30_000, igx._abi.GB_CACHED)
    assert r.limit() == 52_428 - 30_000
    rebuilt = 0
    for k in range(12):
        h, ids = _batch(rng, U, 3_000 * k, 12_000, 300_000)
        before = len(r.gen)
        got, want = r.interval(h, ids, k * 300_000, fresh=(k == 0))
        assert got == want, (k, got, want)
        if k and before > r.limit():
            rebuilt += 1
            assert got == len(np.unique(ids))
    assert rebuilt >= 2
    # more distinct keys than the capacity: the interval fails (ENOSPC) ...
    h, ids = _batch(rng, U, 100_000, 35_500, 1_500_000)
    assert len(ids) > 30_000
    cols = [r.H.to_device(np.ascontiguousarray(h[k])) for k in NAMES]
    r.tab.reset()
    r.tab.update(cols, [0, 1, 2, 3], len(h["op"]), 0)
    with pytest.raises(Exception):
        r.tab.finalize()
    # ... and the next interval is exact (a fresh generation: the overflowing keys are too many to keep)
    h, ids = _batch(rng, U, 50_000, 12_000, 300_000)
    got, want = r.interval(h, ids, 7, fresh=True)
    assert got == want == len(ids)
    r.tab.destroy()


def test_form_switches_and_unfinalized_interval(igx, torch, oracle):
    """partitioned and direct intervals start their own generation; a cached interval after
    them keeps their keys; an interval reset without a finalize ends the generation"""
    A = igx._abi
    rng = np.random.default_rng(0xF0F)
    U = _universe(120_000)
    r = Run(igx, torch, oracle, 80_000, A.GB_CACHED)
    plan = [(A.GB_CACHED, True), (A.GB_CACHED, False), (A.GB_PART, True), (A.GB_CACHED, False),
            (A.GB_DIRECT, True), (A.GB_CACHED, False), (A.GB_CACHED, False)]
    for k, (mode, fresh) in enumerate(plan):
        r.tab.set_mode(mode)
        h, ids = _batch(rng, U, 5_000 * k, 30_000, 400_000)
        got, want = r.interval(h, ids, 0 if k % 2 else 1_000_000 * k, fresh=fresh)
        assert got == want, (k, mode, got, want)
    # an update with no finalize, then a reset: the next interval starts a generation
    h, ids = _batch(rng, U, 0, 30_000, 200_000)
    r.interval(h, ids, 0, finalize=False)
    h, ids = _batch(rng, U, 2_000, 30_000, 400_000)
    got, want = r.interval(h, ids, 5, fresh=True)
    assert got == want == len(ids)
    r.tab.destroy()


def test_auto_state_machine_probers_keep_keys(igx, torch, oracle, monkeypatch):
    """the state-machine probers (IGX_GB_PROBER=1) re-stamp kept keys the same way"""
    monkeypatch.setenv("IGX_GB_PROBER", "1")
    rng = np.random.default_rng(0x5A5)
    U = _universe(100_000)
    r = Run(igx, torch, oracle, 60_000, igx._abi.GB_CACHED)
    for k in range(5):
        h, ids = _batch(rng, U, 4_000 * k, 25_000, 500_000)
        got, want = r.interval(h, ids, 0, fresh=(k == 0))
        assert got == want, (k, got, want)
    r.tab.destroy()


def test_top_tcp_rotating_batches(igx, torch, oracle):
    """the bench's C2 shape at 8M events: two consecutive slices of one stream, alternating;
    each interval against or_top_tcp on its own slice (group count, whole-table checksum,
    top-20), and from the third interval on almost nothing is inserted"""
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    N, G = 8_000_000, 200_000
    cdf = E.zipf_cdf(G, 1.1)
    dcdf = H.to_device(cdf)
    evs = [E.gen_tcp(0xC2, 0, G, dcdf, b * N, N) for b in range(2)]
    # capacity 2 G: the generation's keys (both batches' union) plus a full interval's capacity
    # stay within 4/5 of the 2^20 slots
    tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2], [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)], 2 * G)
    preds = [bench.family_in_pred(A, 7), bench.copied_pred(A, 10, 9)]
    refs = []
    for b in range(2):
        h = oracle.gen_tcp(0xC2, 0, G, cdf, b * N, N)
        refs.append(oracle.top_tcp_mt(h, 20, base_idx=b * N, checksum=True))
    claims = []
    for k in range(6):
        b = k % 2
        ev = evs[b]
        cols = [ev[c] for c in bench.TCP_NAMES] + [ev["size"].view(torch.int32)]
        tab.reset()
        tab.update(cols, list(range(8)), N, b * N, preds)
        fin = tab.finalize()
        top = H.host(tab.gather(tab.sort([(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, True)], 20)))
        rows = H.host(bench.table_rows(E, torch, tab, fin))
        u64 = lambda a, o: a[:, o:o + 8].copy().view(np.uint64).ravel()   # noqa: E731
        cs = oracle.tcp_group_checksum(bench.tcp_fields66(rows), u64(rows, 72), u64(rows, 80), u64(rows, 88))
        Gref, sent, recv, first, ref_cs = refs[b]
        assert fin["n_groups"] == Gref == rows.shape[0], k
        assert cs == ref_cs, k
        assert np.array_equal(u64(top, 88), first) and np.array_equal(u64(top, 72), sent), k
        assert np.array_equal(u64(top, 80), recv), k
        claims.append(tab.info()["claims"])
    assert claims[0] == refs[0][0]
    assert all(c < refs[0][0] // 10 for c in claims[2:]), claims
    tab.destroy()


@pytest.mark.parametrize("prober", ["0", "1"])
def test_seeded_cache_exact(igx, torch, oracle, monkeypatch, prober):
    """The sample-seeded LDS cache (IGX_GB_SEED_MIN=1: every interval of these small streams is
    seeded; IGX_GB_SEED_EVERY=4: the seeds are recomputed every 4 intervals, so most adopt seeds counted
    on an earlier interval's rows -- keys that moved out of the window are simply not found).
    A seeded key may see only LDS hits in an interval: its group must still be listed, with its
    sums and first index, and its `ready` is never re-stamped.  Every interval against the
    oracle; the claims model still holds (seeds are never inserted)."""
    monkeypatch.setenv("IGX_GB_SEED_MIN", "1")
    monkeypatch.setenv("IGX_GB_SEED_EVERY", "4")
    monkeypatch.setenv("IGX_GB_PROBER", prober)
    rng = np.random.default_rng(0x5EED + int(prober))
    U = _universe(150_000)
    r = Run(igx, torch, oracle, 100_000, igx._abi.GB_CACHED)
    claims = []
    for k in range(12):
        h, ids = _batch(rng, U, 3_000 * k, 30_000, 800_000)
        claims.append(r.interval(h, ids, 0 if k % 3 else k * 800_000, fresh=(k == 0)))
    assert all(g == w for g, w in claims), claims
    r.tab.destroy()
