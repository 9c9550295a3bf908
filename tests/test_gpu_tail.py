"""GPU parity of the step tail: the table top-K's device selection (every k regime: the
finish ranks k <= 1024 rows itself, k_sel_rank above; the group count read on the device
after igx_groupby_finalize_async), the slot list of tables past SLOTS_INLINE_TILES tiles
(scan kernel) and below it (in-kernel prefix), and the radix passes on both sides of
SCAN_FREE_TILES.  References: the oracle's Go SliceStable restatement over the canonical
(first-occurrence) order -- SortStats, pkg/columns/sort/sort.go:35-83 -- and numpy.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E(igx):
    return igx.engine


@pytest.fixture(scope="module")
def H(igx):
    return igx.columns


def _go_top(oracle, first, cols, k):
    """first indices of the top k groups: Go SliceStable over the first-occurrence order"""
    order = np.argsort(first, kind="stable")
    perm = oracle.go_sort_entries([(c[order], "uint64", d) for c, d in cols], len(first))
    return first[order][perm.astype(np.int64)][:k]


@pytest.mark.parametrize("sync", [True, False])
def test_table_topk_every_k(oracle, E, H, igx, sync):
    A = igx._abi
    G, n = 8000, 400_000
    ev_h = oracle.gen_tcp(0xC2, 0, G, oracle.zipf_cdf(G, 1.1), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    cols = [ev[k] for k in ("pid", "lport", "family")] + [ev["size"]]
    aggs = [A.Agg(A.AGG_SUM, 3, A.NO_COL, 8, 0), A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)]
    tab = E.Table([4, 2, 2], aggs, 2 * G)
    tab.update(cols, [0, 1, 2], n, 0)
    fin = tab.finalize()
    _, ta, tf = E.table_tensors(tab, fin)
    s, c, f = H.host(ta[0]), H.host(ta[1]), H.host(tf)
    g = fin["n_groups"]
    key_sets = {
        "sum desc, count asc": ([(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, False)], [(s, True), (c, False)]),
        "count desc": ([(A.TSRC_AGG, 1, True)], [(c, True)]),
        "first desc": ([(A.TSRC_FIRST, 0, True)], [(f, True)]),
        "sum asc": ([(A.TSRC_AGG, 0, False)], [(s, False)]),
    }
    row_first = fin["key_bytes"] + 8 * 2   # packed row: key | 2 aggs | first
    for name, (tkeys, okeys) in key_sets.items():
        for k in (1, 20, 300, 1500, 4000):
            if not sync:
                tab.reset()
                tab.update(cols, [0, 1, 2], n, 0)
                assert tab.finalize(sync=False)["n_groups"] is None
            rows = H.host(tab.gather(tab.sort(tkeys, k)))
            if not sync:
                assert tab.wait() == g
            got = rows[:, row_first:row_first + 8].copy().view(np.uint64).ravel()
            want = _go_top(oracle, f, okeys, k)
            assert np.array_equal(got[:len(want)], want), (name, k)
            assert not rows[len(want):].any(), (name, k)
    tab.destroy()


def test_large_table_slot_list(oracle, E, H, igx):
    """a table of more than SLOTS_INLINE_TILES x 8192 slots: the slot list through the scan
    kernel, the read-back from it, top-20 by count -- synchronous and asynchronous"""
    A = igx._abi
    rng = np.random.default_rng(11)
    n, cap = 1_000_000, 30_000_000
    keys = rng.integers(0, 600_000, n, dtype=np.uint32) * np.uint32(2654435761)
    tab = E.Table([4], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], cap)
    kd = H.to_device(keys)
    tab.update([kd], [0], n, 0)
    fin = tab.finalize()
    assert fin["n_slots"] > 4096 * 8192
    uk, first, cnt = np.unique(keys, return_index=True, return_counts=True)
    assert fin["n_groups"] == len(uk)
    tk, _, tf = E.table_tensors(tab, fin)
    assert np.array_equal(np.sort(H.host(tk)[:, :4].copy().view(np.uint32).ravel()), uk)
    want = _go_top(oracle, first.astype(np.uint64), [(cnt.astype(np.uint64), True)], 20)
    for sync in (True, False):
        tab.reset()
        tab.update([kd], [0], n, 0)
        tab.finalize(sync=sync)
        rows = H.host(tab.gather(tab.sort([(A.TSRC_AGG, 0, True)], 20)))
        if not sync:
            assert tab.wait() == len(uk)
        o = fin["key_bytes"] + 8   # packed row: key | count | first
        assert np.array_equal(rows[:, o:o + 8].copy().view(np.uint64).ravel(), want)
    tab.destroy()


@pytest.mark.parametrize("n", [2_000_000, 2_200_000])   # 489 / 538 tiles: scan-free / scan kernels
def test_radix_passes_both_scan_paths(oracle, E, H, n):
    """SortEntries(["b", "-a"]) with ties: b asc, a desc, ties in reverse input order"""
    rng = np.random.default_rng(n)
    a = rng.integers(0, 1 << 20, n, dtype=np.uint32)
    b = rng.integers(0, 64, n, dtype=np.uint32)
    got = H.host(E.sort_perm([(H.to_device(b), False), (H.to_device(a), True)], n)).astype(np.int64)
    want = oracle.go_sort_entries([(b, "uint32", False), (a, "uint32", True)], n).astype(np.int64)
    assert np.array_equal(got, want)


def test_auto_region_overflow_then_exact(E, H, igx):
    """AUTO on a miss-heavy stream with one hot key: cached (measures), then the region
    variant (the hot key's bucket overflows: its extra records merge one by one), then the
    exact variant -- every interval's groups and the hot key's count exact"""
    A = igx._abi
    rng = np.random.default_rng(5)
    n = 4_000_000
    keys = rng.integers(1, 20_000_000, n, dtype=np.uint32)
    keys[rng.random(n) < 0.05] = 0
    uk, first, cnt = np.unique(keys, return_index=True, return_counts=True)
    kd = H.to_device(keys)
    tab = E.Table([4], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], 8_000_000)
    for it in range(4):
        tab.reset()
        tab.update([kd], [0], n, 0)
        fin = tab.finalize()
        assert fin["n_groups"] == len(uk), it
        row = H.host(tab.gather(tab.sort([(A.TSRC_AGG, 0, True)], 1)))[0]
        o = fin["key_bytes"]
        assert row[:4].view(np.uint32)[0] == 0 and row[o:o + 8].view(np.uint64)[0] == cnt[0], it
        assert row[o + 8:o + 16].view(np.uint64)[0] == first[0], it
    tab.destroy()


def test_auto_region_overflow_async_pipeline(E, H, igx):
    """The same stream as test_auto_region_overflow_then_exact, every interval issued without a
    host synchronisation (reset, update, finalize_async, top-1, gather; the count is waited for
    only after the next interval is issued).  The region variant's overflow must still switch
    AUTO to the exact variant within the next two intervals (its read-back is applied with
    its own interval's bookkeeping), and every interval's hot-key row stays exact."""
    A = igx._abi
    rng = np.random.default_rng(5)
    n = 4_000_000
    keys = rng.integers(1, 20_000_000, n, dtype=np.uint32)
    keys[rng.random(n) < 0.05] = 0
    uk, first, cnt = np.unique(keys, return_index=True, return_counts=True)
    kd = H.to_device(keys)
    tab = E.Table([4], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], 8_000_000)
    forms, rows = [], []
    for it in range(7):
        tab.reset()
        tab.update([kd], [0], n, 0)
        forms.append(tab.info())
        fin = tab.finalize(sync=False)
        rows.append(tab.gather(tab.sort([(A.TSRC_AGG, 0, True)], 1)))
    assert tab.wait() == len(uk)
    o = fin["key_bytes"]
    for it, r in enumerate(rows):
        row = H.host(r)[0]
        assert row[:4].view(np.uint32)[0] == 0 and row[o:o + 8].view(np.uint64)[0] == cnt[0], it
        assert row[o + 8:o + 16].view(np.uint64)[0] == first[0], it
    assert forms[0]["form"] == A.GB_CACHED
    region = [i for i, f in enumerate(forms) if f["form"] == A.GB_PART and f["region"]]
    assert region, forms
    r0 = region[0]
    later = forms[r0 + 1:r0 + 4]
    assert any(f["form"] == A.GB_PART and not f["region"] for f in later), forms
    tab.destroy()



def test_auto_reprobe_by_estimate(E, H, igx, oracle):
    """AUTO's re-probe: after a near-uniform stream sends a table to the partitioned form, the
    last interval of each partitioned run replays the LDS cache on a sample (k_gb_estimate)
    instead of running a whole interval cached -- a stream that still misses stays partitioned
    with no cached interval in between; once the stream turns skewed, the probe sends the next
    interval to the cached form.  Every interval's groups and counts exact."""
    A = igx._abi
    rng = np.random.default_rng(9)
    n = 4_000_000
    uni = rng.integers(1, 20_000_000, n, dtype=np.uint32)
    cdf = oracle.zipf_cdf(2000, 1.2)
    skew = (np.searchsorted(cdf, rng.random(n)) + 1).astype(np.uint32)
    tab = E.Table([4], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], 8_000_000)

    def interval(kd, uk, cnt):
        tab.reset()
        tab.update([kd], [0], n, 0)
        f = tab.info()
        fin = tab.finalize()
        assert fin["n_groups"] == len(uk)
        row = H.host(tab.gather(tab.sort([(A.TSRC_AGG, 0, True)], 1)))[0]
        o = fin["key_bytes"]
        assert row[o:o + 8].view(np.uint64)[0] == cnt.max()
        return f

    kd, (uk, cnt) = H.to_device(uni), np.unique(uni, return_counts=True)
    forms = [interval(kd, uk, cnt) for _ in range(40)]
    assert forms[0]["form"] == A.GB_CACHED
    assert all(f["form"] == A.GB_PART for f in forms[1:]), [f["form"] for f in forms]
    kd, (uk, cnt) = H.to_device(skew), np.unique(skew, return_counts=True)
    forms = [interval(kd, uk, cnt) for _ in range(20)]
    cached = [i for i, f in enumerate(forms) if f["form"] == A.GB_CACHED]
    assert cached and cached[0] <= 17, [f["form"] for f in forms]   # within one partitioned run
    assert all(f["form"] == A.GB_CACHED for f in forms[cached[0]:]), [f["form"] for f in forms]
    tab.destroy()
