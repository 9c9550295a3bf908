"""GPU parity of the keyed aggregation (igx_groupby_*) across key layouts, aggregate kinds,
fused predicates, chunked updates and overflow -- against oracle.groupby (igx_oracle.c §4).

Shapes follow the reference's BPF keys: ip_key_t (tcptop.h:8-17), file_id (filetop.h:13-18),
the advise network-policy tuple, single-column keys, plus layouts with
no compile-time kernel (generic path).  Bit-exact: keys, every aggregate, first index.
"""
import ctypes as C
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as T
    return T


@pytest.fixture(scope="module")
def E(igx):
    return igx.engine


@pytest.fixture(scope="module")
def H(igx):
    return igx.columns


def _unpad(keys, widths):
    """device packed key (each column padded to 4 B) -> unpadded concatenation."""
    parts, o = [], 0
    for w in widths:
        parts.append(keys[:, o:o + w])
        o += (w + 3) // 4 * 4
    return np.concatenate(parts, axis=1)


def _pred(A, col, cmp, value, dtype, negate=False):
    b = np.array([value], dtype=dtype).view(np.uint8)
    ref = (C.c_uint8 * A.MAX_REF)(*b.tolist())
    return A.Pred(col, cmp, int(negate), len(b), ref)


def _check(E, H, tab, widths, okeys, oaggs, ofirst):
    fin = tab.finalize()
    keys, aggs, first = E.table_tensors(tab, fin)
    gk = _unpad(H.host(keys), widths)
    distinct = len({bytes(k) for k in gk})
    assert distinct == len(gk), f"{len(gk) - distinct} duplicate groups"
    assert fin["n_groups"] == len(okeys)
    ga = [H.host(a) for a in aggs]
    gf = H.host(first)
    ref = {bytes(k): tuple(int(a[i]) for a in oaggs) + (int(ofirst[i]),) for i, k in enumerate(okeys)}
    got = {bytes(k): tuple(int(a[i]) for a in ga) + (int(gf[i]),) for i, k in enumerate(gk)}
    assert got == ref


def test_top_file_layout(oracle, E, H, igx, torch):
    """top file: key (inode, dev, pid, tid); reads/rbytes/writes/wbytes by op; wbytes wraps u32."""
    A = igx._abi
    G, n = 30_000, 600_000
    ev_h = oracle.gen_file(0xC5, 0, G, oracle.zipf_cdf(G, 1.05), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    names = ("inode", "dev", "pid", "tid", "op", "count")
    widths = [8, 4, 4, 4]
    aggs = [A.Agg(A.AGG_COUNT, 0, 4, 8, 0), A.Agg(A.AGG_SUM, 5, 4, 8, 0),
            A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 4, 1)]
    tab = E.Table(widths, aggs, 2 * G)
    tab.update([ev[k] for k in names], [0, 1, 2, 3], n, 77)
    o = oracle.groupby(oracle.pack_cols(ev_h, names[:4]),
                       [{"kind": "count", "cond": ev_h["op"], "cond_val": 0},
                        {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 0},
                        {"kind": "count", "cond": ev_h["op"], "cond_val": 1},
                        {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 1,
                         "out_width": 4}], base_idx=77)
    _check(E, H, tab, widths, *o)
    tab.destroy()


def test_netpolicy_dedup_layout(oracle, E, H, igx, torch):
    """advise network-policy: distinct (src, pkt type, peer, port) with counts."""
    A = igx._abi
    n = 500_000
    ev_h = oracle.gen_np(0xC4, 5_000, 50_000, 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    names = ("src", "pkt", "peer", "port")
    widths = [4, 1, 4, 2]
    tab = E.Table(widths, [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], n)
    tab.update([ev[k] for k in names], [0, 1, 2, 3], n, 0)
    o = oracle.groupby(oracle.pack_cols(ev_h, names), [{"kind": "count"}])
    _check(E, H, tab, widths, *o)
    tab.destroy()


@pytest.mark.parametrize("col", ["family", "pid", "mntns", "saddr", "dir"])
def test_single_key_layouts(oracle, E, H, igx, torch, col):
    A = igx._abi
    G, n = 3000, 300_000
    ev_h = oracle.gen_tcp(0xC2, 1, G, oracle.zipf_cdf(G, 1.1), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    w = ev_h[col].dtype.itemsize * (ev_h[col].shape[1] if ev_h[col].ndim == 2 else 1)
    tab = E.Table([w], [A.Agg(A.AGG_SUM, 1, A.NO_COL, 8, 0), A.Agg(A.AGG_COUNT, 0, A.NO_COL, 2, 0)], n)
    tab.update([ev[col], ev["size"]], [0], n, 5)
    o = oracle.groupby(oracle.pack_cols(ev_h, (col,)),
                       [{"kind": "sum", "val": ev_h["size"]}, {"kind": "count", "out_width": 2}], base_idx=5)
    _check(E, H, tab, [w], *o)
    tab.destroy()


@pytest.mark.parametrize("names,forced", [(("pid", "lport", "dir"), False),     # 3 words -> generic 4
                                          (("comm", "mntns"), False),           # 6 words
                                          (("daddr", "saddr", "comm", "pid"), False),  # 13 -> 18
                                          (("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport",
                                            "family"), True)])                   # tcp key, generic kernel
def test_generic_layouts(oracle, E, H, igx, torch, monkeypatch, names, forced):
    A = igx._abi
    if forced:
        monkeypatch.setenv("IGX_GB_GENERIC", "1")
    G, n = 20_000, 400_000
    ev_h = oracle.gen_tcp(0xC2, 2, G, oracle.zipf_cdf(G, 1.1), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    widths = [ev_h[k].dtype.itemsize * (ev_h[k].shape[1] if ev_h[k].ndim == 2 else 1) for k in names]
    cols = [ev[k] for k in names] + [ev["size"], ev["dir"]]
    ni = len(names)
    aggs = [A.Agg(A.AGG_SUM, ni, ni + 1, 8, 0), A.Agg(A.AGG_SUM, ni, ni + 1, 8, 1)]
    tab = E.Table(widths, aggs, 2 * G)
    tab.update(cols, list(range(ni)), n, 0)
    o = oracle.groupby(oracle.pack_cols(ev_h, names),
                       [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
                        {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1}])
    _check(E, H, tab, widths, *o)
    tab.destroy()


def test_fused_predicates_signed_and_chunks(oracle, E, H, igx, torch):
    """Two fused predicates (err == 0, NOT pid < 1000), a signed int64 SUM and a signed
    int32 SUM widened to 8 bytes, fed in three chunks with running base_idx."""
    A = igx._abi
    n = 600_000
    ev_h = oracle.gen_open(0xC1, oracle.zipf_cdf(64, 1.0), 0, n)
    ev_h["ret32"] = ev_h["ret"].astype(np.int32)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    names = ("comm", "ret", "ret32", "err", "pid")
    widths = [16]
    aggs = [A.Agg(A.AGG_SUM, 1, A.NO_COL, 8, 0), A.Agg(A.AGG_SUM, 2, A.NO_COL, 8, 0),
            A.Agg(A.AGG_COUNT, 0, A.NO_COL, 4, 0)]
    preds = [_pred(A, 3, A.CMP_EQ, 0, np.int64), _pred(A, 4, A.CMP_LT, 1000, np.uint32, negate=True)]
    tab = E.Table(widths, aggs, 1024)
    cuts = [0, 123_457, 400_000, n]
    for a, b in zip(cuts[:-1], cuts[1:]):
        tab.update([ev[k][a:b] for k in names], [0], b - a, a, preds=preds)
    keep = (ev_h["err"] == 0) & (ev_h["pid"] >= 1000)
    o = oracle.groupby(ev_h["comm"], [{"kind": "sum", "val": ev_h["ret"]},
                                      {"kind": "sum", "val": ev_h["ret32"]},
                                      {"kind": "count", "out_width": 4}], valid=keep)
    _check(E, H, tab, widths, *o)
    # reset = the per-interval Delete loop: the table is empty again and reusable
    tab.reset()
    assert tab.finalize()["n_groups"] == 0
    tab.update([ev[k] for k in names], [0], n, 0, preds=preds)
    _check(E, H, tab, widths, *o)
    tab.destroy()


def test_intervals_and_epoch_wrap(oracle, E, H, igx, torch):
    """Reset = a new epoch (records of older epochs read as empty, claimers re-initialise
    their value records).  Two streams with overlapping key sets alternate across the
    65535-epoch wrap, where reset falls back to a full clear."""
    A = igx._abi
    n = 300_000
    evs = []
    for seed, G in ((0xA1, 3000), (0xB2, 6000)):
        ev_h = oracle.gen_tcp(seed, 0, G, oracle.zipf_cdf(G, 1.0), 0, n)
        o = oracle.groupby(oracle.pack_cols(ev_h, ("pid",)), [{"kind": "count"}, {"kind": "sum", "val": ev_h["size"]}])
        evs.append(({k: H.to_device(ev_h[k]) for k in ("pid", "size")}, o))
    aggs = [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0), A.Agg(A.AGG_SUM, 1, A.NO_COL, 8, 0)]
    tab = E.Table([4], aggs, 8192)

    def interval(which):
        ev, o = evs[which]
        tab.update([ev["pid"], ev["size"]], [0], n, 0)
        _check(E, H, tab, [4], *o)

    interval(0)                       # epoch 1
    tab.reset()
    interval(1)                       # epoch 2
    for _ in range(65532):
        tab.reset()
    assert tab.finalize()["n_groups"] == 0
    tab.reset()
    interval(0)                       # epoch 65535
    tab.reset()
    interval(1)                       # wrapped: full clear, epoch 1
    tab.reset()
    interval(0)                       # epoch 2
    tab.destroy()


def test_occupancy_across_finalize_reset_and_forms(oracle, E, H, igx, torch):
    """The cached form marks its claims in the occupancy byte map, which finalize folds into
    the bitmap (and clears) and reset clears when no finalize did: a reset with no finalize
    drops the interval's groups; updates after a finalize add to them; an interval of the
    cached form then one of the partitioned and one of the direct form list exactly their
    own groups."""
    A = igx._abi
    n = 200_000
    evs = []
    for seed, G in ((0xA7, 20_000), (0xB8, 30_000)):
        ev_h = oracle.gen_tcp(seed, 0, G, oracle.zipf_cdf(G, 0.8), 0, n)
        evs.append((ev_h, {k: H.to_device(ev_h[k]) for k in ("pid", "size")}))
    aggs = [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0), A.Agg(A.AGG_SUM, 1, A.NO_COL, 8, 0)]

    def want(*which):
        pid = np.concatenate([evs[w][0]["pid"] for w in which])
        size = np.concatenate([evs[w][0]["size"] for w in which])
        return oracle.groupby(oracle.pack_cols({"pid": pid}, ("pid",)), [{"kind": "count"}, {"kind": "sum", "val": size}])

    def feed(w, base):
        ev = evs[w][1]
        tab.update([ev["pid"], ev["size"]], [0], n, base)

    tab = E.Table([4], aggs, 65536)
    tab.set_mode(A.GB_CACHED)
    feed(0, 0)
    tab.reset()                        # no finalize: the byte map is cleared here
    feed(1, 0)
    _check(E, H, tab, [4], *want(1))
    feed(0, n)                         # same interval, after a finalize
    _check(E, H, tab, [4], *want(1, 0))
    for mode in (A.GB_CACHED, A.GB_PART, A.GB_DIRECT, A.GB_CACHED):
        tab.reset()
        tab.set_mode(mode)
        feed(0, 0)
        _check(E, H, tab, [4], *want(0))
    tab.destroy()


def test_capacity_overflow_is_reported(oracle, E, H, igx, torch):
    A = igx._abi
    G, n = 5000, 200_000
    ev_h = oracle.gen_tcp(0xC2, 0, G, oracle.zipf_cdf(G, 0.5), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    for cap in (1000, 300):   # over capacity but within slots; and slots exhausted
        tab = E.Table([4], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], cap)
        tab.update([ev["pid"]], [0], n, 0)
        with pytest.raises(A.IgxError) as ei:
            tab.finalize()
        assert ei.value.code == A.IGX_ENOSPC
        tab.destroy()


def test_table_sort_and_gather(oracle, E, H, igx, torch):
    """igx_groupby_sort over the record layout == Go SortStats on first-occurrence order,
    for agg / key / first sources, mixed directions and a wrapped (u16) aggregate."""
    A = igx._abi
    G, n = 8000, 400_000
    ev_h = oracle.gen_tcp(0xC2, 0, G, oracle.zipf_cdf(G, 1.1), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    names = ("pid", "lport", "family")
    widths = [4, 2, 2]
    aggs = [A.Agg(A.AGG_SUM, 3, A.NO_COL, 2, 0), A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)]
    tab = E.Table(widths, aggs, 2 * G)
    tab.update([ev[k] for k in names] + [ev["size"]], [0, 1, 2], n, 0)
    fin = tab.finalize()
    Gn = fin["n_groups"]
    okeys, oaggs, ofirst = oracle.groupby(oracle.pack_cols(ev_h, names),
                                          [{"kind": "sum", "val": ev_h["size"], "out_width": 2},
                                           {"kind": "count"}])
    assert Gn == len(okeys)
    okeys = okeys.copy()
    lport = okeys[:, 4:6].copy().view(np.uint16).ravel()
    pid = okeys[:, 0:4].copy().view(np.uint32).ravel()
    cases = [
        ([(A.TSRC_AGG, 0, True)], [(oaggs[0].astype(np.uint16), "uint16", True)]),
        ([(A.TSRC_AGG, 1, False), (A.TSRC_KEY, (4, 2, A.KIND_UINT), True)],
         [(oaggs[1], "uint64", False), (lport, "uint16", True)]),
        ([(A.TSRC_KEY, (0, 4, A.KIND_UINT), True), (A.TSRC_AGG, 0, True)],
         [(pid, "uint32", True), (oaggs[0].astype(np.uint16), "uint16", True)]),
        ([(A.TSRC_FIRST, 0, True)], [(ofirst, "uint64", True)]),
    ]
    for tkeys, okeys_sort in cases:
        for k in (0, 25):
            slots = tab.sort(tkeys, k)
            rows = H.host(tab.gather(slots))
            got_first = rows[:, -8:].copy().view(np.uint64).ravel()
            perm = oracle.go_sort_entries(okeys_sort, Gn)   # oracle groups are in first order
            want = ofirst[perm.astype(np.int64)]
            if k:
                want = want[:k]
            assert np.array_equal(got_first, want), tkeys
            # wrapped aggregate as gathered
            g16 = rows[:, 12:20].copy().view(np.uint64).ravel()   # key_bytes = 12 (4+4+4 padded)
            assert int(g16.max()) < (1 << 16)
    tab.destroy()


def test_async_finalize_device_count_topk(oracle, E, H, igx, torch):
    """igx_groupby_finalize_async: no host round trip in the interval; the top-K (integer
    keys) reads the group count on the device and equals the synchronous path's, over several
    intervals; fewer groups than k leave 0xFFFFFFFF slots (zero rows from gather); the count
    and a capacity overflow come back from igx_groupby_wait."""
    A = igx._abi
    G, n = 8000, 400_000
    ev_h = oracle.gen_tcp(0xC2, 0, G, oracle.zipf_cdf(G, 1.1), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    names = ("pid", "lport", "family")
    aggs = [A.Agg(A.AGG_SUM, 3, A.NO_COL, 8, 0), A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)]
    cols = [ev[k] for k in names] + [ev["size"]]
    tab = E.Table([4, 2, 2], aggs, 2 * G)
    keys = [(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, False)]
    want = []
    for it in range(3):   # the synchronous path, three intervals of growing size
        tab.reset()
        m = n // (3 - it)
        tab.update(cols, [0, 1, 2], m, 0)
        g = tab.finalize()["n_groups"]
        want.append((g, H.host(tab.gather(tab.sort(keys, 20)))))
    for it in range(3):
        tab.reset()
        m = n // (3 - it)
        tab.update(cols, [0, 1, 2], m, 0)
        fin = tab.finalize(sync=False)
        assert fin["n_groups"] is None
        got = H.host(tab.gather(tab.sort(keys, 20)))
        assert tab.wait() == want[it][0]
        assert np.array_equal(got, want[it][1])
    # fewer groups than k
    tab.reset()
    tab.update([c[:12] for c in cols], [0, 1, 2], 12, 0)
    tab.finalize()
    g_few = tab.fin["n_groups"]
    ref = H.host(tab.gather(tab.sort(keys, 20)))
    tab.reset()
    tab.update([c[:12] for c in cols], [0, 1, 2], 12, 0)
    tab.finalize(sync=False)
    slots = tab.sort(keys, 20)
    rows = H.host(tab.gather(slots))
    assert tab.wait() == g_few < 20
    assert np.array_equal(rows[:g_few], ref[:g_few])
    assert (H.host(slots)[g_few:].view(np.uint32) == 0xFFFFFFFF).all() and not rows[g_few:].any()
    tab.destroy()
    # capacity overflow: reported by wait(), not by finalize(sync=False)
    small = E.Table([4], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], 1000)
    small.update([ev["pid"]], [0], n, 0)
    small.finalize(sync=False)
    with pytest.raises(A.IgxError) as ei:
        small.wait()
    assert ei.value.code == A.IGX_ENOSPC
    # an overflowing interval followed by a clean one with no wait in between: the overflow is
    # reported once -- by the reset that collects it, or else by the next finalize_async, which
    # then does not issue its own interval (a second call does) -- and wait() reports the clean
    # interval's own status and count
    few = int(np.unique(ev_h["pid"][:2000]).size)
    assert few < 1000
    for _ in range(3):
        small.reset()
        small.update([ev["pid"]], [0], n, 0)                  # overflows
        small.finalize(sync=False)
        raised = 0
        try:
            small.reset()
        except A.IgxError as e:
            assert e.code == A.IGX_ENOSPC
            raised += 1
        small.update([ev["pid"][:2000]], [0], 2000, 0)
        try:
            small.finalize(sync=False)
        except A.IgxError as e:
            assert e.code == A.IGX_ENOSPC and "previous interval" in str(e) and "not finalized" in str(e)
            raised += 1
            small.finalize(sync=False)                       # now this interval is issued
        assert raised == 1
        assert small.wait() == few
    small.destroy()


def test_netpolicy_mark_and_masked_distinct(oracle, E, H, igx, torch):
    """igx_np_mark (advisor.go:279-292) + distinct over the kept rows (valid mask)."""
    A = igx._abi
    n = 400_003                      # ragged tail for the 4-rows-per-thread mark kernel
    ev_h = oracle.gen_np(0xC4, 3_000, 30_000, 17, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
    ref_keep = oracle.np_mark(ev_h)
    assert np.array_equal(H.host(keep).astype(bool), ref_keep)
    # columns at an offset (u8 columns 4-B but not 16-B aligned)
    keep4 = E.np_mark(ev["type"][4:], ev["pkt"][4:], ev["hostip"][4:], ev["raddr"][4:])
    assert np.array_equal(H.host(keep4).astype(bool), ref_keep[4:])
    for m in (1, 3, 4, 5, 7, 1027):   # fewer rows than one quad, and a few quads with a tail
        km = E.np_mark(ev["type"][:m], ev["pkt"][:m], ev["hostip"][:m], ev["raddr"][:m])
        assert np.array_equal(H.host(km).astype(bool), ref_keep[:m]), m
    names = ("src", "pkt", "peer", "port")
    tab = E.Table([4, 1, 4, 2], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], n)
    tab.update([ev[k] for k in names], [0, 1, 2, 3], n, 17, valid=keep)
    o = oracle.groupby(oracle.pack_cols(ev_h, names), [{"kind": "count"}], valid=ref_keep, base_idx=17)
    _check(E, H, tab, [4, 1, 4, 2], *o)
    tab.destroy()


def test_merge_partials_on_device(oracle, E, H, igx, torch):
    """Owner-side merge of partial groups (igx_groupby_update_ex with an index column): three
    shards aggregated separately, their gathered rows merged == one aggregation of all."""
    A = igx._abi
    D = igx.dist
    n, G = 300_000, 5_000
    ev_h = oracle.gen_file(0xC5, 0, G, oracle.zipf_cdf(G, 1.05), 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    names = ("inode", "dev", "pid", "tid", "op", "count")
    widths = [8, 4, 4, 4]
    aggs = [A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 4, 1)]
    rows = []
    cuts = [0, 70_001, 190_000, n]
    for a, b in zip(cuts[:-1], cuts[1:]):
        t = E.Table(widths, aggs, 2 * G)
        t.update([ev[k][a:b] for k in names], [0, 1, 2, 3], b - a, a)
        fin = t.finalize()
        slots = t.sort([(A.TSRC_FIRST, 0, False)], 0)
        rows.append(t.gather(slots))
        t.destroy()
    allrows = torch.cat(rows)
    tab = D.merge_partials(allrows, widths, [8, 4], 2 * G)
    o = oracle.groupby(oracle.pack_cols(ev_h, names[:4]),
                       [{"kind": "count", "cond": ev_h["op"], "cond_val": 1},
                        {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 1,
                         "out_width": 4}])
    _check(E, H, tab, widths, *o)
    # the merged table's top-K equals the single-pass one (wbytes DESC)
    slots = tab.sort([(A.TSRC_AGG, 1, True)], 20)
    got_first = H.host(tab.gather(slots))[:, -8:].copy().view(np.uint64).ravel()
    perm = oracle.go_sort_entries([(o[1][1].astype(np.uint32), "uint32", True)], len(o[0]))
    assert np.array_equal(got_first, o[2][perm.astype(np.int64)][:20])
    tab.destroy()


@pytest.mark.parametrize("prober", ["batch", "state-machine", "adaptive"])
@pytest.mark.parametrize("layout", ["tcp", "file", "netpolicy"])
def test_both_prober_forms(oracle, E, H, igx, torch, prober, layout, monkeypatch):
    """Both forms of the miss-resolving waves (batch / state-machine) give the same exact
    table; 'adaptive' lets a miss-heavy first interval switch the table to the
    state-machine form for the second (the kernel's LDS-miss count, read at finalize)."""
    import os
    A = igx._abi
    if prober != "adaptive":
        monkeypatch.setenv("IGX_GB_PROBER", "1" if prober == "state-machine" else "0")
    else:
        monkeypatch.delenv("IGX_GB_PROBER", raising=False)
    n = 1_200_000
    if layout == "tcp":
        G = 200_000                                       # near-uniform: most rows miss LDS
        ev_h = oracle.gen_tcp(0xB7, 0, G, oracle.zipf_cdf(G, 0.2), 0, n)
        names, widths = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family"), \
            [16, 16, 8, 4, 16, 2, 2, 2]
        aggs = [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)]
        extra = ["size", "dir"]
        oaggs = [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
                 {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1}]
    elif layout == "file":
        G = 300_000
        ev_h = oracle.gen_file(0xC5, 0, G, oracle.zipf_cdf(G, 0.3), 0, n)
        names, widths = ("inode", "dev", "pid", "tid"), [8, 4, 4, 4]
        aggs = [A.Agg(A.AGG_COUNT, 0, 5, 8, 0), A.Agg(A.AGG_SUM, 4, 5, 8, 0),
                A.Agg(A.AGG_COUNT, 0, 5, 8, 1), A.Agg(A.AGG_SUM, 4, 5, 4, 1)]
        extra = ["count", "op"]
        oaggs = [{"kind": "count", "cond": ev_h["op"], "cond_val": 0},
                 {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 0},
                 {"kind": "count", "cond": ev_h["op"], "cond_val": 1},
                 {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 1, "out_width": 4}]
    else:
        ev_h = oracle.gen_np(0xC4, 5_000, 50_000, 0, n)
        names, widths = ("src", "pkt", "peer", "port"), [4, 1, 4, 2]
        aggs = [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)]
        extra = []
        oaggs = [{"kind": "count"}]
        G = n
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    cols = [ev[k] for k in list(names) + extra]
    tab = E.Table(widths, aggs, min(2 * G, n))
    o = oracle.groupby(oracle.pack_cols(ev_h, names), oaggs)
    for _ in range(2):                                   # two intervals
        tab.update(cols, list(range(len(names))), n, 0)
        _check(E, H, tab, widths, *o)
        tab.reset()
    tab.destroy()


@pytest.mark.parametrize("layout", ["tcp", "file", "np_distinct", "generic"])
def test_direct_form_matches_oracle(oracle, E, H, igx, torch, monkeypatch, layout):
    """IGX_GB_DIRECT (no LDS cache: every row probes the HBM table, k_groupby_direct) gives
    the same table as the oracle -- keys, every aggregate (incl. a u32 wrap), first index --
    over three chunked updates with a running base index and a nil mask; then AUTO switches
    a miss-heavy stream to the partitioned form after one measured interval and stays exact."""
    A = igx._abi
    n = 450_000
    rng = np.random.default_rng(4)
    if layout == "tcp":
        G = 40_000
        ev_h = oracle.gen_tcp(0xC2, 3, G, oracle.zipf_cdf(G, 0.6), 0, n)
        names, widths = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family"), \
            [16, 16, 8, 4, 16, 2, 2, 2]
        extra = ("size", "dir")
        aggs = [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 4, 1)]
        oaggs = [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
                 {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1, "out_width": 4}]
    elif layout == "file":
        G = 100_000
        ev_h = oracle.gen_file(0xC5, 0, G, oracle.zipf_cdf(G, 0.5), 0, n)
        names, widths, extra = ("inode", "dev", "pid", "tid"), [8, 4, 4, 4], ("op", "count")
        aggs = [A.Agg(A.AGG_COUNT, 0, 4, 8, 0), A.Agg(A.AGG_SUM, 5, 4, 8, 0),
                A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 4, 1)]
        oaggs = [{"kind": "count", "cond": ev_h["op"], "cond_val": 0},
                 {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 0},
                 {"kind": "count", "cond": ev_h["op"], "cond_val": 1},
                 {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 1, "out_width": 4}]
    elif layout == "np_distinct":
        ev_h = oracle.gen_np(0xC4, 5_000, 50_000, 0, n)
        names, widths, extra, aggs, oaggs = ("src", "pkt", "peer", "port"), [4, 1, 4, 2], (), [], []
    else:
        G = 30_000
        ev_h = oracle.gen_tcp(0xC2, 5, G, oracle.zipf_cdf(G, 0.8), 0, n)
        names, widths, extra = ("pid", "lport", "dir"), [4, 2, 1], ("size",)
        aggs = [A.Agg(A.AGG_SUM, 3, A.NO_COL, 8, 0)]
        oaggs = [{"kind": "sum", "val": ev_h["size"]}]
    valid = (rng.random(n) > 0.05).astype(np.uint8)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    cols = [ev[k] for k in names + extra]
    o = oracle.groupby(oracle.pack_cols(ev_h, names), oaggs, valid=valid, base_idx=9)
    tab = E.Table(widths, aggs, n)
    tab.set_mode(A.GB_DIRECT)
    dv = H.to_device(valid)
    cuts = [0, n // 3, 2 * n // 3, n]
    for a, b in zip(cuts, cuts[1:]):
        tab.update([c[a:b] for c in cols], list(range(len(names))), b - a, 9 + a, valid=dv[a:b])
    _check(E, H, tab, widths, *o)
    # AUTO: interval 1 runs cached and measures; a miss-heavy stream runs partitioned next
    tab.set_mode(A.GB_AUTO)
    for _ in range(3):
        tab.reset()
        tab.update(cols, list(range(len(names))), n, 9, valid=dv)
        _check(E, H, tab, widths, *o)
    tab.destroy()


@pytest.mark.parametrize("variant", ["plain", "skewed", "lds_overflow", "index_column", "region", "region_overflow", "uc1"])
@pytest.mark.parametrize("layout", ["tcp", "file", "np_distinct", "generic"])
def test_partitioned_form_matches_oracle(oracle, E, H, igx, torch, monkeypatch, layout, variant):
    """IGX_GB_PART (k_groupby_part.h: count, scan, scatter into hash buckets, LDS aggregation
    per bucket, plain writes into the bucket's own probe regions) gives the oracle's table --
    keys, every aggregate (incl. a u32 wrap), first index -- over three chunked updates with a
    running base index and a nil mask.  'skewed': one key holds a large share of the rows, so
    its bucket is split into several work items that merge with CAS claims and atomics;
    'lds_overflow': an 8-entry LDS table sends most rows down the HBM path; 'index_column':
    global indices from a u64 column (the owner-side merge of igx_dist_exchange_groups).
    'region' / 'region_overflow': the region variant AUTO runs (no count pass, buckets filled
    through cursors), the second with regions of 600 records so that most records take the
    direct find-or-insert path from passes A and B.  'uc1': one record per thread and round in
    pass C (IGX_GBP_UC=1), whose stage buffer is then too small for the dense list of live
    entries on one-quad records, so pass C's flush takes its loop over all entries."""
    A = igx._abi
    if variant.startswith("region"):
        monkeypatch.setenv("IGX_GBP_REGION", "1")
    if variant == "region_overflow":
        monkeypatch.setenv("IGX_GBP_REGSIZE", "600")
    n = 450_000
    rng = np.random.default_rng(11)
    s = 1.3 if variant == "skewed" else 0.5
    if layout == "tcp":
        G = 40_000
        ev_h = oracle.gen_tcp(0xC2, 3, G, oracle.zipf_cdf(G, s), 0, n)
        names, widths = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family"), \
            [16, 16, 8, 4, 16, 2, 2, 2]
        extra = ("size", "dir")
        aggs = [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 4, 1)]
        oaggs = [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
                 {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1, "out_width": 4}]
    elif layout == "file":
        G = 100_000
        ev_h = oracle.gen_file(0xC5, 0, G, oracle.zipf_cdf(G, s), 0, n)
        names, widths, extra = ("inode", "dev", "pid", "tid"), [8, 4, 4, 4], ("op", "count")
        aggs = [A.Agg(A.AGG_COUNT, 0, 4, 8, 0), A.Agg(A.AGG_SUM, 5, 4, 8, 0),
                A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 4, 1)]
        oaggs = [{"kind": "count", "cond": ev_h["op"], "cond_val": 0},
                 {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 0},
                 {"kind": "count", "cond": ev_h["op"], "cond_val": 1},
                 {"kind": "sum", "val": ev_h["count"], "cond": ev_h["op"], "cond_val": 1, "out_width": 4}]
    elif layout == "np_distinct":
        ev_h = oracle.gen_np(0xC4, 5_000 if variant != "skewed" else 40, 50_000, 0, n)
        names, widths, extra, aggs, oaggs = ("src", "pkt", "peer", "port"), [4, 1, 4, 2], (), [], []
    else:
        G = 30_000
        ev_h = oracle.gen_tcp(0xC2, 5, G, oracle.zipf_cdf(G, s + 0.3), 0, n)
        names, widths, extra = ("pid", "lport", "dir"), [4, 2, 1], ("size",)
        aggs = [A.Agg(A.AGG_SUM, 3, A.NO_COL, 8, 0)]
        oaggs = [{"kind": "sum", "val": ev_h["size"]}]
    if variant == "lds_overflow":
        monkeypatch.setenv("IGX_GBP_ENTRIES", "8")
    if variant == "uc1":
        monkeypatch.setenv("IGX_GBP_UC", "1")
    valid = (rng.random(n) > 0.05).astype(np.uint8)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    cols = [ev[k] for k in names + extra]
    idx_h = None
    if variant == "index_column":   # a permutation of global indices, not in row order
        idx_h = (rng.permutation(n).astype(np.uint64) * np.uint64(3) + np.uint64(1000))
        cols = cols + [H.to_device(idx_h)]
    o = oracle.groupby(oracle.pack_cols(ev_h, names), oaggs, valid=valid, base_idx=9)
    if idx_h is not None:   # first = the smallest index column value of the group's rows
        packed = oracle.pack_cols(ev_h, names)
        okeys = [bytes(k) for k in o[0]]
        pos = {k: i for i, k in enumerate(okeys)}
        first = np.full(len(okeys), np.iinfo(np.uint64).max, dtype=np.uint64)
        for r in np.nonzero(valid)[0]:
            i = pos[bytes(packed[r])]
            first[i] = min(first[i], idx_h[r])
        o = (o[0], o[1], first)
    tab = E.Table(widths, aggs, n)
    tab.set_mode(A.GB_PART)
    dv = H.to_device(valid)
    cuts = [0, n // 3, 2 * n // 3, n]
    icol = len(names) + len(extra) if idx_h is not None else None
    for a, b in zip(cuts, cuts[1:]):
        tab.update([c[a:b] for c in cols], list(range(len(names))), b - a, 9 + a, valid=dv[a:b], idx_col=icol)
    _check(E, H, tab, widths, *o)
    tab.reset()                                            # a second interval, one update
    tab.update(cols, list(range(len(names))), n, 9, valid=dv, idx_col=icol)
    _check(E, H, tab, widths, *o)
    tab.destroy()


def test_odd_key_widths_and_unfused_predicates(oracle, E, H, igx, torch):
    """Key columns of 3, 5, 6 and 7 bytes (byte loads in the generic layout, any alignment)
    and more predicates than the kernel fuses -- a string comparison, a regex and four scalar
    ones: the extra ones become a device row mask (k_pred_mask, the filter's evaluator)
    AND-ed with the nil mask.  Exact against the oracle over two chunked updates."""
    A = igx._abi
    rng = np.random.default_rng(21)
    n = 300_000
    k3 = rng.integers(0, 4, (n, 3)).astype(np.uint8)
    k5 = rng.integers(0, 3, (n, 5)).astype(np.uint8)
    k6 = rng.integers(0, 2, (n, 6)).astype(np.uint8)
    k7 = rng.integers(0, 2, (n, 7)).astype(np.uint8)
    v = rng.integers(0, 1000, n).astype(np.uint32)
    p1 = rng.integers(0, 100, n).astype(np.int32)
    p2 = rng.integers(0, 100, n).astype(np.uint16)
    names = np.array([b"bash", b"sshd", b"kworker", b"demo"], dtype="S16")
    comm = np.frombuffer(names[rng.integers(0, 4, n)].tobytes(), np.uint8).reshape(n, 16).copy()
    valid = (rng.random(n) > 0.1).astype(np.uint8)
    cols = [H.to_device(x) for x in (k3, k5, k6, k7, v, p1, p2, comm)]
    ref = (C.c_uint8 * A.MAX_REF)(*b"s.*d")
    preds = [_pred(A, 5, A.CMP_GE, 10, np.int32), _pred(A, 5, A.CMP_LT, 90, np.int32),
             _pred(A, 6, A.CMP_GT, 5, np.uint16), _pred(A, 6, A.CMP_LE, 95, np.uint16, negate=True),
             A.Pred(7, A.CMP_REGEX, 1, 4, ref),                       # !~s.*d
             A.Pred(7, A.CMP_EQ, 1, 0, (C.c_uint8 * A.MAX_REF)())]    # string != 
    comm_s = [bytes(r).split(b"\0")[0].decode() for r in comm]
    keep = (valid.astype(bool) & (p1 >= 10) & (p1 < 90) & (p2 > 5) & ~(p2 <= 95)
            & np.array([re.search("s.*d", c) is None for c in comm_s]) & np.array([c != "" for c in comm_s]))
    widths = [3, 5, 6, 7]
    tab = E.Table(widths, [A.Agg(A.AGG_SUM, 4, A.NO_COL, 8, 0)], 65536)
    dv = H.to_device(valid)
    half = n // 2
    for a, b in ((0, half), (half, n)):
        tab.update([c[a:b] for c in cols], [0, 1, 2, 3], b - a, a, preds=preds, valid=dv[a:b])
    o = oracle.groupby(np.concatenate([k3, k5, k6, k7], axis=1), [{"kind": "sum", "val": v}],
                       valid=keep.astype(np.uint8))
    _check(E, H, tab, widths, *o)
    tab.destroy()
