"""GPU parity: libigx.so (through the C ABI) vs the CPU oracle on identical seeded streams.

Bit-exact for everything (integer counting, keying and ordering).  Sizes are chosen so
the oracle finishes in seconds; the headline config at full size (100M events) is
tests/test_gpu_fullsize.py.
"""
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


def _h(H, d):
    return {k: H.host(v) for k, v in d.items()}


def test_gen_tcp_bit_exact(oracle, E, H, torch):
    G, n = 5000, 200_000
    cdf = oracle.zipf_cdf(G, 1.1)
    for rank, base in [(0, 0), (3, 123_456_789)]:
        ref = oracle.gen_tcp(0xC2, rank, G, cdf, base, n)
        got = _h(H, E.gen_tcp(0xC2, rank, G, H.to_device(cdf), base, n))
        for k in ref:
            assert np.array_equal(ref[k], got[k]), k


def test_gen_others_bit_exact(oracle, E, H, torch):
    n = 100_000
    ccdf = oracle.zipf_cdf(64, 1.0)
    ref = oracle.gen_open(0xC1, ccdf, 7, n)
    got = _h(H, E.gen_open(0xC1, H.to_device(ccdf), 7, n))
    for k in ref:
        assert np.array_equal(ref[k], got[k]), k
    q = oracle.lognormal_quantiles(np.log(2e5), 1.5)
    ref = oracle.gen_bio(0xC3, q, 11, n)
    got = _h(H, E.gen_bio(0xC3, H.to_device(q), 11, n))
    for k in ref:
        assert np.array_equal(ref[k].view(np.uint64), got[k].view(np.uint64)), k
    ref = oracle.gen_np(0xC4, 10_000, 100_000, 5, n)
    got = _h(H, E.gen_np(0xC4, 10_000, 100_000, 5, n))
    for k in ref:
        assert np.array_equal(ref[k], got[k]), k
    fcdf = oracle.zipf_cdf(20_000, 1.05)
    ref = oracle.gen_file(0xC5, 2, 20_000, fcdf, 9, n)
    got = _h(H, E.gen_file(0xC5, 2, 20_000, H.to_device(fcdf), 9, n))
    for k in ref:
        assert np.array_equal(ref[k], got[k]), k


TCP_KEY = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family")


def _tcp_table(E, igx, ev, n, capacity, base=0):
    A = igx._abi
    cols = [ev[k] for k in TCP_KEY] + [ev["size"], ev["dir"]]
    widths = [16, 16, 8, 4, 16, 2, 2, 2]
    aggs = [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)]
    tab = E.Table(widths, aggs, capacity)
    tab.update(cols, list(range(8)), n, base)
    return tab


def _unpad_tcp_keys(keys):
    # device key layout: every column padded to 4 bytes: 16,16,8,4,16,4,4,4 (72 B)
    k = keys[:, :72]
    return np.concatenate([k[:, :60], k[:, 60:62], k[:, 64:66], k[:, 68:70]], axis=1)


@pytest.mark.parametrize("G,n", [(1000, 300_000), (200_000, 400_000)])
def test_groupby_top_tcp(oracle, E, H, igx, torch, G, n):
    cdf = oracle.zipf_cdf(G, 1.1)
    ev_h = oracle.gen_tcp(0xC2, 0, G, cdf, 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    tab = _tcp_table(E, igx, ev, n, capacity=2 * G, base=1000)
    fin = tab.finalize()
    keys, aggs, first = E.table_tensors(tab, fin)
    gk = _unpad_tcp_keys(H.host(keys))
    gs, gr, gf = H.host(aggs[0]), H.host(aggs[1]), H.host(first)
    okeys, oaggs, ofirst = oracle.groupby(
        oracle.pack_cols(ev_h, TCP_KEY),
        [{"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 0},
         {"kind": "sum", "val": ev_h["size"], "cond": ev_h["dir"], "cond_val": 1}],
        base_idx=1000)
    assert fin["n_groups"] == len(okeys)
    ref = {bytes(k): (int(s), int(r), int(f)) for k, s, r, f in zip(okeys, oaggs[0], oaggs[1], ofirst)}
    got = {bytes(k): (int(s), int(r), int(f)) for k, s, r, f in zip(gk, gs, gr, gf)}
    assert got == ref
    tab.destroy()


def test_topk_matches_go_sort(oracle, E, H, igx, torch):
    """top tcp: nextStats -> SortStats(["-sent","-recv"]) -> stats[:20]."""
    G, n = 20_000, 500_000
    cdf = oracle.zipf_cdf(G, 1.1)
    ev_h = oracle.gen_tcp(0xC2, 0, G, cdf, 0, n)
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    tab = _tcp_table(E, igx, ev, n, capacity=2 * G)
    fin = tab.finalize()
    keys, aggs, first = E.table_tensors(tab, fin)
    Gn = fin["n_groups"]
    top = E.sort_perm([(aggs[0], True), (aggs[1], True)], Gn, pos=first, k=20)
    got = H.host(first)[H.host(top).astype(np.int64)]
    Gref, okeys, osent, orecv, ofirst = oracle.top_tcp(ev_h, 20)
    assert Gn == Gref
    assert list(got) == list(ofirst)
    # full sort too, against the Go SliceStable restatement on first-occurrence order
    full = H.host(E.sort_perm([(aggs[0], True), (aggs[1], True)], Gn, pos=first))
    fh = H.host(first)
    order = np.argsort(fh, kind="stable")           # canonical pre-sort order
    sent, recv = H.host(aggs[0])[order], H.host(aggs[1])[order]
    perm = oracle.go_sort_entries([(sent, "uint64", True), (recv, "uint64", True)], Gn)
    assert np.array_equal(fh[full.astype(np.int64)], fh[order][perm.astype(np.int64)])


def test_ties_and_parity(oracle, E, H, torch):
    """Heavy ties, 1-3 keys, mixed directions, signed/unsigned/bytes: exact Go order."""
    rng = np.random.default_rng(7)
    for trial in range(12):
        n = int(rng.integers(1, 5000))
        nk = int(rng.integers(1, 4))
        kinds = rng.choice(["int8", "int64", "uint16", "uint64", "string", "int32"], nk)
        cols_h, keys_d, keys_o = [], [], []
        for kd in kinds:
            desc = bool(rng.random() < 0.6)
            if kd == "string":
                a = np.zeros((n, 8), np.uint8)
                a[:, 0] = rng.integers(97, 100, n)
                a[:, 1] = rng.integers(0, 2, n) * 98
            else:
                a = rng.integers(-3 if kd.startswith("int") else 0, 3, n).astype(kd)
            keys_d.append((H.to_device(a), desc))
            keys_o.append((a, kd, desc))
        got = H.host(E.sort_perm(keys_d, n))
        ref = oracle.go_sort_entries(keys_o, n)
        assert np.array_equal(got, ref), (trial, kinds)
        # top-K (radix-select path when n > 2k): the first k of the same order
        for k in (1, 7, 300):
            if n > k:
                top = H.host(E.sort_perm(keys_d, n, k=k))
                assert np.array_equal(top, ref[:k]), (trial, kinds, k)


def test_filter_c1(oracle, E, H, igx, torch):
    """C1: FilterEntries(["err:0", "pid:>=1000"]) then SortEntries(["comm", "-pid"])."""
    n = 1_000_000
    ccdf = oracle.zipf_cdf(64, 1.0)
    ev_h = oracle.gen_open(0xC1, ccdf, 0, n)
    cols = igx.columns.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"),
                                ("comm", "string", 16), ("ret", "int64"), ("fd", "int64"),
                                ("err", "int64"), ("path", "uint32")])
    batch = igx.columns.EventBatch(cols, {k: H.to_device(v) for k, v in ev_h.items()})
    out = igx.filter.FilterEntries(cols, batch, ["err:0", "pid:>=1000"])
    ocols = {"err": oracle.OCol("err", "int64", 8), "pid": oracle.OCol("pid", "uint32", 4)}
    sel = oracle.match_rows([oracle.parse_filter(ocols, "err:0"),
                             oracle.parse_filter(ocols, "pid:>=1000")], ev_h)
    assert out.n == len(sel)
    assert np.array_equal(H.host(out["pid"]), ev_h["pid"][sel])
    srt = igx.sort.SortEntries(cols, out, ["comm", "-pid"])
    perm = oracle.go_sort_entries([(ev_h["comm"][sel], "string", False),
                                   (ev_h["pid"][sel], "uint32", True)], len(sel))
    assert np.array_equal(H.host(srt["pid"]), ev_h["pid"][sel][perm])
    assert np.array_equal(H.host(srt["comm"]), ev_h["comm"][sel][perm])


def test_take_rows(E, H, torch):
    """igx_take (the compacted batch FilterEntries returns): every width / alignment unit,
    more than one launch's worth of columns, out-of-range indices -> zero rows, empty idx."""
    rng = np.random.default_rng(7)
    n, k = 100_003, 70_001
    specs = [(np.uint8, None), (np.uint16, None), (np.uint32, None), (np.uint64, None),
             (np.int64, None), (np.uint8, 16), (np.uint8, 3), (np.uint8, 24), (np.uint8, 72)] * 2
    cols = []
    for dt, w in specs:
        shape = (n,) if w is None else (n, w)
        cols.append(rng.integers(0, 256 if w else np.iinfo(dt).max, size=shape, dtype=dt))
    idx = rng.integers(0, n, size=k).astype(np.uint32)
    idx[::997] = n + 5                                   # out of range -> zero row
    got = E.take([H.to_device(c) for c in cols], H.to_device(idx), n)
    ok = idx < n
    for c, g in zip(cols, got):
        want = np.zeros((k,) + c.shape[1:], dtype=c.dtype)
        want[ok] = c[idx[ok]]
        assert np.array_equal(H.host(g), want), (c.dtype, c.shape)
    # a byte column whose base address is odd (contiguous, storage offset 5)
    flat = rng.integers(0, 256, size=n * 24 + 5, dtype=np.uint8)
    sub = H.to_device(flat)[5:].view(n, 24)
    got = E.take([sub], H.to_device(idx[ok]), n)[0]
    assert np.array_equal(H.host(got), flat[5:].reshape(n, 24)[idx[ok]])
    assert E.take([H.to_device(cols[0])], H.to_device(np.zeros(0, np.uint32)), n)[0].numel() == 0


def test_take_debug_assert(E, H, torch, monkeypatch):
    """IGX_DEBUG_TAKE=1: an out-of-range row id raises IndexError (as the torch index_select
    igx_take replaced did) unless the caller asked for zero-padded rows."""
    col = H.to_device(np.arange(10, dtype=np.uint32))
    idx = H.to_device(np.array([1, 12, 3], dtype=np.uint32))
    monkeypatch.setenv("IGX_DEBUG_TAKE", "1")
    with pytest.raises(IndexError):
        E.take([col], idx, 10)
    padded = E.take([col], idx, 10, pad=True)[0]
    assert H.host(padded).tolist() == [1, 0, 3]
    assert H.host(E.take([col], H.to_device(np.array([9, 0], dtype=np.uint32)), 10)[0]).tolist() == [9, 0]


@pytest.mark.parametrize("spread", ["all-slots", "high-slots"])
def test_hist_slot_window(oracle, E, H, torch, spread):
    """4096 keys x 27 slots: LDS holds a window of the slots (k_hist header); rows outside
    it go to HBM directly.  Deltas spread over every slot, or concentrated in high slots so
    that the device-chosen window starts above 0."""
    rng = np.random.default_rng(17 if spread == "all-slots" else 18)
    n = 3_000_000
    devs = [(8 << 20) | (16 * k) for k in range(16)]
    dev = np.array(devs, np.uint32)[rng.integers(0, 16, n)]
    cont = rng.integers(0, 256, n).astype(np.uint32)
    if spread == "all-slots":
        delta = (np.exp2(rng.uniform(0, 46, n)) * 1000).astype(np.int64)
    else:
        delta = (np.exp2(rng.normal(30, 1.5, n).clip(0, 60)) * 1000).astype(np.int64)
    delta[::97] = -5                                              # negative: skipped
    got = H.host(E.hist_log2(H.to_device(dev), H.to_device(cont), H.to_device(delta), devs, 256))
    ref = oracle.hist_log2(dev, cont, delta, devs, 256)
    assert np.array_equal(got, ref)
    # one key, one in-window bin, far past the 16-bit LDS counters: window carries
    d1 = torch.full((5_000_000,), 3 << 40, dtype=torch.int64, device="cuda")
    dv = torch.full((5_000_000,), devs[5], dtype=torch.int32, device="cuda").view(torch.uint32)
    cc = torch.full((5_000_000,), 200, dtype=torch.int32, device="cuda").view(torch.uint32)
    h = H.host(E.hist_log2(dv, cc, d1, devs, 256))
    assert int(h[5 * 256 + 200, 26]) == 5_000_000 and int(h.sum()) == 5_000_000


def test_hist_log2_c3(oracle, E, H, torch):
    n = 2_000_000
    q = oracle.lognormal_quantiles(np.log(2e5), 1.5)
    ev_h = oracle.gen_bio(0xC3, q, 0, n)
    devs = [(8 << 20) | (16 * k) for k in range(16)]
    ev = {k: H.to_device(v) for k, v in ev_h.items()}
    got = H.host(E.hist_log2(ev["dev"], ev["cont"], ev["delta"].view(torch.int64), devs, 256))
    ref = oracle.hist_log2(ev_h["dev"], ev_h["cont"], ev_h["delta"], devs, 256)
    assert got.shape == (4096, 27)
    assert np.array_equal(got, ref)
    # reference shape: single key (no per-disk / per-container keys), 27 slots
    got1 = H.host(E.hist_log2(ev["dev"], None, ev["delta"].view(torch.int64), devs[:1], 1))
    ref1 = oracle.hist_log2(ev_h["dev"], np.zeros(n, np.uint32), ev_h["delta"], devs[:1], 1)
    assert np.array_equal(got1, ref1)
    # containers outside [0, ncont) and devices outside devs are not counted; ms divisor
    got2 = H.host(E.hist_log2(ev["dev"], ev["cont"], ev["delta"].view(torch.int64), devs[3:9], 100,
                              divisor=1_000_000))
    ref2 = oracle.hist_log2(ev_h["dev"], ev_h["cont"], ev_h["delta"], devs[3:9], 100, divisor=1_000_000)
    assert np.array_equal(got2, ref2)


def test_float_sort_keys_match_go(oracle, igx, torch):
    """Float sort keys (sort.go:71-74 getLessFunc[float32/float64]): Go's `<` -- -0 == +0
    (a tie), -Inf < finite < +Inf, subnormals ordered -- under ASC / DESC and mixed with an int
    key, against the Go 1.19 SliceStable restatement; heavy ties exercise the closed form's
    tie parity.  A NaN makes the comparison unordered: the order is then SliceStable's own
    (k_gostable.hip runs the algorithm), compared with the C restatement of it."""
    E, H, A = igx.engine, igx.columns, igx._abi
    rng = np.random.default_rng(11)
    n = 50_000
    pool32 = np.array([0.0, -0.0, np.inf, -np.inf, 1.5, -1.5, 1e-45, -1e-45, 3.4e38, -3.4e38, 7.0, 7.0],
                      np.float32)
    pool64 = np.array([0.0, -0.0, np.inf, -np.inf, 2.5, -2.5, 5e-324, -5e-324, 1.7e308, 1.0 / 3.0],
                      np.float64)
    f32 = pool32[rng.integers(0, len(pool32), n)]
    f64 = np.where(rng.random(n) < 0.5, pool64[rng.integers(0, len(pool64), n)], rng.standard_normal(n))
    i8 = rng.integers(-3, 3, n).astype(np.int8)
    d32, d64, di8 = H.to_device(f32), H.to_device(f64), H.to_device(i8)
    cases = [[(0, False)], [(0, True)], [(1, False)], [(1, True)], [(0, True), (2, False)],
             [(2, True), (0, False), (1, True)], [(0, False), (1, False)]]
    cols = [(d32, f32, "float32"), (d64, f64, "float64"), (di8, i8, "int8")]
    for keys in cases:
        got = H.host(E.sort_perm([(cols[c][0], desc) for c, desc in keys], n)).astype(np.int64)
        ref = oracle.go_sort_entries([(cols[c][1], cols[c][2], desc) for c, desc in keys], n).astype(np.int64)
        assert np.array_equal(got, ref), keys
        k = 25
        top = H.host(E.sort_perm([(cols[c][0], desc) for c, desc in keys], n, k=k)).astype(np.int64)
        assert np.array_equal(top, ref[:k]), keys
    bad = f64.copy()
    bad[123] = np.nan
    bad[rng.integers(0, n, 40)] = np.nan
    bad32 = f32.copy()
    bad32[rng.integers(0, n, 300)] = np.nan
    nan_cols = [(H.to_device(bad), bad, "float64"), (H.to_device(bad32), bad32, "float32"), (di8, i8, "int8")]
    for keys in ([(0, False)], [(0, True)], [(1, True), (2, False)], [(2, True), (1, False), (0, True)]):
        got = H.host(E.sort_perm([(nan_cols[c][0], desc) for c, desc in keys], n)).astype(np.int64)
        ref = oracle.go_sort_entries([(nan_cols[c][1], nan_cols[c][2], desc) for c, desc in keys], n).astype(np.int64)
        assert np.array_equal(got, ref), keys
        top = H.host(E.sort_perm([(nan_cols[c][0], desc) for c, desc in keys], n, k=25)).astype(np.int64)
        assert np.array_equal(top, ref[:25]), keys
    # a NaN in a nil row is never compared (sort.go:127-132 returns before reading the field)
    valid = np.ones(n, np.uint8)
    valid[123] = 0
    got = H.host(E.sort_perm([(H.to_device(bad), True)], n, valid=H.to_device(valid))).astype(np.int64)
    ref = oracle.go_sort_entries([(bad, "float64", True)], n, valid=valid).astype(np.int64)
    assert np.array_equal(got, ref)
    valid[rng.integers(0, n, 500)] = 0   # nil rows and NaN rows together
    got = H.host(E.sort_perm([(H.to_device(bad32), False), (di8, True)], n, valid=H.to_device(valid))).astype(np.int64)
    ref = oracle.go_sort_entries([(bad32, "float32", False), (i8, "int8", True)], n, valid=valid).astype(np.int64)
    assert np.array_equal(got, ref)


def test_many_sort_keys(oracle, E, H, torch):
    """More than 8 sort keys (the composed radix key takes up to 32 keys): 12 narrow keys
    with heavy ties and mixed directions, exact Go SliceStable order and top-K."""
    rng = np.random.default_rng(12)
    n = 20_000
    kinds = ["int8", "uint16", "string", "int32", "uint8", "int64", "uint32", "int16", "string", "uint64",
             "int8", "uint8"]
    keys_d, keys_o = [], []
    for kd in kinds:
        desc = bool(rng.random() < 0.5)
        if kd == "string":
            a = np.zeros((n, 4), np.uint8)
            a[:, 0] = rng.integers(97, 99, n)
        else:
            a = rng.integers(-1 if kd.startswith("int") else 0, 2, n).astype(kd)
        keys_d.append((H.to_device(a), desc))
        keys_o.append((a, kd, desc))
    ref = oracle.go_sort_entries(keys_o, n)
    assert np.array_equal(H.host(E.sort_perm(keys_d, n)), ref)
    assert np.array_equal(H.host(E.sort_perm(keys_d, n, k=50)), ref[:50])


def test_nan_sort_hand_derived_vectors(igx, torch):
    """The device NaN path (k_gostable.hip) on the hand-derived Go SliceStable orders of
    tests/test_oracle_golden.py NAN_VECTORS (float64 and float32 keys, nil rows)."""
    from test_oracle_golden import NAN_VECTORS
    E, H = igx.engine, igx.columns
    for keys, valid, want in NAN_VECTORS:
        n = len(want)
        dv = None if valid is None else H.to_device(np.array(valid, np.uint8))
        for dt in (np.float64, np.float32):
            cols = [(H.to_device(np.array(v, dt)), d) for v, d in keys]
            got = H.host(E.sort_perm(cols, n, valid=dv)).astype(np.int64)
            assert list(got) == want, (keys, valid, dt)


def test_device_planned_sort_matches_host_planned(oracle, E, H, torch, monkeypatch):
    """The device-planned LSD passes (IGX_SORT_DEVPLAN=1, k_lsd_*: each pass decides on the device
    whether its digit varies, one launch per pass, tiles chained by tagged counts) against the
    default host-planned passes and the Go SliceStable restatement: 1..8 composed words, ties,
    nil rows, several tiles, and a selection vector whose length stays on the device (both
    paths: the host plan reads the count back with its AND/OR words)."""
    rng = np.random.default_rng(11)
    for trial, n in enumerate([1, 2, 3, 4095, 4096, 4097, 70_000, 300_001]):
        nk = int(rng.integers(1, 4))
        kinds = rng.choice(["int8", "int64", "uint16", "uint32", "string"], nk)
        keys_d, keys_o = [], []
        for kd in kinds:
            desc = bool(rng.random() < 0.5)
            if kd == "string":
                a = np.zeros((n, 12), np.uint8)
                a[:, 0] = rng.integers(97, 103, n)
                a[:, 5] = rng.integers(0, 3, n) * 40
            else:
                lo = -50 if kd.startswith("int") else 0
                a = rng.integers(lo, 50, n).astype(kd)
            keys_d.append((H.to_device(a), desc))
            keys_o.append((a, kd, desc))
        valid = (rng.random(n) < 0.9).astype(np.uint8) if trial % 2 else None
        vd = None if valid is None else H.to_device(valid)
        monkeypatch.setenv("IGX_SORT_DEVPLAN", "1")
        got = H.host(E.sort_perm(keys_d, n, valid=vd))
        monkeypatch.delenv("IGX_SORT_DEVPLAN")
        host = H.host(E.sort_perm(keys_d, n, valid=vd))
        ref = oracle.go_sort_entries(keys_o, n, valid=valid)
        assert np.array_equal(host, ref), (trial, kinds)
        assert np.array_equal(got, ref), (trial, kinds)
        # a selection of m rows (every third row, reversed) of capacity n, its count on the device
        sel = np.arange(n, dtype=np.uint32)[::-3].copy()
        m = len(sel)
        cap = torch.full((n,), 0xFFFF, dtype=torch.int32, device="cuda").view(torch.uint32)
        cap[:m] = H.to_device(sel)
        cnt = torch.tensor([m], dtype=torch.int64, device="cuda").view(torch.uint64)
        sub = [(a[sel], kd, d) for a, kd, d in keys_o]
        want = sel[oracle.go_sort_entries(sub, m, valid=None if valid is None else valid[sel]).astype(np.int64)]
        for devplan in (False, True):
            if devplan:
                monkeypatch.setenv("IGX_SORT_DEVPLAN", "1")
            out = H.host(E.sort_perm(keys_d, n, valid=vd, rowmap=cap, d_count=cnt))[:m]
            monkeypatch.delenv("IGX_SORT_DEVPLAN", raising=False)
            assert np.array_equal(out, want), (trial, kinds, devplan)


def _strings(rng, n, width, distinct):
    """n strings of `width` bytes drawn from exactly `distinct` values over a 3-letter alphabet
    (long shared prefixes), of every length from D = min(8, width) to the field (zero padded, as
    Go compares them), plus the empty string.  A value's last D letters are its index in base 3."""
    D = min(8, width)
    assert distinct <= 3 ** D
    pool = np.zeros((distinct, width), np.uint8)
    for v in range(1, distinct):
        ln = int(rng.integers(D, width + 1))
        pool[v, :ln - D] = rng.integers(97, 100, ln - D)
        pool[v, ln - D:ln] = [97 + (v // 3 ** d) % 3 for d in range(D - 1, -1, -1)]
    assert len(np.unique(pool, axis=0)) == distinct
    return pool[rng.integers(0, distinct, n)]


def test_string_dictionary_sort(oracle, E, H, torch, monkeypatch):
    """String keys of many rows sort through a dictionary of their distinct values (k_dict_*:
    the rank replaces the bytes, one or two live digits instead of one per byte); a dictionary
    over capacity (4 096 values of <= 16 bytes, 2 048 of 32) is void and the raw bytes are
    composed instead.  Same order as IGX_SORT_DICT=0 and as Go's SliceStable restatement: 6-, 8-,
    12-, 16-, 20- and 32-byte strings, ascending and descending, with ties broken by position, nil rows, a
    selection vector with a device count, and exactly-at-capacity / over-capacity value counts."""
    rng = np.random.default_rng(5)
    n = 150_000
    cases = [
        [(16, 64, False), ("uint32", None, True)],            # C1's shape: comm, -pid
        [(16, 4096, True)],                                   # exactly the capacity
        [(16, 4097, False), ("int8", None, False)],           # one over: void, raw bytes
        [(8, 5000, True), (32, 2000, False)],                 # void (8-byte) + valid (32-byte)
        [(12, 300, True), (32, 2049, True), ("int64", None, True)],   # the 32-byte one over capacity
        [(32, 1, False), (16, 3, True)],                      # constant strings
        [(6, 500, False), (20, 700, True), ("uint16", None, False)],   # 2 and 5 words, partial last words
    ]
    for ci, spec in enumerate(cases):
        keys_d, keys_o = [], []
        for kd, distinct, desc in spec:
            if isinstance(kd, int):
                a = _strings(rng, n, kd, distinct)
                keys_o.append((a, "string", desc))
            else:
                a = rng.integers(-40 if kd.startswith("int") else 0, 40, n).astype(kd)
                keys_o.append((a, kd, desc))
            keys_d.append((H.to_device(a), desc))
        valid = (rng.random(n) < 0.93).astype(np.uint8) if ci % 2 else None
        vd = None if valid is None else H.to_device(valid)
        ref = oracle.go_sort_entries(keys_o, n, valid=valid)
        got = H.host(E.sort_perm(keys_d, n, valid=vd))
        monkeypatch.setenv("IGX_SORT_DICT", "0")
        raw = H.host(E.sort_perm(keys_d, n, valid=vd))
        monkeypatch.delenv("IGX_SORT_DICT")
        assert np.array_equal(raw, ref), ci
        assert np.array_equal(got, ref), ci
        # a selection of m rows with its count on the device (FilterEntries' pending view)
        sel = np.sort(rng.choice(n, n // 2 + 1, replace=False)).astype(np.uint32)[::-1].copy()
        m = len(sel)
        cap = torch.full((n,), 0x7FFFFFFF, dtype=torch.int32, device="cuda").view(torch.uint32)
        cap[:m] = H.to_device(sel)
        cnt = torch.tensor([m], dtype=torch.int64, device="cuda").view(torch.uint64)
        sub = [(a[sel], kd, d) for a, kd, d in keys_o]
        want = sel[oracle.go_sort_entries(sub, m, valid=None if valid is None else valid[sel]).astype(np.int64)]
        out = H.host(E.sort_perm(keys_d, n, valid=vd, rowmap=cap, d_count=cnt))[:m]
        assert np.array_equal(out, want), ci
    # high bytes (>= 0x80) compare unsigned, as Go's string comparison does: 900 distinct
    # 16-byte values of random bytes 1..255 (no NUL), two sort directions
    pool = rng.integers(1, 256, (900, 16), dtype=np.uint8)
    pool[::7, 8:] = 0                                       # shorter values, zero padded
    a = pool[rng.integers(0, 900, n)]
    for desc in (False, True):
        got = H.host(E.sort_perm([(H.to_device(a), desc)], n))
        assert np.array_equal(got, oracle.go_sort_entries([(a, "string", desc)], n)), desc
    # no value to rank: every row nil, and an empty slice (a device count of 0)
    a = _strings(rng, n, 16, 10)
    nil = np.zeros(n, np.uint8)
    got = H.host(E.sort_perm([(H.to_device(a), True)], n, valid=H.to_device(nil)))
    assert np.array_equal(got, oracle.go_sort_entries([(a, "string", True)], n, valid=nil))
    cap = torch.zeros((n,), dtype=torch.int32, device="cuda").view(torch.uint32)
    zero = torch.zeros((1,), dtype=torch.int64, device="cuda").view(torch.uint64)
    E.sort_perm([(H.to_device(a), False)], n, rowmap=cap, d_count=zero)
    torch.cuda.synchronize()


@pytest.mark.parametrize("devplan", [False, True])
def test_filter_then_sort_pending_count(oracle, E, H, igx, torch, monkeypatch, devplan):
    """C1's step as the bench runs it: FilterEntries leaves its survivor count on the device and
    SortEntries sorts that pending view (igx_sort_perm_dn: the host plan reads the count back
    with its AND/OR words -- one round trip for the whole step; IGX_SORT_DEVPLAN=1: none); the
    view's length is read only afterwards.  Same rows, same order as the oracle's FilterEntries
    + SortEntries."""
    if devplan:
        monkeypatch.setenv("IGX_SORT_DEVPLAN", "1")
    n = 1_000_000
    ccdf = oracle.zipf_cdf(64, 1.0)
    ev_h = oracle.gen_open(0xC1, ccdf, 0, n)
    cols = igx.columns.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"),
                                ("comm", "string", 16), ("ret", "int64"), ("fd", "int64"),
                                ("err", "int64"), ("path", "uint32")])
    batch = igx.columns.EventBatch(cols, {k: H.to_device(v) for k, v in ev_h.items()})
    for filters, sort_by in ((["err:0", "pid:>=1000"], ["comm", "-pid"]), (["uid:0"], ["-comm", "pid", "-fd"]),
                             (["pid:<0"], ["comm"])):
        out = igx.filter.FilterEntries(cols, batch, filters)
        assert out.pending() is not None
        srt = igx.sort.SortEntries(cols, out, sort_by)
        assert srt.pending() is not None              # the view's length is still on the device
        ocols = {c: oracle.OCol(c, t, w) for c, t, w in (("err", "int64", 8), ("pid", "uint32", 4),
                                                           ("uid", "uint32", 4))}
        sel = oracle.filter_entries(ocols, {k: ev_h[k] for k in ("err", "pid", "uid")}, None, filters)
        kinds = {"comm": "string", "pid": "uint32", "fd": "int64"}
        keys = [(ev_h[s.lstrip("-")][sel], kinds[s.lstrip("-")], s.startswith("-")) for s in sort_by]
        want = sel[oracle.go_sort_entries(keys, len(sel)).astype(np.int64)]
        assert srt.n == len(sel)
        assert np.array_equal(H.host(srt.sel).astype(np.int64), want.astype(np.int64)), filters


@pytest.mark.parametrize("divisor", [1000, 1000000, 7])
def test_hist_slot_boundaries(oracle, E, H, torch, divisor):
    """log2l(delta / divisor) at every boundary D * 2^k - 1, D * 2^k, D * 2^k + 1 (and powers of
    two, zero, negatives): the division-free slot of k_hist (divisors 1000 / 1e6) and the
    generic one agree with biolatency.bpf.c:133-141 / bits.bpf.h:8-29 as the oracle restates it."""
    vals = [0, 1, -1, -5, (1 << 63) - 1]
    for k in range(0, 62):
        for base in (divisor << k, 1 << k):
            for e in (-1, 0, 1):
                v = base + e
                if 0 <= v < (1 << 63):
                    vals.append(v)
    rng = np.random.default_rng(5)
    vals += list(rng.integers(0, 1 << 62, 5000))
    vals += [0] * (-len(vals) % 8192 + 8192 * 4)   # whole 8192-row chunks: the vector path too
    delta = np.array(vals, dtype=np.int64)
    n = len(delta)
    d = H.to_device(delta)
    ref = oracle.hist_log2(None, None, delta, [], 1, divisor=divisor)
    assert ref.sum() == (delta >= 0).sum()
    got = H.host(E.hist_log2(None, None, d, [], 1, divisor=divisor))            # scalar loads
    assert np.array_equal(got, ref)
    devc = H.to_device(np.full(n, 7, np.uint32))
    contc = H.to_device(np.zeros(n, np.uint32))
    got = H.host(E.hist_log2(devc, contc, d, [7], 1, divisor=divisor))          # 16-B loads
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("n", [1_000_003, 16_777_217])
def test_filter_int_mark_and_both_compactions(oracle, E, H, igx, torch, n):
    """igx_filter on integer predicates (the kernel that loads every row's values before it
    compares: signed and unsigned, 1/2/4/8-byte columns, a negated predicate, nil rows) and
    both compactions: up to 16M rows the compaction sums its tile's predecessors itself, above
    that the scan kernel runs first.  Same row ids as numpy, in input order."""
    import ctypes as C
    A = igx._abi
    rng = np.random.default_rng(n)
    i8 = rng.integers(-100, 100, n, dtype=np.int8)
    u16 = rng.integers(0, 60000, n, dtype=np.uint16)
    i32 = rng.integers(-2**31, 2**31 - 1, n, dtype=np.int32)
    i64 = rng.integers(-2**40, 2**40, n, dtype=np.int64)
    valid = (rng.random(n) < 0.97).astype(np.uint8)

    def pred(col, cmp, value, dtype, negate=False):
        b = np.array([value], dtype=dtype).view(np.uint8)
        return A.Pred(col, cmp, int(negate), len(b), (C.c_uint8 * A.MAX_REF)(*b.tolist()))

    cols = [H.to_device(a) for a in (i8, u16, i32, i64)]
    preds = [pred(0, A.CMP_GE, -20, np.int8), pred(1, A.CMP_LT, 45000, np.uint16),
             pred(2, A.CMP_GT, -2**30, np.int32), pred(3, A.CMP_LE, 2**39, np.int64, negate=True)]
    got = H.host(E.filter_rows(cols, preds, n, valid=H.to_device(valid))).astype(np.int64)
    want = np.flatnonzero((i8 >= -20) & (u16 < 45000) & (i32 > -2**30) & ~(i64 <= 2**39) & (valid != 0))
    assert np.array_equal(got, want)
    # MatchAny over the same predicates, no nil mask
    got = H.host(E.filter_rows(cols, preds, n, any=True)).astype(np.int64)
    want = np.flatnonzero((i8 >= -20) | (u16 < 45000) | (i32 > -2**30) | ~(i64 <= 2**39))
    assert np.array_equal(got, want)
