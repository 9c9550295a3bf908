"""The all-cores CPU baselines (oracle/igx_oracle.c §7) equal the single-thread
restatements they are timed against (top tcp, generic group-by + top-k, log2 histograms)."""
import numpy as np


def test_top_tcp_mt_equals_single_thread(oracle):
    O = oracle
    G, n = 5000, 300_000
    cdf = O.zipf_cdf(G, 1.1)
    ev = O.gen_tcp(0xC2, 0, G, cdf, 0, n)
    g1, _, s1, r1, f1 = O.top_tcp(ev, 20)
    for T in (1, 3, 8):
        g2, s2, r2, f2 = O.top_tcp_mt(ev, 20, threads=T)
        assert g2 == g1 and np.array_equal(f2, f1) and np.array_equal(s2, s1) and np.array_equal(r2, r1)


def test_groupby_topk_mt_equals_single_thread(oracle):
    O = oracle
    G, n = 20_000, 200_000
    cdf = O.zipf_cdf(G, 1.05)
    a = O.gen_file(0xC5, 0, G, cdf, 0, n)
    keys = O.pad_keys(a, ("inode", "dev", "pid", "tid"))
    aggs = [{"kind": "count", "cond": a["op"], "cond_val": 0},
            {"kind": "sum", "val": a["count"], "cond": a["op"], "cond_val": 0},
            {"kind": "count", "cond": a["op"], "cond_val": 1},
            {"kind": "sum", "val": a["count"], "cond": a["op"], "cond_val": 1}]
    ok_, oa, of = O.groupby(keys, aggs)
    perm = O.go_sort_entries([(oa[3], "uint64", True)], len(of))[:20].astype(np.int64)
    for T in (1, 5):
        g, first, out = O.groupby_topk_mt(keys, aggs, sort=[(3, True)], k=20, threads=T)
        assert g == len(of) and np.array_equal(first, of[perm]) and np.array_equal(out[:, 3], oa[3][perm])
    e = O.gen_np(0xC4, 300, 3000, 0, n)
    keep = O.np_mark(e)
    rk, _, _ = O.groupby(O.pad_keys(e, ("src", "pkt", "peer", "port")), [{"kind": "count"}], valid=keep)
    g, _, _ = O.groupby_topk_mt(O.pad_keys(e, ("src", "pkt", "peer", "port")), [{"kind": "count"}], valid=keep,
                                threads=4)
    assert g == len(rk)


def test_hist_log2_mt_equals_single_thread(oracle):
    O = oracle
    q = O.lognormal_quantiles(np.log(2e5), 1.5)
    devs = [(8 << 20) | (16 * k) for k in range(16)]
    e = O.gen_bio(0xC3, q, 0, 500_000)
    ref = O.hist_log2(e["dev"], e["cont"], e["delta"], devs, 256)
    assert np.array_equal(O.hist_log2_mt(e["dev"], e["cont"], e["delta"], devs, 256, threads=6), ref)


def test_groupby_checksum_mt_equals_numpy_twin(oracle):
    """The whole-table checksum of or_groupby_topk_mt (C) equals group_checksum (numpy) over
    the single-thread restatement's groups, for any thread count; a changed aggregate, first
    index or key byte changes it (the full-size C4/C5 parity tests rest on this)."""
    O = oracle
    G, n = 20_000, 200_000
    a = O.gen_file(0xC5, 0, G, O.zipf_cdf(G, 1.05), 0, n)
    keys = O.pad_keys(a, ("inode", "dev", "pid", "tid"))
    aggs = [{"kind": "count", "cond": a["op"], "cond_val": 0},
            {"kind": "sum", "val": a["count"], "cond": a["op"], "cond_val": 1}]
    ok, oa, of = O.groupby(keys, aggs, base_idx=7)
    ref = O.group_checksum(ok, list(oa), of)
    for T in (1, 3):
        assert O.groupby_topk_mt(keys, aggs, base_idx=7, threads=T, checksum=True)[3] == ref
    oa2 = oa.copy()
    oa2[1][5] += 1
    assert O.group_checksum(ok, list(oa2), of) != ref
    of2 = of.copy()
    of2[9] += 1
    assert O.group_checksum(ok, list(oa), of2) != ref
    ok2 = ok.copy()
    ok2[3, 2] ^= 1
    assert O.group_checksum(ok2, list(oa), of) != ref
    e = O.gen_np(0xC4, 300, 3000, 0, n)
    keep = O.np_mark(e)
    nk = O.pad_keys(e, ("src", "pkt", "peer", "port"))
    rk, _, rf = O.groupby(nk, [], valid=keep)
    assert O.groupby_topk_mt(nk, [], valid=keep, threads=4, checksum=True)[3] == O.group_checksum(rk, [], rf)
