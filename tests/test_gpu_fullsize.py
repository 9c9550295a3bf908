"""C2 at the exact bench size (BASELINE.json configs[1]: 100M events, 1M keys, Zipf 1.1,
family filter, top-20 by ["-sent","-recv"]) against the oracle:
  - group count;
  - the WHOLE group table through an order-independent checksum: every group's key fields,
    sent, recv and first index fingerprinted (oracle group_csum) and summed -- the device
    table is gathered to the host and fingerprinted by the numpy twin, the oracle computes
    its own inside the all-cores restatement (or_top_tcp_mt);
  - the top-20 rows bit-exact (first, sent, recv) -- the tie order of the reference sort.
"""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, G, K = 100_000_000, 1_000_000, 20


def test_c2_full_size_table_and_topk(oracle, igx, torch):
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    cdf = E.zipf_cdf(G, 1.1)
    ev = E.gen_tcp(0xC2, 0, G, H.to_device(cdf), 0, N)
    cols = [ev[k] for k in bench.TCP_NAMES] + [ev["size"].view(torch.int32)]
    tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2], [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)],
                  G + G // 4)
    tab.update(cols, list(range(8)), N, 0, [bench.family_in_pred(A, 7), bench.copied_pred(A, 10, 9)])
    fin = tab.finalize()
    top = H.host(tab.gather(tab.sort([(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, True)], K)))
    rows = H.host(bench.table_rows(E, torch, tab, fin))
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()
    # device packed key: saddr 0:16 daddr 16:32 mntns 32:40 pid 40:44 comm 44:60 lport 60:62
    # dport 64:66 family 68:70 (each column padded to 4 B) | sent 72 | recv 80 | first 88
    fields = np.concatenate([rows[:, 0:62], rows[:, 64:66], rows[:, 68:70]], axis=1)
    u64 = lambda o: rows[:, o:o + 8].copy().view(np.uint64).ravel()   # noqa: E731
    dev_cs = oracle.tcp_group_checksum(fields, u64(72), u64(80), u64(88))
    h = oracle.gen_tcp(0xC2, 0, G, cdf, 0, N)
    Gref, sent, recv, first, ref_cs = oracle.top_tcp_mt(h, K, checksum=True)
    assert fin["n_groups"] == Gref == rows.shape[0]
    assert dev_cs == ref_cs
    t64 = lambda o: top[:, o:o + 8].copy().view(np.uint64).ravel()    # noqa: E731
    assert np.array_equal(t64(88), first) and np.array_equal(t64(72), sent) and np.array_equal(t64(80), recv)


# ------------------------------------------------------------------------------------
# C3 / C4 / C5 at the bench's per-GPU size (125M events = the 8-GPU configs' 1B / 8), on the
# exact streams, table capacities and group-by modes bench.py runs
# ------------------------------------------------------------------------------------
NC = 125_000_000


def _table_check(oracle, E, H, torch, bench, tab, fin, naggs):
    """Whole device table -> (G, checksum) with the oracle's generic group fingerprint."""
    rows = H.host(bench.table_rows(E, torch, tab, fin))
    kb = fin["key_bytes"]
    u64 = lambda o: rows[:, o:o + 8].copy().view(np.uint64).ravel()   # noqa: E731
    cs = oracle.group_checksum(rows[:, :kb], [u64(kb + 8 * a) for a in range(naggs)], u64(kb + 8 * naggs))
    return rows.shape[0], cs


def test_c3_full_size_histogram(oracle, igx, torch):
    """profile block-io at 125M events: the whole u32[16*256][27] histogram equal to
    or_hist_log2_mt (biolatency.bpf.c:100-154 per event), including the slot-window path."""
    E, H = igx.engine, igx.columns
    bench = importlib.import_module("bench")
    q = E.lognormal_quantiles(*bench.C3_LOGNORMAL)
    ev = E.gen_bio(0xC3, H.to_device(q), 0, NC)
    hist = E.hist_log2(ev["dev"], ev["cont"], ev["delta"].view(torch.int64), bench.C3_DEVS, bench.C3_NCONT)
    hist2 = E.hist_log2(ev["dev"], ev["cont"], ev["delta"].view(torch.int64), bench.C3_DEVS, bench.C3_NCONT,
                        hist=hist.clone())          # accumulates onto a non-zero histogram
    got, got2 = H.host(hist), H.host(hist2)
    del ev
    torch.cuda.empty_cache()
    h = oracle.gen_bio(0xC3, q, 0, NC)
    ref = oracle.hist_log2_mt(h["dev"], h["cont"], h["delta"], bench.C3_DEVS, bench.C3_NCONT)
    assert int(ref.astype(np.uint64).sum()) > NC // 2
    assert np.array_equal(got, ref)
    assert np.array_equal(got2, (ref.astype(np.uint64) * 2).astype(np.uint32))


def test_c4_full_size_distinct(oracle, igx, torch):
    """advise network-policy at 125M events, cap 11M: the distinct-tuple count and a checksum
    of every (tuple, first index) equal or_groupby_topk_mt's (advisor.go:302-320, first event
    wins), for the bench's AUTO sequence (interval 1 cached and measured, then the
    capacity-derived partitioned plan) and each explicit form."""
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    ev = E.gen_np(*bench.C4_GEN, 0, NC)
    cols = [ev[k] for k in bench.C4_NAMES]
    tab = E.Table(bench.C4_WIDTHS, [], bench.C4_CAP)
    got = []
    for mode in (A.GB_AUTO, A.GB_AUTO, A.GB_AUTO, A.GB_CACHED, A.GB_PART, A.GB_DIRECT):
        tab.reset()
        tab.set_mode(mode)
        keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
        tab.update(cols, [0, 1, 2, 3], NC, 0, valid=keep)
        fin = tab.finalize()
        got.append((fin["n_groups"],) + _table_check(oracle, E, H, torch, bench, tab, fin, 0))
    tab.destroy()
    del ev, cols, keep
    torch.cuda.empty_cache()
    h = oracle.gen_np(*bench.C4_GEN, 0, NC)
    keys = oracle.pad_keys(h, bench.C4_NAMES)
    valid = oracle.np_mark(h)
    del h
    G, _, _, cs = oracle.groupby_topk_mt(keys, [], valid=valid, checksum=True)
    assert G > 10_000_000
    for i, (ng, nrows, dcs) in enumerate(got):
        assert ng == nrows == G, (i, ng, nrows, G)
        assert dcs == cs, i


def test_c5_full_size_table_and_topk(oracle, igx, torch):
    """top file at 125M events over 10M Zipf(1.05) keys, cap 12.5M: group count, a checksum of
    every (key, reads, rbytes, writes, wbytes, first) and the top-20 by [-wbytes] bit-exact vs
    or_groupby_topk_mt (filetop.bpf.c:68-92, SortStats), cached (AUTO) and partitioned."""
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    cdf = E.zipf_cdf(bench.C5_KEYS, bench.C5_ZIPF)
    ev = E.gen_file(0xC5, 0, bench.C5_KEYS, H.to_device(cdf), 0, NC)
    cols = [ev[k] for k in bench.C5_NAMES]
    tab = E.Table(bench.C5_WIDTHS, bench.c5_aggs(A), bench.C5_CAP)
    got = []
    for mode in (A.GB_AUTO, A.GB_AUTO, A.GB_PART):
        tab.reset()
        tab.set_mode(mode)
        tab.update(cols, [0, 1, 2, 3], NC, 0)
        fin = tab.finalize()
        top = H.host(tab.gather(tab.sort([(A.TSRC_AGG, 3, True)], bench.C5_TOPK)))
        got.append((fin["n_groups"],) + _table_check(oracle, E, H, torch, bench, tab, fin, 4) + (top,))
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()
    h = oracle.gen_file(0xC5, 0, bench.C5_KEYS, cdf, 0, NC)
    keys = oracle.pad_keys(h, ("inode", "dev", "pid", "tid"))
    G, first, aggs, cs = oracle.groupby_topk_mt(keys, bench.c5_oracle_aggs(h), sort=[(3, True)],
                                                k=bench.C5_TOPK, checksum=True)
    assert G > 5_000_000
    for i, (ng, nrows, dcs, top) in enumerate(got):
        assert ng == nrows == G, (i, ng, nrows, G)
        assert dcs == cs, i
        t64 = lambda o: top[:, o:o + 8].copy().view(np.uint64).ravel()    # noqa: E731
        assert np.array_equal(t64(52), first), i
        for a in range(4):
            assert np.array_equal(t64(20 + 8 * a), aggs[:, a]), (i, a)


# ------------------------------------------------------------------------------------
# the bench's own measured step, verbatim: bench.run_c2 / run_c5 at their default sizes with
# back-to-back asynchronous intervals (finalize(sync=False), the device-count top-K, no host
# sync inside a step; AUTO's loader / form switching between intervals), then bench's
# post-run check of the LAST interval against the oracle
# ------------------------------------------------------------------------------------
def _bench_ctx(igx, torch):
    import torch.distributed as dist
    bench = importlib.import_module("bench")
    return bench, bench.make_ctx(torch, dist, igx, 0, 1, torch.device("cuda", 0), True)


def test_bench_c2_async_intervals_match_oracle(igx, torch):
    bench, ctx = _bench_ctx(igx, torch)
    a = bench.parse(["--steps", "5", "--warmup", "1", "--cpu-sample", "0"])
    out = bench.run_c2(a, ctx)
    ck = out["check"]
    assert ck["groups_equal"] and ck["table_checksum_equal"] and ck["topk_equal"], ck
    assert ck["bit_exact"] is True


def test_bench_c5_async_intervals_match_oracle(igx, torch):
    bench, ctx = _bench_ctx(igx, torch)
    a = bench.parse(["--config-steps", "5", "--cpu-sample", "0"])
    out = bench.run_c5(a, ctx)
    ck = out["check"]
    assert ck["groups_equal"] and ck["table_checksum_equal"] and ck["topk_equal"], ck
    assert ck["bit_exact"] is True
    torch.cuda.empty_cache()


def test_auto_loader_choice_has_a_band(igx, torch):
    """AUTO's cached-form wave roles (igx_groupby_info: loaders, miss_permille): C2's stream
    (~35 % LDS misses) keeps 8 loader waves over 5 intervals; C5's (~42 %) moves to 7 after its
    first interval and stays there -- the switch has a band (on above 39 %, off below 37 %)."""
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    cdf = E.zipf_cdf(G, 1.1)
    ev = E.gen_tcp(0xC2, 0, G, H.to_device(cdf), 0, N)
    cols = [ev[k] for k in bench.TCP_NAMES] + [ev["size"].view(torch.int32)]
    tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2], [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)],
                  G + G // 4)
    c2 = []
    for _ in range(5):
        tab.reset()
        tab.update(cols, list(range(8)), N, 0, [bench.family_in_pred(A, 7), bench.copied_pred(A, 10, 9)])
        tab.finalize()
        c2.append(tab.info())
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()
    cdf5 = E.zipf_cdf(bench.C5_KEYS, bench.C5_ZIPF)
    ev = E.gen_file(0xC5, 0, bench.C5_KEYS, H.to_device(cdf5), 0, NC)
    cols = [ev[k] for k in bench.C5_NAMES]
    tab = E.Table(bench.C5_WIDTHS, bench.c5_aggs(A), bench.C5_CAP)
    c5 = []
    for _ in range(5):
        tab.reset()
        tab.update(cols, [0, 1, 2, 3], NC, 0)
        tab.finalize()
        c5.append(tab.info())
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()
    print("c2", [(i["loaders"], i["miss_permille"]) for i in c2], "c5", [(i["loaders"], i["miss_permille"]) for i in c5])
    assert all(i["form"] == A.GB_CACHED for i in c2 + c5)
    assert all(i["loaders"] == 8 for i in c2), c2
    assert all(300 < i["miss_permille"] < 370 for i in c2), c2
    assert all(i["loaders"] == 7 for i in c5), c5
    assert all(i["miss_permille"] > 390 for i in c5), c5
