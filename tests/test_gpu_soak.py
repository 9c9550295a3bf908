"""Soak: the bench's streams (C2, C4, C5 at their bench sizes) aggregated again and again into
the same table, interval after interval, exactly as bench.py steps them (reset, update,
finalize(sync=False), device-count top-K).  Every interval must produce the same table: the
group count, an order-independent fingerprint of every group's row (key | aggregates | first
index, hashed and summed on the device) and the top-K rows.  The protocol's races -- claims
published a round late, the occupancy byte map, LDS adoption, the miss and update rings --
would show here as an interval that differs; so would AUTO's switches between intervals
(C5: 8 -> 7 loader waves after the first interval; C4: cached, then the partitioned form with
its sampled re-probe every 17th interval), which must not change a single bit.  The first
interval of each stream is checked against the oracle by tests/test_gpu_fullsize.py.
"""
import importlib

import pytest

pytestmark = pytest.mark.gpu

INTERVALS = 100


def _fingerprint(torch, rows):
    """sum over rows of a 64-bit mix of the row's words (wrapping int64 arithmetic)."""
    G, rb = rows.shape
    wb = (rb + 7) // 8 * 8
    r = torch.zeros((G, wb), dtype=torch.uint8, device=rows.device)
    r[:, :rb] = rows
    w = r.view(torch.int64)
    x = torch.full((G,), 0x243F6A8885A308D3, dtype=torch.int64, device=rows.device)
    for j in range(w.shape[1]):
        x = (x ^ w[:, j]) * 0x100000001B3
        x = x ^ (x >> 29)
    return int(x.sum().item())


def _soak(torch, bench, E, tab, feed, sort, K):
    got = []
    for i in range(INTERVALS):
        tab.reset()
        feed()
        tab.finalize(sync=False)
        cand = tab.gather(tab.sort(sort, K)) if K else None
        G = tab.wait()
        rows = bench.table_rows(E, torch, tab, tab.fin)
        got.append((G, rows.shape[0], _fingerprint(torch, rows),
                    None if cand is None else cand.cpu().numpy().tobytes()))
        del rows
    for i, g in enumerate(got):
        assert g[0] == g[1] == got[0][0], (i, g[:2], got[0][0])
        assert g[2] == got[0][2], f"interval {i}: table fingerprint differs from interval 0"
        assert g[3] == got[0][3], f"interval {i}: top-K rows differ from interval 0"
    return got[0][0]


def test_soak_c2_intervals_identical(igx, torch):
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    fs = importlib.import_module("test_gpu_fullsize")
    cdf = E.zipf_cdf(fs.G, 1.1)
    ev = E.gen_tcp(0xC2, 0, fs.G, H.to_device(cdf), 0, fs.N)
    cols = [ev[k] for k in bench.TCP_NAMES] + [ev["size"].view(torch.int32)]
    tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2], [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)],
                  fs.G + fs.G // 4)
    preds = [bench.family_in_pred(A, 7), bench.copied_pred(A, 10, 9)]
    G = _soak(torch, bench, E, tab, lambda: tab.update(cols, list(range(8)), fs.N, 0, preds),
              [(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, True)], 20)
    assert G > 500_000
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()


def test_soak_c5_intervals_identical(igx, torch):
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    fs = importlib.import_module("test_gpu_fullsize")
    cdf = E.zipf_cdf(bench.C5_KEYS, bench.C5_ZIPF)
    ev = E.gen_file(0xC5, 0, bench.C5_KEYS, H.to_device(cdf), 0, fs.NC)
    cols = [ev[k] for k in bench.C5_NAMES]
    tab = E.Table(bench.C5_WIDTHS, bench.c5_aggs(A), bench.C5_CAP)
    G = _soak(torch, bench, E, tab, lambda: tab.update(cols, [0, 1, 2, 3], fs.NC, 0),
              [(A.TSRC_AGG, 3, True)], bench.C5_TOPK)
    assert G > 5_000_000
    assert tab.info()["loaders"] == 7   # AUTO moved C5 to 7 loader waves after interval 1
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()


def test_soak_c4_intervals_identical_across_forms(igx, torch):
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    fs = importlib.import_module("test_gpu_fullsize")
    ev = E.gen_np(*bench.C4_GEN, 0, fs.NC)
    cols = [ev[k] for k in bench.C4_NAMES]
    tab = E.Table(bench.C4_WIDTHS, [], bench.C4_CAP)
    forms = []

    def feed():
        keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
        tab.update(cols, [0, 1, 2, 3], fs.NC, 0, valid=keep)
        forms.append(tab.info()["form"])

    G = _soak(torch, bench, E, tab, feed, (), 0)
    assert G > 10_000_000
    assert forms[0] == A.GB_CACHED and A.GB_PART in forms, forms   # both forms, identical tables
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()
