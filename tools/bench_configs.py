"""Per-config throughput of the other SURVEY.md §8(d) workloads on one MI355X (C1, C3, C4,
C5; C2 is bench.py's headline).  Each line: events/s, device ms per pass, algorithmic bytes
and the %-of-HBM-peak they imply, plus a bit-exact check of a reduced-size run against the
oracle.  Inputs are generated on the device (resident in HBM before timing).

    python tools/bench_configs.py [--only c1,c3,c4,c5] [--reps 5]

Per-GPU sizes are the 8-GPU configs' shares (1B events / 8 = 125M), weak-scaling style.
"""
import argparse
import ctypes as C
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def timed(torch, fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def line(name, n, ms, alg_bytes, extra):
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    d = {"config": name, "events": n, "ms": ms, "events_per_s": n / (ms * 1e-3),
         "alg_bytes": alg_bytes, "achieved_GBs": gbs, "hbm_frac": gbs / PEAK}
    d.update(extra)
    print(json.dumps(d), flush=True)


def c1(igx, O, torch, reps):
    """pkg/columns FilterEntries(["err:0","pid:>=1000"]) + SortEntries(["comm","-pid"]), 1M."""
    E, H, A = igx.engine, igx.columns, igx._abi
    n = 1_000_000
    ccdf = H.to_device(O.zipf_cdf(64, 1.0))
    ev = E.gen_open(0xC1, ccdf, 0, n)
    cols = igx.columns.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"),
                                ("comm", "string", 16), ("ret", "int64"), ("fd", "int64"),
                                ("err", "int64"), ("path", "uint32")])
    specs = igx.filter.GetFiltersFromStrings(cols, ["err:0", "pid:>=1000"])
    preds = [s.pred for s in specs]
    tcols = [ev[c.Name] for c in cols.GetOrderedColumns()]
    state = {}

    def run():
        idx = E.filter_rows(tcols, preds, n)
        comm, pid = E.take([ev["comm"], ev["pid"]], idx, n)
        state["perm"] = E.sort_perm([(comm, False), (pid, True)], idx.numel())
        state["idx"] = idx
    ms = timed(torch, run, reps)
    sel = state["idx"].numel()
    h = {k: H.host(v) for k, v in ev.items()}
    ocols = {"err": O.OCol("err", "int64", 8), "pid": O.OCol("pid", "uint32", 4)}
    osel = O.match_rows([O.parse_filter(ocols, "err:0"), O.parse_filter(ocols, "pid:>=1000")], h)
    operm = O.go_sort_entries([(h["comm"][osel], "string", False), (h["pid"][osel], "uint32", True)], len(osel))
    got = H.host(state["idx"]).astype(np.int64)[H.host(state["perm"]).astype(np.int64)]
    ok = bool(np.array_equal(got, osel[operm.astype(np.int64)]))
    line("C1 filter+sort", n, ms, n * 12 + sel * 24, {"selected": sel, "bit_exact_vs_oracle": ok,
                                                     "note": "launch-bound at 1M rows"})


def c3(igx, O, torch, reps, n):
    E, H = igx.engine, igx.columns
    q = O.lognormal_quantiles(np.log(2e5), 1.5)
    devs = [(8 << 20) | (16 * k) for k in range(16)]
    ev = E.gen_bio(0xC3, H.to_device(q), 0, n)
    delta = ev["delta"].view(torch.int64)
    hist = torch.zeros((4096, 27), dtype=torch.uint32, device="cuda")

    def run():
        hist.zero_()
        E.hist_log2(ev["dev"], ev["cont"], delta, devs, 256, hist=hist)
    ms = timed(torch, run, reps)
    m = 2_000_000
    h = {k: H.host(v[:m]) for k, v in ev.items()}
    small = H.host(E.hist_log2(ev["dev"][:m], ev["cont"][:m], delta[:m], devs, 256))
    ok = bool(np.array_equal(small, O.hist_log2(h["dev"], h["cont"], h["delta"], devs, 256)))
    line("C3 block-io log2 hist (4096 keys x 27)", n, ms, n * 16 + 4096 * 27 * 4,
         {"bit_exact_vs_oracle_2M": ok, "total": int(H.host(hist).sum())})


def c4(igx, O, torch, reps, n):
    E, H, A = igx.engine, igx.columns, igx._abi
    ev = E.gen_np(0xC4, 10_000, 100_000, 0, n)
    names = ("src", "pkt", "peer", "port")
    tab = E.Table([4, 1, 4, 2], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], 11_000_000)
    st = {}

    def run():
        tab.reset()
        keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
        tab.update([ev[k] for k in names], [0, 1, 2, 3], n, 0, valid=keep)
        st["fin"] = tab.finalize()
    ms = timed(torch, run, reps)
    ng = st["fin"]["n_groups"]
    tab.destroy()
    m = 1_000_000
    t2 = E.Table([4, 1, 4, 2], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], m)
    sub = {k: v[:m] for k, v in ev.items()}
    keep = E.np_mark(sub["type"], sub["pkt"], sub["hostip"], sub["raddr"])
    t2.update([sub[k] for k in names], [0, 1, 2, 3], m, 0, valid=keep)
    fin = t2.finalize()
    keys, aggs, first = E.table_tensors(t2, fin)
    h = {k: H.host(v) for k, v in sub.items()}
    ok_, oa, of = O.groupby(O.pad_keys(h, names), [{"kind": "count"}], valid=O.np_mark(h))
    got = {bytes(k): (int(a), int(f)) for k, a, f in zip(H.host(keys), H.host(aggs[0]), H.host(first))}
    ok = got == {bytes(k): (int(a), int(f)) for k, a, f in zip(ok_, oa[0], of)}
    t2.destroy()
    line("C4 network-policy distinct (mark + dedup + finalize)", n, ms, n * 24 + ng * 20,
         {"distinct": ng, "bit_exact_vs_oracle_1M": bool(ok)})


def c5(igx, O, torch, reps, n, G):
    E, H, A = igx.engine, igx.columns, igx._abi
    cdf = H.to_device(O.zipf_cdf(G, 1.05))
    ev = E.gen_file(0xC5, 0, G, cdf, 0, n)
    names = ("inode", "dev", "pid", "tid", "op", "count")
    aggs = [A.Agg(A.AGG_COUNT, 0, 4, 8, 0), A.Agg(A.AGG_SUM, 5, 4, 8, 0),
            A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 8, 1)]
    tab = E.Table([8, 4, 4, 4], aggs, G + G // 4)
    st = {}

    def run():
        tab.reset()
        tab.update([ev[k] for k in names], [0, 1, 2, 3], n, 0)
        st["fin"] = tab.finalize()
        slots = tab.sort([(A.TSRC_AGG, 3, True)], 20)    # ["-wbytes"]
        st["rows"] = tab.gather(slots)
    ms = timed(torch, run, reps)
    ng = st["fin"]["n_groups"]
    tab.destroy()
    line("C5 top file (group-by 4 aggs + top-20 -wbytes)", n, ms, n * 25 + ng * 60,
         {"keys": G, "groups": ng})


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--only", default="c1,c3,c4,c5")
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--events", type=int, default=125_000_000)
    a = p.parse_args()
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    from oracle import oracle as O
    todo = a.only.split(",")
    if "c1" in todo:
        c1(igx, O, torch, a.reps)
    if "c3" in todo:
        c3(igx, O, torch, a.reps, a.events)
    if "c4" in todo:
        c4(igx, O, torch, a.reps, a.events)
    if "c5" in todo:
        c5(igx, O, torch, a.reps, a.events, 1_250_000)


if __name__ == "__main__":
    main()
