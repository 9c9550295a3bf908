"""Diagnostics: the group-by forms (cached / direct / partitioned) on the bench configs' update
step, timed with HIP events; group counts printed so the forms can be compared.  Not part of
the product path or the tests.

    python tools/ablate_forms.py [--configs c2,c4,c5] [--forms cached,direct,part] [--reps 3]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def setups(E, H, A, torch, which):
    if which == "c2":
        n, G = 100_000_000, 1_000_000
        ev = E.gen_tcp(0xC2, 0, G, H.to_device(E.zipf_cdf(G, 1.1)), 0, n)
        cols = [ev[k] for k in ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family", "size", "dir")]
        return dict(n=n, widths=[16, 16, 8, 4, 16, 2, 2, 2], cols=cols, keys=list(range(8)),
                    aggs=[A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)], cap=G + G // 4, valid=None)
    if which == "c4":
        n = 125_000_000
        ev = E.gen_np(0xC4, 10_000, 100_000, 0, n)
        keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
        return dict(n=n, widths=[4, 1, 4, 2], cols=[ev[k] for k in ("src", "pkt", "peer", "port")],
                    keys=[0, 1, 2, 3], aggs=[], cap=11_000_000, valid=keep)
    n, G = 125_000_000, 10_000_000
    ev = E.gen_file(0xC5, 0, G, H.to_device(E.zipf_cdf(G, 1.05)), 0, n)
    return dict(n=n, widths=[8, 4, 4, 4], cols=[ev[k] for k in ("inode", "dev", "pid", "tid", "op", "count")],
                keys=[0, 1, 2, 3], cap=G + G // 4, valid=None,
                aggs=[A.Agg(A.AGG_COUNT, 0, 4, 8, 0), A.Agg(A.AGG_SUM, 5, 4, 8, 0),
                      A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 8, 1)])


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="c2,c4,c5")
    p.add_argument("--forms", default="cached,direct,part")
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    E, H, A = igx.engine, igx.columns, igx._abi
    modes = {"cached": A.GB_CACHED, "direct": A.GB_DIRECT, "part": A.GB_PART}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for c in a.configs.split(","):
        s = setups(E, H, A, torch, c)
        out = {"config": c, "events": s["n"]}
        for f in a.forms.split(","):
            tab = E.Table(s["widths"], s["aggs"], s["cap"])
            tab.set_mode(modes[f])
            ts = []
            for r in range(a.reps + 1):
                tab.reset()
                e0.record()
                tab.update(s["cols"], s["keys"], s["n"], 0, valid=s["valid"])
                e1.record()
                torch.cuda.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
            fin = tab.finalize()
            out[f + "_ms"] = float(np.median(ts))
            out[f + "_groups"] = fin["n_groups"]
            if s["aggs"]:   # a checksum of every aggregate, to compare the forms
                keys, aggs, first = E.table_tensors(tab, fin)
                out[f + "_sum"] = [int(H.host(x).astype(np.uint64).sum()) for x in aggs] + \
                                  [int(H.host(first).astype(np.uint64).sum())]
            else:
                keys, aggs, first = E.table_tensors(tab, fin)
                out[f + "_sum"] = [int(H.host(first).astype(np.uint64).sum())]
            tab.destroy()
            torch.cuda.empty_cache()
            print(json.dumps(out), flush=True)
        del s
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
