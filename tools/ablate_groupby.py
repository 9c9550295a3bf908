"""Diagnostics: time k_groupby variants in one process (interleaved rounds) to find where
the time goes.  Not part of the product path or the tests.

    python tools/ablate_groupby.py --events 100000000 --keys 1000000 --zipf 1.1
    python tools/ablate_groupby.py --layout file --events 125000000 --keys 10000000 --zipf 1.05 --variants 0
Variants (IGX_GB_DEBUG bits, read per launch; the top-file key only in an IGX_GB_DEBUG_FILE build): 0 full, 1 load+hash only, 2 stop after the
LDS lookup (misses dropped), 4 no HBM atomics on misses, 8 full + hit/miss counters.
"""
import argparse
import ctypes as C
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--events", type=int, default=100_000_000)
    p.add_argument("--keys", type=int, default=1_000_000)
    p.add_argument("--zipf", type=float, default=1.1)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--variants", default="0,1,2,4,8")
    p.add_argument("--noreset", action="store_true", help="keep the table between launches (no new keys after the first)")
    p.add_argument("--layout", choices=("tcp", "file"), default="tcp")
    a = p.parse_args()
    variants = [int(x) for x in a.variants.split(",")]
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    from oracle import oracle as O
    E, H, A = igx.engine, igx.columns, igx._abi
    N, G = a.events, a.keys
    cdf = H.to_device(O.zipf_cdf(G, a.zipf))
    if a.layout == "tcp":
        ev = E.gen_tcp(0xC2, 0, G, cdf, 0, N)
        names = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family", "size", "dir")
        cols = [ev[k] for k in names]
        tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2],
                      [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)], G + G // 4)
        nkey = 8
    else:   # bench.py's C5: file_id key, reads / rbytes / writes / wbytes
        bench = importlib.import_module("bench")
        ev = E.gen_file(0xC5, 0, G, cdf, 0, N)
        cols = [ev[k] for k in bench.C5_NAMES]
        tab = E.Table(bench.C5_WIDTHS, bench.c5_aggs(A), G + G // 4)
        nkey = 4
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for r in range(a.rounds):
        for v in variants:
            os.environ["IGX_GB_DEBUG"] = str(v)
            if not a.noreset:
                tab.reset()
            elif r == 0 and v == variants[0]:
                tab.update(cols, list(range(nkey)), N, 0)   # populate: later launches find every key
            e0.record()
            tab.update(cols, list(range(nkey)), N, 0)
            e1.record()
            if not a.noreset:
                tab.finalize()   # lists the groups: the next reset keeps the keys (a generation)
            torch.cuda.synchronize()
            res.setdefault(v, []).append(e0.elapsed_time(e1))
            if v & (8 | 65536 | 262144):
                cnt = (C.c_uint64 * 32)()
                tab.ctx.check(tab.ctx.L.igx_groupby_debug_counts(tab.h, cnt))
                if v & 8:
                    res.setdefault("hits_misses", []).append([cnt[0], cnt[1]])
                if v & 65536:
                    res.setdefault("waits_lfull_pempty_ufull_sidle", []).append([cnt[4], cnt[5], cnt[6], cnt[7]])
                if v & 262144:
                    res.setdefault("atomics", []).append(
                        {"server_updates": cnt[8], "server_minima": cnt[9], "server_record_requests": cnt[10],
                         "server_line_requests": cnt[11], "server_straddles": cnt[12],
                         "server_pairs_by_32_16_8_lanes": [cnt[13], cnt[14], cnt[15]], "flush_updates": cnt[16],
                         "flush_record_requests": cnt[18], "flush_minima": cnt[20],
                         "claims": tab.info()["claims"]})
    os.environ.pop("IGX_GB_DEBUG", None)
    out = {str(k): (float(np.median(v)) if not isinstance(k, str) else (v if k.startswith("atomics") else v[-1]))
           for k, v in res.items()}
    out["launch_ms"] = {str(k): v for k, v in res.items() if not isinstance(k, str)}
    if hasattr(tab, "info"):
        out["claims_last"] = tab.info()["claims"]
    out.update({"events": N, "keys": G, "zipf": a.zipf, "layout": a.layout, "noreset": a.noreset})
    print(json.dumps(out))
    tab.destroy()


if __name__ == "__main__":
    main()
