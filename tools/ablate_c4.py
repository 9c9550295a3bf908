"""Diagnostics: C4 (advise network-policy distinct) group-by forms, timed with HIP events.
Not part of the product path or the tests.

    python tools/ablate_c4.py [--events 125000000]
Prints ms per update for: cached / direct form, distinct (0 aggs) / COUNT, and the direct
form on a table that already holds every key (no claims: the probe-only cost)."""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--events", type=int, default=125_000_000)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    E, A = igx.engine, igx._abi
    n = a.events
    ev = E.gen_np(0xC4, 10_000, 100_000, 0, n)
    cols = [ev[k] for k in ("src", "pkt", "peer", "port")]
    keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {"events": n}
    for name, aggs, mode, reset in [("cached_distinct", [], A.GB_CACHED, True),
                                    ("direct_distinct", [], A.GB_DIRECT, True),
                                    ("direct_count", [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], A.GB_DIRECT, True),
                                    ("direct_distinct_noclaims", [], A.GB_DIRECT, False)]:
        tab = E.Table([4, 1, 4, 2], aggs, 11_000_000)
        tab.set_mode(mode)
        ts = []
        for r in range(a.reps + 1):
            if reset or r == 0:
                tab.reset()
            e0.record()
            tab.update(cols, [0, 1, 2, 3], n, 0, valid=keep)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        out[name] = float(np.median(ts))
        out[name + "_groups"] = tab.finalize()["n_groups"]
        tab.destroy()
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
