"""Diagnostics: the partitioned group-by form's passes on the bench configs, by stopping the
pipeline early / skipping work with IGX_GBP_DEBUG (results invalid except for dbg 0).
Not part of the product path or the tests.

    python tools/ablate_part.py [--configs c4,c5] [--dbg 0,257,256,512,516,8,32,64,16]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ablate_forms import setups  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="c4,c5")
    p.add_argument("--dbg", default="0,257,256,512,516,8,32,64,16")
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    E, H, A = igx.engine, igx.columns, igx._abi
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for c in a.configs.split(","):
        s = setups(E, H, A, torch, c)
        tab = E.Table(s["widths"], s["aggs"], s["cap"])
        tab.set_mode(A.GB_PART)
        out = {"config": c}
        for d in a.dbg.split(","):
            os.environ["IGX_GBP_DEBUG"] = d
            ts = []
            for r in range(a.reps + 1):
                tab.reset()
                e0.record()
                tab.update(s["cols"], s["keys"], s["n"], 0, valid=s["valid"])
                e1.record()
                torch.cuda.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
            out[d] = round(float(np.median(ts)), 3)
            if d == "0":
                out["groups"] = tab.finalize()["n_groups"]
        os.environ.pop("IGX_GBP_DEBUG", None)
        print(json.dumps(out), flush=True)
        tab.destroy()
        del s
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
