"""Diagnostics (not product, not tests): where FilterEntries' wall time goes as the batch grows
(tools/filter_scale.py saw 0.12 ms at 4M rows and 21 ms at 16M).  Per size, the median over
reps of each phase, with a device synchronisation after each:
  cols   batch.tensors_in_schema_order()
  call   engine.filter_rows(..., device_count=True)  (igx_filter_ex: mark + compaction launches)
  sync   torch.cuda.synchronize() after the call (the kernels)
  count  reading the selected count (.item())
    python tools/filter_cliff.py [--sizes 4000000,8000000,12000000,16000000]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=9)
    p.add_argument("--sizes", default="4000000,8000000,12000000,16000000")
    a = p.parse_args()
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    E, H = igx.engine, igx.columns
    cols = igx.columns.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"), ("comm", "string", 16),
                                ("ret", "int64"), ("fd", "int64"), ("err", "int64"), ("path", "uint32")])
    for n in [int(x) for x in a.sizes.split(",")]:
        ev = E.gen_open(0xC1, H.to_device(E.zipf_cdf(64, 1.0)), 0, n)
        batch = igx.columns.EventBatch(cols, ev)
        specs = [igx.filter.GetFilterFromString(cols, f) for f in ("err:0", "pid:>=1000")]
        ph = {"cols": [], "call": [], "sync": [], "count": [], "whole": []}
        torch.cuda.synchronize()
        for r in range(a.reps + 2):
            t0 = time.perf_counter()
            ts = batch.tensors_in_schema_order()
            t1 = time.perf_counter()
            idx, cnt = E.filter_rows(ts, [s.pred for s in specs], batch.n, batch.valid, device_count=True)
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            m = int(cnt.item())
            t4 = time.perf_counter()
            f = igx.filter.FilterEntries(cols, batch, ["err:0", "pid:>=1000"])
            _ = f.n
            t5 = time.perf_counter()
            if r >= 2:
                for k, v in (("cols", t1 - t0), ("call", t2 - t1), ("sync", t3 - t2), ("count", t4 - t3),
                             ("whole", t5 - t4)):
                    ph[k].append(v * 1e3)
        print(json.dumps({"rows": n, "selected": m,
                          "ms": {k: round(sorted(v)[len(v) // 2], 4) for k, v in ph.items()}}), flush=True)
        del ev, batch, idx, cnt, f
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
