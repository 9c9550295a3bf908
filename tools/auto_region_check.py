"""Diagnostics: AUTO on a miss-heavy stream with one hot key (5% of the rows).  Interval 1
runs cached and measures the misses, interval 2 the partitioned region variant (the hot
key's bucket overflows its region), later ones the exact variant.  Prints ms per interval
and checks every interval's group count against numpy.

  python tools/auto_region_check.py            AUTO
  IGX_GB_MODE=1 python tools/auto_region_check.py                       cached every interval
  IGX_GB_MODE=3 IGX_GBP_REGION=1 python tools/auto_region_check.py      interval 0: region variant
                                                                        with overflow, then exact"""
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
igx = importlib.import_module("inspektor-gadget_amd")
E, H, A = igx.engine, igx.columns, igx._abi
n = 20_000_000
rng = np.random.default_rng(5)
keys = rng.integers(1, 50_000_000, n, dtype=np.uint32)
keys[rng.random(n) < 0.05] = 0
want = len(np.unique(keys))
kd = H.to_device(keys)
tab = E.Table([4], [A.Agg(A.AGG_COUNT, 0, A.NO_COL, 8, 0)], 30_000_000)
for it in range(5):
    tab.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tab.update([kd], [0], n, 0)
    g = tab.finalize()["n_groups"]
    torch.cuda.synchronize()
    print(f"interval {it}: {1e3 * (time.perf_counter() - t0):.2f} ms, groups {g} (want {want})", flush=True)
    assert g == want
tab.destroy()
