"""C1 step alone (FilterEntries + SortEntries of 1M trace-open events, bench.py's run_c1), for
kernel traces and A/Bs: python tools/c1_step.py [steps].  Prints ms per step."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    igx = importlib.import_module("inspektor-gadget_amd")
    E, H = igx.engine, igx.columns
    n = 1_000_000
    ev = E.gen_open(0xC1, H.to_device(E.zipf_cdf(64, 1.0)), 0, n)
    cols = igx.columns.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"),
                                ("comm", "string", 16), ("ret", "int64"), ("fd", "int64"),
                                ("err", "int64"), ("path", "uint32")])
    batch = igx.columns.EventBatch(cols, ev)
    out = None
    for i in range(steps + 3):
        if i == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        out = igx.sort.SortEntries(cols, igx.filter.FilterEntries(cols, batch, ["err:0", "pid:>=1000"]), ["comm", "-pid"])
    torch.cuda.synchronize()
    print(f"c1 {1e3 * (time.perf_counter() - t0) / steps:.3f} ms/step, {out.n} rows")


if __name__ == "__main__":
    main()
