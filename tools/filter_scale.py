"""ADVICE r05 (k_filter.hip k_filter_compact_sf): the fused compaction sums its tile's
predecessors itself, so its work grows with the square of the tile count.  Time
FilterEntries([err:0, pid:>=1000]) over 1M / 4M / 16M trace-open events with the fused form
(up to IGX_FILTER_SF_MAX tiles) and with the two-kernel scan + compaction (IGX_FILTER_SF_MAX=0),
interleaved on one GPU, and check both give the same rows.  Prints one JSON line.
    python tools/filter_scale.py [--reps 30]
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
    p.add_argument("--reps", type=int, default=30)
    p.add_argument("--sizes", default="1000000,4000000,16000000")
    a = p.parse_args()
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    E, H = igx.engine, igx.columns
    cols = igx.columns.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"), ("comm", "string", 16),
                                ("ret", "int64"), ("fd", "int64"), ("err", "int64"), ("path", "uint32")])
    out = {}
    for n in [int(x) for x in a.sizes.split(",")]:
        ev = E.gen_open(0xC1, H.to_device(E.zipf_cdf(64, 1.0)), 0, n)
        batch = igx.columns.EventBatch(cols, ev)
        res, sels = {}, {}
        for rep in range(a.reps + 2):
            for v, env in (("fused", None), ("two_kernel", "0")):
                if env is None:
                    os.environ.pop("IGX_FILTER_SF_MAX", None)
                else:
                    os.environ["IGX_FILTER_SF_MAX"] = env
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                f = igx.filter.FilterEntries(cols, batch, ["err:0", "pid:>=1000"])
                m = f.n
                dt = (time.perf_counter() - t0) * 1e3
                if rep >= 2:
                    res.setdefault(v, []).append(dt)
                sels[v] = (m, H.host(f.sel[:m]).tobytes() if f.sel is not None else b"")
        os.environ.pop("IGX_FILTER_SF_MAX", None)
        tiles = (n + 1023) // 1024
        out[str(n)] = {"tiles": tiles, "ms": {k: sorted(v)[len(v) // 2] for k, v in res.items()},
                       "same_rows": sels["fused"] == sels["two_kernel"], "selected": sels["fused"][0]}
        del ev, batch
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
