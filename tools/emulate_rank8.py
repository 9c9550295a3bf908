"""Rank 0 of an 8-GPU C4 / C5 step, emulated on one GPU: what the N > 1
step adds on each rank besides the aggregation itself, with the xGMI transfer left out.

For each config, eight slices of ONE global stream (bench.py's shapes: 125M events per rank,
batch 0) are aggregated into a partial table in turn; each is partitioned by owner straight from
the table (igx_partition_groups) and the rows owner 0 would receive are kept.  Then rank 0's
step after its own update is timed over `--reps` repetitions, each phase with HIP events on the
library's stream:
  finalize   igx_groupby_finalize_async of rank 0's partial table
  partition  igx_partition_groups(8) + the send counts read back (the step's one host read)
  merge      the owner merge of the 8 received parts: reset + update_ex + finalize_async, into a
             table sized from the owner's share (dist.owner_capacity for C5; C4 keeps its
             capacity: its tuple universe is not bounded by one rank's)
  topk       C5: the owner's top-20 (device count) + gather
and the update itself for scale.  Writes profiles/r06/emulated_rank8.json (--out).
    python tools/emulate_rank8.py [--events 125000000] [--reps 10]
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
    p.add_argument("--events", type=int, default=125_000_000)
    p.add_argument("--ranks", type=int, default=8)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--configs", default="c5,c4")
    p.add_argument("--merge-mode", default="cached", choices=("auto", "cached", "direct", "part"),
                   help="the owner table's group-by form (igx_groupby_set_mode)")
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "emulated_rank8.json"))
    a = p.parse_args()
    import torch
    igx = importlib.import_module("inspektor-gadget_amd")
    bench = importlib.import_module("bench")
    E, H, A, D = igx.engine, igx.columns, igx._abi, igx.dist
    torch.cuda.set_device(0)
    n, WS = a.events, a.ranks
    res = {"ranks": WS, "events_per_rank": n, "reps": a.reps, "merge_mode": a.merge_mode,
           "what": __doc__.split("\n\n")[1].strip()}

    def ev_ms(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        return out, (e0, e1)

    for cfg in a.configs.split(","):
        if cfg == "c5":
            cdf = H.to_device(E.zipf_cdf(bench.C5_KEYS, bench.C5_ZIPF))
            names, widths, aggs, cap = bench.C5_NAMES, bench.C5_WIDTHS, bench.c5_aggs(A), bench.C5_CAP
            gen = lambda r: E.gen_file(0xC5, 0, bench.C5_KEYS, cdf, r * n, n)   # noqa: E731
            own_cap, ow = D.owner_capacity(cap, WS), [8, 8, 8, 8]
            own_aggs = [A.Agg(A.AGG_SUM, 4 + x, A.NO_COL, 8, 0) for x in range(4)]
        else:
            names, widths, aggs, cap = bench.C4_NAMES, bench.C4_WIDTHS, [], bench.C4_CAP
            gen = lambda r: E.gen_np(*bench.C4_GEN, r * n, n)                   # noqa: E731
            own_cap, ow, own_aggs = cap, [], []
        tab = E.Table(widths, aggs, cap)

        def update(ev, r):
            if cfg == "c4":
                keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
                tab.update([ev[k] for k in names], [0, 1, 2, 3], n, r * n, valid=keep)
            else:
                tab.update([ev[k] for k in names], [0, 1, 2, 3], n, r * n)

        recv = []
        for r in range(WS - 1, -1, -1):          # rank 0's slice last: its table stays for the timing
            ev = gen(r)
            tab.reset()
            update(ev, r)
            tab.finalize(sync=False)
            rows, cnt = tab.partition(WS)
            counts = cnt.cpu().tolist()
            recv.append(rows[:counts[0]].clone())
            if r:
                del ev
        mine = torch.cat(recv[::-1])
        own = E.Table(widths, own_aggs, own_cap)
        own.set_mode({"auto": A.GB_AUTO, "cached": A.GB_CACHED, "direct": A.GB_DIRECT, "part": A.GB_PART}[a.merge_mode])
        t = {"update": [], "finalize": [], "partition": [], "merge": [], "topk": [], "wall_after_update": []}
        for rep in range(a.reps + 2):
            torch.cuda.synchronize()
            tab.reset()
            _, eu = ev_ms(lambda: update(ev, 0))
            torch.cuda.synchronize()
            w0 = time.perf_counter()
            _, ef = ev_ms(lambda: tab.finalize(sync=False))
            (rows, cnt), ep = ev_ms(lambda: tab.partition(WS))
            counts = cnt.cpu().tolist()
            _, em = ev_ms(lambda: D.merge_partials(mine, widths, ow, own_cap, table=own, sync=False))
            ek = None
            if cfg == "c5":
                _, ek = ev_ms(lambda: own.gather(own.sort([(A.TSRC_AGG, 3, True)], bench.C5_TOPK)))
            torch.cuda.synchronize()
            wall = (time.perf_counter() - w0) * 1e3
            if rep < 2:
                continue
            for k, e in (("update", eu), ("finalize", ef), ("partition", ep), ("merge", em), ("topk", ek)):
                if e is not None:
                    t[k].append(e[0].elapsed_time(e[1]))
            t["wall_after_update"].append(wall)
        G, Gown = tab.wait(), own.wait()
        avg = {k: (sum(v) / len(v) if v else None) for k, v in t.items()}
        added = sum(avg[k] for k in ("finalize", "partition", "merge", "topk") if avg[k] is not None)
        res[cfg] = {"ms": avg, "added_ms": added, "partial_groups": G, "sent_to_owner0": counts[0],
                    "received_rows": int(mine.shape[0]), "owner_groups": Gown, "owner_capacity": own_cap,
                    "partial_capacity": cap}
        print(cfg, json.dumps(res[cfg]), flush=True)
        tab.destroy()
        own.destroy()
        del mine, recv, ev
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
