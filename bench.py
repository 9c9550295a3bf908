"""Headline bench: top-tcp interval aggregation (BASELINE.json configs[1]).

One step = one `top tcp` interval over a resident batch of synthetic events:
  reset the device table (the per-interval map drain, tracer.go:154-171)
  -> keyed group-by of every event on the 8-field ip_key_t, summing sent / recv
     (tcptop.bpf.c:33-110; family filter :54-55 fused into the scan)
  -> stable top-20 by ["-sent","-recv"] with the reference's tie order (top.go:39-41)
  -> N>1: all-gather of the per-rank top-20 candidates over RCCL + exact global merge.
Events are hash-partitioned across GPUs at ingest (each rank owns its own key universe),
so per-GPU work is fixed as N grows ("scaling": "weak").

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` for the
group-by kernel (HIP events on the stream it runs on) and `cpu_baseline` (the oracle's
single-thread restatement of the reference's CPU path on a bounded sample, rank 0, N=1).
"""
import argparse
import importlib
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
METRIC = "events aggregated/sec (filter+group-by+top-K) at 1/2/4/8 MI355X; % HBM peak"   # BASELINE.json
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01", "traffic.json")   # tools/pmc_traffic.py
EV_BYTES = 71                  # saddr16 daddr16 mntns8 pid4 comm16 lport2 dport2 family2 size4 dir1
GROUP_BYTES = 90               # key 66 + sent 8 + recv 8 + first_idx 8


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--events", type=int, default=100_000_000, help="events per GPU per step")
    p.add_argument("--keys", type=int, default=1_000_000, help="key universe per GPU")
    p.add_argument("--zipf", type=float, default=1.1)
    p.add_argument("--topk", type=int, default=20)
    p.add_argument("--cpu-sample", type=int, default=48_000_000,
                   help="events in the CPU-baseline sample (0 = skip); ~10 s single-thread")
    p.add_argument("--check", action="store_true", help="verify the top-K against the oracle")
    return p.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    igx = importlib.import_module("inspektor-gadget_amd")
    from oracle import oracle as O   # only for the CDF table helper and the CPU baseline
    E, H, A = igx.engine, igx.columns, igx._abi

    N, G, K = a.events, a.keys, a.topk
    cdf_h = O.zipf_cdf(G, a.zipf)
    cdf = H.to_device(cdf_h, dev)
    base = rank * N                                   # global event index of row 0
    ev = E.gen_tcp(0xC2, rank, G, cdf, base, N)
    names = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family", "size", "dir")
    cols = [ev[k] for k in names]
    widths = [16, 16, 8, 4, 16, 2, 2, 2]
    aggs = [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)]
    tab = E.Table(widths, aggs, capacity=G + G // 4)
    # BPF probe filter: family in {AF_INET, AF_INET6} (tcptop.bpf.c:54-55) -> family <= 10
    fam = A.Pred()
    fam.col, fam.cmp, fam.negate, fam.ref_len = 7, A.CMP_LE, 0, 2
    fam.ref[0] = 10
    preds = [fam]
    torch.cuda.synchronize()

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gb_ms = []

    def step(record):
        tab.reset()
        if record:
            ev0.record()
        tab.update(cols, list(range(8)), N, base, preds)
        if record:
            ev1.record()
        fin = tab.finalize()                          # syncs: group count for the top-K
        Gn = fin["n_groups"]
        # SortStats(["-sent","-recv"]) over the table's groups, first K slots
        slots = tab.sort([(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, True)], K)
        cand = tab.gather(slots)                      # K rows: key 72 | sent | recv | first
        if world > 1:
            out = [torch.empty_like(cand) for _ in range(world)]
            dist.all_gather(out, cand)
            allc = torch.cat(out)
            cand = merge_candidates(E, H, allc, K)
        if record:
            gb_ms.append(ev0.elapsed_time(ev1))
        return cand, Gn

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        cand, Gn = step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_step = dt * 1000.0 / a.steps
    value = world * N * a.steps / dt

    gb_avg_ms = float(np.mean(gb_ms)) if gb_ms else float("nan")
    alg_bytes = N * EV_BYTES + Gn * GROUP_BYTES
    achieved = alg_bytes / (gb_avg_ms * 1e-3) / 1e9

    traffic, traffic_src = load_traffic(N, G, a.zipf)

    check = None
    if a.check and rank == 0 and world == 1:
        check = verify(O, cdf_h, G, N, K, cand, H)

    if rank == 0:
        cpu = None
        if a.cpu_sample and world == 1:
            cpu = cpu_baseline(O, cdf_h, G, a.cpu_sample, K)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "events/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based SplitMix64 stream, Zipf key ranks)",
            "config": {
                "workload": "top-tcp: filter family, group-by ip_key_t(saddr,daddr,mntns,pid,"
                            "comm,lport,dport,family) sum sent/recv, stable top-20 by "
                            "[-sent,-recv]",
                "events_per_gpu": N, "keys_per_gpu": G, "zipf_s": a.zipf, "topk": K,
                "groups_per_gpu": Gn,
                "parallelism": f"ingest-partitioned x{world}, RCCL all-gather top-K merge",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": "k_groupby<ip_key_t>", "kernel_ms": gb_avg_ms,
                "alg_bytes_per_launch": alg_bytes,
                "alg_bytes_def": f"{EV_BYTES} B/event x events + {GROUP_BYTES} B/group x groups",
                "traffic_source": traffic_src,
                "hbm_pct_of_peak_whole_step": 100.0 * alg_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
            },
            "cpu_baseline": cpu,
        }
        if check is not None:
            line["check"] = check
        print(json.dumps(line), flush=True)
    tab.destroy()
    if world > 1:
        dist.destroy_process_group()


def load_traffic(N, G, zipf):
    """HBM bytes per group-by launch measured by rocprofv3 PMC passes for this exact config
    (tools/pmc_traffic.py output, committed under profiles/); None when absent."""
    try:
        with open(TRAFFIC_FILE) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, None
    c = t.get("config", {})
    if (c.get("events"), c.get("keys"), c.get("zipf")) != (N, G, zipf):
        return None, None
    return t["traffic_bytes_per_launch"], os.path.relpath(TRAFFIC_FILE, ROOT) + " (bytes per launch)"


def merge_candidates(E, H, allc, K):
    """Exact global top-K over all ranks' candidates (keys are rank-disjoint)."""
    import torch
    sent = allc[:, 72:80].contiguous().view(torch.uint64).flatten()
    recv = allc[:, 80:88].contiguous().view(torch.uint64).flatten()
    first = allc[:, 88:96].contiguous().view(torch.uint64).flatten()
    idx = E.sort_perm([(sent, True), (recv, True)], allc.shape[0], pos=first, k=K)
    return E.take([allc], idx)[0]


def verify(O, cdf_h, G, N, K, cand, H):
    ev = O.gen_tcp(0xC2, 0, G, cdf_h, 0, N)
    Gref, keys, sent, recv, first = O.top_tcp(ev, K)
    c = H.host(cand)
    got_first = c[:, 88:96].copy().view(np.uint64).flatten()
    got_sent = c[:, 72:80].copy().view(np.uint64).flatten()
    ok = bool(np.array_equal(got_first, first) and np.array_equal(got_sent, sent))
    return {"oracle_groups": int(Gref), "topk_bit_exact": ok}


def cpu_baseline(O, cdf_h, G, S, K):
    """Single-thread restatement of the reference CPU path (BPF-map group-by per event,
    nextStats drain, SortEntries(-sent,-recv) via Go SliceStable, truncate) on S events."""
    ev = O.gen_tcp(0xC2, 0, G, cdf_h, 0, S)
    t0 = time.perf_counter()
    O.top_tcp(ev, K)
    dt = time.perf_counter() - t0
    try:
        cpu_model = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":")[1].strip()
    except Exception:
        cpu_model = platform.processor()
    return {"value": S / dt, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"{S} events of the same stream (keys {G}, zipf), oracle/igx_oracle.c "
                      f"or_top_tcp single thread, {dt:.2f} s",
            "cpu": cpu_model, "nproc": os.cpu_count()}


if __name__ == "__main__":
    main()
