"""Headline bench: top-tcp interval aggregation (BASELINE.json configs[1]), plus the other
SURVEY.md §8(d) configs in the same run.

One headline step = one `top tcp` interval over a resident batch of synthetic events:
  reset the device table (the per-interval map drain, tracer.go:154-171)
  -> keyed group-by of every event on the 8-field ip_key_t, summing sent / recv, with the
     probes' checks fused in (tcptop.bpf.c:33-131; `family in {AF_INET, AF_INET6}` :54-55 as
     an IGX_CMP_IN predicate, the receive probe's `copied <= 0` drop :127-128 as a guarded
     `copied > 0`, the same ones gadgets.TopTcpTracer uses)
  -> stable top-20 by ["-sent","-recv"] with the reference's tie order (top.go:39-41)
  -> N>1: all-gather of the per-rank top-20 candidates over RCCL + exact global merge.
Events are hash-partitioned across GPUs at ingest (each rank owns its own key universe),
so per-GPU work is fixed as N grows ("scaling": "weak").

The other configs (`--configs`, default c1,c3,c4,c5) run after the headline with their own
timed steps and land in the line's "configs" object, each with its roofline and (rank 0,
N=1) CPU baselines.  At N>1 their collectives are inside the timed region: C3 all-reduces
the histogram, C4 and C5 exchange partial groups by key owner (every rank holds a slice of
ONE global stream and key universe), C5 all-gathers the owners' top-20.

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` for the
group-by kernel (HIP events on the stream it runs on) and `cpu_baseline` (the oracle's
restatement of the reference's CPU path on a bounded sample, all host cores, with the
single-thread number beside it; rank 0, N=1).

After each config's timed loop (outside the timed region) the LAST timed interval's output --
the very tables, histogram and top-K the measured steps produced -- is checked against the
oracle on the same stream (`check` in each config, `check` at the top level for C2; default on,
`--no-check` skips it).  A mismatch makes the process exit 3 after the line is printed.
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
PROFILE_DIR = os.path.join(ROOT, "profiles", "r06")
EV_BYTES = 71                  # saddr16 daddr16 mntns8 pid4 comm16 lport2 dport2 family2 size4 dir1
GROUP_BYTES = 90               # key 66 + sent 8 + recv 8 + first_idx 8
TCP_NAMES = ("saddr", "daddr", "mntns", "pid", "comm", "lport", "dport", "family", "size", "dir")
# per-config inputs (shared with tests/test_gpu_fullsize.py, which checks these exact streams)
C3_DEVS = [(8 << 20) | (16 * k) for k in range(16)]
C3_NCONT = 256
C3_LOGNORMAL = (float(np.log(2e5)), 1.5)
C4_GEN = (0xC4, 10_000, 100_000)               # seed, sources, peers
C4_NAMES, C4_WIDTHS, C4_CAP = ("src", "pkt", "peer", "port"), [4, 1, 4, 2], 11_000_000
C5_KEYS, C5_ZIPF, C5_TOPK = 10_000_000, 1.05, 20
C5_NAMES, C5_WIDTHS = ("inode", "dev", "pid", "tid", "op", "count"), [8, 4, 4, 4]
C5_CAP = C5_KEYS + C5_KEYS // 4


def c5_aggs(A):
    """filetop.bpf.c:68-92: reads / rbytes (op 0 = READ), writes / wbytes (op 1 = WRITE)."""
    return [A.Agg(A.AGG_COUNT, 0, 4, 8, 0), A.Agg(A.AGG_SUM, 5, 4, 8, 0),
            A.Agg(A.AGG_COUNT, 0, 4, 8, 1), A.Agg(A.AGG_SUM, 5, 4, 8, 1)]


def c5_oracle_aggs(h):
    return [{"kind": "count", "cond": h["op"], "cond_val": 0},
            {"kind": "sum", "val": h["count"], "cond": h["op"], "cond_val": 0},
            {"kind": "count", "cond": h["op"], "cond_val": 1},
            {"kind": "sum", "val": h["count"], "cond": h["op"], "cond_val": 1}]


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--events", type=int, default=100_000_000, help="events per GPU per step")
    p.add_argument("--keys", type=int, default=1_000_000, help="key universe per GPU")
    p.add_argument("--zipf", type=float, default=1.1)
    p.add_argument("--topk", type=int, default=20)
    p.add_argument("--cpu-sample", type=int, default=48_000_000,
                   help="events in the C2 CPU-baseline sample (0 = skip every CPU baseline)")
    p.add_argument("--configs", default="c1,c3,c4,c5",
                   help="other configs to run after the headline ('' = none)")
    p.add_argument("--config-events", type=int, default=125_000_000,
                   help="events per GPU for C3/C4/C5 (the 8-GPU configs' 1B / 8)")
    p.add_argument("--config-steps", type=int, default=20,
                   help="timed steps per other config (C1 at 5 steps: 0.20-0.22 ms, at 50: 0.17 -- the "
                        "closing synchronisation weighs on a 0.2 ms step)")
    p.add_argument("--batches", type=int, default=0,
                   help="C2 / C5: pre-generated batches the intervals step through -- consecutive slices of one "
                        "stream (same key universe and Zipf law, different events), so the keys an interval finds "
                        "already in the table recur because the stream repeats them, never because a batch is "
                        "replayed.  0 = one slice per interval (warmup + steps), as many as --input-gb holds; "
                        "past that the slices rotate")
    p.add_argument("--input-gb", type=float, default=150.0,
                   help="HBM for the C2 / C5 input slices (--batches 0)")
    p.add_argument("--no-check", dest="check", action="store_false",
                   help="skip the post-run check of each config's last timed interval against the oracle")
    p.add_argument("--transport", choices=("igx", "torch"), default="torch",
                   help="N>1 exchanges: torch's collectives (RCCL on the nccl group; the default until "
                        "the igx_dist_* send/recv loops have run with two or more GPUs) or the igx_dist_* "
                        "C ABI over RCCL (falls back to torch's if igx_dist_init fails on any rank)")
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="N>1 process group: nccl (RCCL over xGMI, one GPU per rank) or gloo -- a rehearsal of the "
                        "N>1 path whose ranks may share one GPU (tests/test_gpu_bench_dist.py); the product's "
                        "igx_dist_* transport needs one GPU per rank and is then reported unavailable")
    p.add_argument("--launch-dry-run", action="store_true",
                   help="launcher self-test: each rank prints its RANK/WORLD_SIZE and exits, no GPU")
    return p.parse_args(argv)


def n_batches(a, steps, event_bytes, n):
    """Slices of the stream a config steps through: one per interval when they fit --input-gb."""
    if a.batches > 0:
        return a.batches
    fit = int(a.input_gb * 1e9 // (event_bytes * n))
    return max(2, min(steps, fit))


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a):
    """`--gpus N` (N > 1) without a torch.distributed launcher: start N rank processes of this
    script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each), before this process
    makes any torch or HIP call.  Rank 0 prints the JSON line; the exit status is the first
    failing rank's (the others are then terminated), else 0."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    return status


class Timer:
    """Wall time of K steps bracketed by barrier + synchronize, max over ranks; plus the
    dominant kernel's HIP-event time on the stream it runs on."""

    def __init__(self, torch, dist, world, dev):
        self.torch, self.dist, self.world, self.dev = torch, dist, world, dev

    def sync(self):
        self.torch.cuda.synchronize()
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def run(self, step, steps, warmup):
        for _ in range(warmup):
            step(False)
        self.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(True)
        self.sync()
        dt = time.perf_counter() - t0
        if self.world > 1:
            t = self.torch.tensor([dt], dtype=self.torch.float64, device=self.dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt


class KernelClock:
    """HIP events around the dominant kernel's launch on torch's current stream (the stream
    libigx launches on: runtime.Context binds it); read after the timed loop, so timing adds
    no host synchronisation to a step."""

    def __init__(self, torch):
        self.torch = torch
        self.pairs = []
        self.on = False

    def __enter__(self):
        if self.on:
            e0 = self.torch.cuda.Event(enable_timing=True)
            e0.record()
            self.pairs.append([e0, None])
        return self

    def __exit__(self, *exc):
        if self.on:
            e1 = self.torch.cuda.Event(enable_timing=True)
            e1.record()
            self.pairs[-1][1] = e1
        return False

    def avg(self):
        if not self.pairs:
            return float("nan")
        self.torch.cuda.synchronize()
        return float(np.mean([e0.elapsed_time(e1) for e0, e1 in self.pairs]))


def roofline(alg_bytes, kernel_ms, kernel, alg_def, traffic_key, match):
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic, src = load_traffic(traffic_key, match)
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kernel, "kernel_ms": kernel_ms,
            "alg_bytes_per_launch": alg_bytes, "alg_bytes_def": alg_def, "traffic_source": src}


def load_traffic(key, match):
    """HBM bytes per launch of a config's dominant kernel, from the rocprofv3 PMC passes
    committed under profiles/ (tools/pmc_traffic.py); None when absent or another config."""
    path = os.path.join(PROFILE_DIR, f"traffic_{key}.json")
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, None
    if any(t.get("config", {}).get(k) != v for k, v in match.items()):
        return None, None
    return t["traffic_bytes_per_launch"], os.path.relpath(path, ROOT) + " (bytes per launch)"


def cpu_model():
    try:
        return [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":")[1].strip()
    except Exception:
        return platform.processor()


def cpu_entry(units, single, multi, threads, unit, sample):
    """cpu_baseline object: value = all host cores (the fair baseline), single_core beside it."""
    return {"value": units / multi, "unit": unit, "cores": threads, "kind": "port", "sample": sample,
            "single_core": {"value": units / single, "unit": unit, "cores": 1, "seconds": single},
            "seconds": multi, "cpu": cpu_model(), "nproc": os.cpu_count()}


# ------------------------------------------------------------------------------------
# post-run parity checks (outside every timed region; the oracle is the checker only)
# ------------------------------------------------------------------------------------
def check_threads(ctx):
    """Host threads for one rank's oracle check: the rank's share of the CPUs it may use
    (a launcher may set OMP_NUM_THREADS=1, which would make a 100M-event check crawl)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(32, n // max(1, ctx["world"])))


def u64_col(rows, off):
    return rows[:, off:off + 8].copy().view(np.uint64).ravel()


def tcp_fields66(rows):
    """Device packed ip_key_t (each column padded to 4 B: saddr 0:16 daddr 16:32 mntns 32:40
    pid 40:44 comm 44:60 lport 60:62 dport 64:66 family 68:70) -> the 66 field bytes."""
    return np.concatenate([rows[:, 0:62], rows[:, 64:66], rows[:, 68:70]], axis=1)


def topk_equal(cand_rows, off_aggs, off_first, first, aggs):
    """A device top-K (packed rows) against the oracle's (first (k,), aggs [(k,)...])."""
    if cand_rows.shape[0] != len(first):
        return False
    if not np.array_equal(u64_col(cand_rows, off_first), np.asarray(first, np.uint64)):
        return False
    return all(np.array_equal(u64_col(cand_rows, o), np.asarray(a, np.uint64)) for o, a in zip(off_aggs, aggs))


def gather_checks(ctx, obj):
    """Every rank's check record on every rank (torch all_gather_object: the check does not
    ride the product's own transport)."""
    if ctx["world"] == 1:
        return [obj]
    out = [None] * ctx["world"]
    ctx["dist"].all_gather_object(out, obj)
    return out


def merge_rank_topk(O, recs, K):
    """The oracle's global top-K from every rank's top-K (rank-disjoint key universes): the
    union ordered by SortStats(["-sent","-recv"]) with the global first index as the
    pre-sort position (Go SliceStable via the oracle).  Returns (sent, recv, first) of the first
    K.  tests/test_bench_check.py checks it against the oracle run over the union's events."""
    S = np.concatenate([r["sent"] for r in recs])
    R = np.concatenate([r["recv"] for r in recs])
    F = np.concatenate([r["first"] for r in recs])
    order = np.argsort(F, kind="stable")              # pre-sort position = global first index
    perm = O.go_sort_entries([(S[order], "uint64", True), (R[order], "uint64", True)], len(F))
    sel = order[perm[:K].astype(np.int64)]
    return S[sel], R[sel], F[sel]


def sum_rank_hists(refs):
    """Every rank's oracle histogram summed with u32 wrap, like the device's all-reduce."""
    return np.sum([r.astype(np.uint64) for r in refs], axis=0).astype(np.uint32)


def fingerprint(torch, rows):
    """Order-independent fingerprint of packed rows on the device: the sum over rows of a 64-bit
    mix of each row's words (wrapping int64 arithmetic; tests/test_gpu_soak.py's)."""
    G, rb = rows.shape
    if G == 0:
        return 0
    wb = (rb + 7) // 8 * 8
    r = torch.zeros((G, wb), dtype=torch.uint8, device=rows.device)
    r[:, :rb] = rows
    w = r.view(torch.int64)
    x = torch.full((G,), 0x243F6A8885A308D3, dtype=torch.int64, device=rows.device)
    for j in range(w.shape[1]):
        x = (x ^ w[:, j]) * 0x100000001B3
        x = x ^ (x >> 29)
    return int(x.sum().item())


IGX_CHECK_TIMEOUT_MS = 30000


def transport_check(ctx, what, fn):
    """N > 1, after a config's timed loop (outside it): the config's exchange run once through
    torch's collectives and once through the product's own igx_dist_* C ABI (IgxComm: RCCL inside
    libigx.so, the entry points a cgo caller binds), the results compared byte for byte on every
    rank; the ranks agree through an all-reduce (MIN).  fn(transport) -> a device u8 tensor.  A
    C-ABI transport that cannot be opened on some rank is reported (transport_igx_equal None);
    one that opens and then fails or differs is a mismatch (False: bench.py exits 3)."""
    torch, dist, D = ctx["torch"], ctx["dist"], ctx["D"]
    if ctx["world"] == 1:
        return None
    rec = {"what": what + ": torch.distributed (nccl = RCCL) vs igx_dist_* (C ABI, RCCL in libigx.so)"}
    ref = fn(D.TorchComm(dist))
    if "igx_comm" not in ctx:
        # the deadline bounds igx_dist_init too (a rank whose context failed leaves its peers in
        # ncclCommInitRankConfig until it passes), not only the later collectives
        old = os.environ.get("IGX_DIST_TIMEOUT_MS")
        os.environ["IGX_DIST_TIMEOUT_MS"] = str(IGX_CHECK_TIMEOUT_MS)
        try:
            ctx["igx_comm"] = D.IgxComm(dist, timeout_ms=IGX_CHECK_TIMEOUT_MS)
        except Exception as e:   # noqa: BLE001 -- agreed on below
            ctx["igx_comm"], ctx["igx_comm_error"] = None, repr(e)[:300]
        finally:
            if old is None:
                os.environ.pop("IGX_DIST_TIMEOUT_MS", None)
            else:
                os.environ["IGX_DIST_TIMEOUT_MS"] = old
        up = torch.tensor([1 if ctx["igx_comm"] is not None else 0], dtype=torch.int32, device=ctx["dev"])
        dist.all_reduce(up, op=dist.ReduceOp.MIN)
        if not int(up.item()) and ctx["igx_comm"] is not None:
            ctx["igx_comm"].close()
            ctx["igx_comm"] = None
    ic = ctx["igx_comm"]
    if ic is None:
        rec["transport_igx_equal"] = None
        rec["igx_error"] = ctx.get("igx_comm_error", "igx_dist_init failed on another rank")
        return rec
    ok = True
    try:
        got = fn(ic)
        ok = got.shape == ref.shape and bool(torch.equal(got, ref))
    except Exception as e:   # noqa: BLE001 -- a failed collective (IGX_EIO within the deadline)
        ok = False
        rec["igx_error"] = repr(e)[:300]
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=ctx["dev"])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    rec["transport_igx_equal"] = bool(int(flag.item()))
    rec["bytes"] = int(ref.numel())
    return rec


def check_c2(a, ctx, tab, cand, cdf_h, Gn, base):
    """C2's last timed interval vs or_top_tcp_mt on the same stream: this rank's group count
    and whole-table checksum (key fields, sent, recv, first index of every group), and the
    top-20 (first, sent, recv) -- at N>1 the global top-20 against the oracle's merge of every
    rank's top-20 (rank-disjoint key universes; the position is the global first index)."""
    torch, E, H, O = ctx["torch"], ctx["E"], ctx["H"], ctx["O"]
    rank, world = ctx["rank"], ctx["world"]
    N, G, K = a.events, a.keys, a.topk
    rows = H.host(table_rows(E, torch, tab, tab.fin))
    dev_cs = O.tcp_group_checksum(tcp_fields66(rows), u64_col(rows, 72), u64_col(rows, 80), u64_col(rows, 88))
    del rows
    h = O.gen_tcp(0xC2, rank, G, cdf_h, base, N)
    Gref, sent, recv, first, cs = O.top_tcp_mt(h, K, base_idx=base, threads=check_threads(ctx), checksum=True)
    del h
    recs = gather_checks(ctx, {"groups": int(Gn), "oracle_groups": int(Gref), "checksum_equal": dev_cs == cs,
                               "sent": sent, "recv": recv, "first": first})
    if rank != 0:
        return None
    S, R, F = merge_rank_topk(O, recs, K)
    c = H.host(cand)
    top_ok = topk_equal(c, (72, 80), 88, F, (S, R))
    groups_ok = all(r["groups"] == r["oracle_groups"] for r in recs)
    cs_ok = all(r["checksum_equal"] for r in recs)
    return {"bit_exact": bool(groups_ok and cs_ok and top_ok), "groups_equal": bool(groups_ok),
            "table_checksum_equal": bool(cs_ok), "topk_equal": bool(top_ok),
            "groups": [r["groups"] for r in recs], "oracle_groups": [r["oracle_groups"] for r in recs],
            "batch_base": base,
            "what": "last timed interval vs oracle or_top_tcp_mt on its own batch: per-rank group count and "
                    "whole-table checksum (66 key bytes + sent + recv + first of every group), global top-"
                    f"{K} (first, sent, recv)" + (" vs the oracle merge of every rank's top-K" if world > 1 else "")}


def check_table(a, ctx, tab, cand, keys_h, oaggs, valid, naggs, sort, K, base=0):
    """C4 / C5 (N=1): the last timed interval's table -- group count and a checksum of every
    (key, aggregates, first index) -- and, with `sort`, its top-K against or_groupby_topk_mt."""
    torch, E, H, O = ctx["torch"], ctx["E"], ctx["H"], ctx["O"]
    fin = tab.fin
    rows = H.host(table_rows(E, torch, tab, fin))
    kb = fin["key_bytes"]
    dev_cs = O.group_checksum(rows[:, :kb], [u64_col(rows, kb + 8 * x) for x in range(naggs)],
                              u64_col(rows, kb + 8 * naggs))
    ng = rows.shape[0]
    del rows
    Gref, first, aggs, cs = O.groupby_topk_mt(keys_h, oaggs, valid=valid, base_idx=base, sort=sort, k=K,
                                              threads=check_threads(ctx), checksum=True)
    out = {"groups": int(fin["n_groups"]), "oracle_groups": int(Gref), "groups_equal": fin["n_groups"] == Gref == ng,
           "table_checksum_equal": dev_cs == cs}
    ok = out["groups_equal"] and out["table_checksum_equal"]
    if sort:
        out["topk_equal"] = topk_equal(H.host(cand), [kb + 8 * x for x in range(naggs)], kb + 8 * naggs,
                                       first, [aggs[:, x] for x in range(naggs)])
        ok = ok and out["topk_equal"]
    out["bit_exact"] = bool(ok)
    return {k: (bool(v) if isinstance(v, (bool, np.bool_)) else v) for k, v in out.items()}


# ------------------------------------------------------------------------------------
# C2: the headline
# ------------------------------------------------------------------------------------
def family_in_pred(A, col):
    """tcptop.bpf.c:54-55: drop unless family is AF_INET (2) or AF_INET6 (10)."""
    p = A.Pred()
    p.col, p.cmp, p.negate, p.ref_len = col, A.CMP_IN, 0, 4
    for i, b in enumerate((2).to_bytes(2, "little") + (10).to_bytes(2, "little")):
        p.ref[i] = b
    return p


def copied_pred(A, col, dir_col):
    """tcptop.bpf.c:124-130: the receive probe returns when `int copied <= 0`; sends have no
    such check -- `copied > 0` guarded by dir == 1 (gadgets.copied_pred)."""
    p = A.Pred()
    p.col, p.cmp, p.negate, p.ref_len = col, A.CMP_GT, 0, 4
    p.guard_col, p.guard_len, p.guard_ref[0] = dir_col, 1, 1
    return p


def run_c2(a, ctx):
    torch, E, H, A, D, T = ctx["torch"], ctx["E"], ctx["H"], ctx["A"], ctx["D"], ctx["timer"]
    rank, world = ctx["rank"], ctx["world"]
    N, G, K = a.events, a.keys, a.topk
    cdf_h = E.zipf_cdf(G, a.zipf)
    cdf_d = H.to_device(cdf_h, ctx["dev"])
    # batch b = events [(b * world + rank) * N, ... + N) of one stream: the global event index of
    # row 0 (the first-index position), so every interval's events are distinct
    bases = [(b * world + rank) * N for b in range(n_batches(a, a.steps + a.warmup, EV_BYTES, N))]
    colsets = []
    for b in bases:
        ev = E.gen_tcp(0xC2, rank, G, cdf_d, b, N)
        colsets.append([ev[k] for k in TCP_NAMES] + [ev["size"].view(torch.int32)])   # 10: `int copied`
    del ev
    aggs = [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)]
    tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2], aggs, capacity=G + G // 4)
    preds = [family_in_pred(A, 7), copied_pred(A, 10, 9)]
    clk = KernelClock(torch)
    st = {"i": 0}

    def step(record):
        b = st["i"] % len(bases)
        st["i"] += 1
        st["b"] = b
        tab.reset()
        clk.on = record
        with clk:
            tab.update(colsets[b], list(range(8)), N, bases[b], preds)
        tab.finalize(sync=False)                      # the group count stays on the device
        # SortStats(["-sent","-recv"]) over the table's groups, first K slots (the device top-K
        # reads the count there: the step has no host round trip)
        cand = tab.gather(tab.sort([(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, True)], K))
        if world > 1:
            st["local"] = cand
            cand = D.merge_topk(cand, 72, 2, [(0, True), (1, True)], K)
        st["cand"] = cand

    torch.cuda.synchronize()
    dt = T.run(step, a.steps, a.warmup)
    Gn = tab.wait()                                   # the last interval's group count
    alg = N * EV_BYTES + Gn * GROUP_BYTES
    out = {"value": world * N * a.steps / dt, "ms_per_step": dt * 1000.0 / a.steps, "groups_per_gpu": Gn,
           "batches": len(bases), "claims_per_interval": tab.info()["claims"],
           "roofline": roofline(alg, clk.avg(), "k_groupby<ip_key_t>",
                                f"{EV_BYTES} B/event x events + {GROUP_BYTES} B/group x groups", "c2",
                                {"events": N, "keys": G, "zipf": a.zipf})}
    out["roofline"]["hbm_pct_of_peak_whole_step"] = 100.0 * alg / (out["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS
    if a.check:
        out["check"] = check_c2(a, ctx, tab, st["cand"], cdf_h, Gn, bases[st["b"]])
        if world > 1:   # every rank takes part; rank 0 records it
            tr = transport_check(ctx, "C2 all-gather of the per-rank top-K candidates",
                                 lambda c: D.allgather_rows(st["local"], c).flatten())
            if out["check"] is not None:
                out["check"]["transport"] = tr
    if rank == 0 and world == 1 and a.cpu_sample:
        O = ctx["O"]
        S = a.cpu_sample
        evh = O.gen_tcp(0xC2, 0, G, cdf_h, 0, S)
        t0 = time.perf_counter()
        r1 = O.top_tcp(evh, K)
        single = time.perf_counter() - t0
        thr = O.cpu_threads()
        t0 = time.perf_counter()
        r2 = O.top_tcp_mt(evh, K, threads=thr)
        multi = time.perf_counter() - t0
        assert np.array_equal(r1[4], r2[3]), "all-cores baseline disagrees with the single-thread one"
        out["cpu_baseline"] = cpu_entry(
            S, single, multi, thr, "events/s",
            f"{S} events of the same stream (keys {G}, zipf {a.zipf}): oracle/igx_oracle.c or_top_tcp_mt "
            f"(hash-partitioned Go-map restatement + per-thread SliceStable top-K + merge) on {thr} threads; "
            f"single_core = or_top_tcp (BPF-map group-by, nextStats, SortEntries via Go SliceStable)")
    tab.destroy()
    return out


# ------------------------------------------------------------------------------------
# C1: pkg/columns FilterEntries + SortEntries over 1M trace-open events
# ------------------------------------------------------------------------------------
def run_c1(a, ctx):
    torch, E, H, T = ctx["torch"], ctx["E"], ctx["H"], ctx["timer"]
    igx = ctx["igx"]
    n = 1_000_000
    ev = E.gen_open(0xC1, H.to_device(E.zipf_cdf(64, 1.0), ctx["dev"]), ctx["rank"] * n, n)
    cols = igx.columns.Columns([("pid", "uint32"), ("uid", "uint32"), ("mntns", "uint64"),
                                ("comm", "string", 16), ("ret", "int64"), ("fd", "int64"),
                                ("err", "int64"), ("path", "uint32")])
    batch = igx.columns.EventBatch(cols, ev)
    filters, sort_by = ["err:0", "pid:>=1000"], ["comm", "-pid"]
    st = {}

    def step(record):
        out = igx.filter.FilterEntries(cols, batch, filters)
        st["out"] = igx.sort.SortEntries(cols, out, sort_by)

    dt = T.run(step, a.config_steps, 1)
    sel = st["out"].n
    ms = dt * 1000.0 / a.config_steps
    alg = n * 12 + sel * 24
    out = {"workload": "FilterEntries([err:0, pid:>=1000]) + SortEntries([comm, -pid]) of 1M trace-open events",
           "events_per_gpu": n, "value": ctx["world"] * n / (ms * 1e-3), "unit": "events/s",
           "ms_per_step": ms, "selected": sel,
           "hbm_pct_of_peak_whole_step": 100.0 * alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "note": "launch- and sync-bound at 1M rows (several kernels, one host sync per filter)"}
    if a.check and ctx["rank"] == 0:
        # the last timed step's view: its selection vector, in SortEntries order, against the
        # oracle's FilterEntries (one or_filter per filter, filter.go:294-325) + SortEntries
        # (Go SliceStable per key, sort.go:35-83) of this rank's batch
        O = ctx["O"]
        h = O.gen_open(0xC1, O.zipf_cdf(64, 1.0), ctx["rank"] * n, n)
        ocols = {"err": O.OCol("err", "int64", 8), "pid": O.OCol("pid", "uint32", 4)}
        osel = O.filter_entries(ocols, {"err": h["err"], "pid": h["pid"]}, None, filters)
        perm = O.go_sort_entries([(h["comm"][osel], "string", False), (h["pid"][osel], "uint32", True)], len(osel))
        want = osel[perm.astype(np.int64)]
        got = H.host(st["out"].sel).astype(np.int64) if st["out"].sel is not None else np.arange(sel)
        ok = bool(np.array_equal(got, want))
        out["check"] = {"bit_exact": ok, "selected": int(sel), "oracle_selected": int(len(want)),
                        "what": "rank 0's last timed step: selected row ids in output order vs oracle "
                                "filter_entries + go_sort_entries"}
    if ctx["rank"] == 0 and ctx["world"] == 1 and a.cpu_sample:
        O = ctx["O"]
        h = O.gen_open(0xC1, O.zipf_cdf(64, 1.0), 0, n)
        ocols = {"err": O.OCol("err", "int64", 8), "pid": O.OCol("pid", "uint32", 4)}
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            osel = O.match_rows([O.parse_filter(ocols, "err:0")], h)
            osel = osel[O.match_rows([O.parse_filter(ocols, "pid:>=1000")], {"pid": h["pid"][osel]})]
            O.go_sort_entries([(h["comm"][osel], "string", False), (h["pid"][osel], "uint32", True)], len(osel))
        single = (time.perf_counter() - t0) / reps
        out["cpu_baseline"] = {"value": n / single, "unit": "events/s", "cores": 1, "kind": "port",
                               "sample": f"the full 1M-event batch x{reps}: oracle or_filter per filter + "
                                         "or_sort_entries (Go SliceStable, one pass per key) -- the reference "
                                         "path is single-threaded Go, so no all-cores variant",
                               "cpu": cpu_model(), "nproc": os.cpu_count()}
    return out


# ------------------------------------------------------------------------------------
# C3: profile block-io log2 histograms, all-reduce at N>1
# ------------------------------------------------------------------------------------
def run_c3(a, ctx):
    torch, E, H, D, T = ctx["torch"], ctx["E"], ctx["H"], ctx["D"], ctx["timer"]
    rank, world, n = ctx["rank"], ctx["world"], a.config_events
    q = E.lognormal_quantiles(*C3_LOGNORMAL)
    devs = C3_DEVS
    ev = E.gen_bio(0xC3, H.to_device(q, ctx["dev"]), rank * n, n)
    delta = ev["delta"].view(torch.int64)
    hist = torch.zeros((4096, 27), dtype=torch.uint32, device=ctx["dev"])
    clk = KernelClock(torch)

    def step(record):
        hist.zero_()
        clk.on = record
        with clk:
            E.hist_log2(ev["dev"], ev["cont"], delta, devs, C3_NCONT, hist=hist)
        D.allreduce_hist(hist)

    dt = T.run(step, a.config_steps, 1)
    ms = dt * 1000.0 / a.config_steps
    alg = n * 16 + 4096 * 27 * 4
    out = {"workload": "profile block-io: log2 latency histograms, 16 devs x 256 containers x 27 slots"
                       + (", RCCL all-reduce" if world > 1 else ""),
           "events_per_gpu": n, "value": world * n / (ms * 1e-3), "unit": "events/s", "ms_per_step": ms,
           "roofline": roofline(alg, clk.avg(), "k_hist", "16 B/event (dev 4, cont 4, delta 8) + 442 KB out",
                                "c3", {"events": n}),
           "total_counted": int(H.host(hist).astype(np.uint64).sum())}
    if a.check:
        # the last timed step's histogram (all-reduced at N>1) vs the sum of every rank's
        # oracle histogram (or_hist_log2_mt: biolatency.bpf.c:100-154 per event)
        O = ctx["O"]
        hh = O.gen_bio(0xC3, q, rank * n, n)
        ref = O.hist_log2_mt(hh["dev"], hh["cont"], hh["delta"], devs, C3_NCONT, threads=check_threads(ctx))
        del hh
        refs = gather_checks(ctx, ref)
        tr = None
        if world > 1:
            loc = torch.zeros_like(hist)
            E.hist_log2(ev["dev"], ev["cont"], delta, devs, C3_NCONT, hist=loc)   # this rank's own histogram
            tr = transport_check(ctx, "C3 all-reduce of the u32[4096][27] histogram",
                                 lambda c: D.allreduce_hist(loc.clone(), c).flatten().view(torch.uint8))
        if rank == 0:
            tot = sum_rank_hists(refs)
            ok = bool(np.array_equal(H.host(hist), tot))
            out["check"] = {"bit_exact": ok, "what": "last timed step's whole u32[4096][27] histogram vs the sum "
                                                     f"of {world} rank(s)' oracle histograms"}
            if tr is not None:
                out["check"]["transport"] = tr
    if rank == 0 and world == 1 and a.cpu_sample:
        O = ctx["O"]
        S = 40_000_000
        h = O.gen_bio(0xC3, q, 0, S)
        t0 = time.perf_counter()
        r1 = O.hist_log2(h["dev"], h["cont"], h["delta"], devs, 256)
        single = time.perf_counter() - t0
        thr = O.cpu_threads()
        t0 = time.perf_counter()
        r2 = O.hist_log2_mt(h["dev"], h["cont"], h["delta"], devs, 256, threads=thr)
        multi = time.perf_counter() - t0
        assert np.array_equal(r1, r2)
        out["cpu_baseline"] = cpu_entry(S, single, multi, thr, "events/s",
                                        f"{S} events of the same stream: or_hist_log2_mt (private histograms per "
                                        f"thread, summed) on {thr} threads; single_core = or_hist_log2 "
                                        "(biolatency.bpf.c:100-154 + bits.bpf.h log2l per event)")
    return out


# ------------------------------------------------------------------------------------
# C4: advise network-policy distinct tuples, all-to-all by key owner at N>1
# ------------------------------------------------------------------------------------
def run_c4(a, ctx):
    torch, E, H, A, D, T = ctx["torch"], ctx["E"], ctx["H"], ctx["A"], ctx["D"], ctx["timer"]
    rank, world, n = ctx["rank"], ctx["world"], a.config_events
    names, widths = C4_NAMES, C4_WIDTHS
    ev = E.gen_np(*C4_GEN, rank * n, n, device=ctx["dev"])   # a slice of ONE global stream
    cols = [ev[k] for k in names]
    cap = C4_CAP
    # distinct only, as the reference: graph.c:102-114 (BPF_NOEXIST, first timestamp wins),
    # advisor.go:307-319 (first event per tuple); nothing is counted
    tab = E.Table(widths, [], cap)
    # an owner receives about 1/N of the global distinct tuples, but C4's tuple universe is not
    # bounded by one rank's capacity (every rank's slice adds tuples), so its table keeps it
    own = D.owner_table(widths, [], cap) if world > 1 else None
    clk = KernelClock(torch)
    st = {}

    def step(record):
        tab.reset()
        clk.on = record
        with clk:   # the bracket holds every kernel that reads the 24 B/event: np_mark and the update
            keep = E.np_mark(ev["type"], ev["pkt"], ev["hostip"], ev["raddr"])
            tab.update(cols, [0, 1, 2, 3], n, rank * n, valid=keep)
        tab.finalize(sync=False)                      # the distinct count stays on the device
        if world > 1:
            # the partial groups, grouped by owner straight from the table (the device count
            # sizes the passes); the send counts are the step's one host read, then the
            # exchange's own plan all-gather, then the owner merge, finalized asynchronously
            rows, cnt = tab.partition(world)
            counts = cnt.cpu().tolist()
            mine = D.exchange_partitioned(rows, counts)
            D.merge_partials(mine, widths, [], cap, table=own, sync=False)
            st["part"] = (rows, counts)

    dt = T.run(step, a.config_steps, 1)
    ms = dt * 1000.0 / a.config_steps
    ng = own.wait() if world > 1 else tab.wait()
    alg = n * 24 + ng * 20
    out = {"workload": "advise network-policy: np_mark + distinct (src, dir, peer, port) with first index"
                       + (", partial groups all-to-all by key owner + owner merge" if world > 1 else ""),
           "events_per_gpu": n, "value": world * n / (ms * 1e-3), "unit": "events/s", "ms_per_step": ms,
           "distinct_on_rank0": ng,
           "roofline": roofline(n * 24 + ng * 20, clk.avg(),
                                "k_np_mark + igx_groupby_update on the np tuple (AUTO: the partitioned form's "
                                "passes k_gbp_count/csum/scan/offs/a/b/c after the first, measured, interval)",
                                "24 B/event (src 4, peer 4, port 2, pkt 1, type 1, proto 1, hostip 4, raddr 4, "
                                "+3 pad) + 20 B/distinct tuple (key 12 + first 8)", "c4", {"events": n})}
    out["roofline"]["alg_bytes_per_launch"] = alg
    if a.check and world == 1:
        O = ctx["O"]
        h = O.gen_np(*C4_GEN, 0, n)
        keys, valid = O.pad_keys(h, names), O.np_mark(h)
        del h
        out["check"] = check_table(a, ctx, tab, None, keys, [], valid, 0, (), 0)
        out["check"]["what"] = ("last timed interval's table vs oracle or_groupby_topk_mt distinct on the same "
                                "stream: distinct count + checksum of every (tuple, first index)")
        del keys, valid
    elif a.check:
        scratch = D.owner_table(widths, [], cap)

        def c4x(c):
            mine = D.exchange_partitioned(st["part"][0], st["part"][1], c)
            t = D.merge_partials(mine, widths, [], cap, table=scratch)
            fp = fingerprint(torch, table_rows(E, torch, t, t.fin))
            return torch.cat([mine.flatten(), torch.tensor([fp], dtype=torch.int64, device=mine.device).view(torch.uint8)])

        tr = transport_check(ctx, "C4 all-to-all of the partial groups by key owner + the owner merge", c4x)
        scratch.destroy()
        if rank == 0:
            out["check"] = {"skipped": "N>1: the owners' tables span every rank's slice; checked at N=1 and by "
                                       "tests/test_gpu_dist.py", "transport": tr}
    if rank == 0 and world == 1 and a.cpu_sample:
        O = ctx["O"]
        # the reference's own path: GeneratePolicies builds a localPodKey / networkPeerKey string
        # per event (label keys sorted, fmt.Sprintf) and dedups in string-keyed maps
        # (advisor.go:130-159, 279-320) -- or_np_advise_strings, single-threaded like the Go code
        SS = 4_000_000
        hs = O.gen_np(*C4_GEN, 0, SS)
        t0 = time.perf_counter()
        gs = O.np_advise_strings(hs)
        strings = time.perf_counter() - t0
        assert gs == O.groupby(O.pad_keys(hs, names), [], valid=O.np_mark(hs))[0].shape[0]
        del hs
        # the same dedup over pre-packed integer keys (a lower bound of the CPU's cost)
        S = 20_000_000
        h = O.gen_np(*C4_GEN, 0, S)
        keys = O.pad_keys(h, names)
        keep = O.np_mark(h)
        t0 = time.perf_counter()
        k1, _, _ = O.groupby(keys, [], valid=keep)
        single = time.perf_counter() - t0
        thr = O.cpu_threads()
        t0 = time.perf_counter()
        g2, _, _ = O.groupby_topk_mt(keys, [], valid=keep, threads=thr)
        multi = time.perf_counter() - t0
        assert g2 == len(k1)
        out["cpu_baseline"] = {
            "value": SS / strings, "unit": "events/s", "cores": 1, "kind": "port", "seconds": strings,
            "sample": f"{SS} events of the same stream through oracle/igx_oracle.c or_np_advise_strings: "
                      "GeneratePolicies on the reference's string keys (localPodKey / networkPeerKey per "
                      "event with sorted label keys, string-keyed first-event-wins maps, advisor.go:130-159, "
                      "279-320), single-threaded like the Go code; same distinct count as the device",
            "cpu": cpu_model(), "nproc": os.cpu_count(),
            "prepacked": cpu_entry(S, single, multi, thr, "events/s",
                                   f"{S} events, keys pre-packed as integers (not timed): or_groupby_topk_mt "
                                   f"distinct on {thr} threads; single_core = or_groupby -- a lower bound of the "
                                   "CPU path's cost, not the reference's shape")}
    tab.destroy()
    if own is not None:
        own.destroy()
    return out


def table_rows(E, torch, tab, fin):
    """every occupied group of a finalized table as packed rows (key | aggs | first)."""
    G = fin["n_groups"]
    slots = torch.empty(max(1, G), dtype=torch.int32, device="cuda")[:G]
    if G:
        tab.ctx.check(tab.ctx.L.igx_memcpy_d2d(tab.ctx.h, slots.data_ptr(), fin["groups_ptr"], G * 4))
    return tab.gather(slots)


# ------------------------------------------------------------------------------------
# C5: top file, 10M distinct keys, owner exchange + all-gather top-K at N>1
# ------------------------------------------------------------------------------------
def run_c5(a, ctx):
    torch, E, H, A, D, T = ctx["torch"], ctx["E"], ctx["H"], ctx["A"], ctx["D"], ctx["timer"]
    rank, world, n = ctx["rank"], ctx["world"], a.config_events
    G, K = C5_KEYS, C5_TOPK
    names, widths = C5_NAMES, C5_WIDTHS
    cdf_h = E.zipf_cdf(G, C5_ZIPF)
    cdf_d = H.to_device(cdf_h, ctx["dev"])
    # one global key universe; batch b is the b-th chunk of one global stream, this rank's slice
    bases = [(b * world + rank) * n for b in range(n_batches(a, a.config_steps + 1, 25, n))]
    colsets = []
    for b in bases:
        ev = E.gen_file(0xC5, 0, G, cdf_d, b, n)
        colsets.append([ev[k] for k in names])
    del ev
    aggs = c5_aggs(A)
    cap = C5_CAP
    tab = E.Table(widths, aggs, cap)
    # C5's key universe is global (C5_CAP bounds it), so an owner holds about 1/N of it
    own_cap = D.owner_capacity(cap, world)
    own = D.owner_table(widths, [8, 8, 8, 8], own_cap) if world > 1 else None
    clk = KernelClock(torch)
    st = {"i": 0}

    def step(record):
        b = st["i"] % len(bases)
        st["i"] += 1
        st["b"] = b
        tab.reset()
        clk.on = record
        with clk:
            tab.update(colsets[b], [0, 1, 2, 3], n, bases[b])
        t = tab
        tab.finalize(sync=False)                      # the group count stays on the device
        if world > 1:
            # as C4: partition straight from the table, one host read (the send counts), the
            # exchange, the owner merge finalized asynchronously (its top-K reads its count there)
            rows, cnt = tab.partition(world)
            counts = cnt.cpu().tolist()
            mine = D.exchange_partitioned(rows, counts)
            t = D.merge_partials(mine, widths, [8, 8, 8, 8], own_cap, table=own, sync=False)
            st["part"] = (rows, counts)
        cand = t.gather(t.sort([(A.TSRC_AGG, 3, True)], K))       # ["-wbytes"]
        if world > 1:
            st["local"] = cand
            cand = D.merge_topk(cand, 20, 4, [(3, True)], K)
        st["cand"] = cand

    dt = T.run(step, a.config_steps, 1)
    ms = dt * 1000.0 / a.config_steps
    ng = own.wait() if world > 1 else tab.wait()
    alg = n * 25 + ng * 60
    out = {"workload": "top file: group-by (inode, dev, pid, tid) with reads/rbytes/writes/wbytes, top-20 by "
                       "[-wbytes]" + (", partial groups all-to-all by key owner, owners' top-20 all-gathered"
                                      if world > 1 else ""),
           "events_per_gpu": n, "keys": G, "value": world * n / (ms * 1e-3), "unit": "events/s",
           "ms_per_step": ms, "groups_on_rank0": ng, "batches": len(bases),
           "owner_capacity": own_cap if world > 1 else None,
           "claims_per_interval": tab.info()["claims"] if world == 1 else None,
           "roofline": roofline(alg, clk.avg(), "k_groupby<file_id>",
                                "25 B/event (inode 8, dev 4, pid 4, tid 4, op 1, count 4) + 60 B/group", "c5",
                                {"events": n, "keys": G})}
    if a.check and world == 1:
        O = ctx["O"]
        base = bases[st["b"]]
        h = O.gen_file(0xC5, 0, G, cdf_h, base, n)
        keys = O.pad_keys(h, ("inode", "dev", "pid", "tid"))
        out["check"] = check_table(a, ctx, tab, st["cand"], keys, c5_oracle_aggs(h), None, 4, [(3, True)], K, base)
        out["check"]["batch_base"] = base
        out["check"]["what"] = ("last timed interval's table vs oracle or_groupby_topk_mt on its own batch: "
                                "group count, checksum of every (key, reads, rbytes, writes, wbytes, first), "
                                "top-20 by [-wbytes] (first + 4 aggregates)")
        del h, keys
    elif a.check:
        scratch = D.owner_table(widths, [8, 8, 8, 8], own_cap)

        def c5x(c):
            mine = D.exchange_partitioned(st["part"][0], st["part"][1], c)
            t = D.merge_partials(mine, widths, [8, 8, 8, 8], own_cap, table=scratch)
            allc = D.allgather_rows(t.gather(t.sort([(A.TSRC_AGG, 3, True)], K)), c)
            return torch.cat([mine.flatten(), allc.flatten()])

        tr = transport_check(ctx, "C5 all-to-all of the partial groups by key owner + owner merge + all-gather "
                                  "of the owners' top-20", c5x)
        scratch.destroy()
        if rank == 0:
            out["check"] = {"skipped": "N>1: the owners' tables span every rank's slice; checked at N=1 and by "
                                       "tests/test_gpu_dist.py", "transport": tr}
    if rank == 0 and world == 1 and a.cpu_sample:
        O = ctx["O"]
        S = 10_000_000
        h = O.gen_file(0xC5, 0, G, cdf_h, 0, S)
        keys = O.pad_keys(h, ("inode", "dev", "pid", "tid"))
        oaggs = c5_oracle_aggs(h)
        t0 = time.perf_counter()
        _, oa, of = O.groupby(keys, oaggs)
        perm = O.go_sort_entries([(oa[3], "uint64", True)], len(of))
        single = time.perf_counter() - t0
        thr = O.cpu_threads()
        t0 = time.perf_counter()
        _, first, _ = O.groupby_topk_mt(keys, oaggs, sort=[(3, True)], k=K, threads=thr)
        multi = time.perf_counter() - t0
        assert np.array_equal(first, of[perm[:K].astype(np.int64)])
        out["cpu_baseline"] = cpu_entry(S, single, multi, thr, "events/s",
                                        f"{S} events of the same stream (keys pre-packed, not timed): "
                                        f"or_groupby_topk_mt on {thr} threads; single_core = or_groupby + "
                                        "SortEntries([-wbytes]) via Go SliceStable over every group")
    tab.destroy()
    if own is not None:
        own.destroy()
    return out


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:
            sys.exit(launch_ranks(a))
    elif int(os.environ["WORLD_SIZE"]) != a.gpus:
        print(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {a.gpus}", file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.launch_dry_run:
        print(json.dumps({"rank": rank, "local_rank": local, "world": world,
                          "master": [os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")]}), flush=True)
        return
    import torch
    import torch.distributed as dist

    local = local % max(1, torch.cuda.device_count())   # a gloo rehearsal may run more ranks than GPUs
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    transport = None
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    igx = importlib.import_module("inspektor-gadget_amd")
    if world > 1:
        transport = igx.dist.select_transport(a.transport)
    ctx = make_ctx(torch, dist, igx, rank, world, dev, a.check or (rank == 0 and world == 1 and a.cpu_sample))

    c2 = run_c2(a, ctx)
    configs = {}
    for name in [c for c in a.configs.split(",") if c]:
        fn = {"c1": run_c1, "c3": run_c3, "c4": run_c4, "c5": run_c5}[name]
        configs[name] = fn(a, ctx)
        torch.cuda.empty_cache()

    failed = []
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": c2["value"],
            "unit": "events/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": c2["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based SplitMix64 stream, Zipf key ranks)",
            "config": {
                "workload": "top-tcp: filter family in {AF_INET, AF_INET6}, group-by ip_key_t(saddr,daddr,mntns,"
                            "pid,comm,lport,dport,family) sum sent/recv, stable top-20 by [-sent,-recv]",
                "events_per_gpu": a.events, "keys_per_gpu": a.keys, "zipf_s": a.zipf, "topk": a.topk,
                "groups_per_gpu": c2["groups_per_gpu"],
                "batches": c2["batches"],
                "claims_per_interval": c2["claims_per_interval"],
                "parallelism": (f"ingest-partitioned x{world}, all-gather top-K merge over "
                                + ("igx_dist_* (RCCL, C ABI)" if transport == "igx" else
                                   "torch.distributed (nccl = RCCL)")) if world > 1 else "single GPU",
            },
            "roofline": c2["roofline"],
            "cpu_baseline": c2.get("cpu_baseline"),
            "configs": configs,
            "library": os.path.relpath(igx._abi.LIB_PATH, ROOT),
        }
        if "check" in c2:
            line["check"] = c2["check"]
            line["check"]["configs"] = {k: v["check"].get("bit_exact", "skipped")
                                        for k, v in configs.items() if "check" in v}
            failed = [k for k, v in [("c2", c2)] + list(configs.items())
                      if v.get("check", {}).get("bit_exact") is False
                      or (v.get("check", {}).get("transport") or {}).get("transport_igx_equal") is False]
            if world > 1:
                line["check"]["transport_igx_equal"] = {
                    k: (v.get("check", {}).get("transport") or {}).get("transport_igx_equal")
                    for k, v in [("c2", c2)] + list(configs.items())}
            line["check"]["all_bit_exact"] = not failed
        print(json.dumps(line), flush=True)
    if world > 1:
        if ctx.get("igx_comm") is not None:
            ctx["igx_comm"].close()
        igx.dist.shutdown()
        dist.destroy_process_group()
    if failed:
        print(f"bench.py: results differ from the oracle in {failed}", file=sys.stderr, flush=True)
        sys.exit(3)


def make_ctx(torch, dist, igx, rank, world, dev, need_oracle):
    """The per-process handles every run_cX takes (tests/test_gpu_fullsize.py builds the same
    one to run the bench's exact steps)."""
    O = None
    if need_oracle:
        from oracle import oracle as O   # CPU baselines and the post-run check only (test infrastructure)
    return {"torch": torch, "dist": dist, "igx": igx, "E": igx.engine, "H": igx.columns, "A": igx._abi,
            "D": igx.dist, "O": O, "rank": rank, "world": world, "dev": dev, "timer": Timer(torch, dist, world, dev)}


if __name__ == "__main__":
    main()
