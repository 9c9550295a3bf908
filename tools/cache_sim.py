"""Per-CU simulation of the cached group-by kernel's LDS key cache: one CU's
share of a Zipf stream, E entries in sets of `ways`, admission on the k-th miss seen through a
direct-mapped ghost table of recent miss keys, no eviction -- the shipped policy is 8 ways,
second miss, 1 024 ghost entries.  Prints the miss share per variant and the ideal top-E hit
share.  CPU only; about a minute per variant.

  python tools/cache_sim.py c2     # 1M keys, Zipf 1.1, 100M / 256 events per CU, E = 1 048
  python tools/cache_sim.py c5     # 10M keys, Zipf 1.05, 125M / 256 events per CU, E = 1 568
  python tools/cache_sim.py c2 seeded   # + the cache pre-filled from a 1 % / 2 % row sample
"""
import sys

import numpy as np

CONFIGS = {"c2": (1_000_000, 1.1, 390_000, 1048), "c5": (10_000_000, 1.05, 488_000, 1568)}


def stream(G, s, n, seed=1):
    rng = np.random.default_rng(seed)
    p = np.arange(1, G + 1, dtype=np.float64) ** -s
    p /= p.sum()
    keys = np.searchsorted(np.cumsum(p), rng.random(n))
    h = rng.permutation(G)[keys].astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)   # wraps: a hash
    return p, keys, h


def simulate(keys, h, E, ways, kth, ghost):
    sets = E // ways
    cache = [set() for _ in range(sets)]
    gk = np.full(ghost, -1, np.int64)
    gc = np.zeros(ghost, np.int64)
    hs = (h >> np.uint64(32)).astype(np.int64) % sets
    hg = (h >> np.uint64(20)).astype(np.int64) & (ghost - 1)
    miss = 0
    for i in range(len(keys)):
        k, c = keys[i], cache[hs[i]]
        if k in c:
            continue
        miss += 1
        if len(c) >= ways:
            continue
        if kth <= 1:
            c.add(k)
            continue
        g = hg[i]
        if gk[g] == k:
            gc[g] += 1
            if gc[g] + 1 >= kth:
                c.add(k)
        else:
            gk[g], gc[g] = k, 0
    return miss / len(keys)


def simulate_seeded(keys, h, E, ways, ghost, pinned_keys, pinned_h):
    """the cache starts with the keys a row sample of the whole interval
    counted most often (pinned: their sets filled in sample-count order, never evicted), and the
    shipped second-miss admission fills what is left.  Same per-CU stream as simulate()."""
    sets = E // ways
    cache = [set() for _ in range(sets)]
    for k, hh in zip(pinned_keys, pinned_h):
        c = cache[int(hh >> np.uint64(32)) % sets]
        if len(c) < ways:
            c.add(int(k))
    gk = np.full(ghost, -1, np.int64)
    gc = np.zeros(ghost, np.int64)
    hs = (h >> np.uint64(32)).astype(np.int64) % sets
    hg = (h >> np.uint64(20)).astype(np.int64) & (ghost - 1)
    miss = 0
    for i in range(len(keys)):
        k, c = int(keys[i]), cache[hs[i]]
        if k in c:
            continue
        miss += 1
        if len(c) >= ways:
            continue
        g = hg[i]
        if gk[g] == k:
            gc[g] += 1
            if gc[g] + 1 >= 2:
                c.add(k)
        else:
            gk[g], gc[g] = k, 0
    return miss / len(keys)


def sample_top(G, s, sample_rows, E, seed=7):
    """The keys a sample of `sample_rows` rows of the interval (all CUs' rows: a 1-2 % sample
    of 100M is 1-2M rows) counts most often, hottest first, with their hashes (the same key ->
    hash map as stream())."""
    rng = np.random.default_rng(seed)
    p = np.arange(1, G + 1, dtype=np.float64) ** -s
    p /= p.sum()
    ks = np.searchsorted(np.cumsum(p), rng.random(sample_rows))
    cnt = np.bincount(ks, minlength=G)
    top = np.argsort(-cnt, kind="stable")[: 4 * E]
    return top[cnt[top] > 0]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    G, s, n, E = CONFIGS[cfg]
    p, keys, h = stream(G, s, n)
    print(f"ideal top-{E} miss share {1 - p[:E].sum():.4f}")
    if len(sys.argv) > 2 and sys.argv[2] == "seeded":
        # the permutation stream() applied to ranks, to hash the sample's keys the same way
        rng = np.random.default_rng(1)
        rng.random(n)
        perm = rng.permutation(G)
        print(f"shipped (8 ways, second miss, ghost 1024): miss share {simulate(keys, h, E, 8, 2, 1024):.4f}")
        for frac in (0.01, 0.02):
            rows = int(frac * n * 256)       # the interval's rows: every CU's share
            top = sample_top(G, s, rows, E)
            ph = perm[top].astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
            r = simulate_seeded(keys, h, E, 8, 1024, top, ph)
            print(f"sample-seeded {frac:.0%} of the interval ({rows} rows), top keys pinned: miss share {r:.4f}")
        return
    for ways, kth, ghost in ((8, 2, 1024), (8, 1, 1024), (8, 3, 1024), (8, 3, 4096), (16, 2, 1024), (E, 2, 1024)):
        print(f"ways {ways:5d} admit on miss {kth} ghost {ghost:5d}: miss share {simulate(keys, h, E, ways, kth, ghost):.4f}")


if __name__ == "__main__":
    main()
