"""bench.py's N > 1 path, rehearsed on one GPU: `--gpus 2 --dist-backend gloo` starts two rank
processes that share cuda:0 over a gloo group (host-staged collectives; RCCL refuses two ranks
on one device).  Every config runs its N > 1 step -- C2's all-gathered top-K, C3's all-reduce,
C4 / C5's partition straight from the table, exchange and asynchronously finalized owner
merge -- and the line's checks must hold: C2's per-rank tables and merged global top-20 and
C3's all-reduced histogram against the oracle.  The product's igx_dist_* transport cannot open
two ranks on one device, so the transport comparison must report it unavailable (None), not
fail or hang.  The real 8-GPU run is the driver's.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_rehearsal():
    env = dict(os.environ, OMP_NUM_THREADS="4", IGX_DIST_TIMEOUT_MS="20000")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--events", "4000000", "--keys", "100000", "--config-events", "3000000", "--steps", "3",
           "--warmup", "1", "--config-steps", "2", "--cpu-sample", "0", "--configs", "c3,c4,c5",
           "--input-gb", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert r.returncode == 0 and lines, (r.stdout[-3000:], r.stderr[-3000:])
    d = json.loads(lines[-1])
    assert d["n_gpus"] == 2
    assert d["check"]["all_bit_exact"] is True, d["check"]
    assert d["check"]["bit_exact"] is True
    assert d["check"]["configs"]["c3"] is True
    tr = d["check"]["transport_igx_equal"]
    assert set(tr) == {"c2", "c3", "c4", "c5"}, tr
    assert all(v is None for v in tr.values()), tr       # unavailable on a shared GPU, reported
    assert d["configs"]["c5"]["owner_capacity"] < 12_500_000
    for c in ("c4", "c5"):
        assert d["configs"][c]["check"]["transport"]["transport_igx_equal"] is None
