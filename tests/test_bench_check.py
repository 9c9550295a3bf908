"""bench.py's multi-rank post-run check on CPU (gloo, world 2): the rank records travel over
the process group and rank 0's oracle merge equals the oracle over the union of the ranks'
events -- C2's global top-20 (rank-disjoint key universes, global first index as position)
and C3's summed histogram.  The GPU side of the check is exercised at N=1 by
tests/test_gpu_fullsize.py::test_bench_c2_async_intervals_match_oracle."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_check_world2_gloo():
    env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "bench_check_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "BENCH_CHECK_OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
