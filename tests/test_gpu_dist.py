"""Multi-rank merges on the GPU.

test_world2_product_merges: tests/dist_worker_gpu.py under torch.distributed.run, two ranks
sharing cuda:0 over gloo (host-staged; RCCL refuses two ranks on one device): per-rank
aggregation, partition, owner merge and top-K merge are libigx.so, checked against the oracle
on the union of both ranks' events (C2, C3, C4, C5).

test_igx_dist_rccl_single_rank: the igx_dist_* C ABI over RCCL with a one-rank communicator
(the only RCCL shape a one-GPU box allows): unique id -> init -> all-reduce, all-gather, all-to-
all (size queries and data), exchange_groups, capacity errors, barrier, destroy.
"""
import ctypes as C
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_world2_product_merges():
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_worker_gpu.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "DIST_GPU_OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])


def test_igx_dist_rccl_single_rank(igx, torch, oracle):
    A, E, H = igx._abi, igx.engine, igx.columns
    ctx = igx.runtime.context()
    L = ctx.L
    uid = (C.c_uint8 * A.DIST_ID_BYTES)()
    assert L.igx_dist_get_unique_id(uid) == 0
    h = C.c_void_p()
    ctx.check(L.igx_dist_init(ctx.h, uid, 1, 0, C.byref(h)))
    try:
        r, n = C.c_int(-1), C.c_int(-1)
        ctx.check(L.igx_dist_rank(h, C.byref(r), C.byref(n)))
        assert (r.value, n.value) == (0, 1)
        hist = torch.arange(4096 * 27, dtype=torch.int64, device="cuda").to(torch.int32).view(torch.uint32)
        before = H.host(hist).copy()
        ctx.check(L.igx_dist_allreduce_u32(h, C.c_void_p(hist.data_ptr()), hist.numel()))
        torch.cuda.synchronize()
        assert np.array_equal(H.host(hist), before)
        rows = torch.randint(0, 256, (1000, 96), dtype=torch.uint8, device="cuda")
        cnt = (C.c_uint64 * 1)()
        ctx.check(L.igx_dist_allgather_rows(h, C.c_void_p(rows.data_ptr()), 1000, 96, None, 0, cnt))
        assert cnt[0] == 1000
        out = torch.empty_like(rows)
        assert L.igx_dist_allgather_rows(h, C.c_void_p(rows.data_ptr()), 1000, 96, C.c_void_p(out.data_ptr()),
                                         999, cnt) == A.IGX_ENOSPC
        ctx.check(L.igx_dist_allgather_rows(h, C.c_void_p(rows.data_ptr()), 1000, 96, C.c_void_p(out.data_ptr()),
                                            1000, cnt))
        torch.cuda.synchronize()
        assert torch.equal(out, rows)
        sc = (C.c_uint64 * 1)(1000)
        rc = (C.c_uint64 * 1)()
        ctx.check(L.igx_dist_alltoallv_rows(h, C.c_void_p(rows.data_ptr()), sc, 96, None, 0, rc))
        assert rc[0] == 1000
        out2 = torch.empty_like(rows)
        ctx.check(L.igx_dist_alltoallv_rows(h, C.c_void_p(rows.data_ptr()), sc, 96, C.c_void_p(out2.data_ptr()),
                                            1000, rc))
        torch.cuda.synchronize()
        assert torch.equal(out2, rows)
        # an argument error (null rows with rows to send) fails through the plan, and leaves
        # the communicator usable
        assert L.igx_dist_alltoallv_rows(h, None, sc, 96, C.c_void_p(out2.data_ptr()), 1000, rc) == A.IGX_EINVAL
        assert L.igx_dist_allgather_rows(h, C.c_void_p(rows.data_ptr()), 1000, 0, C.c_void_p(out.data_ptr()),
                                         1000, cnt) == A.IGX_EINVAL
        got = C.c_uint64()
        out3 = torch.empty_like(rows)
        ctx.check(L.igx_dist_exchange_groups(h, C.c_void_p(rows.data_ptr()), 1000, 96, 72,
                                             C.c_void_p(out3.data_ptr()), 1000, C.byref(got)))
        torch.cuda.synchronize()
        assert got.value == 1000 and torch.equal(out3, rows)   # one rank owns every key, order kept
        ctx.check(L.igx_dist_barrier(h))
        # a broken communicator: every call fails with IGX_EIO before entering a collective,
        # the all-reduce included
        ctx.check(L.igx_dist_mark_broken(h))
        assert L.igx_dist_allreduce_u32(h, C.c_void_p(hist.data_ptr()), hist.numel()) == A.IGX_EIO
        assert L.igx_dist_allgather_rows(h, C.c_void_p(rows.data_ptr()), 1000, 96, None, 0, cnt) == A.IGX_EIO
        assert L.igx_dist_alltoallv_rows(h, C.c_void_p(rows.data_ptr()), sc, 96, None, 0, rc) == A.IGX_EIO
        assert L.igx_dist_barrier(h) == A.IGX_EIO
    finally:
        ctx.check(L.igx_dist_destroy(h))


DEADLINE_CHILD = r'''
import ctypes as C, importlib, sys, time
sys.path.insert(0, ROOT)
print("start", flush=True)
import torch
igx = importlib.import_module("inspektor-gadget_amd")
A = igx._abi
torch.cuda.set_device(0)
ctx = igx.runtime.context()
L = ctx.L
ctx.bind_stream()
uid = (C.c_uint8 * A.DIST_ID_BYTES)()
assert L.igx_dist_get_unique_id(uid) == 0
h = C.c_void_p()
ctx.check(L.igx_dist_init(ctx.h, uid, 1, 0, C.byref(h)))
ctx.check(L.igx_dist_barrier(h))                         # healthy first
ctx.check(L.igx_dist_set_timeout(h, 1000))
tok = C.c_void_p()
ctx.check(L.igx_debug_hold_stream(ctx.h, 8000, C.byref(tok)))   # the stream stops here (<= ~8 s)
t0 = time.time()
rc = L.igx_dist_barrier(h)                               # its all-gather queues behind the held wave
dt = time.time() - t0
msg = L.igx_last_error(ctx.h).decode()
assert rc == A.IGX_EIO, (rc, msg)
assert "timed out after 1000 ms" in msg, msg
print(f"barrier returned {rc} after {dt:.3f}s: {msg}", flush=True)
assert 0.9 < dt < 5.0, dt                                # the deadline, not the held wave's ~8 s
# broken: every later call fails at once, without entering a collective
t1 = time.time()
assert L.igx_dist_barrier(h) == A.IGX_EIO
assert L.igx_dist_wait(h) == A.IGX_EIO
assert L.igx_dist_allreduce_u32(h, None, 0) == A.IGX_EIO
assert time.time() - t1 < 0.5
how = C.c_uint32()
t2 = time.time()
ctx.check(L.igx_debug_release(ctx.h, tok, C.byref(how)))   # release the wave, stream drains
print(f"released after {time.time() - t0:.3f}s (wave ended {how.value}), drained in {time.time() - t2:.3f}s", flush=True)
assert how.value == 1, how.value
ctx.check(L.igx_dist_destroy(h))
# a fresh communicator on the same context works again
h2 = C.c_void_p()
assert L.igx_dist_get_unique_id(uid) == 0
ctx.check(L.igx_dist_init(ctx.h, uid, 1, 0, C.byref(h2)))
ctx.check(L.igx_dist_barrier(h2))
ctx.check(L.igx_dist_wait(h2))
ctx.check(L.igx_dist_destroy(h2))
print(f"DEADLINE_OK {dt:.2f}s")
'''


def test_igx_dist_deadline_aborts_instead_of_hanging():
    """Failure detection (ncclCommGetAsyncError + timeout; the reference drops a
    silent node after its TTL, snapshotcombiner.go:91-100): a collective that cannot complete --
    here a one-rank barrier queued behind a wave held on a host-mapped flag, as a dead peer
    would hold it -- returns IGX_EIO within the communicator's deadline with the communicator
    aborted and broken, instead of hanging in hipStreamSynchronize.  In a child process."""
    code = f"ROOT = {ROOT!r}\n" + DEADLINE_CHILD
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=150)
    print(r.stdout[-1500:])
    assert r.returncode == 0 and "DEADLINE_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_igx_comm_transport_single_rank():
    """dist.IgxComm (the bench's N > 1 transport) built through a real one-rank "nccl" group:
    rank 0's unique id + status byte broadcast, igx_dist_init, an all-reduce, close -- in a
    child process so the process group does not outlive the test."""
    code = (
        "import os, sys, torch, torch.distributed as d\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import importlib; igx = importlib.import_module('inspektor-gadget_amd')\n"
        "from importlib import import_module\n"
        "dist = import_module('inspektor-gadget_amd.dist')\n"
        "torch.cuda.set_device(0)\n"
        "d.init_process_group('nccl', rank=0, world_size=1)\n"
        "c = dist.IgxComm(d)\n"
        "h = torch.arange(27 * 4, dtype=torch.int32, device='cuda').view(torch.uint32).view(4, 27)\n"
        "ref = h.clone()\n"
        "c.allreduce_u32(h)\n"
        "torch.cuda.synchronize()\n"
        "assert torch.equal(h.view(torch.int32), ref.view(torch.int32))\n"
        "c.close()\n"
        "d.destroy_process_group()\n"
        "print('igx comm ok')\n")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "igx comm ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
