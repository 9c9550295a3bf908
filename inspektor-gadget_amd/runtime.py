"""Device context: one igx_ctx per process/GPU, bound to torch's current HIP stream.

torch provides device memory and the stream (plumbing); every byte of event work runs
in libigx.so.  There is no CPU fallback: without the library or a GPU this raises.
"""
import ctypes as C

from ._abi import IgxError, lib, Col, SortKey, Pred

_ctx_cache = {}


def torch_mod():
    import torch
    return torch


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


class Context:
    """igx_open / igx_close wrapper.  All calls are enqueued on torch's current stream of
    the context's device, so torch ops and igx kernels are ordered with no extra syncs."""

    def __init__(self, device=0, stream=None):
        torch = torch_mod()
        if not torch.cuda.is_available():
            raise IgxError(-2, "no GPU visible: the igx path runs only on MI355X (gfx950)")
        self.device = device
        self.L = lib()
        h = C.c_void_p()
        rc = self.L.igx_open(device, 0, C.byref(h))
        if rc:
            raise IgxError(rc, "igx_open failed (gfx950 GPU required)")
        self.h = h
        self.stream = stream       # a fixed torch stream (None: follow torch's current one)
        self.bind_stream()

    def bind_stream(self, stream=None):
        torch = torch_mod()
        s = stream if stream is not None else (self.stream if self.stream is not None
                                               else torch.cuda.current_stream(self.device))
        self.check(self.L.igx_set_stream(self.h, C.c_void_p(s.cuda_stream)))

    def check(self, rc):
        if rc:
            msg = self.L.igx_last_error(self.h)
            raise IgxError(rc, msg.decode() if msg else "")
        return rc

    def sync(self):
        self.check(self.L.igx_sync(self.h))

    def close(self):
        if self.h:
            self.L.igx_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def context(device=None):
    """Process-wide context for `device` (default: torch's current device)."""
    torch = torch_mod()
    if device is None:
        device = torch.cuda.current_device()
    ctx = _ctx_cache.get(device)
    if ctx is None:
        ctx = Context(device)
        _ctx_cache[device] = ctx
    else:
        ctx.bind_stream()
    return ctx


def col_of(t, kind, width=None):
    """igx_col for a device tensor: scalars (n,) or fixed-width bytes (n, W) uint8."""
    if width is None:
        width = t.shape[1] if t.dim() == 2 else t.element_size()
    return Col(C.c_void_p(t.data_ptr()), width, kind)


def cols_array(cols):
    arr = (Col * max(1, len(cols)))(*cols)
    return arr


def dtype_kind(t):
    """igx kind of a torch tensor column."""
    torch = torch_mod()
    from . import _abi
    if t.dim() == 2:
        return _abi.KIND_BYTES
    if t.dtype in (torch.int8, torch.int16, torch.int32, torch.int64):
        return _abi.KIND_INT
    if t.dtype in (torch.uint8, torch.uint16, torch.uint32, torch.uint64):
        return _abi.KIND_UINT
    if t.dtype in (torch.float32, torch.float64):
        return _abi.KIND_FLOAT
    if t.dtype == torch.bool:
        return _abi.KIND_BOOL
    return _abi.KIND_OTHER
