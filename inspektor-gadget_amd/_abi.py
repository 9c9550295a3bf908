"""ctypes mirror of include/igx.h (the C ABI of libigx.so).

This is the same surface a Go caller binds with cgo; the Python host
layer uses it so the parity tests exercise exactly what a drop-in caller would call.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IGX_LIB") or os.path.join(HERE, "libigx.so")   # IGX_LIB: A/B builds
if os.environ.get("IGX_LIB"):
    # an experimental build replaces the in-tree one for the whole process: say so, and
    # bench.py records the path in its JSON line (`library`)
    import sys as _sys
    print(f"inspektor-gadget_amd: IGX_LIB={LIB_PATH}", file=_sys.stderr, flush=True)

IGX_OK = 0
IGX_ENOENT = -2
IGX_EIO = -5
IGX_ENOMEM = -12
IGX_EINVAL = -22
IGX_ENOSPC = -28
IGX_ENOTSUP = -95

KIND_INT, KIND_UINT, KIND_FLOAT, KIND_BYTES, KIND_BOOL, KIND_OTHER = range(6)
CMP_EQ, CMP_REGEX, CMP_LT, CMP_LE, CMP_GT, CMP_GE, CMP_IN = range(7)
COL_VIRTUAL, COL_EXTRACTOR = 1, 2
NO_COL = 0xFFFFFFFF
MAX_REF = 256
AGG_COUNT, AGG_SUM = 0, 1
FILTER_ANY, FILTER_NIL_MATCH = 1, 2
GB_AUTO, GB_CACHED, GB_DIRECT, GB_PART = 0, 1, 2, 3


class SchemaCol(C.Structure):
    _fields_ = [("name", C.c_char_p), ("kind", C.c_uint32), ("width", C.c_uint32),
                ("flags", C.c_uint32), ("raw_kind", C.c_uint32)]


class Col(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("width", C.c_uint32), ("kind", C.c_uint32)]


class Pred(C.Structure):
    _fields_ = [("col", C.c_uint32), ("cmp", C.c_uint32), ("negate", C.c_uint32),
                ("ref_len", C.c_uint32), ("ref", C.c_uint8 * MAX_REF),
                ("guard_col", C.c_uint32), ("guard_len", C.c_uint32), ("guard_ref", C.c_uint8 * 8)]


class SortKey(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("width", C.c_uint32), ("kind", C.c_uint32),
                ("desc", C.c_uint32), ("col", C.c_uint32)]


class GroupbyInfo(C.Structure):
    _fields_ = [("form", C.c_uint32), ("region", C.c_uint32), ("part_left", C.c_uint32),
                ("exact_left", C.c_uint32), ("sm_probers", C.c_uint32), ("loaders", C.c_uint32),
                ("rows", C.c_uint64), ("miss_permille", C.c_uint32), ("persist", C.c_uint32),
                ("claims", C.c_uint64), ("gen_keys", C.c_uint64)]


class Agg(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("col", C.c_uint32), ("cond_col", C.c_uint32),
                ("out_width", C.c_uint32), ("cond_val", C.c_uint64), ("divisor", C.c_uint64)]


class TableView(C.Structure):
    _fields_ = [("n_groups", C.c_uint64), ("n_slots", C.c_uint64), ("key_bytes", C.c_uint32),
                ("key_stride", C.c_uint32), ("val_stride", C.c_uint32), ("naggs", C.c_uint32),
                ("keys", C.c_void_p),
                ("aggs", C.c_void_p * 16), ("first_idx", C.c_void_p), ("groups", C.c_void_p),
                ("d_n_groups", C.c_void_p)]


TSRC_AGG, TSRC_FIRST, TSRC_KEY, TSRC_CONST, TSRC_IPTEXT = 0, 1, 2, 3, 4
IPTEXT_WIDTH = 40


class TSortKey(C.Structure):
    _fields_ = [("src", C.c_uint32), ("index", C.c_uint32), ("offset", C.c_uint32),
                ("width", C.c_uint32), ("kind", C.c_uint32), ("desc", C.c_uint32)]


class OpenCols(C.Structure):
    """igx_open_cols: device outputs of igx_ingest_open_events (NULL = skipped)."""
    _fields_ = [(f, C.c_void_p) for f in ("timestamp", "pid", "uid", "mntns", "ret", "fd", "err",
                                           "comm", "path")]


OPEN_SAMPLE_BYTES = 304
DIST_ID_BYTES = 128
DIST_MAX_RANKS = 64
DIST_F_BADARG, DIST_F_QUERY = 1, 2


class DistPlan(C.Structure):
    """igx_dist_plan: the all-ranks decision and row offsets of a row exchange."""
    _fields_ = [("status", C.c_int32), ("culprit", C.c_int32), ("total_rows", C.c_uint64),
                ("recv_counts", C.c_uint64 * DIST_MAX_RANKS), ("send_off", C.c_uint64 * DIST_MAX_RANKS),
                ("recv_off", C.c_uint64 * DIST_MAX_RANKS)]


class IgxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"igx error {code}: {msg}")
        self.code = code


# (name, restype, argtypes) for every symbol of include/igx.h
_VP, _U32, _U64, _SZ, _I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
SIGNATURES = [
    ("igx_open", _I, [_I, _U32, C.POINTER(_VP)]),
    ("igx_close", _I, [_VP]),
    ("igx_last_error", C.c_char_p, [_VP]),
    ("igx_set_stream", _I, [_VP, _VP]),
    ("igx_get_stream", _VP, [_VP]),
    ("igx_sync", _I, [_VP]),
    ("igx_malloc", _I, [_VP, _SZ, C.POINTER(_VP)]),
    ("igx_free", _I, [_VP, _VP]),
    ("igx_memcpy_h2d", _I, [_VP, _VP, _VP, _SZ]),
    ("igx_memcpy_d2h", _I, [_VP, _VP, _VP, _SZ]),
    ("igx_memcpy_d2d", _I, [_VP, _VP, _VP, _SZ]),
    ("igx_version", _I, []),
    ("igx_filter_parse", _I, [C.POINTER(SchemaCol), _U32, C.c_char_p, C.POINTER(Pred),
                              C.c_char_p, _SZ]),
    ("igx_regex_compile_blob", _I, [C.c_char_p, _SZ, _VP, _SZ, C.POINTER(_SZ), C.c_char_p, _SZ]),
    ("igx_filter", _I, [_VP, C.POINTER(Col), _U32, C.POINTER(Pred), _U32, _VP, _U64, _VP, _VP]),
    ("igx_filter_any", _I, [_VP, C.POINTER(Col), _U32, C.POINTER(Pred), _U32, _VP, _U64, _VP, _VP]),
    ("igx_filter_ex", _I, [_VP, C.POINTER(Col), _U32, C.POINTER(Pred), _U32, _VP, _U64, _U32, _VP,
                           _VP]),
    ("igx_take", _I, [_VP, C.POINTER(Col), _U32, _U64, _VP, _U64, C.POINTER(_VP)]),
    ("igx_sort_prepare", _I, [C.POINTER(SchemaCol), _U32, C.POINTER(C.c_char_p), _U32,
                              C.POINTER(SortKey), C.POINTER(_U32), C.POINTER(_U32)]),
    ("igx_sort_perm", _I, [_VP, C.POINTER(SortKey), _U32, _U64, _VP, _VP, _VP]),
    ("igx_sort_perm_ex", _I, [_VP, C.POINTER(SortKey), _U32, _U64, _VP, _VP, _VP, _VP]),
    ("igx_sort_perm_dn", _I, [_VP, C.POINTER(SortKey), _U32, _U64, _VP, _VP, _VP, _VP, _VP]),
    ("igx_topk", _I, [_VP, C.POINTER(SortKey), _U32, _U64, _VP, _U32, _VP]),
    ("igx_groupby_create", _I, [_VP, C.POINTER(_U32), _U32, C.POINTER(Agg), _U32, _U64,
                                C.POINTER(_VP)]),
    ("igx_groupby_update", _I, [_VP, C.POINTER(Col), _U32, C.POINTER(_U32), C.POINTER(Pred),
                                _U32, _U64, _U64]),
    ("igx_groupby_update_ex", _I, [_VP, C.POINTER(Col), _U32, C.POINTER(_U32), C.POINTER(Pred),
                                   _U32, _VP, _U32, _U64, _U64]),
    ("igx_groupby_finalize", _I, [_VP, C.POINTER(TableView)]),
    ("igx_groupby_finalize_async", _I, [_VP, C.POINTER(TableView)]),
    ("igx_groupby_wait", _I, [_VP, C.POINTER(C.c_uint64)]),
    ("igx_groupby_info", _I, [_VP, C.POINTER(GroupbyInfo)]),
    ("igx_groupby_gather", _I, [_VP, _VP, _U64, _VP]),
    ("igx_groupby_sort", _I, [_VP, C.POINTER(TSortKey), _U32, _U32, _VP]),
    ("igx_segment_fsum", _I, [_VP, _VP, _U32, _U32, _VP, _U64, _VP, _VP, _U32, _VP]),
    ("igx_ip_text", _I, [_VP, _VP, _U32, _VP, _U32, _VP, _U64, _VP]),
    ("igx_groupby_reset", _I, [_VP]),
    ("igx_groupby_set_mode", _I, [_VP, _U32]),
    ("igx_groupby_destroy", _I, [_VP]),
    ("igx_groupby_debug_counts", _I, [_VP, _VP]),
    ("igx_groupby_topk_counts", _I, [_VP, _VP]),
    ("igx_np_mark", _I, [_VP, _VP, _VP, _VP, _VP, _U64, _VP]),
    ("igx_hist_log2", _I, [_VP, _VP, _VP, _VP, _U64, C.POINTER(_U32), _U32, _U32, _U64, _U32,
                           _VP]),
    ("igx_log2_slots", _I, [_VP, _VP, _U64, _U64, _U32, _VP, _VP]),
    ("igx_partition_rows", _I, [_VP, _VP, _U64, _U32, _U32, _U32, _VP, _VP]),
    ("igx_partition_groups", _I, [_VP, _VP, _VP, _U32, _VP, _U64, _VP]),
    ("igx_dist_get_unique_id", _I, [_VP]),
    ("igx_dist_init", _I, [_VP, _VP, _I, _I, C.POINTER(_VP)]),
    ("igx_dist_destroy", _I, [_VP]),
    ("igx_dist_rank", _I, [_VP, C.POINTER(_I), C.POINTER(_I)]),
    ("igx_dist_barrier", _I, [_VP]),
    ("igx_dist_mark_broken", _I, [_VP]),
    ("igx_dist_set_timeout", _I, [_VP, _I]),
    ("igx_dist_wait", _I, [_VP]),
    ("igx_dist_allreduce_u32", _I, [_VP, _VP, _U64]),
    ("igx_dist_allgather_rows", _I, [_VP, _VP, _U64, _U32, _VP, _U64, C.POINTER(_U64)]),
    ("igx_dist_alltoallv_rows", _I, [_VP, _VP, C.POINTER(_U64), _U32, _VP, _U64, C.POINTER(_U64)]),
    ("igx_dist_exchange_groups", _I, [_VP, _VP, _U64, _U32, _U32, _VP, _U64, C.POINTER(_U64)]),
    ("igx_dist_plan_alltoallv", _I, [_I, _I, C.POINTER(_U64), C.POINTER(DistPlan)]),
    ("igx_dist_plan_allgather", _I, [_I, _I, C.POINTER(_U64), C.POINTER(DistPlan)]),
    ("igx_ingest_open_events", _I, [_VP, _VP, _U64, _U32, C.c_int64, C.POINTER(OpenCols)]),
    ("igx_ingest_aos", _I, [_VP, _VP, _U64, _U32, C.POINTER(_U32), C.POINTER(_U32), _U32,
                            C.POINTER(_VP)]),
    ("igx_debug_hold_stream", _I, [_VP, _U32, C.POINTER(_VP)]),
    ("igx_debug_release", _I, [_VP, _VP, C.POINTER(_U32)]),
    ("igx_gen_tcp", _I, [_VP, _U64, _U64, _U64, _U64, _U64, _VP, _U64, _U64] + [_VP] * 10),
    ("igx_gen_open", _I, [_VP, _U64, _VP, _U64, _U64] + [_VP] * 8),
    ("igx_gen_bio", _I, [_VP, _U64, _VP, _U64, _U64, _U64, _VP, _VP, _VP]),
    ("igx_gen_np", _I, [_VP, _U64, _U64, _U64, _U64, _U64] + [_VP] * 8),
    ("igx_gen_file", _I, [_VP, _U64, _U64, _U64, _U64, _U64, _VP, _U64, _U64] + [_VP] * 6),
]

_lib = None


def lib():
    """Load libigx.so.  There is no fallback: the product path fails loudly without it."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() "
                              "(or `make -C inspektor-gadget_amd/csrc`)")
        # torch bundles its own libamdhip64 / libhsa-runtime64 / librccl under the same
        # sonames as /opt/rocm's.  Whichever loads first serves the process, so torch goes
        # first: libigx.so loaded before it pulls in /opt/rocm's runtime, and torch on top
        # of that runtime leaves hipGetDeviceCount failing inside libigx (igx_open ENOENT).
        import torch  # noqa: F401
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib
