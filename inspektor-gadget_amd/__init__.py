"""igx: MI355X-native event aggregation for Inspektor Gadget's hot path.

Mirrors the reference's pkg/columns (filter / sort / group), pkg/gadgets/top and the
keyed aggregations behind top tcp/file/block-io, profile block-io and advise
network-policy.  All event work runs in libigx.so (HIP kernels for gfx950) through the C
ABI declared in include/igx.h; torch supplies device memory, streams and RCCL.

The directory name contains a hyphen, so import it by string:

    igx = importlib.import_module("inspektor-gadget_amd")
"""
from ._abi import IgxError, lib  # noqa: F401  (loads libigx.so eagerly: fail loudly)

lib()

from . import runtime, engine  # noqa: E402,F401
from . import columns, filter, sort, group, top, dist, advisor, gadgets, parser, wire, textcolumns, operators  # noqa: E402,F401

__all__ = ["IgxError", "lib", "runtime", "engine", "columns", "filter", "sort", "group", "top",
           "dist", "advisor", "gadgets", "parser", "wire", "textcolumns", "operators"]
