// igx_internal.h -- shared host/device declarations for libigx.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>

#include "../../include/igx.h"

#define IGX_VERSION 1

struct igx_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // grow-only scratch arena (kernels never hipMalloc inside a call once warmed up)
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    // pinned host staging for small readbacks
    void *pinned = nullptr;
    size_t pinned_bytes = 0;
    // compiled regex automata on the device, by pattern (freed by igx_close)
    std::map<std::string, void *> regex;
    // igx_set_stream: the new stream waits on this event recorded on the old one
    hipEvent_t handoff = nullptr;
    // the sort's NaN flag: one device word, zero between sorts (k_andor_final clears it)
    uint32_t *nan_word = nullptr;
    // device-planned LSD passes (k_sort.hip): per-tile digit counts published by tag, so the
    // array is the context's own (never scratch: a stale word must never carry a live tag)
    uint64_t *lsd_status = nullptr;
    size_t lsd_status_words = 0;
    uint32_t lsd_epoch = 0;
};

// sets ctx->err and returns code
int igx_fail(igx_ctx *ctx, int code, const char *fmt, ...);
// hipError_t -> IGX_EIO with message
#define IGX_HIP(ctx, expr)                                                            \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return igx_fail((ctx), IGX_EIO, "%s: %s", #expr, hipGetErrorString(e_));  \
    } while (0)

// scratch: returns a device pointer with at least `bytes` (16-B aligned sub-buffers are
// carved by the caller).  May synchronise the stream when it has to grow.
int igx_scratch(igx_ctx *ctx, size_t bytes, void **out);
int igx_pinned(igx_ctx *ctx, size_t bytes, void **out);

static inline size_t igx_align(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------------
// device-side predicate (compiled igx_pred + column), passed by value in kernargs
// ---------------------------------------------------------------------------------
#define IGX_KMAX_PREDS 4
struct DevPred {
    const uint8_t *ptr;
    uint32_t width, kind, cmp, negate;
    uint32_t ref_len, pad;
    const uint8_t *dfa;   // IGX_CMP_REGEX: device regex automaton (igx_regex.h blob)
    const uint8_t *gptr;  // guard column (igx_pred.guard_*): the test applies where it equals gref
    uint64_t gref;
    uint32_t gwidth, gpad;   // gwidth 0: unguarded
    uint8_t ref[IGX_MAX_REF];
};
struct DevPreds {
    uint32_t n, pad;
    DevPred p[IGX_KMAX_PREDS];
};
int igx_build_preds(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred *preds,
                    uint32_t npreds, DevPreds *out);
// a predicate's guard (igx_pred.guard_*): validated against the columns; its value as u64
int igx_check_guard(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, const igx_pred &p);
uint64_t igx_guard_ref(const igx_pred &p);

// ---------------------------------------------------------------------------------
// launchers (defined in the k_*.hip files)
// ---------------------------------------------------------------------------------
int launch_filter(igx_ctx *ctx, const DevPreds &dp, const uint8_t *valid, uint64_t nrows,
                  uint32_t *out_idx, uint64_t *out_n);
int launch_filter_chunks(igx_ctx *ctx, const DevPreds *dps, uint32_t nchunks, uint32_t any,
                         uint32_t nil_match, const uint8_t *valid, uint64_t nrows, uint32_t *out_idx,
                         uint64_t *out_n);

struct SortPlanKey {
    const uint8_t *ptr;
    uint32_t width, kind, desc_eff, words, stride;
    uint32_t direct;   // row r reads this key at r even when a rowmap is given
};
// IP text of n rows (rowmap nullable) -> out, n x IGX_IPTEXT_WIDTH bytes (k_sort.hip)
int launch_ip_text(igx_ctx *ctx, const uint8_t *addr, uint32_t astride, const uint8_t *fam, uint32_t fstride,
                   const uint32_t *rowmap, uint64_t n, uint8_t *out);
// One sort pass as sort.go runs it (raw sortBy order and direction), for the exact SliceStable
// path (k_gostable.hip) that a NaN in a float key needs.
struct GoSortKey {
    const uint8_t *ptr;
    uint32_t width, kind, stride;
    uint32_t asc;     // no '-' prefix (columns.OrderAsc)
    uint32_t konst;   // constant column (no data): a pass that compares every row equal
};
// rowmap (device, nullable): row r reads its keys / pos at rowmap[r] and the permutation
// reports rowmap[r] (used to sort a table's groups through its slot list).  gokeys (nullable):
// every pass in sortBy order, for the exact path when a float key holds a NaN (without them that
// case returns IGX_ENOTSUP).  d_nrows (device, nullable): the row count lives on the device and
// nrows is only its upper bound -- top-K without a float key or nil mask only (the device
// selection); out_perm entries past the count are 0xFFFFFFFF.
// A table's top-K hint (k_sort.hip, the device selection over a table's groups): the slots
// of its last top-K.  The k smallest composed keys of ALL groups are <= the k-th smallest of
// ANY k groups, so the groups at or below that bound hold the top-K whatever the hints are:
// hints only decide how tight the bound is (how few rows are ranked), never the result.
constexpr uint32_t TK_MAXK = 1024;
constexpr size_t TK_STATE_BYTES = 64 + 2048 * 4;   // counters + bound, then the candidates
struct TopkHint {
    uint32_t *slots;       // device, TK_MAXK words: read, then rewritten with this call's top-K
    uint32_t nh;           // slots held (0: none yet); the call sets it to its k
    const uint32_t *occ;   // the interval's occupancy bitmap: a hint counts iff its slot is a group
    uint64_t nslots;
    uint32_t *state;       // device, TK_STATE_BYTES
};
int launch_sort_perm(igx_ctx *ctx, const SortPlanKey *keys, uint32_t nkeys, uint64_t nrows,
                     const uint64_t *pos, bool pos_not, const uint8_t *valid,
                     uint32_t *out_perm, uint32_t limit, const uint32_t *rowmap,
                     uint32_t pos_stride = 8, const GoSortKey *gokeys = nullptr, uint32_t ngokeys = 0,
                     const uint64_t *d_nrows = nullptr, TopkHint *hint = nullptr);
// data (device, n rows in the pre-sort order) sorted in place by Go 1.19 SliceStable, pass by pass
int launch_go_stable(igx_ctx *ctx, const GoSortKey *keys, uint32_t nkeys, uint64_t nrows, const uint8_t *valid,
                     uint32_t *data);
// closed-form planning + launch (igx_host.cpp); strides per key (nullable = widths)
int sort_common_rows(igx_ctx *ctx, const igx_sortkey *keys, const uint32_t *strides, uint32_t nkeys,
                     uint64_t nrows, const uint32_t *rowmap, const uint64_t *pos, uint32_t pos_stride,
                     uint32_t limit, uint32_t *out, uint32_t direct_mask = 0, const uint64_t *d_nrows = nullptr,
                     TopkHint *hint = nullptr);

int launch_hist_log2(igx_ctx *ctx, const uint32_t *dev, const uint32_t *cont,
                     const int64_t *delta, uint64_t nrows, const uint32_t *devs, uint32_t ndev,
                     uint32_t ncont, uint64_t divisor, uint32_t nslots, uint32_t *hist);
int launch_log2_slots(igx_ctx *ctx, const int64_t *delta, uint64_t n, uint64_t divisor, uint32_t nslots,
                      uint8_t *slot, uint8_t *keep);
