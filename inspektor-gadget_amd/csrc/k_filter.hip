// k_filter.hip -- SoA filter scan + order-preserving compaction (kernel (1)).
//
// Restates FilterEntries / FilterSpecs.MatchAll (pkg/columns/filter/filter.go:266-325):
// every predicate is `(field OP ref) != negate`, predicates AND together, nil rows are
// skipped, and survivors keep input order.
//
// Two or three launches, each a straight HBM stream:
//   mark     one pass over the predicate columns; one 64-bit ballot word per wave-row-group
//            (1 bit per row) + one survivor count per 1024-row tile
//   scan     exclusive scan of the tile counts (one workgroup; up to 16M rows the compaction
//            sums its tile's predecessors itself instead)
//   compact  re-reads only the bitmask (n/8 bytes) and writes the u32 row ids
// Algorithmic bytes per row = sum of predicate column widths + 4 per survivor.
#include <cstdlib>

#include "k_common.h"

namespace {

constexpr int TB = 256;            // threads per block
constexpr int RPT = 4;             // rows per thread per tile
constexpr int TILE = TB * RPT;     // 1024 rows per tile
constexpr int WPT = TILE / 64;     // mask words per tile

// any = 0: AND of dp's predicates (MatchAll); any = 1: OR (MatchAny).  acc = 1 combines the
// tile's bits (AND / OR) with the mask an earlier launch wrote (more than IGX_KMAX_PREDS
// specs); the counts are always those of the combined mask.  nil_bit is what a nil row
// (valid == 0) yields for this chunk: 0 for FilterEntries, which skips nil entries
// (filter.go:310-314); the AND (MatchAll) or OR (MatchAny) of the chunk's negate flags for
// FilterSpecs.Match(nil) == negate (filter.go:286-291).
__global__ __launch_bounds__(TB) void k_filter_mark(DevPreds dp, const uint8_t *__restrict__ valid,
                                                    uint64_t n, uint64_t *__restrict__ mask,
                                                    uint32_t *__restrict__ tile_cnt, uint32_t any,
                                                    uint32_t acc, uint32_t nil_bit) {
    __shared__ uint32_t wcnt[TB / 64];
    const uint64_t tile = blockIdx.x;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        uint64_t row = tile * TILE + (uint64_t)j * TB + threadIdx.x;
        bool ok = row < n;
        if (ok && valid && valid[row] == 0) ok = nil_bit != 0;
        else if (ok) ok = any ? preds_match_any(dp, row) : preds_match_all(dp, row);
        uint64_t b = __ballot(ok);
        if (lane == 0) {
            if (acc) {
                const uint64_t prev = mask[tile * WPT + j * (TB / 64) + wave];
                b = any ? (b | prev) : (b & prev);
            }
            mask[tile * WPT + j * (TB / 64) + wave] = b;
            cnt += __popcll(b);
        }
    }
    if (lane == 0) wcnt[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int w = 0; w < TB / 64; ++w) s += wcnt[w];
        tile_cnt[tile] = s;
    }
}

// The same mark for chunks of integer predicates only (1/2/4/8-byte columns, no guard, no
// regex): every row's predicate values -- and its nil byte -- are loaded, zero-extended,
// before any is compared, so a tile's loads retire under one wait.  (The generic kernel's
// short-circuit AND puts each predicate's load behind the previous one's branch: C1's two
// predicates over 1M rows, 17 us.)
__device__ __forceinline__ bool pred_eval_int(const DevPred &d, uint64_t a) {
    const bool sign = d.kind == IGX_KIND_INT;
    if (sign && d.width < 8) {
        const uint64_t m = 1ull << (8 * d.width - 1);
        a = (a ^ m) - m;
    }
    const uint64_t b = ref_scalar(d, sign);
    const int c = sign ? ((int64_t)a < (int64_t)b ? -1 : ((int64_t)a > (int64_t)b ? 1 : 0))
                       : (a < b ? -1 : (a > b ? 1 : 0));
    bool r;
    switch (d.cmp) {
    case IGX_CMP_EQ: r = c == 0; break;
    case IGX_CMP_LT: r = c < 0; break;
    case IGX_CMP_LE: r = c <= 0; break;
    case IGX_CMP_GT: r = c > 0; break;
    case IGX_CMP_GE: r = c >= 0; break;
    default: r = false;
    }
    return r != (d.negate != 0);
}

__global__ __launch_bounds__(TB) void k_filter_mark_int(DevPreds dp, const uint8_t *__restrict__ valid,
                                                        uint64_t n, uint64_t *__restrict__ mask,
                                                        uint32_t *__restrict__ tile_cnt, uint32_t any,
                                                        uint32_t acc, uint32_t nil_bit) {
    __shared__ uint32_t wcnt[TB / 64];
    const uint64_t tile = blockIdx.x;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint64_t v[RPT][IGX_KMAX_PREDS];
    uint32_t nb[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const uint64_t row = tile * TILE + (uint64_t)j * TB + threadIdx.x;
        const uint64_t r = row < n ? row : n - 1;
        nb[j] = valid ? valid[r] : 1u;
#pragma unroll
        for (int p = 0; p < IGX_KMAX_PREDS; ++p)
            v[j][p] = (uint32_t)p < dp.n ? ld_scalar(dp.p[p].ptr, dp.p[p].width, r, false) : 0ull;
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const uint64_t row = tile * TILE + (uint64_t)j * TB + threadIdx.x;
        bool ok = row < n;
        if (ok && nb[j] == 0) {
            ok = nil_bit != 0;
        } else if (ok) {
            bool m = !any;
#pragma unroll
            for (int p = 0; p < IGX_KMAX_PREDS; ++p) {
                if ((uint32_t)p < dp.n) {
                    const bool r = pred_eval_int(dp.p[p], v[j][p]);
                    m = any ? (m || r) : (m && r);
                }
            }
            ok = m;
        }
        uint64_t b = __ballot(ok);
        if (lane == 0) {
            if (acc) {
                const uint64_t prev = mask[tile * WPT + j * (TB / 64) + wave];
                b = any ? (b | prev) : (b & prev);
            }
            mask[tile * WPT + j * (TB / 64) + wave] = b;
            cnt += __popcll(b);
        }
    }
    if (lane == 0) wcnt[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int w = 0; w < TB / 64; ++w) s += wcnt[w];
        tile_cnt[tile] = s;
    }
}

// exclusive scan of cnt[0..m) -> off[0..m), total -> *total (u64); one block of 1024
__global__ __launch_bounds__(1024) void k_scan_counts(const uint32_t *__restrict__ cnt, uint64_t m,
                                                      uint64_t *__restrict__ off,
                                                      uint64_t *__restrict__ total) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (m + 1023) / 1024;
    const uint64_t b = threadIdx.x * per, e = min(m, b + per);
    uint64_t s = 0;
    for (uint64_t i = b; i < e; ++i) s += cnt[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (uint64_t i = b; i < e; ++i) {
        off[i] = run;
        run += cnt[i];
    }
    if (threadIdx.x == 1023) *total = part[1023];
}

__global__ __launch_bounds__(TB) void k_filter_compact(const uint64_t *__restrict__ mask,
                                                       const uint64_t *__restrict__ tile_off,
                                                       uint64_t n, uint32_t *__restrict__ out) {
    __shared__ uint32_t wpre[WPT];
    const uint64_t tile = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    if (threadIdx.x < WPT) {
        // prefix over the tile's 16 words (tiny; each thread sums its predecessors)
        uint32_t s = 0;
        for (int w = 0; w < (int)threadIdx.x; ++w) s += __popcll(mask[tile * WPT + w]);
        wpre[threadIdx.x] = s;
    }
    __syncthreads();
    const uint64_t base = tile_off[tile];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        uint32_t k = j * TB + threadIdx.x;       // row within tile
        uint32_t w = k >> 6;                      // == j*4 + wave
        uint64_t m = mask[tile * WPT + w];
        if ((m >> lane) & 1ull) {
            uint64_t pos = base + wpre[w] + __popcll(m & lanemask_lt());
            out[pos] = (uint32_t)(tile * TILE + k);
        }
    }
}

// k_scan_counts + k_filter_compact in one launch, for up to SF_MAX_TILES tiles: each tile
// sums the counts of the tiles before it itself (at most SF_MAX_TILES / TB loads per thread),
// and the last tile writes the survivor count.  That work grows with the square of the tile
// count; measured per kernel (profiles/r06/filter_scale.txt): 1M rows 7.3 us fused
// vs 4.6 + 5.6 split, 4M 13.9 vs 9.4 + 5.6, 16M 58.4 vs 26.7 + 5.6 -- so the fused form stops
// at 4M rows.
constexpr uint64_t SF_MAX_TILES = 4096;
__global__ __launch_bounds__(TB) void k_filter_compact_sf(const uint64_t *__restrict__ mask,
                                                          const uint32_t *__restrict__ cnt, uint64_t ntiles,
                                                          uint32_t *__restrict__ out, uint64_t *__restrict__ out_n) {
    __shared__ uint32_t wpre[WPT];
    __shared__ uint64_t red[TB / 64];
    const uint64_t tile = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t s = 0;
#pragma unroll 4
    for (uint64_t i = threadIdx.x; i < tile; i += TB) s += cnt[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) red[wave] = s;
    if (threadIdx.x < WPT) {
        uint32_t p = 0;
#pragma unroll
        for (int w = 0; w < WPT; ++w)
            if (w < (int)threadIdx.x) p += __popcll(mask[tile * WPT + w]);
        wpre[threadIdx.x] = p;
    }
    __syncthreads();
    uint64_t base = 0;
#pragma unroll
    for (int w = 0; w < TB / 64; ++w) base += red[w];
    if (tile == ntiles - 1 && threadIdx.x == 0) *out_n = base + cnt[tile];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const uint32_t k = j * TB + threadIdx.x;   // row within tile
        const uint32_t w = k >> 6;                 // == j*4 + wave
        const uint64_t m = mask[tile * WPT + w];
        if ((m >> lane) & 1ull) out[base + wpre[w] + __popcll(m & lanemask_lt())] = (uint32_t)(tile * TILE + k);
    }
}

}  // namespace

int launch_filter(igx_ctx *ctx, const DevPreds &dp, const uint8_t *valid, uint64_t nrows,
                  uint32_t *out_idx, uint64_t *out_n) {
    return launch_filter_chunks(ctx, &dp, 1, 0, 0, valid, nrows, out_idx, out_n);
}

int launch_filter_chunks(igx_ctx *ctx, const DevPreds *dps, uint32_t nchunks, uint32_t any,
                         uint32_t nil_match, const uint8_t *valid, uint64_t nrows, uint32_t *out_idx,
                         uint64_t *out_n) {
    if (nrows == 0) {
        IGX_HIP(ctx, hipMemsetAsync(out_n, 0, sizeof(uint64_t), ctx->stream));
        return IGX_OK;
    }
    const uint64_t ntiles = (nrows + TILE - 1) / TILE;
    size_t mask_b = igx_align(ntiles * WPT * 8, 256);
    size_t cnt_b = igx_align(ntiles * 4, 256);
    size_t off_b = igx_align(ntiles * 8, 256);
    void *s;
    int rc = igx_scratch(ctx, mask_b + cnt_b + off_b, &s);
    if (rc) return rc;
    auto *mask = reinterpret_cast<uint64_t *>(s);
    auto *cnt = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(s) + mask_b);
    auto *off = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(s) + mask_b + cnt_b);
    for (uint32_t c = 0; c < nchunks; ++c) {
        // Match(nil) == negate, combined over the chunk like the predicates themselves
        uint32_t nil_bit = any ? 0u : 1u;
        for (uint32_t p = 0; p < dps[c].n; ++p)
            nil_bit = any ? (nil_bit | (dps[c].p[p].negate != 0)) : (nil_bit & (dps[c].p[p].negate != 0));
        if (!nil_match) nil_bit = 0;
        bool ints = true;   // integer predicates only: the kernel that loads before it compares
        for (uint32_t p = 0; p < dps[c].n; ++p) {
            const DevPred &d = dps[c].p[p];
            ints = ints && (d.kind == IGX_KIND_INT || d.kind == IGX_KIND_UINT) && d.gwidth == 0 &&
                   (d.width == 1 || d.width == 2 || d.width == 4 || d.width == 8) &&
                   (d.cmp == IGX_CMP_EQ || d.cmp == IGX_CMP_LT || d.cmp == IGX_CMP_LE || d.cmp == IGX_CMP_GT ||
                    d.cmp == IGX_CMP_GE);
        }
        if (ints)
            hipLaunchKernelGGL(k_filter_mark_int, dim3(ntiles), dim3(TB), 0, ctx->stream, dps[c], valid, nrows,
                               mask, cnt, any, c > 0 ? 1u : 0u, nil_bit);
        else
            hipLaunchKernelGGL(k_filter_mark, dim3(ntiles), dim3(TB), 0, ctx->stream, dps[c], valid, nrows,
                               mask, cnt, any, c > 0 ? 1u : 0u, nil_bit);
    }
    uint64_t sf_max = SF_MAX_TILES;
    if (const char *e = std::getenv("IGX_FILTER_SF_MAX")) sf_max = std::strtoull(e, nullptr, 0);   // A/B knob
    if (ntiles <= sf_max) {
        hipLaunchKernelGGL(k_filter_compact_sf, dim3(ntiles), dim3(TB), 0, ctx->stream, mask, cnt, ntiles, out_idx,
                           out_n);
    } else {
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, ctx->stream, cnt, ntiles, off, out_n);
        hipLaunchKernelGGL(k_filter_compact, dim3(ntiles), dim3(TB), 0, ctx->stream, mask, off, nrows,
                           out_idx);
    }
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

// ---- row gather (the compacted batch FilterEntries returns) ---------------------------------
// One thread per (row, column): copies the row's width bytes in the widest unit that divides
// the width and both base addresses.  Output rows are consecutive, so writes coalesce; reads
// follow idx (ascending after a filter).  Indices >= nrows produce zero rows.
namespace {

constexpr uint32_t TAKE_MAXC = 16;

struct TakeArgs {
    const uint8_t *src[TAKE_MAXC];
    uint8_t *dst[TAKE_MAXC];
    uint32_t width[TAKE_MAXC];
    uint32_t unit[TAKE_MAXC];
};

template <typename U>
__device__ __forceinline__ void take_copy(const uint8_t *s, uint8_t *d, uint32_t width, bool ok) {
    const U *su = reinterpret_cast<const U *>(s);
    U *du = reinterpret_cast<U *>(d);
    for (uint32_t w = 0; w < width / sizeof(U); ++w) du[w] = ok ? su[w] : U{};
}

__global__ __launch_bounds__(TB) void k_take(TakeArgs a, const uint32_t *__restrict__ idx, uint64_t k,
                                             uint64_t nrows, uint64_t r0) {
    const uint64_t r = r0 + (uint64_t)blockIdx.x * TB + threadIdx.x;
    if (r >= k) return;
    const uint32_t c = blockIdx.y;
    const uint32_t width = a.width[c];
    const uint64_t g = idx[r];
    const bool ok = g < nrows;
    const uint8_t *s = a.src[c] + (ok ? g : 0) * width;
    uint8_t *d = a.dst[c] + r * width;
    switch (a.unit[c]) {
    case 16: take_copy<uint4>(s, d, width, ok); break;
    case 8: take_copy<uint64_t>(s, d, width, ok); break;
    case 4: take_copy<uint32_t>(s, d, width, ok); break;
    case 2: take_copy<uint16_t>(s, d, width, ok); break;
    default: take_copy<uint8_t>(s, d, width, ok); break;
    }
}

}  // namespace

extern "C" int igx_take(igx_ctx *ctx, const igx_col *cols, uint32_t ncols, uint64_t nrows,
                        const uint32_t *idx, uint64_t k, void *const *out) {
    if (!ctx) return IGX_EINVAL;
    if (k == 0 || ncols == 0) return IGX_OK;
    if (!cols || !idx || !out) return igx_fail(ctx, IGX_EINVAL, "take: null argument");

    for (uint32_t c0 = 0; c0 < ncols; c0 += TAKE_MAXC) {
        const uint32_t nc = ncols - c0 < TAKE_MAXC ? ncols - c0 : TAKE_MAXC;
        TakeArgs a{};
        for (uint32_t j = 0; j < nc; ++j) {
            const igx_col &col = cols[c0 + j];
            if (!col.ptr || !out[c0 + j] || col.width == 0)
                return igx_fail(ctx, IGX_EINVAL, "take: column %u has no data", c0 + j);
            a.src[j] = static_cast<const uint8_t *>(col.ptr);
            a.dst[j] = static_cast<uint8_t *>(out[c0 + j]);
            a.width[j] = col.width;
            const uint64_t al = (uint64_t)(uintptr_t)col.ptr | (uint64_t)(uintptr_t)out[c0 + j] | col.width;
            a.unit[j] = (al & 15) == 0 ? 16 : (al & 7) == 0 ? 8 : (al & 3) == 0 ? 4 : (al & 1) == 0 ? 2 : 1;
        }
        // at most 2^20 blocks per launch (a grid dimension is capped at 2^32 - 1 work-items)
        constexpr uint64_t ROWS = (1ull << 20) * TB;
        for (uint64_t r0 = 0; r0 < k; r0 += ROWS) {
            const uint64_t m = std::min<uint64_t>(ROWS, k - r0);
            hipLaunchKernelGGL(k_take, dim3((unsigned)((m + TB - 1) / TB), nc), dim3(TB), 0, ctx->stream, a, idx, k,
                               nrows, r0);
        }
    }
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
