// k_filter.hip -- SoA filter scan + order-preserving compaction (kernel (1)).
//
// Restates FilterEntries / FilterSpecs.MatchAll (pkg/columns/filter/filter.go:266-325):
// every predicate is `(field OP ref) != negate`, predicates AND together, nil rows are
// skipped, and survivors keep input order.
//
// Three launches, each a straight HBM stream:
//   mark     one pass over the predicate columns; one 64-bit ballot word per wave-row-group
//            (1 bit per row) + one survivor count per 1024-row tile
//   scan     exclusive scan of the tile counts (one workgroup)
//   compact  re-reads only the bitmask (n/8 bytes) and writes the u32 row ids
// Algorithmic bytes per row = sum of predicate column widths + 4 per survivor.
#include "k_common.h"

namespace {

constexpr int TB = 256;            // threads per block
constexpr int RPT = 4;             // rows per thread per tile
constexpr int TILE = TB * RPT;     // 1024 rows per tile
constexpr int WPT = TILE / 64;     // mask words per tile

__global__ __launch_bounds__(TB) void k_filter_mark(DevPreds dp, const uint8_t *__restrict__ valid,
                                                    uint64_t n, uint64_t *__restrict__ mask,
                                                    uint32_t *__restrict__ tile_cnt) {
    __shared__ uint32_t wcnt[TB / 64];
    const uint64_t tile = blockIdx.x;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        uint64_t row = tile * TILE + (uint64_t)j * TB + threadIdx.x;
        bool ok = row < n;
        if (ok && valid) ok = valid[row] != 0;
        if (ok) ok = preds_match_all(dp, row);
        uint64_t b = __ballot(ok);
        if (lane == 0) {
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

}  // namespace

int launch_filter(igx_ctx *ctx, const DevPreds &dp, const uint8_t *valid, uint64_t nrows,
                  uint32_t *out_idx, uint64_t *out_n) {
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
    hipLaunchKernelGGL(k_filter_mark, dim3(ntiles), dim3(TB), 0, ctx->stream, dp, valid, nrows,
                       mask, cnt);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, ctx->stream, cnt, ntiles, off, out_n);
    hipLaunchKernelGGL(k_filter_compact, dim3(ntiles), dim3(TB), 0, ctx->stream, mask, off, nrows,
                       out_idx);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
