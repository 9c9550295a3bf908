// k_partition.hip -- data movement on either side of the aggregation path.
//
// igx_partition_rows: the sender side of the group-by all-to-all:
//   every packed row (key | partial aggregates | first index) goes to the rank that owns
//   its key, owner = FNV-1a over the key's u32 words mod nparts (the same value on every
//   rank and device).  Rows come out grouped by owner, stable within an owner, so one
//   all-to-all moves them.  Two passes over fixed row chunks: an owner histogram per chunk,
//   a scan, then a stable scatter (ranks within a wave by ballot over the owners present,
//   across waves through LDS).
// igx_ingest_aos: the step before the path: records in the
//   reference's wire formats -- BPF map dumps of {key struct, value struct}
//   (`tcptopIpKeyT` 72 B + `tcptopTrafficT` 16 B, `filetopFileId` 24 B, `biotopInfoT` 40 B,
//   `biolatencyHistKey` 8 B; `*_bpfel_x86.go`) or perf-ring event structs -- are cut into
//   the SoA columns the kernels stream.  Field = (byte offset in the record, width).
#include <algorithm>
#include <vector>

#include "k_common.h"

namespace {

constexpr int PTB = 1024;           // threads per block
constexpr uint32_t PMAXP = 64;      // parts

__device__ __forceinline__ uint32_t row_owner(const uint8_t *row, uint32_t key_words, uint32_t nparts) {
    uint32_t h = 0x811C9DC5u;
    for (uint32_t w = 0; w < key_words; ++w) h = (h ^ reinterpret_cast<const uint32_t *>(row)[w]) * 16777619u;
    return h % nparts;
}

__global__ __launch_bounds__(PTB) void k_part_hist(const uint8_t *__restrict__ rows, uint64_t n, uint32_t row_bytes,
                                                   uint32_t key_words, uint32_t nparts, uint64_t chunk,
                                                   uint32_t *__restrict__ hist /* [nparts][nblocks] */) {
    __shared__ uint32_t cnt[PMAXP];
    if (threadIdx.x < PMAXP) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk, b1 = min(n, b0 + chunk);
    for (uint64_t r = b0 + threadIdx.x; r < b1; r += PTB)
        atomicAdd(&cnt[row_owner(rows + r * row_bytes, key_words, nparts)], 1u);
    __syncthreads();
    if (threadIdx.x < nparts) hist[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = cnt[threadIdx.x];
}

// exclusive scan of hist in [part][block] order (one block; nparts * nblocks <= 65536)
__global__ __launch_bounds__(PTB) void k_part_scan(uint32_t *__restrict__ v, uint32_t m, uint32_t nparts,
                                                   uint32_t nblocks, uint64_t *__restrict__ part_counts) {
    __shared__ uint32_t part[PTB];
    const uint32_t per = (m + PTB - 1) / PTB;
    const uint32_t b = threadIdx.x * per, e = min(m, b + per);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += v[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < PTB; d <<= 1) {
        const uint32_t x = threadIdx.x >= (uint32_t)d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (uint32_t i = b; i < e; ++i) {
        const uint32_t c = v[i];
        v[i] = run;
        run += c;
    }
    __syncthreads();
    // rows per part = next part's first offset - this part's first offset
    if (threadIdx.x < nparts) {
        const uint32_t lo = v[threadIdx.x * nblocks];
        const uint32_t hi = threadIdx.x + 1 < nparts ? v[(threadIdx.x + 1) * nblocks] : part[PTB - 1];
        part_counts[threadIdx.x] = hi - lo;
    }
}

__global__ __launch_bounds__(PTB) void k_part_scatter(const uint8_t *__restrict__ rows, uint64_t n, uint32_t row_bytes,
                                                      uint32_t key_words, uint32_t nparts, uint64_t chunk,
                                                      const uint32_t *__restrict__ off, uint8_t *__restrict__ out) {
    __shared__ uint32_t base[PMAXP];              // running output offset per part
    __shared__ uint32_t wcnt[PTB / 64][PMAXP];    // per-wave counts of this tile
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < nparts) base[threadIdx.x] = off[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x];
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk, b1 = min(n, b0 + chunk);
    for (uint64_t t0 = b0; t0 < b1; t0 += PTB) {
        for (uint32_t i = threadIdx.x; i < (PTB / 64) * PMAXP; i += PTB) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        const uint64_t r = t0 + threadIdx.x;
        const bool in = r < b1;
        const uint32_t o = in ? row_owner(rows + r * row_bytes, key_words, nparts) : 0xFFFFFFFFu;
        // rank within the wave among rows of the same owner (lanes in order)
        uint32_t rank = 0;
        uint64_t todo = __ballot(in);
        while (todo) {
            const uint32_t leader = (uint32_t)__ffsll((long long)todo) - 1;
            const uint32_t lo = __shfl(o, (int)leader);
            const uint64_t m = __ballot(o == lo);
            if (o == lo) rank = (uint32_t)__popcll(m & lanemask_lt());
            if (lane == 0) wcnt[wave][lo] = (uint32_t)__popcll(m);
            todo &= ~m;
        }
        __syncthreads();
        if (in) {
            uint32_t before = 0;
            for (uint32_t w = 0; w < wave; ++w) before += wcnt[w][o];
            const uint64_t dst = (uint64_t)base[o] + before + rank;
            const uint32_t *src = reinterpret_cast<const uint32_t *>(rows + r * row_bytes);
            uint32_t *d = reinterpret_cast<uint32_t *>(out + dst * row_bytes);
            for (uint32_t w = 0; w < row_bytes / 4; ++w) d[w] = src[w];
        }
        __syncthreads();
        if (threadIdx.x < nparts) {
            uint32_t tot = 0;
            for (uint32_t w = 0; w < PTB / 64; ++w) tot += wcnt[w][threadIdx.x];
            base[threadIdx.x] += tot;
        }
        __syncthreads();
    }
}

// ---- the same partition straight from a finalized table (igx_partition_groups) ---------
// The rows are the table's groups -- key words | aggregates masked to their out_width | first
// index, igx_groupby_gather's layout -- read through the slot list, and their number is the
// group count on the device, so an asynchronously finalized table is partitioned without a
// host round trip: both passes size their chunks from that count.
struct GroupSrc {
    const uint8_t *keys, *vals;
    const uint32_t *groups;
    const uint64_t *ng;
    uint64_t cap;                 // rows the output holds
    uint32_t key_stride, val_stride, key_words, naggs;
    uint32_t m[16];               // (lo, hi) masks per aggregate
};

__device__ __forceinline__ uint64_t src_rows(const GroupSrc &g) { return min(*g.ng, g.cap); }

__device__ __forceinline__ uint32_t src_word(const GroupSrc &g, uint32_t slot, uint32_t w) {
    if (w < g.key_words) return reinterpret_cast<const uint32_t *>(g.keys + (uint64_t)slot * g.key_stride)[w];
    const uint32_t *v = reinterpret_cast<const uint32_t *>(g.vals + (uint64_t)slot * g.val_stride);
    const uint32_t a = w - g.key_words;
    return a < 2 * g.naggs ? v[2 + a] & g.m[a] : v[a - 2 * g.naggs];
}

// The owner of every row, computed once: each thread takes GH rows at a time, their slots
// first, then their keys' first words, so GH scattered key reads are in flight at once (a
// dependent slot -> key -> owner chain per row left the pass latency-bound); owners go to a byte
// array the scatter reads back in order.
constexpr int GH = 4;
constexpr uint32_t GKW = 8;   // key words loaded up front (longer keys read the rest in a loop)

__global__ __launch_bounds__(PTB) void k_gpart_hist(GroupSrc g, uint32_t nparts, uint32_t *__restrict__ hist,
                                                    uint8_t *__restrict__ owner) {
    __shared__ uint32_t cnt[PMAXP];
    if (threadIdx.x < PMAXP) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t n = src_rows(g), chunk = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = min(n, (uint64_t)blockIdx.x * chunk), b1 = min(n, b0 + chunk);
    for (uint64_t r0 = b0 + threadIdx.x; r0 < b1; r0 += GH * PTB) {
        uint32_t slot[GH];
#pragma unroll
        for (int u = 0; u < GH; ++u) {
            const uint64_t r = r0 + (uint64_t)u * PTB;
            slot[u] = r < b1 ? g.groups[r] : 0u;
        }
        uint32_t kw[GH][GKW];
#pragma unroll
        for (int u = 0; u < GH; ++u) {
            const uint32_t *k = reinterpret_cast<const uint32_t *>(g.keys + (uint64_t)slot[u] * g.key_stride);
#pragma unroll
            for (uint32_t w = 0; w < GKW; ++w) kw[u][w] = w < g.key_words ? k[w] : 0u;
        }
        uint32_t o[GH];
#pragma unroll
        for (int u = 0; u < GH; ++u) {   // FNV-1a over the key words: row_owner's function
            const uint32_t *k = reinterpret_cast<const uint32_t *>(g.keys + (uint64_t)slot[u] * g.key_stride);
            uint32_t h = 0x811C9DC5u;
#pragma unroll
            for (uint32_t w = 0; w < GKW; ++w)
                if (w < g.key_words) h = (h ^ kw[u][w]) * 16777619u;
            for (uint32_t w = GKW; w < g.key_words; ++w) h = (h ^ k[w]) * 16777619u;
            o[u] = h % nparts;
        }
#pragma unroll
        for (int u = 0; u < GH; ++u) {
            const uint64_t r = r0 + (uint64_t)u * PTB;
            if (r < b1) {
                atomicAdd(&cnt[o[u]], 1u);
                owner[r] = (uint8_t)o[u];
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < nparts) hist[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = cnt[threadIdx.x];
}

// k_part_scatter's wave / LDS ranking over the table's rows; a row's words are written by
// consecutive lanes of one store (one lane per word, rows of a wave side by side)
__global__ __launch_bounds__(PTB) void k_gpart_scatter(GroupSrc g, uint32_t nparts, const uint32_t *__restrict__ off,
                                                       const uint8_t *__restrict__ owner, uint8_t *__restrict__ out) {
    __shared__ uint32_t base[PMAXP];
    __shared__ uint32_t wcnt[PTB / 64][PMAXP];
    __shared__ uint32_t dst_slot[PTB][2];         // per row of the tile: output row, table slot
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t row_words = g.key_words + 2 * g.naggs + 2;
    if (threadIdx.x < nparts) base[threadIdx.x] = off[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x];
    const uint64_t n = src_rows(g), chunk = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = min(n, (uint64_t)blockIdx.x * chunk), b1 = min(n, b0 + chunk);
    for (uint64_t t0 = b0; t0 < b1; t0 += PTB) {
        for (uint32_t i = threadIdx.x; i < (PTB / 64) * PMAXP; i += PTB) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        const uint64_t r = t0 + threadIdx.x;
        const bool in = r < b1;
        const uint32_t slot = in ? g.groups[r] : 0u;
        const uint32_t o = in ? (uint32_t)owner[r] : 0xFFFFFFFFu;
        uint32_t rank = 0;
        uint64_t todo = __ballot(in);
        while (todo) {
            const uint32_t leader = (uint32_t)__ffsll((long long)todo) - 1;
            const uint32_t lo = __shfl(o, (int)leader);
            const uint64_t m = __ballot(o == lo);
            if (o == lo) rank = (uint32_t)__popcll(m & lanemask_lt());
            if (lane == 0) wcnt[wave][lo] = (uint32_t)__popcll(m);
            todo &= ~m;
        }
        __syncthreads();
        if (in) {
            uint32_t before = 0;
            for (uint32_t w = 0; w < wave; ++w) before += wcnt[w][o];
            dst_slot[threadIdx.x][0] = base[o] + before + rank;
            dst_slot[threadIdx.x][1] = slot;
        }
        __syncthreads();
        // one lane per output word, 8 words in flight per lane (their loads before any store)
        const uint32_t tile = (uint32_t)min<uint64_t>(PTB, b1 - t0), words = tile * row_words;
        for (uint32_t i0 = threadIdx.x; i0 < words; i0 += 8 * PTB) {
            uint32_t v[8];
            uint64_t d[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t i = i0 + u * PTB;
                const uint32_t j = i / row_words, w = i - j * row_words;
                d[u] = i < words ? (uint64_t)dst_slot[j][0] * row_words + w : ~0ull;
                v[u] = i < words ? src_word(g, dst_slot[j][1], w) : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (d[u] != ~0ull) reinterpret_cast<uint32_t *>(out)[d[u]] = v[u];
        }
        __syncthreads();
        if (threadIdx.x < nparts) {
            uint32_t tot = 0;
            for (uint32_t w = 0; w < PTB / 64; ++w) tot += wcnt[w][threadIdx.x];
            base[threadIdx.x] += tot;
        }
        __syncthreads();
    }
}

// ---- AoS -> SoA -----------------------------------------------------------------------
struct IngestArgs {
    const uint8_t *rec;
    uint64_t n;
    uint32_t rec_bytes, nf;
    uint32_t off[16], width[16];
    uint8_t *dst[16];
};

// one thread per (record, field); a wave covers 64 consecutive records of one field, so
// the SoA stores are contiguous; the record reads are strided but every record's line is
// read by the fields' waves back to back (L2 hits)
__global__ __launch_bounds__(256) void k_ingest(IngestArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t total = (a.n + 63) / 64 * 64 * a.nf;   // whole 64-record groups
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const uint32_t f = (uint32_t)((i / 64) % a.nf);
        const uint64_t r = (i / 64 / a.nf) * 64 + (i % 64);
        if (r >= a.n) continue;
        const uint8_t *s = a.rec + r * a.rec_bytes + a.off[f];
        uint8_t *d = a.dst[f] + r * a.width[f];
        const uint32_t w = a.width[f];
        if (w == 16 && ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
            *reinterpret_cast<uint4 *>(d) = *reinterpret_cast<const uint4 *>(s);
        } else if (w == 8 && ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 7) == 0) {
            *reinterpret_cast<uint64_t *>(d) = *reinterpret_cast<const uint64_t *>(s);
        } else if (w == 4 && ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 3) == 0) {
            *reinterpret_cast<uint32_t *>(d) = *reinterpret_cast<const uint32_t *>(s);
        } else {
            for (uint32_t b = 0; b < w; ++b) d[b] = s[b];
        }
    }
}

}  // namespace

extern "C" int igx_partition_rows(igx_ctx *ctx, const uint8_t *rows, uint64_t nrows, uint32_t row_bytes,
                                  uint32_t key_bytes, uint32_t nparts, uint8_t *out, uint64_t *part_counts) {
    if (!ctx) return IGX_EINVAL;
    if (nparts == 0 || nparts > PMAXP) return igx_fail(ctx, IGX_EINVAL, "partition: nparts must be 1..%u", PMAXP);
    if (row_bytes == 0 || row_bytes % 4 || key_bytes % 4 || key_bytes > row_bytes)
        return igx_fail(ctx, IGX_EINVAL, "partition: rows and keys are whole u32 words");
    if (nrows >= (1ull << 32)) return igx_fail(ctx, IGX_EINVAL, "partition: more than 2^32 rows");
    if (!part_counts || (nrows && (!rows || !out))) return igx_fail(ctx, IGX_EINVAL, "partition: null argument");
    if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(out)) & 3)
        return igx_fail(ctx, IGX_EINVAL, "partition: rows must be 4-byte aligned");
    if (nrows == 0) {
        IGX_HIP(ctx, hipMemsetAsync(part_counts, 0, nparts * sizeof(uint64_t), ctx->stream));
        return IGX_OK;
    }
    const uint32_t nblocks = (uint32_t)std::min<uint64_t>(std::max(1, ctx->num_cus * 2), (nrows + PTB - 1) / PTB);
    const uint64_t chunk = (nrows + nblocks - 1) / nblocks;
    void *scratch;
    int rc = igx_scratch(ctx, (size_t)nparts * nblocks * 4, &scratch);
    if (rc) return rc;
    uint32_t *hist = static_cast<uint32_t *>(scratch);
    const uint32_t kw = key_bytes / 4;
    hipLaunchKernelGGL(k_part_hist, dim3(nblocks), dim3(PTB), 0, ctx->stream, rows, nrows, row_bytes, kw, nparts,
                       chunk, hist);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(PTB), 0, ctx->stream, hist, nparts * nblocks, nparts, nblocks,
                       part_counts);
    hipLaunchKernelGGL(k_part_scatter, dim3(nblocks), dim3(PTB), 0, ctx->stream, rows, nrows, row_bytes, kw, nparts,
                       chunk, hist, out);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_partition_groups(igx_ctx *ctx, const igx_table_view *view, const uint32_t *out_widths,
                                    uint32_t nparts, uint8_t *out, uint64_t cap_rows, uint64_t *part_counts) {
    if (!ctx) return IGX_EINVAL;
    if (!view || !part_counts) return igx_fail(ctx, IGX_EINVAL, "partition_groups: null argument");
    if (nparts == 0 || nparts > PMAXP) return igx_fail(ctx, IGX_EINVAL, "partition_groups: nparts must be 1..%u", PMAXP);
    if (view->naggs > 8 || view->key_bytes % 4 || !view->groups || !view->d_n_groups || !view->keys ||
        !view->first_idx)
        return igx_fail(ctx, IGX_EINVAL, "partition_groups: not a finalized table view");
    if (cap_rows >= (1ull << 32)) return igx_fail(ctx, IGX_EINVAL, "partition_groups: more than 2^32 rows");
    if (cap_rows == 0) {
        IGX_HIP(ctx, hipMemsetAsync(part_counts, 0, nparts * sizeof(uint64_t), ctx->stream));
        return IGX_OK;
    }
    if (!out || (reinterpret_cast<uintptr_t>(out) & 3)) return igx_fail(ctx, IGX_EINVAL, "partition_groups: out");
    GroupSrc g{};
    g.keys = view->keys;
    g.vals = reinterpret_cast<const uint8_t *>(view->first_idx);
    g.groups = view->groups;
    g.ng = view->d_n_groups;
    g.cap = cap_rows;
    g.key_stride = view->key_stride;
    g.val_stride = view->val_stride;
    g.key_words = view->key_bytes / 4;
    g.naggs = view->naggs;
    for (uint32_t x = 0; x < view->naggs; ++x) {
        const uint32_t ow = out_widths ? out_widths[x] : 8;
        const uint64_t m = (ow == 0 || ow >= 8) ? ~0ull : ((1ull << (8 * ow)) - 1);
        g.m[2 * x] = (uint32_t)m;
        g.m[2 * x + 1] = (uint32_t)(m >> 32);
    }
    // blocks: as igx_partition_rows would pick for the most rows the output holds
    const uint32_t nblocks = (uint32_t)std::min<uint64_t>(std::max(1, ctx->num_cus * 2), (cap_rows + PTB - 1) / PTB);
    void *scratch;
    const size_t hist_b = igx_align((size_t)nparts * nblocks * 4, 256);
    int rc = igx_scratch(ctx, hist_b + cap_rows, &scratch);
    if (rc) return rc;
    uint32_t *hist = static_cast<uint32_t *>(scratch);
    uint8_t *owner = static_cast<uint8_t *>(scratch) + hist_b;   // each row's owner, from the first pass
    hipLaunchKernelGGL(k_gpart_hist, dim3(nblocks), dim3(PTB), 0, ctx->stream, g, nparts, hist, owner);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(PTB), 0, ctx->stream, hist, nparts * nblocks, nparts, nblocks,
                       part_counts);
    hipLaunchKernelGGL(k_gpart_scatter, dim3(nblocks), dim3(PTB), 0, ctx->stream, g, nparts, hist, owner, out);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

// ---- trace open perf samples -> Event columns (one wave per sample) --------------------------
namespace {
constexpr uint32_t OPEN_SAMPLE = 304;   // sizeof(struct event), 8-byte aligned

// FromCString over a row held as one dword per lane (lanes [0, nl)): keeps the bytes before the
// first NUL (bytes at index >= lim count as NUL), zeroes the rest
__device__ __forceinline__ uint32_t cstring_cut(uint32_t v, uint32_t lane, uint32_t nl, uint32_t lim) {
    uint32_t first = 4;   // first NUL byte in this lane's dword (4 = none)
    for (int j = 3; j >= 0; --j) {
        const bool nul = ((v >> (8 * j)) & 0xFFu) == 0 || 4 * lane + j >= lim;
        if (nul) first = (uint32_t)j;
    }
    const uint64_t m = __ballot(lane < nl && first < 4);
    const uint32_t L = m ? (uint32_t)__ffsll((long long)m) - 1 : 64u;
    if (lane > L) return 0;
    if (lane == L) return first == 0 ? 0u : (v & (0xFFFFFFFFu >> (32 - 8 * first)));
    return v;
}

__global__ __launch_bounds__(256) void k_ingest_open(const uint8_t *__restrict__ s, uint64_t n, uint32_t sb,
                                                     int64_t boot, igx_open_cols o) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wpb = 256 / 64;
    for (uint64_t r = (uint64_t)blockIdx.x * wpb + (threadIdx.x >> 6); r < n; r += (uint64_t)gridDim.x * wpb) {
        const uint8_t *rec = s + r * sb;
        const uint32_t *d = reinterpret_cast<const uint32_t *>(rec);
        // fname: bytes 48..303 = dword 12 + lane; byte 255 of the row is the struct's padding
        const uint32_t f = __builtin_nontemporal_load(d + 12 + lane);
        const uint32_t pf = cstring_cut(f, lane, 64, 255);
        if (o.path) reinterpret_cast<uint32_t *>(o.path + r * 256)[lane] = pf;
        const uint32_t c = lane < 4 ? d[8 + lane] : 0u;
        const uint32_t pc = cstring_cut(c, lane, 4, 16);
        if (o.comm && lane < 4) reinterpret_cast<uint32_t *>(o.comm + r * 16)[lane] = pc;
        if (lane == 0) {
            const uint64_t ts = *reinterpret_cast<const uint64_t *>(rec);
            const int64_t ret = (int64_t) * reinterpret_cast<const int32_t *>(rec + 24);
            if (o.timestamp) o.timestamp[r] = (int64_t)(ts + (uint64_t)boot);
            if (o.pid) o.pid[r] = d[2];
            if (o.uid) o.uid[r] = d[3];
            if (o.mntns) o.mntns[r] = *reinterpret_cast<const uint64_t *>(rec + 16);
            if (o.ret) o.ret[r] = ret;
            if (o.fd) o.fd[r] = ret >= 0 ? ret : 0;
            if (o.err) o.err[r] = ret < 0 ? -ret : 0;
        }
    }
}
}  // namespace

extern "C" int igx_ingest_open_events(igx_ctx *ctx, const uint8_t *samples, uint64_t n, uint32_t sample_bytes,
                                      int64_t boot_to_wall_ns, const igx_open_cols *out) {
    if (!ctx) return IGX_EINVAL;
    if (!out) return igx_fail(ctx, IGX_EINVAL, "ingest_open: null output");
    if (n == 0) return IGX_OK;
    if (!samples) return igx_fail(ctx, IGX_EINVAL, "ingest_open: null samples");
    if (sample_bytes < OPEN_SAMPLE || sample_bytes % 8 || reinterpret_cast<uintptr_t>(samples) % 8)
        return igx_fail(ctx, IGX_EINVAL, "ingest_open: samples must be >= %u bytes, 8-byte aligned", OPEN_SAMPLE);
    if ((out->path && reinterpret_cast<uintptr_t>(out->path) % 4) || (out->comm && reinterpret_cast<uintptr_t>(out->comm) % 4))
        return igx_fail(ctx, IGX_EINVAL, "ingest_open: comm / path columns must be 4-byte aligned");
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((uint64_t)ctx->num_cus * 8, (n + 3) / 4);
    hipLaunchKernelGGL(k_ingest_open, dim3(blocks), dim3(256), 0, ctx->stream, samples, n, sample_bytes,
                       boot_to_wall_ns, *out);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}

extern "C" int igx_ingest_aos(igx_ctx *ctx, const void *records, uint64_t nrec, uint32_t rec_bytes,
                              const uint32_t *field_off, const uint32_t *field_width, uint32_t nfields,
                              void *const *out_cols) {
    if (!ctx) return IGX_EINVAL;
    if (nfields == 0 || nfields > 16) return igx_fail(ctx, IGX_EINVAL, "ingest: 1..16 fields");
    if (nrec && (!records || !field_off || !field_width || !out_cols))
        return igx_fail(ctx, IGX_EINVAL, "ingest: null argument");
    IngestArgs a{};
    a.rec = static_cast<const uint8_t *>(records);
    a.n = nrec;
    a.rec_bytes = rec_bytes;
    a.nf = nfields;
    for (uint32_t f = 0; f < nfields; ++f) {
        if (field_width[f] == 0 || field_off[f] + field_width[f] > rec_bytes)
            return igx_fail(ctx, IGX_EINVAL, "ingest: field %u [%u, +%u) outside the %u-byte record", f,
                            field_off[f], field_width[f], rec_bytes);
        a.off[f] = field_off[f];
        a.width[f] = field_width[f];
        a.dst[f] = static_cast<uint8_t *>(out_cols[f]);
        if (nrec && !a.dst[f]) return igx_fail(ctx, IGX_EINVAL, "ingest: null output column %u", f);
    }
    if (nrec == 0) return IGX_OK;
    const uint64_t total = (nrec + 63) / 64 * 64 * nfields;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((uint64_t)ctx->num_cus * 8, (total + 255) / 256);
    hipLaunchKernelGGL(k_ingest, dim3(blocks), dim3(256), 0, ctx->stream, a);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
