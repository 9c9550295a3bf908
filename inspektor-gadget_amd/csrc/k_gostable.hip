// k_gostable.hip -- Go 1.19 sort.SliceStable executed step for step, for sort passes whose
// comparison is no strict weak order.
//
// Reference: ColumnSorterCollection.Sort (pkg/columns/sort/sort.go:35-83) runs one
// sort.SliceStable per key under getLessFunc (:125-135), `!(a < b) != order`.  For a float key
// holding NaN, `<` is unordered, so the pass's result depends on which pairs SliceStable
// compares: insertionSort_func on blocks of 20, then symMerge_func / rotate_func
// (sort/zsortfunc.go).  k_sort's closed form cannot reproduce that; this file runs the algorithm
// itself on the device, with the same comparisons in the same places, for every pass of such a
// sort:
//   * insertion sort: one thread per block of 20 rows, staged in LDS;
//   * the merges of one block size: level by level.  A task (a, m, b) does the binary searches of
//     symMerge_func on the current array, records its rotation and its two sub-merges; the
//     rotations of a level touch disjoint ranges and run next (one workgroup each); then the
//     sub-merges form the next level.  Searches, rotations and recursion order are Go's, so the
//     array after each level is the one Go's depth-first recursion reaches (sub-merges of one
//     task only read and write their own ranges).
// Host round trips: one per level (task counts).  This path runs only when k_sort's composed-key
// scan saw a NaN in a float key of a non-nil row.
#include "k_common.h"

namespace {

struct GoKey {
    const uint8_t *ptr;
    uint32_t width, kind, stride;
    uint32_t asc;     // columns.OrderAsc (no '-' prefix)
    uint32_t konst;   // a column that is the same for every row (sort_common's width-0 key)
};

__device__ __forceinline__ bool go_value_lt(const GoKey &k, uint32_t ra, uint32_t rb) {
    if (k.konst) return false;   // v < v
    const uint8_t *pa = k.ptr + (uint64_t)ra * k.stride, *pb = k.ptr + (uint64_t)rb * k.stride;
    if (k.kind == IGX_KIND_BYTES) {
        for (uint32_t i = 0; i < k.width; ++i)
            if (pa[i] != pb[i]) return pa[i] < pb[i];
        return false;
    }
    if (k.kind == IGX_KIND_FLOAT) {
        if (k.width == 4) return *reinterpret_cast<const float *>(pa) < *reinterpret_cast<const float *>(pb);
        return *reinterpret_cast<const double *>(pa) < *reinterpret_cast<const double *>(pb);
    }
    const uint64_t x = ld_scalar(pa, k.width, 0, false), y = ld_scalar(pb, k.width, 0, false);
    if (k.kind == IGX_KIND_INT) {
        const uint32_t sh = 64u - 8u * k.width;
        return (int64_t)(x << sh) < (int64_t)(y << sh);
    }
    return x < y;
}

// getLessFunc(i, j) on the rows at positions i and j: nil entries are never less, and a non-nil
// entry is less than a nil one (sort.go:127-132)
__device__ __forceinline__ bool go_less(const GoKey &k, const uint8_t *valid, uint32_t ra, uint32_t rb) {
    if (valid && !valid[ra]) return false;
    if (valid && !valid[rb]) return true;
    return !go_value_lt(k, ra, rb) != (k.asc != 0);
}

constexpr uint32_t INS = 20;   // insertionSort_func block size of stable_func
constexpr uint32_t ITB = 128;

__global__ __launch_bounds__(ITB) void k_go_insertion(uint32_t *data, uint32_t n, GoKey k, const uint8_t *valid) {
    __shared__ uint32_t blk[ITB * INS];
    const uint32_t a = (blockIdx.x * ITB + threadIdx.x) * INS;
    if (a >= n) return;
    const uint32_t len = min(INS, n - a);
    uint32_t *d = blk + threadIdx.x * INS;
    for (uint32_t i = 0; i < len; ++i) d[i] = data[a + i];
    for (uint32_t i = 1; i < len; ++i)
        for (uint32_t j = i; j > 0 && go_less(k, valid, d[j], d[j - 1]); --j) {
            const uint32_t t = d[j];
            d[j] = d[j - 1];
            d[j - 1] = t;
        }
    for (uint32_t i = 0; i < len; ++i) data[a + i] = d[i];
}

// the merges of block size bs: (a, a + bs, min(a + 2 bs, n)) for every a = 2 bs t with a + bs < n
__global__ void k_go_pairs(uint4 *tasks, uint32_t ntasks, uint32_t bs, uint32_t n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntasks) return;
    const uint32_t a = 2 * bs * t;
    tasks[t] = make_uint4(a, a + bs, min(a + 2 * bs, n), 0);
}

// one level of symMerge_func: searches on the current array, the rotation it asks for, its
// sub-merges.  A single-element side is a rotation by one (Go's swap loops).
__global__ void k_go_symmerge(const uint32_t *data, const uint4 *tasks, uint32_t ntasks, GoKey k,
                              const uint8_t *valid, uint4 *rots, uint32_t *nrot, uint4 *next, uint32_t *nnext) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntasks) return;
    const uint32_t a = tasks[t].x, m = tasks[t].y, b = tasks[t].z;
    if (m - a == 1) {
        uint32_t i = m, j = b;
        while (i < j) {
            const uint32_t h = (i + j) >> 1;
            if (go_less(k, valid, data[h], data[a])) i = h + 1;
            else j = h;
        }
        // swaps a..i-2 move data[a] to i-1: rotate [a, i) left by one
        if (i - 1 > a) rots[atomicAdd(nrot, 1u)] = make_uint4(a, a + 1, i, 0);
        return;
    }
    if (b - m == 1) {
        uint32_t i = a, j = m;
        while (i < j) {
            const uint32_t h = (i + j) >> 1;
            if (!go_less(k, valid, data[m], data[h])) i = h + 1;
            else j = h;
        }
        // swaps m..i+1 move data[m] to i: rotate [i, m + 1) so that its last element comes first
        if (m > i) rots[atomicAdd(nrot, 1u)] = make_uint4(i, m, m + 1, 0);
        return;
    }
    const uint32_t mid = (a + b) >> 1, nn = mid + m;
    uint32_t start, r;
    if (m > mid) {
        start = nn - b;
        r = mid;
    } else {
        start = a;
        r = m;
    }
    const uint32_t p = nn - 1;
    while (start < r) {
        const uint32_t c = (start + r) >> 1;
        if (!go_less(k, valid, data[p - c], data[c])) start = c + 1;
        else r = c;
    }
    const uint32_t end = nn - start;
    if (start < m && m < end) rots[atomicAdd(nrot, 1u)] = make_uint4(start, m, end, 0);
    if (a < start && start < mid) next[atomicAdd(nnext, 1u)] = make_uint4(a, start, mid, 0);
    if (mid < end && end < b) next[atomicAdd(nnext, 1u)] = make_uint4(mid, end, b, 0);
}

// rotate_func(s, m, e): [m, e) then [s, m); one workgroup per rotation, through tmp
__global__ __launch_bounds__(256) void k_go_rotate(uint32_t *data, uint32_t *tmp, const uint4 *rots) {
    const uint32_t s = rots[blockIdx.x].x, m = rots[blockIdx.x].y, e = rots[blockIdx.x].z;
    const uint32_t len = e - s, sh = m - s;
    for (uint32_t i = threadIdx.x; i < len; i += 256) tmp[s + i] = data[s + i];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < len; i += 256) {
        uint32_t j = i + sh;
        if (j >= len) j -= len;
        data[s + i] = tmp[s + j];
    }
}

}  // namespace

// data (device, n rows, already in the pre-sort order) is sorted in place by every pass of keys
// (sortBy order; the last key's pass runs first), exactly as ColumnSorterCollection.Sort does.
int launch_go_stable(igx_ctx *ctx, const GoSortKey *keys, uint32_t nkeys, uint64_t nrows, const uint8_t *valid,
                     uint32_t *data) {
    if (nrows < 2 || nkeys == 0) return IGX_OK;
    if (nrows >= (1ull << 31)) return igx_fail(ctx, IGX_ENOTSUP, "sort: too many rows for the exact NaN path");
    const uint32_t n = (uint32_t)nrows;
    const uint32_t maxt = n / 2 + 2;
    void *buf = nullptr;
    const size_t bytes = (size_t)n * 4 + 3ull * maxt * 16 + 64;
    IGX_HIP(ctx, hipMalloc(&buf, bytes));
    uint32_t *tmp = static_cast<uint32_t *>(buf);
    uint4 *T[2] = {reinterpret_cast<uint4 *>(tmp + n), reinterpret_cast<uint4 *>(tmp + n) + maxt};
    uint4 *rots = T[1] + maxt;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(rots + maxt);   // [0] rotations, [1] next tasks
    uint32_t *hcnt = nullptr;
    int rc = igx_pinned(ctx, 16, reinterpret_cast<void **>(&hcnt));
    for (int ki = (int)nkeys - 1; ki >= 0 && !rc; --ki) {
        GoKey k{keys[ki].ptr, keys[ki].width, keys[ki].kind, keys[ki].stride, keys[ki].asc, keys[ki].konst};
        hipLaunchKernelGGL(k_go_insertion, dim3((n + INS * ITB - 1) / (INS * ITB)), dim3(ITB), 0, ctx->stream, data, n, k,
                           valid);
        for (uint64_t bs = INS; bs < n && !rc; bs *= 2) {
            uint32_t nt = (uint32_t)((n - bs + 2 * bs - 1) / (2 * bs));   // pairs with a + bs < n
            int cur = 0;
            hipLaunchKernelGGL(k_go_pairs, dim3((nt + 255) / 256), dim3(256), 0, ctx->stream, T[0], nt, (uint32_t)bs, n);
            while (nt) {
                if (hipMemsetAsync(cnt, 0, 8, ctx->stream) != hipSuccess) { rc = IGX_EIO; break; }
                hipLaunchKernelGGL(k_go_symmerge, dim3((nt + 255) / 256), dim3(256), 0, ctx->stream, data, T[cur], nt, k,
                                   valid, rots, cnt, T[cur ^ 1], cnt + 1);
                if (hipMemcpyAsync(hcnt, cnt, 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                    hipStreamSynchronize(ctx->stream) != hipSuccess) {
                    rc = IGX_EIO;
                    break;
                }
                if (hcnt[0]) hipLaunchKernelGGL(k_go_rotate, dim3(hcnt[0]), dim3(256), 0, ctx->stream, data, tmp, rots);
                nt = hcnt[1];
                cur ^= 1;
            }
        }
    }
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(buf);
    if (rc) return igx_fail(ctx, rc, "sort: exact SliceStable path failed");
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
