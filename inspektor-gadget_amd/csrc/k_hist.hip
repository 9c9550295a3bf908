// k_hist.hip -- log2 latency histograms in LDS (kernel (4)).
//
// Reference: ig_profio_done (pkg/gadgets/profile/block-io/tracer/bpf/biolatency.bpf.c:100-154)
//   delta = ts_complete - ts_start (s64), negative -> skipped;
//   v = delta / 1000 (usecs; 1e6 with targ_ms);  slot = log2l(v) (bits.bpf.h:8-29) clamped
//   to MAX_SLOTS-1 = 26;  __sync_fetch_and_add(&slots[slot], 1) (u32).
// log2l(v) == floor(log2 v) for v >= 1 and 0 for v == 0, i.e. 63 - clz64(v).
// The reference keys the histogram by hist_key{cmd_flags, dev}; C3 keys it by
// (dev, container) -- dense key = dev_index * ncont + cont.
//
// Layout: hist is [nkeys][nslots] u32 in HBM.  Each workgroup privatises a slice of it
// in LDS (u32 counters, up to 120 KB); when the whole histogram does not fit, the key
// space is split into P partitions and P workgroups that share an XCD (blockIdx % 8,
// speed only) sweep the same input chunks, each counting its own partition -- the
// repeated reads are L2 hits.  Small histograms are replicated per wave to spread LDS
// atomic contention.  Commit: one coalesced HBM atomic add per non-zero bin per WG.
#include <algorithm>
#include <vector>

#include "k_common.h"

namespace {

constexpr int TB = 1024;
constexpr uint32_t LDS_BUDGET = 120 * 1024;
constexpr uint64_t CHUNK = 1 << 16;   // rows per chunk

struct HistArgs {
    const uint32_t *dev;
    const uint32_t *cont;
    const int64_t *delta;
    uint64_t n;
    uint32_t devs_sorted[64];
    uint32_t devs_index[64];
    uint32_t ndev, ncont, nslots;
    uint32_t P;          // key partitions
    uint32_t Kp;         // keys per partition
    uint32_t R;          // LDS replicas
    uint32_t ngroups;    // chunk groups (multiple of 8)
    uint64_t divisor;
    uint32_t *hist;
};

template <int DIV>
__device__ __forceinline__ uint64_t divide(uint64_t v, uint64_t d) {
    if constexpr (DIV == 1000) return v / 1000ull;
    else if constexpr (DIV == 1000000) return v / 1000000ull;
    else return v / d;
}

template <int DIV>
__global__ __launch_bounds__(TB) void k_hist(HistArgs a) {
    extern __shared__ uint32_t h[];
    const uint32_t part_bins = a.Kp * a.nslots;
    for (uint32_t i = threadIdx.x; i < part_bins * a.R; i += TB) h[i] = 0;
    __shared__ uint32_t sdev[64], sidx[64];
    if (threadIdx.x < 64) {
        sdev[threadIdx.x] = a.devs_sorted[threadIdx.x];
        sidx[threadIdx.x] = a.devs_index[threadIdx.x];
    }
    __syncthreads();
    const uint32_t b = blockIdx.x, xcd = b & 7, j = b >> 3;
    const uint32_t p = j % a.P, g = j / a.P;
    const uint32_t cgroup = g * 8 + xcd;
    const uint32_t kbase = p * a.Kp;
    const uint32_t rep = (threadIdx.x >> 6) % a.R;
    uint32_t *hr = h + rep * part_bins;
    const uint64_t nchunks = (a.n + CHUNK - 1) / CHUNK;
    for (uint64_t c = cgroup; c < nchunks; c += a.ngroups) {
        const uint64_t end = min(a.n, (c + 1) * CHUNK);
        for (uint64_t row = c * CHUNK + threadIdx.x; row < end; row += TB) {
            const uint32_t dv = a.dev[row];
            // binary search in the sorted device table
            uint32_t lo = 0, hi = a.ndev;
            while (lo < hi) {
                uint32_t mid = (lo + hi) >> 1;
                if (sdev[mid] < dv) lo = mid + 1; else hi = mid;
            }
            if (lo >= a.ndev || sdev[lo] != dv) continue;
            const uint32_t ci = a.cont ? a.cont[row] : 0u;
            if (ci >= a.ncont) continue;   // unknown container: not counted
            const uint32_t key = sidx[lo] * a.ncont + ci;
            if (key - kbase >= a.Kp) continue;
            const int64_t d = a.delta[row];
            if (d < 0) continue;
            const uint64_t v = divide<DIV>((uint64_t)d, a.divisor);
            uint32_t slot = v ? 63u - (uint32_t)__clzll(v) : 0u;
            slot = min(slot, a.nslots - 1);
            atomicAdd(&hr[(key - kbase) * a.nslots + slot], 1u);
        }
    }
    __syncthreads();
    const uint32_t nkeys_here = min(a.Kp, a.ndev * a.ncont - min(kbase, a.ndev * a.ncont));
    for (uint32_t i = threadIdx.x; i < nkeys_here * a.nslots; i += TB) {
        uint32_t s = 0;
        for (uint32_t r = 0; r < a.R; ++r) s += h[r * part_bins + i];
        if (s) atomicAdd(&a.hist[(uint64_t)kbase * a.nslots + i], s);
    }
}

}  // namespace

int launch_hist_log2(igx_ctx *ctx, const uint32_t *dev, const uint32_t *cont, const int64_t *delta,
                     uint64_t nrows, const uint32_t *devs, uint32_t ndev, uint32_t ncont,
                     uint64_t divisor, uint32_t nslots, uint32_t *hist) {
    if (nrows == 0) return IGX_OK;
    if (ndev == 0 || ndev > 64) return igx_fail(ctx, IGX_EINVAL, "hist: ndev must be 1..64");
    if (ncont == 0 || (!cont && ncont != 1)) return igx_fail(ctx, IGX_EINVAL, "hist: bad ncont");
    if (nslots == 0 || nslots > 64 || divisor == 0) return igx_fail(ctx, IGX_EINVAL, "hist: bad nslots/divisor");
    HistArgs a{};
    a.dev = dev;
    a.cont = cont;
    a.delta = delta;
    a.n = nrows;
    std::vector<std::pair<uint32_t, uint32_t>> dv;
    for (uint32_t i = 0; i < ndev; ++i) dv.push_back({devs[i], i});
    std::sort(dv.begin(), dv.end());
    for (uint32_t i = 1; i < ndev; ++i)
        if (dv[i].first == dv[i - 1].first) return igx_fail(ctx, IGX_EINVAL, "hist: duplicate device");
    for (uint32_t i = 0; i < 64; ++i) {
        a.devs_sorted[i] = i < ndev ? dv[i].first : 0xFFFFFFFFu;
        a.devs_index[i] = i < ndev ? dv[i].second : 0;
    }
    a.ndev = ndev;
    a.ncont = ncont;
    a.nslots = nslots;
    const uint64_t nkeys = (uint64_t)ndev * ncont;
    const uint64_t keys_fit = LDS_BUDGET / (4ull * nslots);
    a.P = (uint32_t)((nkeys + keys_fit - 1) / keys_fit);
    a.Kp = (uint32_t)((nkeys + a.P - 1) / a.P);
    const uint32_t part_bytes = a.Kp * nslots * 4;
    a.R = std::max<uint32_t>(1, std::min<uint32_t>(TB / 64, LDS_BUDGET / part_bytes));
    // small histograms: keep several workgroups per CU
    uint32_t bpc = (part_bytes * a.R <= 32 * 1024) ? 2 : 1;
    if (a.R > 4 && bpc == 2) a.R = 4;
    uint32_t blocks = (uint32_t)ctx->num_cus * bpc;
    blocks = std::max<uint32_t>(8 * a.P, blocks / (8 * a.P) * (8 * a.P));
    a.ngroups = blocks / a.P;
    a.divisor = divisor;
    a.hist = hist;
    const size_t lds = (size_t)part_bytes * a.R;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_hist<1000>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BUDGET);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_hist<1000000>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BUDGET);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_hist<0>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BUDGET);
        attr_set = true;
    }
    if (divisor == 1000)
        hipLaunchKernelGGL(k_hist<1000>, dim3(blocks), dim3(TB), lds, ctx->stream, a);
    else if (divisor == 1000000)
        hipLaunchKernelGGL(k_hist<1000000>, dim3(blocks), dim3(TB), lds, ctx->stream, a);
    else
        hipLaunchKernelGGL(k_hist<0>, dim3(blocks), dim3(TB), lds, ctx->stream, a);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
