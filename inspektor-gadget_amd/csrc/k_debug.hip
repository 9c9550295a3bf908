// k_debug.hip -- test hooks for the failure paths (not used by the aggregation path).
//
// igx_debug_hold_stream enqueues one wave that waits on a host-mapped flag, so a test can keep
// a stream busy on purpose -- e.g. to make a collective behind it miss igx_dist's deadline the
// way a dead peer would -- and then release it.  The wait is bounded twice: by the flag and by
// an iteration budget sized from max_ms, so the wave always exits and the grid drains.
#include "igx_internal.h"

struct igx_hold {
    uint32_t *flag = nullptr;   // pinned, device-visible host word: 0 = hold, 1 = release
};

__global__ void __launch_bounds__(64) k_hold(const uint32_t *flag, uint64_t max_iters, uint32_t *seen) {
    uint64_t it = 0;
    for (; it < max_iters; ++it) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
        __builtin_amdgcn_s_sleep(127);   // ~8K cycles per poll
    }
    if (threadIdx.x == 0) seen[0] = it < max_iters ? 1u : 2u;   // 1 released, 2 budget spent
}

extern "C" int igx_debug_hold_stream(igx_ctx *ctx, uint32_t max_ms, void **token) {
    if (!ctx || !token || max_ms == 0) return IGX_EINVAL;
    *token = nullptr;
    auto *h = new igx_hold();
    // word 0: the flag; word 1: how the wave ended (for igx_debug_release)
    if (hipHostMalloc(reinterpret_cast<void **>(&h->flag), 64, hipHostMallocCoherent | hipHostMallocMapped) !=
        hipSuccess) {
        delete h;
        return igx_fail(ctx, IGX_ENOMEM, "debug_hold_stream: host flag");
    }
    __atomic_store_n(&h->flag[0], 0u, __ATOMIC_RELEASE);
    h->flag[1] = 0;
    // ~3.4 us per poll at 2.4 GHz: the budget ends the wave near max_ms even if never released
    const uint64_t iters = (uint64_t)max_ms * 300;
    hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, ctx->stream, h->flag, iters, h->flag + 1);
    IGX_HIP(ctx, hipGetLastError());
    *token = h;
    return IGX_OK;
}

// Releases the held wave, waits for the context's stream to drain (bounded by the wave's own
// budget), frees the flag.  *how = 1 if the wave saw the release, 2 if its budget ran out.
extern "C" int igx_debug_release(igx_ctx *ctx, void *token, uint32_t *how) {
    if (!ctx || !token) return IGX_EINVAL;
    auto *h = static_cast<igx_hold *>(token);
    __atomic_store_n(&h->flag[0], 1u, __ATOMIC_RELEASE);
    IGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (how) *how = __atomic_load_n(&h->flag[1], __ATOMIC_ACQUIRE);
    (void)hipHostFree(h->flag);
    delete h;
    return IGX_OK;
}
