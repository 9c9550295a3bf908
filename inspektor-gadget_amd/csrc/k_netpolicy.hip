// k_netpolicy.hip -- the advise network-policy event filter (advisor.go:279-292) as a
// device pass producing the row mask that igx_groupby_update_ex consumes.
//
// GeneratePolicies keeps an event iff Type == "normal", PktType is HOST or OUTGOING, and
// not (PktType == HOST and PodHostIP == RemoteAddr) -- a pod's own node cannot be blocked.
// Events arrive dictionary-encoded: pkt = Linux PACKET_* code (HOST 0, OUTGOING 4),
// type = 0 for "normal", PodHostIP / RemoteAddr as ids of one shared address dictionary.
#include "k_common.h"

namespace {

constexpr uint32_t PKT_HOST = 0, PKT_OUTGOING = 4;

// 4 rows per thread: u8 columns are read as one dword per thread, the u32 columns as uint4
__global__ __launch_bounds__(256) void k_np_mark(const uint8_t *__restrict__ typ, const uint8_t *__restrict__ pkt,
                                                 const uint32_t *__restrict__ hostip,
                                                 const uint32_t *__restrict__ raddr, uint64_t n,
                                                 uint8_t *__restrict__ keep) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t r0 = 4 * q;
    if (r0 >= n) return;
    if (r0 + 4 <= n) {
        const uint32_t t4 = reinterpret_cast<const uint32_t *>(typ)[q];
        const uint32_t p4 = reinterpret_cast<const uint32_t *>(pkt)[q];
        const uint4 h4 = reinterpret_cast<const uint4 *>(hostip)[q];
        const uint4 a4 = reinterpret_cast<const uint4 *>(raddr)[q];
        const uint32_t h[4] = {h4.x, h4.y, h4.z, h4.w}, a[4] = {a4.x, a4.y, a4.z, a4.w};
        uint32_t out = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t t = (t4 >> (8 * j)) & 255u, p = (p4 >> (8 * j)) & 255u;
            const bool k = t == 0 && (p == PKT_HOST || p == PKT_OUTGOING) && !(p == PKT_HOST && h[j] == a[j]);
            out |= (k ? 1u : 0u) << (8 * j);
        }
        reinterpret_cast<uint32_t *>(keep)[q] = out;
    } else {
        for (uint64_t r = r0; r < n; ++r) {
            const uint32_t p = pkt[r];
            keep[r] = typ[r] == 0 && (p == PKT_HOST || p == PKT_OUTGOING) && !(p == PKT_HOST && hostip[r] == raddr[r]);
        }
    }
}

}  // namespace

extern "C" int igx_np_mark(igx_ctx *ctx, const uint8_t *typ, const uint8_t *pkt, const uint32_t *hostip,
                           const uint32_t *raddr, uint64_t nrows, uint8_t *keep) {
    if (!ctx) return IGX_EINVAL;
    if (nrows == 0) return IGX_OK;
    if (!typ || !pkt || !hostip || !raddr || !keep) return igx_fail(ctx, IGX_EINVAL, "np_mark: null argument");
    const uintptr_t al = reinterpret_cast<uintptr_t>(typ) | reinterpret_cast<uintptr_t>(pkt) |
                         reinterpret_cast<uintptr_t>(keep);
    const uintptr_t al16 = reinterpret_cast<uintptr_t>(hostip) | reinterpret_cast<uintptr_t>(raddr);
    if ((al & 3) || (al16 & 15)) return igx_fail(ctx, IGX_EINVAL, "np_mark: misaligned columns");
    const uint64_t threads = (nrows + 3) / 4;
    hipLaunchKernelGGL(k_np_mark, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, ctx->stream, typ, pkt, hostip,
                       raddr, nrows, keep);
    IGX_HIP(ctx, hipGetLastError());
    return IGX_OK;
}
