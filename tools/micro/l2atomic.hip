// Microbenchmark (diagnostics only): where do 64-bit atomics execute?  Random u64 atomic adds
// into per-XCD table regions of T bytes (blocks b and b+8 share an XCD and a region), agent
// scope vs workgroup scope (no sc1: performed in the XCD's L2 when the line is cached there).
// The workgroup-scope runs are checked: every region is touched by one XCD only, so the sum
// over the table after the kernel (kernel end writes L2 back) must equal the adds issued.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7u;
}

template <int SCOPE>
__global__ void k_atomic(unsigned long long *tab, uint64_t words_per_region, uint64_t per) {
    const uint32_t x = xcc_id();
    unsigned long long *reg = tab + (uint64_t)x * words_per_region;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = 0; i < per; ++i) {
        const uint64_t r = mix(gid * per + i) % words_per_region;
        __hip_atomic_fetch_add(&reg[r], 1ull, __ATOMIC_RELAXED, SCOPE);
    }
}

// 32-bit adds (no return / returning) and 64-bit returning adds, same pattern
template <int RET>
__global__ void k_atomic32(unsigned int *tab, uint64_t words_per_region, uint64_t per, uint32_t *sink) {
    const uint32_t x = xcc_id();
    unsigned int *reg = tab + (uint64_t)x * words_per_region;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t i = 0; i < per; ++i) {
        const uint64_t r = mix(gid * per + i) % words_per_region;
        if (RET) acc += __hip_atomic_fetch_add(&reg[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_add(&reg[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 0x12345678u) sink[0] = 1;
}
__global__ void k_atomic64r(unsigned long long *tab, uint64_t words_per_region, uint64_t per, uint32_t *sink) {
    const uint32_t x = xcc_id();
    unsigned long long *reg = tab + (uint64_t)x * words_per_region;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long acc = 0;
    for (uint64_t i = 0; i < per; ++i) {
        const uint64_t r = mix(gid * per + i) % words_per_region;
        acc += __hip_atomic_fetch_add(&reg[r], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 0x12345678ull) sink[0] = 1;
}

// random plain 8-B loads within the XCD's region
__global__ void k_load(const unsigned long long *tab, uint64_t words_per_region, uint64_t per, uint32_t *sink) {
    const uint32_t x = xcc_id();
    const unsigned long long *reg = tab + (uint64_t)x * words_per_region;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long acc = 0;
    for (uint64_t i = 0; i < per; i += 4) {
        unsigned long long v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = reg[mix(gid * per + i + u) % words_per_region];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    if (acc == 0x12345678ull) sink[0] = 1;
}

// random read-modify-write with plain 8-B loads and stores (no atomicity; the rate bound of an
// owner-exclusive region update)
__global__ void k_rmw(unsigned long long *tab, uint64_t words_per_region, uint64_t per) {
    const uint32_t x = xcc_id();
    unsigned long long *reg = tab + (uint64_t)x * words_per_region;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = 0; i < per; i += 4) {
        uint64_t r[4];
        unsigned long long v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { r[u] = mix(gid * per + i + u) % words_per_region; v[u] = reg[r[u]]; }
#pragma unroll
        for (int u = 0; u < 4; ++u) reg[r[u]] = v[u] + 1;
    }
}

__global__ void k_sum(const unsigned long long *tab, uint64_t n, unsigned long long *out) {
    unsigned long long s = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) s += tab[i];
    atomicAdd(out, s);
}

int main() {
    const uint64_t MAXB = 8ull << 30;
    unsigned long long *tab, *sum;
    uint32_t *sink;
    hipMalloc(&tab, MAXB);
    hipMalloc(&sum, 8);
    hipMalloc(&sink, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 4, threads = 256;
    const uint64_t lanes = (uint64_t)blocks * threads, per = 64;
    auto timeit = [&](auto fn) {
        fn();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        fn();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        return ms;
    };
    for (uint64_t rb : {256ull << 10, 1ull << 20, 2ull << 20, 3ull << 20, 8ull << 20, 32ull << 20, 256ull << 20, 1ull << 30}) {
        const uint64_t w = rb / 8;
        float ma = timeit([&] { k_atomic<__HIP_MEMORY_SCOPE_AGENT><<<blocks, threads>>>(tab, w, per); });
        hipMemset(tab, 0, 8 * rb);
        float mw = timeit([&] { k_atomic<__HIP_MEMORY_SCOPE_WORKGROUP><<<blocks, threads>>>(tab, w, per); });
        hipMemset(sum, 0, 8);
        k_sum<<<1024, 256>>>(tab, 8 * w, sum);
        unsigned long long got = 0;
        hipMemcpy(&got, sum, 8, hipMemcpyDeviceToHost);
        float ml = timeit([&] { k_load<<<blocks, threads>>>(tab, w, per, sink); });
        float mr = timeit([&] { k_rmw<<<blocks, threads>>>(tab, w, per); });
        float m32 = timeit([&] { k_atomic32<0><<<blocks, threads>>>((unsigned int *)tab, 2 * w, per, sink); });
        float m32r = timeit([&] { k_atomic32<1><<<blocks, threads>>>((unsigned int *)tab, 2 * w, per, sink); });
        float m64r = timeit([&] { k_atomic64r<<<blocks, threads>>>(tab, w, per, sink); });
        const double ops = (double)lanes * per;
        printf("region %7.2f MiB x8: atomics u32 %6.1f G/s  u32 returning %6.1f G/s  u64 returning %6.1f G/s\n", rb / 1048576.0,
               ops / m32 / 1e6, ops / m32r / 1e6, ops / m64r / 1e6);
        printf("region %7.2f MiB x8: atomics agent %6.1f G/s  workgroup %6.1f G/s (sum %s: %llu of %.0f)  loads %6.1f G/s  plain rmw %6.1f G/s\n",
               rb / 1048576.0, ops / ma / 1e6, ops / mw / 1e6, got == (unsigned long long)(2 * ops) ? "ok" : "MISMATCH", got,
               2 * ops, ops / ml / 1e6, ops / mr / 1e6);
    }
    return 0;
}
