// Microbenchmark (diagnostics only): random-access rates on MI355X that bound the
// high-cardinality group-by designs -- random R-byte reads over a T-byte table, random 8-byte
// atomics (agent scope and workgroup scope), and a streaming read for reference.
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

// each lane: `per` random records of R bytes (R/16 dwordx4 loads), xor-reduce
template <int Q>
__global__ void k_rand_read(const uint4 *tab, uint64_t nrec, uint64_t per, uint32_t *sink) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t i = 0; i < per; ++i) {
        const uint64_t r = mix(gid * per + i) % nrec;
        uint4 v[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) v[q] = tab[r * Q + q];
#pragma unroll
        for (int q = 0; q < Q; ++q) acc ^= v[q].x ^ v[q].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_rand_atomic(unsigned long long *tab, uint64_t n, uint64_t per, int wg_scope) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = 0; i < per; ++i) {
        const uint64_t r = mix(gid * per + i) % n;
        if (wg_scope)
            __hip_atomic_fetch_add(&tab[r], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
            __hip_atomic_fetch_add(&tab[r], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_stream(const uint4 *a, uint64_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = a[i];
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t TB = 1ull << 30;   // 1 GiB table
    uint4 *tab;
    uint32_t *sink;
    hipMalloc(&tab, 4 * TB);
    hipMalloc(&sink, 64);
    hipMemset(tab, 1, 4 * TB);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8, threads = 256;
    const uint64_t lanes = (uint64_t)blocks * threads;
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
    for (uint64_t tbytes : {TB / 32, TB / 16, TB / 8, TB / 4, TB / 2, TB, 4 * TB}) {
        const uint64_t per = 64;
        const uint64_t acc = lanes * per;
        float m16 = timeit([&] { k_rand_read<1><<<blocks, threads>>>(tab, tbytes / 16, per, sink); });
        float m32 = timeit([&] { k_rand_read<2><<<blocks, threads>>>(tab, tbytes / 32, per, sink); });
        float m64 = timeit([&] { k_rand_read<4><<<blocks, threads>>>(tab, tbytes / 64, per, sink); });
        float m128 = timeit([&] { k_rand_read<8><<<blocks, threads>>>(tab, tbytes / 128, per, sink); });
        printf("table %6.0f MiB: random reads  16B %.2f G/s  32B %.2f G/s  64B %.2f G/s (%.0f GB/s)  128B %.2f G/s (%.0f GB/s)\n",
               tbytes / 1048576.0, acc / m16 / 1e6, acc / m32 / 1e6, acc / m64 / 1e6, acc * 64 / m64 / 1e6,
               acc / m128 / 1e6, acc * 128 / m128 / 1e6);
        float ma = timeit([&] { k_rand_atomic<<<blocks, threads>>>((unsigned long long *)tab, tbytes / 8, 16, 0); });
        float mw = timeit([&] { k_rand_atomic<<<blocks, threads>>>((unsigned long long *)tab, tbytes / 8, 16, 1); });
        printf("table %6.0f MiB: random 8B atomics agent %.2f G/s  workgroup-scope %.2f G/s\n", tbytes / 1048576.0,
               lanes * 16 / ma / 1e6, lanes * 16 / mw / 1e6);
    }
    float ms = timeit([&] { k_stream<<<256 * 8, 256>>>(tab, 4 * TB / 16, sink); });
    printf("stream read 4 GiB: %.0f GB/s\n", 4.0 * TB / ms / 1e6);
    return 0;
}
