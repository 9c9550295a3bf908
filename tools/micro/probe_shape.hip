// Microbenchmark (diagnostics only): the shape of a random 96-B key-record probe.  Each lane
// probes random 128-B records of a T-byte table: (a) six 16-B loads per lane (the group-by's
// probe), (b) one 16-B load per lane (the request floor), (c) six lanes per record, one 16-B
// load each (cooperative: one 96-B request per record).  Reports records probed per second.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

template <int MODE>
__global__ void k_probe(const uint4 *tab, uint64_t nrec, uint64_t per, uint32_t *sink) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t acc = 0;
    for (uint64_t i = 0; i < per; ++i) {
        if (MODE == 0) {
            const uint64_t r = mix(gid * per + i) % nrec;
            uint4 q[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) q[j] = tab[r * 8 + j];
#pragma unroll
            for (int j = 0; j < 6; ++j) acc ^= q[j].x ^ q[j].w;
        } else if (MODE == 1) {
            const uint64_t r = mix(gid * per + i) % nrec;
            const uint4 q = tab[r * 8];
            acc ^= q.x ^ q.w;
        } else {
            // 60 lanes: 10 records x 6 quads per instruction; six instructions = 60 records per wave
            // (vs 64 in mode 0, normalised below)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const uint32_t rl = lane / 6, qd = lane % 6;
                const uint64_t r = mix((gid / 64) * per * 64 + i * 64 + j * 10 + rl) % nrec;
                if (lane < 60) {
                    const uint4 q = tab[r * 8 + qd];
                    acc ^= q.x ^ q.w;
                }
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = 1;
}

int main(int argc, char **argv) {
    uint4 *tab;
    uint32_t *sink;
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 256ull) << 20;
    hipMalloc(&tab, bytes);
    hipMemset(tab, 1, bytes);
    hipMalloc(&sink, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8, threads = 256;
    const uint64_t per = 32, nrec = bytes / 128;
    auto run = [&](auto k, double recs_per_lane_iter) {
        hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, tab, nrec, per, sink);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, tab, nrec, per, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double recs = (double)blocks * threads * per * recs_per_lane_iter;
        return recs / ms / 1e6;
    };
    printf("table %llu MiB: six 16-B loads per lane %.1f G records/s\n", (unsigned long long)(bytes >> 20),
           run(k_probe<0>, 1.0));
    printf("table %llu MiB: one 16-B load per lane  %.1f G records/s\n", (unsigned long long)(bytes >> 20),
           run(k_probe<1>, 1.0));
    printf("table %llu MiB: six lanes per record    %.1f G records/s\n", (unsigned long long)(bytes >> 20),
           run(k_probe<2>, 60.0 / 64.0));
    return 0;
}
