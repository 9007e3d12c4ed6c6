// Returning 32-bit atomicAdd throughput on random addresses vs the size of
// the counter array (L2-, MALL- or HBM-resident), one lane per atomic: does a
// smaller (coarser) bucket histogram make the count pass cheaper?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_atomics(unsigned *cnt, uint32_t mask, unsigned *out, uint32_t iters) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        x = x * 1664525u + 1013904223u;                      // LCG per lane
        const uint32_t h = (x ^ (x >> 13)) * 0x9E3779B1u;
        acc += atomicAdd(&cnt[h & mask], 1u);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    const uint32_t nthreads = 1u << 22, iters = 64;  // 268 M atomics per size
    unsigned *cnt, *out;
    hipMalloc(&cnt, (size_t)1 << 32);  // up to 1 Gi counters
    hipMalloc(&out, (size_t)nthreads * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int lg = 16; lg <= 30; lg += 2) {
        const uint32_t mask = (1u << lg) - 1;
        hipMemset(cnt, 0, ((size_t)1 << lg) * 4);
        k_atomics<<<nthreads / 256, 256>>>(cnt, mask, out, 4);  // warm
        hipEventRecord(a);
        k_atomics<<<nthreads / 256, 256>>>(cnt, mask, out, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double n = (double)nthreads * iters;
        printf("{\"counters\": %u, \"bytes_MB\": %.1f, \"ms\": %.3f, \"G_atomics_s\": %.2f}\n",
               1u << lg, (double)(4ull << lg) / 1e6, ms, n / ms / 1e6);
    }
    return 0;
}
