// Microbenchmark: LDS atomic add throughput (f32, u32, u64) vs plain RMW.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(512) void k(float* out, int iters, int sep) {
  extern __shared__ float lds[];
  unsigned* ldu = (unsigned*)lds;
  unsigned long long* ldq = (unsigned long long*)lds;
  for (int i = threadIdx.x; i < 8 * 3200; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kx = lane >> 3, ky = lane & 7;
  float v = 1.0f + lane;
  unsigned uv = lane + 1;
  int base = sep ? wave * 3200 / 8 * 0 + (wave & 7) * 400 : (wave & 3) * 3;
  for (int it = 0; it < iters; ++it) {
    int off = (kx + (it & 3)) * 40 + ky + base;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int o = sep ? off : q * 3200 + off;
      if (MODE == 0) { atomicAdd(&lds[o], v); atomicAdd(&lds[o + 1600 * (1 - sep)], v); }
      if (MODE == 2) { lds[o] += v; lds[o + 1600 * (1 - sep)] += v; }
      if (MODE == 3) { atomicAdd(&ldu[o], uv); atomicAdd(&ldu[o + 1600 * (1 - sep)], uv); }
      if (MODE == 4) { atomicAdd(&ldq[o >> 1], (unsigned long long)uv); atomicAdd(&ldq[(o >> 1) + 800], (unsigned long long)uv); }
    }
    v += 1e-3f; uv += 3;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[5];
}
template <int M> void run(const char* name, int threads, int sep, float* out) {
  size_t lds = 8 * 3200 * 4; int iters = 1000, nblk = 256;
  hipFuncSetAttribute((const void*)k<M>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(a); k<M><<<nblk, threads, lds>>>(out, iters, sep); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double lane_ops = (double)nblk * threads * iters * 16;
    if (rep) printf("%-10s threads %d sep %d: %8.3f ms  per-CU %6.2f lanes/clk (2.4GHz)\n", name, threads, sep, ms, lane_ops / (ms * 1e-3) / 256 / 2.4e9);
  }
}
int main() {
  float* out; (void)hipMalloc(&out, 4096 * 4);
  for (int sep = 0; sep < 2; ++sep) for (int th : {256, 512}) {
    run<0>("ds_add_f32", th, sep, out); run<3>("ds_add_u32", th, sep, out);
    run<4>("ds_add_u64", th, sep, out); run<2>("plain_rmw", th, sep, out);
  }
  return 0;
}
