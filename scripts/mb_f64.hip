// Microbenchmark: v_mfma_f64_16x16x4_f64 and v_fma_f64 issue rates on one
// GPU (cycles per instruction per SIMD), for sizing the fp64 NUFFT kernels.
// hipcc --offload-arch=gfx950 -O3 scripts/mb_f64.hip -o scripts/mb_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double doublex4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void k_mfma(double *out, int iters, double a0, double b0) {
    doublex4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = doublex4{0, 0, 0, 0};
    double a = a0 + threadIdx.x * 1e-9, b = b0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma(double *out, int iters, double a0, double b0) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = a0 + i + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fma(x[i], b0, a0);
    }
    double s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double *out;
    hipMalloc(&out, sizeof(double) * 1024 * 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    for (int wps = 1; wps <= 2; ++wps) {
        // one workgroup of 4*wps waves per CU: wps waves per SIMD
        const int blocks = cus, threads = 256 * wps;
        k_mfma<4><<<blocks, threads>>>(out, 10, 1.0, 1.0);
        hipEventRecord(e0);
        k_mfma<4><<<blocks, threads>>>(out, iters, 1.0, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double n_per_simd = (double)iters * 4 * wps;
        printf("mfma_f64_16x16x4: %d wave/SIMD: %.3f ms, %.2f ns per MFMA per SIMD, %.1f TFLOP/s\n",
               wps, ms, ms * 1e6 / n_per_simd,
               (double)blocks * 4 * n_per_simd * 2048 / (ms * 1e-3) / 1e12);
        k_fma<<<blocks, threads>>>(out, 10, 1.0, 1.0);
        hipEventRecord(e0);
        k_fma<<<blocks, threads>>>(out, iters, 1.0, 0.999);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        const double f_per_simd = (double)iters * 8 * wps;
        printf("v_fma_f64:        %d wave/SIMD: %.3f ms, %.2f ns per wave-FMA per SIMD, %.1f TFLOP/s\n",
               wps, ms, ms * 1e6 / f_per_simd,
               (double)blocks * 4 * f_per_simd * 128 / (ms * 1e-3) / 1e12);
    }
    return 0;
}
