"""Generate scripts/micro/fx_fft_check.hip: the fused x-FFT kernels' Stockham
transform (device code copied from csrc/wstack.hip) checked against hipFFT."""
import os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
s=open(os.path.join(ROOT, 'ska-sdp-func-python_amd', 'csrc', 'wstack.hip')).read()
def seg(a,b):
    i=s.index(a); j=s.index(b,i); return s[i:j]
fx=seg('__device__ __forceinline__ float2 cmulf','// pass 0\'s inputs v[r]')
body=r'''
template <int LOGN, int SG>
__global__ __launch_bounds__(FxShape<LOGN>::T) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_fft_only(const float2 *__restrict__ in, float2 *__restrict__ out, const float2 *__restrict__ twt) {
    using S = FxShape<LOGN>;
    extern __shared__ float2 fbuf[];
    const int t = threadIdx.x;
    float2 *const twl = fx_twl<LOGN>(fbuf, twt, t);
    const float2 *row = in + (size_t)blockIdx.x * S::N;
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = row[t + r * S::T];
    fx_fft<LOGN, SG>(v, fbuf, twl, t);
    for (int i = t; i < S::N; i += S::T) out[(size_t)blockIdx.x * S::N + i] = fbuf[fx_pad(i)];
}

template <int LOGN>
static std::vector<float2> twiddles() {
    using S = FxShape<LOGN>;
    std::vector<float2> h(S::TW);
    auto root = [](long num, long den) {
        const long double a = 2.0L * 3.14159265358979323846264338327950288L * num / den;
        return make_float2((float)std::cos(a), (float)std::sin(a));
    };
    for (int p = 1, ns = 16; p < S::P16; ++p, ns *= 16)
        for (int k = 0; k < ns; ++k) {
            h[S::tw_off(p) + 2 * k] = root(k, 16L * ns);
            h[S::tw_off(p) + 2 * k + 1] = root(4L * k, 16L * ns);
        }
    for (int t = 0; t < S::T; ++t) h[S::tw_off(S::P16) + t] = root(t, S::N);
    return h;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

template <int LOGN, int SG>
static int run(int rows) {
    using S = FxShape<LOGN>;
    const int N = S::N;
    std::vector<float2> h((size_t)rows * N);
    srand(1234 + LOGN);
    for (auto &x : h) x = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
    std::vector<float2> tw = twiddles<LOGN>();
    float2 *din, *dout, *dtw, *dref;
    double2 *dz;
    CK(hipMalloc(&din, h.size() * 8)); CK(hipMalloc(&dout, h.size() * 8)); CK(hipMalloc(&dref, h.size() * 8));
    CK(hipMalloc(&dtw, tw.size() * 8)); CK(hipMalloc(&dz, h.size() * 16));
    CK(hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice));
    const size_t lds = S::lds_bytes();
    CK(hipFuncSetAttribute((const void *)k_fft_only<LOGN, SG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k_fft_only<LOGN, SG><<<rows, S::T, lds>>>(din, dout, dtw);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    // references: hipFFT fp32 and fp64
    std::vector<double2> hz(h.size());
    for (size_t i = 0; i < h.size(); ++i) hz[i] = make_double2(h[i].x, h[i].y);
    CK(hipMemcpy(dz, hz.data(), hz.size() * 16, hipMemcpyHostToDevice));
    hipfftHandle p32, p64;
    hipfftPlan1d(&p32, N, HIPFFT_C2C, rows);
    hipfftPlan1d(&p64, N, HIPFFT_Z2Z, rows);
    const int dir = SG > 0 ? HIPFFT_BACKWARD : HIPFFT_FORWARD;
    hipfftExecC2C(p32, (hipfftComplex *)din, (hipfftComplex *)dref, dir);
    hipfftExecZ2Z(p64, (hipfftDoubleComplex *)dz, (hipfftDoubleComplex *)dz, dir);
    CK(hipDeviceSynchronize());
    std::vector<float2> o(h.size()), r32(h.size());
    CK(hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r32.data(), dref, r32.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hz.data(), dz, hz.size() * 16, hipMemcpyDeviceToHost));
    double e_f = 0, e_h = 0, nrm = 0;
    for (size_t i = 0; i < h.size(); ++i) {
        const double ax = o[i].x - hz[i].x, ay = o[i].y - hz[i].y;
        const double bx = r32[i].x - hz[i].x, by = r32[i].y - hz[i].y;
        e_f += ax * ax + ay * ay;
        e_h += bx * bx + by * by;
        nrm += hz[i].x * hz[i].x + hz[i].y * hz[i].y;
    }
    // timing
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) k_fft_only<LOGN, SG><<<rows, S::T, lds>>>(din, dout, dtw);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms_f; CK(hipEventElapsedTime(&ms_f, a, b));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipfftExecC2C(p32, (hipfftComplex *)din, (hipfftComplex *)dref, dir);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms_h; CK(hipEventElapsedTime(&ms_h, a, b));
    const bool ok = sqrt(e_f / nrm) < 3.0 * sqrt(e_h / nrm) + 1e-7;
    printf("N=%d sign=%+d rows=%d  relRMS fused %.3e  hipfft32 %.3e  ms fused %.4f hipfft %.4f  %s\n", N, SG, rows,
           sqrt(e_f / nrm), sqrt(e_h / nrm), ms_f / reps, ms_h / reps, ok ? "OK" : "FAIL");
    hipfftDestroy(p32); hipfftDestroy(p64);
    hipFree(din); hipFree(dout); hipFree(dref); hipFree(dtw); hipFree(dz);
    return ok ? 0 : 1;
}

int main() {
    int bad = 0;
    bad += run<7, 1>(512); bad += run<7, -1>(512);
    bad += run<8, 1>(512); bad += run<9, -1>(512);
    bad += run<10, 1>(512); bad += run<10, -1>(512);
    bad += run<11, 1>(512); bad += run<11, -1>(512);
    bad += run<12, 1>(512); bad += run<12, -1>(512);
    bad += run<13, 1>(4096); bad += run<13, -1>(4096);
    bad += run<14, 1>(512); bad += run<14, -1>(512);
    printf(bad ? "FAILED %d\n" : "ALL OK\n", bad);
    return bad ? 1 : 0;
}
'''
hdr='''// Standalone check of the fused x-FFT's Stockham transform against hipFFT
// fp32 / fp64.  Generated by scripts/micro/make_fx_fft_check.py from the
// device code in csrc/wstack.hip (cmulf .. fx_twl); do not edit.
// Build on the GPU box: hipcc --offload-arch=gfx950 -O3 -std=c++17 fx_fft_check.hip -lhipfft
#include <hip/hip_runtime.h>
#include <hipfft/hipfft.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
'''
open(os.path.join(ROOT, 'scripts', 'micro', 'fx_fft_check.hip'),'w').write(hdr+fx+body)
