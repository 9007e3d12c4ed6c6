// Sky-component DFT predict for gfx950: sdp_hip_dft_point_v00 (drop-in for
// ska_sdp_func.visibility.dft_point_v00 and the reference's cupy dft_kernel,
// src/ska_sdp_func_python/imaging/dft.py:173-178, :185-262) and
// sdp_hip_dft_point_metres (uvw in metres + frequencies, lambda scaling fused).
//
//   vis[row, chan, pol] = sum_c flux[c, chan|0, pol] exp(-2 pi i (u l + v m + w (n-1)))
//
// Components are staged through LDS in chunks (direction cosines as fp64,
// fluxes as fp32 complex).  The phase u l + v m + w (n - 1) is an fp64 MFMA
// product (k_dft_mfma below), reduced to turns in fp64 (v_fract_f64) before
// the hardware v_sin_f32 / v_cos_f32 (which take revolutions), so SKA-scale
// u ~ 1e6 wavelengths lose no phase precision; the component sum accumulates
// in fp32 for complex64 output and in fp64 for complex128 output (the
// reference's dft_cpu_looped sums in complex128, imaging/dft.py:265-285).
// C3 (1000 components x 10 Mvis, one channel): 3.36 ms = 2,970 G comp*vis/s,
// against 4.43 - 4.49 ms for the previous one-thread-per-visibility VALU
// kernel (fp64 phase by FMAs, rint) on one box (profiles/r06_dft_mfma_ab.txt).
#include <type_traits>

#include "sdp_common.h"

namespace sdp {
namespace dft {

constexpr double kCLight = 299792458.0;
constexpr int kThreads = 256;

__device__ __forceinline__ float2 to_f2(const double2 v) { return make_float2((float)v.x, (float)v.y); }
__device__ __forceinline__ void put(float2 *p, float re, float im) { *p = make_float2(re, im); }
__device__ __forceinline__ void put(double2 *p, double re, double im) { *p = make_double2(re, im); }

// MFMA form: the phase product (u, v, w) . (l, m, n - 1) of 16 visibilities x
// 16 components is one v_mfma_f64_16x16x4_f64 (exact fp64 FMAs; A = the
// visibilities' uvw_lambda with K = 4 (the fourth zero), B = the components'
// direction cosines), so the VALU keeps only the reduction to turns
// (v_fract_f64), the fp32 sin / cos and the flux multiply-add.  Lane l of the
// product holds visibility rows (l >> 4) + 4 i (i = 0..3) against component
// l & 15 (the f64 16x16 output layout: register i of lane l is row
// (l >> 4) + 4 i); the lanes sum over their 16 components at the end (a
// 16-lane butterfly).  A workgroup holds 4 waves x T tiles of 16 rows of ONE channel
// (blockIdx.y), so a per-channel flux is one value per component and lane.
typedef double doublex4 __attribute__((ext_vector_type(4)));
constexpr int kMfmaChunk = 256;  // components staged per LDS chunk (a multiple of 16)

template <int NPOL, class OT, bool kMetres, int T>
__global__ __launch_bounds__(kThreads) void k_dft_mfma(int ncomp, const double *__restrict__ dc,
                                                       const double2 *__restrict__ flux,
                                                       int fnchan, int64_t nrow, int nchan,
                                                       const double *__restrict__ uvw,
                                                       const double *__restrict__ freq,
                                                       OT *__restrict__ vis) {
    __shared__ double s_b[kMfmaChunk * 4];  // (l, m, n - 1, 0) per component
    // c128 output: fp64 flux, sincos and sums (the reference's numpy fp64
    // arithmetic for that dtype); c64: fp32 sincos of the fp64-reduced phase
    constexpr bool kF64 = std::is_same<OT, double2>::value;
    using FT2 = typename std::conditional<kF64, double2, float2>::type;
    __shared__ FT2 s_fl[kMfmaChunk * NPOL];
    using AT = typename std::conditional<kF64, double, float>::type;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int chan = blockIdx.y;
    const int k = lane >> 4, r16 = lane & 15;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * (16 * T);
    // A operands: uvw_lambda of row row0 + 16 t + r16, component k (k = 3: 0)
    double aop[T];
    const double s = kMetres ? freq[chan] / kCLight : 1.0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int64_t row = row0 + 16 * t + r16;
        double a = 0.0;
        if (row < nrow && k < 3)
            a = kMetres ? uvw[row * 3 + k] * s : uvw[(row * nchan + chan) * 3 + k];
        aop[t] = a;
    }
    AT ar[T][4][NPOL], ai[T][4][NPOL];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int p = 0; p < NPOL; ++p) ar[t][i][p] = ai[t][i][p] = (AT)0;
    const int fch = fnchan == 1 ? 0 : chan;
    for (int c0 = 0; c0 < ncomp; c0 += kMfmaChunk) {
        const int nc = min(kMfmaChunk, ncomp - c0);
        const int ncp = (nc + 15) & ~15;  // padded: zero flux, zero direction
        __syncthreads();
        for (int i = threadIdx.x; i < ncp * 4; i += kThreads) {
            const int c = i >> 2, q = i & 3;
            s_b[i] = (c < nc && q < 3) ? dc[(int64_t)(c0 + c) * 3 + q] : 0.0;
        }
        for (int i = threadIdx.x; i < ncp * NPOL; i += kThreads) {
            const int c = i / NPOL, p = i - c * NPOL;
            if constexpr (kF64)
                s_fl[i] = c < nc ? flux[((int64_t)(c0 + c) * fnchan + fch) * NPOL + p]
                                 : make_double2(0.0, 0.0);
            else
                s_fl[i] = c < nc ? to_f2(flux[((int64_t)(c0 + c) * fnchan + fch) * NPOL + p])
                                 : make_float2(0.0f, 0.0f);
        }
        __syncthreads();
        for (int ct = 0; ct < ncp; ct += 16) {
            const int c = ct + r16;  // this lane's component
            const double bop = s_b[c * 4 + k];
            FT2 f[NPOL];
#pragma unroll
            for (int p = 0; p < NPOL; ++p) f[p] = s_fl[c * NPOL + p];
            doublex4 ph[T];
#pragma unroll
            for (int t = 0; t < T; ++t)
                ph[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop[t], bop,
                                                             doublex4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    // the phase in turns, reduced to [0, 1) in fp64
                    if constexpr (kF64) {
                        double sn, cs;
                        sincospi(2.0 * __builtin_amdgcn_fract(ph[t][i]), &sn, &cs);
#pragma unroll
                        for (int p = 0; p < NPOL; ++p) {
                            ar[t][i][p] = fma(f[p].y, sn, fma(f[p].x, cs, ar[t][i][p]));
                            ai[t][i][p] = fma(-f[p].x, sn, fma(f[p].y, cs, ai[t][i][p]));
                        }
                    } else {
                        const float x = (float)__builtin_amdgcn_fract(ph[t][i]);
                        const float sn = __builtin_amdgcn_sinf(x);  // sin(2 pi x)
                        const float cs = __builtin_amdgcn_cosf(x);
#pragma unroll
                        for (int p = 0; p < NPOL; ++p) {
                            // f * exp(-2 pi i x) = f * (cs - i sn); fp32 sums
                            // as two fused multiply-adds per part (packed pairs)
                            ar[t][i][p] = fmaf(f[p].y, sn, fmaf(f[p].x, cs, ar[t][i][p]));
                            ai[t][i][p] = fmaf(-f[p].x, sn, fmaf(f[p].y, cs, ai[t][i][p]));
                        }
                    }
                }
        }
    }
    // sum over the 16 components of each lane group, then lane (k, i) writes
    // row 16 t + k + 4 i
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int p = 0; p < NPOL; ++p)
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    ar[t][i][p] += __shfl_xor(ar[t][i][p], o, 64);
                    ai[t][i][p] += __shfl_xor(ai[t][i][p], o, 64);
                }
        const int64_t row = row0 + 16 * t + k + 4 * r16;
        if (r16 < 4 && row < nrow) {
#pragma unroll
            for (int p = 0; p < NPOL; ++p) {
                AT xr = ar[t][0][p], xi = ai[t][0][p];
#pragma unroll
                for (int i = 1; i < 4; ++i)
                    if (r16 == i) {
                        xr = ar[t][i][p];
                        xi = ai[t][i][p];
                    }
                put(vis + (row * nchan + chan) * NPOL + p, xr, xi);
            }
        }
    }
}

template <class OT, bool kMetres, int NPOL>
static void launch_mfma(int ncomp, const double *dc, const double2 *flux, int fnchan,
                        int64_t nrow, int nchan, const double *uvw, const double *freq, OT *out,
                        hipStream_t st) {
    constexpr int T = NPOL == 1 ? 4 : NPOL == 2 ? 2 : 1;
    const int64_t rows_per = 4 * 16 * T;
    const int64_t nbx = (nrow + rows_per - 1) / rows_per;
    SDP_REQUIRE(nchan <= 65535 && nbx < 2147483647, "too many channels or rows for one DFT call");
    k_dft_mfma<NPOL, OT, kMetres, T><<<dim3((unsigned)nbx, (unsigned)nchan), kThreads, 0, st>>>(
        ncomp, dc, flux, fnchan, nrow, nchan, uvw, freq, out);
}

template <class OT, bool kMetres>
static void launch(int ncomp, const double *dc, const double2 *flux, int fnchan, int npol,
                   int64_t nrow, int nchan, const double *uvw, const double *freq, void *vis,
                   hipStream_t st) {
    OT *out = static_cast<OT *>(vis);
    switch (npol) {
        case 1: launch_mfma<OT, kMetres, 1>(ncomp, dc, flux, fnchan, nrow, nchan, uvw, freq, out, st); break;
        case 2: launch_mfma<OT, kMetres, 2>(ncomp, dc, flux, fnchan, nrow, nchan, uvw, freq, out, st); break;
        case 4: launch_mfma<OT, kMetres, 4>(ncomp, dc, flux, fnchan, nrow, nchan, uvw, freq, out, st); break;
        default: throw Error(SDP_HIP_ERR_INVALID_ARG, "npol must be 1, 2 or 4");
    }
    SDP_HIP_CHECK(hipGetLastError());
}

static void run(bool metres, int ncomp, const double *dc, const void *fluxes, int fnchan,
                int npol, int64_t nrow, int nchan, const double *uvw, const double *freq,
                void *vis, int vis_dtype, hipStream_t st) {
    SDP_REQUIRE(ncomp >= 0 && nrow >= 0 && nchan > 0, "bad sizes");
    SDP_REQUIRE(fnchan == 1 || fnchan == nchan, "flux channels must be 1 or nchan");
    SDP_REQUIRE(vis != nullptr && (ncomp == 0 || (dc && fluxes)) && (nrow == 0 || uvw),
                "null pointer argument");
    SDP_REQUIRE(!metres || freq != nullptr, "freq required with uvw in metres");
    if (nrow == 0) return;
    const double2 *flux = static_cast<const double2 *>(fluxes);
    if (vis_dtype == SDP_HIP_C128) {
        if (metres)
            launch<double2, true>(ncomp, dc, flux, fnchan, npol, nrow, nchan, uvw, freq, vis, st);
        else
            launch<double2, false>(ncomp, dc, flux, fnchan, npol, nrow, nchan, uvw, freq, vis, st);
    } else if (vis_dtype == SDP_HIP_C64) {
        if (metres)
            launch<float2, true>(ncomp, dc, flux, fnchan, npol, nrow, nchan, uvw, freq, vis, st);
        else
            launch<float2, false>(ncomp, dc, flux, fnchan, npol, nrow, nchan, uvw, freq, vis, st);
    } else {
        throw Error(SDP_HIP_ERR_INVALID_ARG, "vis must be complex64 or complex128");
    }
}

}  // namespace dft
}  // namespace sdp

extern "C" {

int sdp_hip_dft_point_v00(int ncomp, const double *direction_cosines, const void *fluxes,
                          int flux_nchan, int npol, int64_t nrow, int nchan,
                          const double *uvw_lambda, void *vis, int vis_dtype, void *stream,
                          char *errbuf, size_t errbuf_len) {
    return sdp::guarded(errbuf, errbuf_len, [&] {
        sdp::dft::run(false, ncomp, direction_cosines, fluxes, flux_nchan, npol, nrow, nchan,
                      uvw_lambda, nullptr, vis, vis_dtype, sdp::as_stream(stream));
    });
}

int sdp_hip_dft_point_metres(int ncomp, const double *direction_cosines, const void *fluxes,
                             int flux_nchan, int npol, int64_t nrow, int nchan,
                             const double *uvw, const double *freq, void *vis, int vis_dtype,
                             void *stream, char *errbuf, size_t errbuf_len) {
    return sdp::guarded(errbuf, errbuf_len, [&] {
        sdp::dft::run(true, ncomp, direction_cosines, fluxes, flux_nchan, npol, nrow, nchan, uvw,
                      freq, vis, vis_dtype, sdp::as_stream(stream));
    });
}

}  // extern "C"
