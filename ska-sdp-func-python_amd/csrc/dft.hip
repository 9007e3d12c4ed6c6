// Sky-component DFT predict for gfx950: sdp_hip_dft_point_v00 (drop-in for
// ska_sdp_func.visibility.dft_point_v00 and the reference's cupy dft_kernel,
// src/ska_sdp_func_python/imaging/dft.py:173-178, :185-262) and
// sdp_hip_dft_point_metres (uvw in metres + frequencies, lambda scaling fused).
//
//   vis[row, chan, pol] = sum_c flux[c, chan|0, pol] exp(-2 pi i (u l + v m + w (n-1)))
//
// One thread per visibility; components are staged through LDS in chunks
// (direction cosines as fp64, fluxes as fp32 complex).  The phase is formed in
// fp64 and reduced to turns (t - rint(t)) before the hardware v_sin_f32 /
// v_cos_f32 (which take revolutions), so SKA-scale u ~ 1e6 wavelengths lose
// no phase precision; the component sum accumulates in fp32 for complex64
// output and in fp64 for complex128 output (the reference's dft_cpu_looped
// sums in complex128, imaging/dft.py:265-285).
#include <type_traits>

#include "sdp_common.h"

namespace sdp {
namespace dft {

constexpr double kCLight = 299792458.0;
constexpr int kThreads = 256;
constexpr int kCompChunk = 256;

__device__ __forceinline__ float2 to_f2(const double2 v) { return make_float2((float)v.x, (float)v.y); }
__device__ __forceinline__ void put(float2 *p, float re, float im) { *p = make_float2(re, im); }
__device__ __forceinline__ void put(double2 *p, double re, double im) { *p = make_double2(re, im); }

template <int NPOL, class OT, bool kMetres>
__global__ __launch_bounds__(kThreads) void k_dft(int ncomp, const double *__restrict__ dc,
                                                  const double2 *__restrict__ flux, int fnchan,
                                                  int64_t nrow, int nchan,
                                                  const double *__restrict__ uvw,
                                                  const double *__restrict__ freq,
                                                  OT *__restrict__ vis) {
    __shared__ double s_dc[kCompChunk * 3];
    __shared__ float2 s_fl[kCompChunk * NPOL];
    const int64_t nvis = nrow * (int64_t)nchan;
    const int64_t v = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    const bool ok = v < nvis;
    const int64_t row = ok ? v / nchan : 0;
    const int chan = ok ? (int)(v - row * nchan) : 0;
    double u = 0.0, vv = 0.0, w = 0.0;
    if (ok) {
        if (kMetres) {
            const double s = freq[chan] / kCLight;
            u = uvw[row * 3] * s;
            vv = uvw[row * 3 + 1] * s;
            w = uvw[row * 3 + 2] * s;
        } else {
            u = uvw[v * 3];
            vv = uvw[v * 3 + 1];
            w = uvw[v * 3 + 2];
        }
    }
    using AT = typename std::conditional<std::is_same<OT, double2>::value, double, float>::type;
    AT ar[NPOL], ai[NPOL];
#pragma unroll
    for (int p = 0; p < NPOL; ++p) ar[p] = ai[p] = (AT)0;
    const bool shared_flux = fnchan == 1;
    for (int c0 = 0; c0 < ncomp; c0 += kCompChunk) {
        const int nc = min(kCompChunk, ncomp - c0);
        __syncthreads();
        for (int i = threadIdx.x; i < nc * 3; i += kThreads) s_dc[i] = dc[(int64_t)c0 * 3 + i];
        if (shared_flux)
            for (int i = threadIdx.x; i < nc * NPOL; i += kThreads)
                s_fl[i] = to_f2(flux[(int64_t)c0 * NPOL + i]);
        __syncthreads();
        for (int c = 0; c < nc; ++c) {
            double ph = u * s_dc[3 * c] + vv * s_dc[3 * c + 1] + w * s_dc[3 * c + 2];
            ph -= rint(ph);
            const float t = (float)ph;
            const float sn = __builtin_amdgcn_sinf(t);  // sin(2 pi t), t in turns
            const float cs = __builtin_amdgcn_cosf(t);
#pragma unroll
            for (int p = 0; p < NPOL; ++p) {
                const float2 f = shared_flux
                                     ? s_fl[c * NPOL + p]
                                     : to_f2(flux[((int64_t)(c0 + c) * fnchan + chan) * NPOL + p]);
                // f * exp(-2 pi i t) = f * (cs - i sn): the fp32 products
                // summed in the accumulator's precision
                ar[p] += (AT)(f.x * cs + f.y * sn);
                ai[p] += (AT)(f.y * cs - f.x * sn);
            }
        }
    }
    if (ok) {
#pragma unroll
        for (int p = 0; p < NPOL; ++p) put(vis + v * NPOL + p, ar[p], ai[p]);
    }
}

template <class OT, bool kMetres>
static void launch(int ncomp, const double *dc, const double2 *flux, int fnchan, int npol,
                   int64_t nrow, int nchan, const double *uvw, const double *freq, void *vis,
                   hipStream_t st) {
    const unsigned nb = grid1d(nrow * (int64_t)nchan, kThreads);
    OT *out = static_cast<OT *>(vis);
    switch (npol) {
        case 1:
            k_dft<1, OT, kMetres><<<nb, kThreads, 0, st>>>(ncomp, dc, flux, fnchan, nrow, nchan,
                                                          uvw, freq, out);
            break;
        case 2:
            k_dft<2, OT, kMetres><<<nb, kThreads, 0, st>>>(ncomp, dc, flux, fnchan, nrow, nchan,
                                                          uvw, freq, out);
            break;
        case 4:
            k_dft<4, OT, kMetres><<<nb, kThreads, 0, st>>>(ncomp, dc, flux, fnchan, nrow, nchan,
                                                          uvw, freq, out);
            break;
        default:
            throw Error(SDP_HIP_ERR_INVALID_ARG, "npol must be 1, 2 or 4");
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
