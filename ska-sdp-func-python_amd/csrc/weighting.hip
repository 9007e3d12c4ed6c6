// Imaging weights for gfx950: sdp_hip_grid_weights / sdp_hip_reweight /
// sdp_hip_taper, replacing the chan x pol x row Python loops of the
// reference's
//   grid_visibility_weight_to_griddata   src/ska_sdp_func_python/grid_data/gridding.py:258-334
//   griddata_visibility_reweight         gridding.py:362-499
//   taper_visibility_gaussian / _tukey   src/ska_sdp_func_python/imaging/weighting.py:71-136
// (weight_visibility, weighting.py:35-68, is the grid + reweight pair).
//
// Layout: weights / flags / imaging weights are the Visibility's
// [nrow, nchan, npol] arrays (nrow = ntimes * nbaselines), uvw [nrow, 3]
// metres, the weight grid real f64 [g_nchan, npol, ny, nx].
//
// One thread owns kChan consecutive channels x all pols of one row (a
// contiguous span of the weight array), so a wave reads whole cache lines.
// The nearest-cell mapping is the reference's (gridding.py:49-57, :148-157):
//   u = uvw_u * (freq / c);  pu = round_half_even((u - crval) / cdelt + crpix - 1)
// evaluated with the same IEEE operations in the same order (fp contraction
// is off in this file), so cell indices are bit-identical to numpy's.
// Gridding aggregates runs of consecutive channels that land in the same cell
// (every short baseline does) in registers and issues one fp64 atomic per run
// and cell; the HBM-bound read of the weights stays the floor.
#include "sdp_common.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

#pragma clang fp contract(off)

namespace sdp {
namespace weighting {

constexpr int kThreads = 256;
constexpr int kChan = 8;
constexpr double kC = 299792458.0;
constexpr int kMaxLdsSum = 256;  // g_nchan * npol entries summed in LDS
constexpr int kMaxLdsK = 1024;   // channels whose freq / c lives in LDS

struct Geom {
    int64_t nrow;
    int nchan, npol, g_nchan, ny, nx;
    double u_val, u_del, u_pix, v_val, v_del, v_pix;
    int flag_bytes;  // 0: no flags, else 1 / 4 / 8 byte integers
    int zero_val;    // crval_u == crval_v == 0: one division gives cell and conjugate
    int win, win_u0, win_v0;  // LDS-privatised uv window (win x win cells), 0 = none
    int nt;                   // threads per block of k_grid_weights (256 or 1024)
    int mirror;               // conjugate cell == mirror of the cell about (cu2/2, cv2/2)
    long long cu2, cv2;       //   (crval 0, integral crpix): grid only the cell, fold later
};

__device__ __forceinline__ double nan_to_num(double x) {
    if (isnan(x)) return 0.0;
    if (isinf(x)) return x > 0 ? DBL_MAX : -DBL_MAX;
    return x;
}

// numpy.round(...).astype(int); values far outside any grid map to -1
// (astype's result there is unspecified and always off-grid).
__device__ __forceinline__ long long round_pix(double p) {
    p = rint(p);
    return fabs(p) < 4.0e18 ? (long long)p : -1;
}

struct Cell {
    long long pu, pv, puc, pvc;
};

// world2pix: (world - crval) / cdelt + crpix - 1.  With crval == 0,
// (-u - 0) / cdelt == -(u / cdelt) exactly, so the conjugate cell reuses the
// quotient -- still the reference's IEEE result, bit for bit.
__device__ __forceinline__ Cell map_cell(const Geom &g, double uu, double vv, double k) {
    const double u = nan_to_num(uu * k), v = nan_to_num(vv * k);
    if (g.zero_val) {
        const double qu = u / g.u_del, qv = v / g.v_del;
        return {round_pix(qu + g.u_pix - 1.0), round_pix(qv + g.v_pix - 1.0),
                round_pix(-qu + g.u_pix - 1.0), round_pix(-qv + g.v_pix - 1.0)};
    }
    return {round_pix((u - g.u_val) / g.u_del + g.u_pix - 1.0),
            round_pix((v - g.v_val) / g.v_del + g.v_pix - 1.0),
            round_pix((-u - g.u_val) / g.u_del + g.u_pix - 1.0),
            round_pix((-v - g.v_val) / g.v_del + g.v_pix - 1.0)};
}

__device__ __forceinline__ bool in_grid(const Geom &g, const Cell &c) {
    return c.pv >= 0 && c.pv < g.ny && c.pu >= 0 && c.pu < g.nx && c.pvc >= 0 &&
           c.pvc < g.ny && c.puc >= 0 && c.puc < g.nx;
}

__device__ __forceinline__ double flag_of(const void *flags, int bytes, size_t i) {
    if (bytes == 8) return (double)static_cast<const int64_t *>(flags)[i];
    if (bytes == 4) return (double)static_cast<const int32_t *>(flags)[i];
    if (bytes == 1) return (double)static_cast<const int8_t *>(flags)[i];
    return 0.0;
}

// flagged_weight = weight * (1 - flags)  (datamodels' visibility_acc)
__device__ __forceinline__ double flagged(const double *w, const void *flags, int bytes, size_t i) {
    return bytes ? w[i] * (1.0 - flag_of(flags, bytes, i)) : w[i];
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// first element of span s (spans tile each row in kChan-channel pieces)
__device__ __forceinline__ int64_t span_elem(int64_t s, int nspan, int rowlen, int np) {
    const int64_t row = s / nspan;
    return row * rowlen + (s - row * nspan) * (int64_t)(kChan * np);
}

// ---- grid_visibility_weight_to_griddata -----------------------------------
// Persistent blocks (1024 threads, one per CU) walk tiles of spans; each
// thread loads its span's weights and flags with 16-B loads and walks the
// channels, merging runs that stay in one cell.  Three measures cut the
// fp64 atomics, which execute memory-side and dominate this kernel:
//  * cells inside the central uv window (where the short baselines of a
//    dense core pile up: 78% of the C2 samples land in the central 128x128
//    cells) accumulate in block-private LDS (128 KB), written out as
//    per-block partials and summed by k_window_flush;
//  * with crval = 0 and an integral crpix the conjugate cell is the mirror
//    of the cell except at exact rounding ties, so only the cell is gridded
//    (into g1) and k_mirror_fold adds g1 + mirror(g1) to the grid; tie
//    samples add both cells to the grid directly;
//  * the remaining cells take one global atomic per run.
// C2 (123.6 Mvis, 4096^2): 11.3 ms with plain atomics -> 1.9 ms.
template <int NP, int NT>
__global__ __launch_bounds__(NT) void k_grid_weights(Geom g, int64_t ntiles,
                                                           const double *__restrict__ uvw,
                                                           const double *__restrict__ freq,
                                                           const double *__restrict__ wt,
                                                           const void *__restrict__ flags,
                                                           const int32_t *__restrict__ vis_to_im,
                                                           double *grid, double *g1,
                                                           double *sumwt, double *win_partial,
                                                           unsigned long long *nskipped) {
    // g1: where run cells go (== grid unless g.mirror, then only the direct
    // cell is gridded and k_mirror_fold adds g1 and its mirror image to grid)
    extern __shared__ double lds[];
    double *s_win = lds;                                   // nplanes * win * win
    const int nplanes = g.g_nchan * NP;
    const int nwin = g.win ? nplanes * g.win * g.win : 0;
    __shared__ double s_sum[kMaxLdsSum];
    __shared__ double s_k[kMaxLdsK];
    __shared__ unsigned long long s_skip;
    const bool lds_sum = nplanes <= kMaxLdsSum;
    const bool lds_k = g.nchan <= kMaxLdsK;
    if (lds_k)
        for (int i = threadIdx.x; i < g.nchan; i += NT) s_k[i] = freq[i] / kC;
    for (int i = threadIdx.x; i < nwin; i += NT) s_win[i] = 0.0;
    if (lds_sum)
        for (int i = threadIdx.x; i < nplanes; i += NT) s_sum[i] = 0.0;
    if (threadIdx.x == 0) s_skip = 0;

    const int nspan = (g.nchan + kChan - 1) / kChan;
    const int rowlen = g.nchan * NP;
    const int64_t nspans = g.nrow * nspan;
    unsigned long long skipped = 0;

    __syncthreads();
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t s0 = tile * NT;
        const int64_t sp = s0 + threadIdx.x;
        if (sp >= nspans) continue;
        double w[kChan * NP];
        const int64_t e = span_elem(sp, nspan, rowlen, NP);
        const int ne = min(kChan, g.nchan - (int)(sp % nspan) * kChan) * NP;
        if (ne == kChan * NP && ((e & 1) == 0)) {
            // full span, 16-B aligned: vector loads (a wave's loads cover one
            // contiguous range; lines are reused from L1 across the group)
            const double2 *w2 = reinterpret_cast<const double2 *>(wt + e);
#pragma unroll
            for (int i = 0; i < kChan * NP / 2; ++i) {
                const double2 x = w2[i];
                w[2 * i] = x.x;
                w[2 * i + 1] = x.y;
            }
            if (g.flag_bytes == 8) {
                const longlong2 *f2 =
                    reinterpret_cast<const longlong2 *>(static_cast<const int64_t *>(flags) + e);
#pragma unroll
                for (int i = 0; i < kChan * NP / 2; ++i) {
                    const longlong2 f = f2[i];
                    w[2 * i] *= 1.0 - (double)f.x;
                    w[2 * i + 1] *= 1.0 - (double)f.y;
                }
            } else if (g.flag_bytes) {
#pragma unroll
                for (int i = 0; i < kChan * NP; ++i)
                    w[i] *= 1.0 - flag_of(flags, g.flag_bytes, (size_t)(e + i));
            }
        } else {
#pragma unroll
            for (int i = 0; i < kChan * NP; ++i)
                w[i] = i < ne ? flagged(wt, flags, g.flag_bytes, (size_t)(e + i)) : 0.0;
        }
        const int64_t row = sp / nspan;
        const int c0 = (int)(sp - row * nspan) * kChan;
        const int nc = min(kChan, g.nchan - c0);
        const double uu = uvw[3 * row], vv = uvw[3 * row + 1];

        Cell cur{};
        int cur_ic = -1, sum_ic = -1;
        double acc[NP], ssum[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) acc[p] = ssum[p] = 0.0;
        auto add_cell = [&](int plane0, long long pu, long long pv, const double *a) {
            const long long du = pu - g.win_u0, dv = pv - g.win_v0;
            if (g.win && du >= 0 && du < g.win && dv >= 0 && dv < g.win) {
#pragma unroll
                for (int p = 0; p < NP; ++p)
                    atomicAdd(&s_win[((plane0 + p) * g.win + dv) * g.win + du], a[p]);
            } else {
#pragma unroll
                for (int p = 0; p < NP; ++p)
                    atomicAdd(g1 + ((size_t)(plane0 + p) * g.ny + pv) * g.nx + pu, a[p]);
            }
        };
        auto flush = [&]() {
            if (cur_ic < 0) return;
            add_cell(cur_ic * NP, cur.pu, cur.pv, acc);
            if (!g.mirror) add_cell(cur_ic * NP, cur.puc, cur.pvc, acc);
#pragma unroll
            for (int p = 0; p < NP; ++p) acc[p] = 0.0;
        };
        auto flush_sum = [&]() {
            if (sum_ic < 0) return;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                if (lds_sum) atomicAdd(&s_sum[sum_ic * NP + p], ssum[p]);
                else atomicAdd(&sumwt[sum_ic * NP + p], ssum[p]);
                ssum[p] = 0.0;
            }
        };
        for (int c = 0; c < nc; ++c) {
            const int ch = c0 + c;
            const Cell cell = map_cell(g, uu, vv, lds_k ? s_k[ch] : freq[ch] / kC);
            if (!in_grid(g, cell)) {
                skipped += NP;
                continue;
            }
            const int ic = vis_to_im[ch];
            if (g.mirror && (cell.pu + cell.puc != g.cu2 || cell.pv + cell.pvc != g.cv2)) {
                // rounding tie: the conjugate is not the mirror cell; both go
                // straight to the output grid
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    double *gp = grid + (size_t)(ic * NP + p) * g.ny * g.nx;
                    atomicAdd(gp + cell.pv * g.nx + cell.pu, w[c * NP + p]);
                    atomicAdd(gp + cell.pvc * g.nx + cell.puc, w[c * NP + p]);
                }
                if (ic != sum_ic) {
                    flush_sum();
                    sum_ic = ic;
                }
#pragma unroll
                for (int p = 0; p < NP; ++p) ssum[p] += w[c * NP + p] * 2;
                continue;
            }
            if (ic != cur_ic || cell.pu != cur.pu || cell.pv != cur.pv || cell.puc != cur.puc ||
                cell.pvc != cur.pvc) {
                flush();
                if (ic != sum_ic) {
                    flush_sum();
                    sum_ic = ic;
                }
                cur = cell;
                cur_ic = ic;
            }
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                acc[p] += w[c * NP + p];
                ssum[p] += w[c * NP + p] * 2;
            }
        }
        flush();
        flush_sum();
    }
    if (skipped) atomicAdd(&s_skip, skipped);
    __syncthreads();
    if (lds_sum)
        for (int i = threadIdx.x; i < nplanes; i += NT)
            if (s_sum[i] != 0.0) atomicAdd(&sumwt[i], s_sum[i]);
    for (int i = threadIdx.x; i < nwin; i += NT)
        win_partial[(size_t)blockIdx.x * nwin + i] = s_win[i];
    if (threadIdx.x == 0 && s_skip) atomicAdd(nskipped, s_skip);
}

// grid += g1 + mirror(g1): the conjugate half of every non-tie sample.
__global__ __launch_bounds__(kThreads) void k_mirror_fold(Geom g, int64_t ncell,
                                                          const double *__restrict__ g1,
                                                          double *grid) {
    const int64_t plane_n = (int64_t)g.ny * g.nx;
    for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < ncell;
         i += (int64_t)gridDim.x * kThreads) {
        const int64_t plane = i / plane_n, r = i - plane * plane_n;
        const long long y = r / g.nx, x = r - y * g.nx;
        const long long my = g.cv2 - y, mx = g.cu2 - x;
        double s = g1[i];
        if (my >= 0 && my < g.ny && mx >= 0 && mx < g.nx) s += g1[plane * plane_n + my * g.nx + mx];
        if (s != 0.0) grid[i] += s;
    }
}

// g1[window] += sum over blocks of the LDS partials (one writer per cell).
// Block = 16 cells x 16 block-stripes, stripes combined in LDS.
__global__ __launch_bounds__(kThreads) void k_window_flush(Geom g, int nplanes, int nblocks,
                                                           const double *__restrict__ win_partial,
                                                           double *grid) {
    __shared__ double s_part[kThreads];
    const int nwin = nplanes * g.win * g.win;
    const int cl = threadIdx.x & 15, stripe = threadIdx.x >> 4;
    const int i = blockIdx.x * 16 + cl;
    double s = 0.0;
    if (i < nwin)
        for (int b = stripe; b < nblocks; b += 16) s += win_partial[(size_t)b * nwin + i];
    s_part[threadIdx.x] = s;
    __syncthreads();
    if (stripe == 0 && i < nwin) {
        for (int k = 1; k < 16; ++k) s += s_part[k * 16 + cl];
        if (s != 0.0) {
            const int plane = i / (g.win * g.win), r = i - plane * g.win * g.win;
            const int dv = r / g.win, du = r - dv * g.win;
            grid[((size_t)plane * g.ny + g.win_v0 + dv) * g.nx + g.win_u0 + du] += s;
        }
    }
}

// ---- reductions for the robust weighting constant --------------------------
// mode 0: sum of x^2 (sumlocwt = sum(real_gd**2), gridding.py:410)
// mode 1: sum of flagged weights (sumwt = sum(flagged_weight), :412-414)
__global__ __launch_bounds__(kThreads) void k_reduce(const double *__restrict__ x,
                                                     const void *__restrict__ flags,
                                                     int flag_bytes, size_t n, int mode,
                                                     double *partial) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n;
         i += (size_t)gridDim.x * kThreads) {
        if (mode == 0) s += x[i] * x[i];
        else s += flagged(x, flags, flag_bytes, i);
    }
    __shared__ double s_w[kThreads / 64];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = 0.0;
        for (int i = 0; i < kThreads / 64; ++i) b += s_w[i];
        partial[blockIdx.x] = b;
    }
}

// f2 = coef * sumwt / sumlocwt, coef = (5 * 10^-robustness)^2 (gridding.py:415)
__global__ __launch_bounds__(64) void k_robust_f2(const double *__restrict__ sq_part, int nsq,
                                                  const double *__restrict__ wt_part, int nwt,
                                                  const double *__restrict__ sumwt, int n_sumwt,
                                                  double coef, double *f2) {
    double sq = 0.0, tot = 0.0;
    for (int i = threadIdx.x; i < nsq; i += 64) sq += sq_part[i];
    if (sumwt) {
        for (int i = threadIdx.x; i < n_sumwt; i += 64) tot += sumwt[i];
    } else {
        for (int i = threadIdx.x; i < nwt; i += 64) tot += wt_part[i];
    }
    sq = wave_sum(sq);
    tot = wave_sum(tot);
    if (threadIdx.x == 0) *f2 = coef * (sumwt ? tot : tot * 2) / sq;
}

// ---- griddata_visibility_reweight -----------------------------------------
// mode 0 natural (imaging_weight = weight), 1 uniform, 2 robust.  One
// element of the [nrow, nchan, npol] arrays per thread (coalesced); the
// gathered grid weights of a dense core stay in L2 / MALL.
template <int NP>
__global__ __launch_bounds__(kThreads) void k_reweight(Geom g, int mode, const double *__restrict__ uvw,
                                                       const double *__restrict__ freq,
                                                       const double *__restrict__ wt,
                                                       const void *__restrict__ flags,
                                                       const int32_t *__restrict__ vis_to_im,
                                                       const double *__restrict__ grid,
                                                       const double *__restrict__ f2p,
                                                       double *imw) {
    const int rowlen = g.nchan * NP;
    const int64_t n = g.nrow * rowlen;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    if (mode == 0) {
        for (int64_t e = blockIdx.x * (int64_t)kThreads + threadIdx.x; e < n; e += stride)
            imw[e] = wt[e];
        return;
    }
    const double f2 = mode == 2 ? *f2p : 0.0;
    const bool small = n < (int64_t(1) << 32);
    __shared__ double s_k[kMaxLdsK];
    const bool lds_k = g.nchan <= kMaxLdsK;
    if (lds_k)
        for (int i = threadIdx.x; i < g.nchan; i += kThreads) s_k[i] = freq[i] / kC;
    __syncthreads();
    for (int64_t e = blockIdx.x * (int64_t)kThreads + threadIdx.x; e < n; e += stride) {
        int64_t row;
        int rem;
        if (small) {
            const uint32_t eu = (uint32_t)e, r = eu / (uint32_t)rowlen;
            row = r;
            rem = (int)(eu - r * (uint32_t)rowlen);
        } else {
            row = e / rowlen;
            rem = (int)(e - row * rowlen);
        }
        const int ch = rem / NP, p = rem - (rem / NP) * NP;
        const Cell cell = map_cell(g, uvw[3 * row], uvw[3 * row + 1], lds_k ? s_k[ch] : freq[ch] / kC);
        double out = 0.0;
        if (in_grid(g, cell)) {
            const double gw =
                grid[(((size_t)vis_to_im[ch] * NP + p) * g.ny + cell.pv) * g.nx + cell.pu];
            if (gw > 0.0) {
                const double fw = flagged(wt, flags, g.flag_bytes, (size_t)e);
                out = mode == 1 ? fw / gw : fw / (1 + f2 * gw);
            } else if (!(gw <= 0.0)) {
                // NaN grid weight: the reference leaves flagged_imaging_weight
                out = flagged(imw, flags, g.flag_bytes, (size_t)e);
            }
        }
        imw[e] = out;
    }
}

// ---- tapers ---------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_max_radius(const double *__restrict__ uvw, int64_t nrow,
                                                         unsigned long long *rmax_bits) {
    double r = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < nrow;
         i += (int64_t)gridDim.x * kThreads) {
        const double u = uvw[3 * i], v = uvw[3 * i + 1];
        r = fmax(r, sqrt(u * u + v * v));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r = fmax(r, __shfl_xor(r, o, 64));
    // non-negative doubles order like their bit patterns
    if ((threadIdx.x & 63) == 0) atomicMax(rmax_bits, (unsigned long long)__double_as_longlong(r));
}

// kind 0: gaussian, param = scale_factor = pi^2 beam^2 / (4 ln 2)   (weighting.py:86-99)
// kind 1: tukey, param = r; radius / max radius per channel        (weighting.py:120-134)
__global__ __launch_bounds__(kThreads) void k_taper(int64_t nrow, int nchan, int npol, int kind,
                                                    double param, const double *__restrict__ uvw,
                                                    const double *__restrict__ freq,
                                                    const void *__restrict__ flags, int flag_bytes,
                                                    const unsigned long long *__restrict__ rmax_bits,
                                                    double *imw) {
    const int64_t t = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (t >= nrow * nchan) return;
    const int64_t row = t / nchan;
    const int ch = (int)(t - row * nchan);
    const double u = uvw[3 * row], v = uvw[3 * row + 1];
    const double wave = kC / freq[ch];
    double wt;
    if (kind == 0) {
        const double uvdistsq = (u * u + v * v) / (wave * wave);
        wt = exp(-param * uvdistsq);
    } else {
        const double rmax = __longlong_as_double((long long)*rmax_bits) / wave;
        const double x = (sqrt(u * u + v * v) / wave) / rmax;
        const double r = param;
        if (0.0 <= x && x < r / 2.0) wt = 0.5 * (1.0 + cos(2.0 * M_PI * (x - r / 2.0) / r));
        else if (1 - r / 2.0 <= x && x <= 1.0) wt = 0.5 * (1.0 + cos(2.0 * M_PI * (x - 1 + r / 2.0) / r));
        else wt = 1.0;
    }
    const size_t base = ((size_t)row * nchan + ch) * npol;
    for (int p = 0; p < npol; ++p) imw[base + p] = flagged(imw, flags, flag_bytes, base + p) * wt;
}

Geom make_geom(int64_t nrow, int nchan, int npol, int g_nchan, int ny, int nx, const double *wcs,
               int flag_bytes) {
    SDP_REQUIRE(nrow >= 0 && nchan > 0, "nrow must be >= 0 and nchan > 0");
    SDP_REQUIRE(npol == 1 || npol == 2 || npol == 4, "npol must be 1, 2 or 4");
    SDP_REQUIRE(g_nchan > 0 && ny > 0 && nx > 0, "grid dimensions must be positive");
    SDP_REQUIRE(flag_bytes == 0 || flag_bytes == 1 || flag_bytes == 4 || flag_bytes == 8,
                "flag element size must be 0, 1, 4 or 8 bytes");
    SDP_REQUIRE(wcs != nullptr && wcs[1] != 0.0 && wcs[4] != 0.0, "grid wcs cdelt must be non-zero");
    Geom g{nrow, nchan, npol, g_nchan, ny, nx, wcs[0], wcs[1], wcs[2], wcs[3], wcs[4], wcs[5],
           flag_bytes, wcs[0] == 0.0 && wcs[3] == 0.0, 0, 0, 0, 1024, 0, 0, 0};
    if (const char *e = std::getenv("SDP_HIP_WEIGHT_NT")) g.nt = std::atoi(e) == 256 ? 256 : 1024;
    if (g.zero_val && wcs[2] == std::floor(wcs[2]) && wcs[5] == std::floor(wcs[5]) &&
        std::fabs(wcs[2]) < 1e9 && std::fabs(wcs[5]) < 1e9 && !std::getenv("SDP_HIP_WEIGHT_NOMIRROR")) {
        g.mirror = 1;
        g.cu2 = 2 * ((long long)wcs[2] - 1);
        g.cv2 = 2 * ((long long)wcs[5] - 1);
    }
    return g;
}

// Central window: up to 32 KB of LDS per block over all (image channel, pol)
// planes, centred on the cell of u = v = 0 and clipped to the grid.
void choose_window(Geom &g) {
    const int planes = g.g_nchan * g.npol;
    int win = 128;
    size_t budget = g.nt == 1024 ? 131072 : 32768;
    if (const char *e = std::getenv("SDP_HIP_WEIGHT_WIN")) win = std::atoi(e);
    if (const char *e = std::getenv("SDP_HIP_WEIGHT_WIN_KB")) budget = (size_t)std::atoi(e) * 1024;
    while (win >= 8 && ((size_t)planes * win * win * 8 > budget || win > g.nx || win > g.ny)) win /= 2;
    if (win < 8) {
        g.win = 0;
        return;
    }
    auto centre = [](double val, double del, double pix) {
        return (long long)std::nearbyint((0.0 - val) / del + pix - 1.0);
    };
    long long u0 = centre(g.u_val, g.u_del, g.u_pix) - win / 2;
    long long v0 = centre(g.v_val, g.v_del, g.v_pix) - win / 2;
    u0 = std::max(0LL, std::min<long long>(u0, g.nx - win));
    v0 = std::max(0LL, std::min<long long>(v0, g.ny - win));
    g.win = win;
    g.win_u0 = (int)u0;
    g.win_v0 = (int)v0;
}

unsigned elem_blocks(const Geom &g) {
    const int64_t n = g.nrow * g.nchan * g.npol;
    return (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, 8192);
}

}  // namespace weighting
}  // namespace sdp

extern "C" {

int sdp_hip_grid_weights(int64_t nrow, int nchan, int npol, const double *uvw, const double *freq,
                         const double *weight, const void *flags, int flag_bytes,
                         const int32_t *vis_to_im, const double *grid_wcs, double *grid,
                         int g_nchan, int ny, int nx, double *sumwt, int64_t *nskipped,
                         void *stream, char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    using namespace sdp::weighting;
    return guarded(errbuf, errbuf_len, [&] {
        const Geom g = make_geom(nrow, nchan, npol, g_nchan, ny, nx, grid_wcs, flags ? flag_bytes : 0);
        if (nrow == 0) return;
        SDP_REQUIRE(uvw && freq && weight && vis_to_im && grid && sumwt && nskipped,
                    "null pointer argument");
        const hipStream_t st = as_stream(stream);
        auto *sk = reinterpret_cast<unsigned long long *>(nskipped);
        Geom gw = g;
        choose_window(gw);
        const int nspan = (nchan + kChan - 1) / kChan;
        int dev = 0, ncu = 0;
        SDP_HIP_CHECK(hipGetDevice(&dev));
        SDP_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        const int nplanes = g_nchan * npol;
        const int nwin = gw.win ? nplanes * gw.win * gw.win : 0;
        const size_t lds = (size_t)nwin * sizeof(double);
        int per_cu = 1;
        const bool big = gw.nt == 1024;
        const void *fn = big ? (npol == 1 ? (const void *)k_grid_weights<1, 1024>
                                : npol == 2 ? (const void *)k_grid_weights<2, 1024>
                                            : (const void *)k_grid_weights<4, 1024>)
                             : (npol == 1 ? (const void *)k_grid_weights<1, 256>
                                : npol == 2 ? (const void *)k_grid_weights<2, 256>
                                            : (const void *)k_grid_weights<4, 256>);
        SDP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, gw.nt, lds));
        const int64_t ntiles = (nrow * nspan + gw.nt - 1) / gw.nt;
        const unsigned nb = (unsigned)std::min<int64_t>(ntiles, (int64_t)std::max(per_cu, 1) * ncu);
        double *partial = nwin ? scratch<double>("weight_window", (size_t)nb * nwin) : nullptr;
        const int64_t ncell = (int64_t)nplanes * ny * nx;
        double *g1 = grid;
        if (gw.mirror) {
            g1 = scratch<double>("weight_direct", (size_t)ncell);
            SDP_HIP_CHECK(hipMemsetAsync(g1, 0, (size_t)ncell * sizeof(double), st));
        }
#define SDP_GW_LAUNCH(NPV, NTV) \
    k_grid_weights<NPV, NTV><<<nb, NTV, lds, st>>>(gw, ntiles, uvw, freq, weight, flags, vis_to_im, grid, g1, sumwt, partial, sk)
        if (big) {
            if (npol == 1) SDP_GW_LAUNCH(1, 1024);
            else if (npol == 2) SDP_GW_LAUNCH(2, 1024);
            else SDP_GW_LAUNCH(4, 1024);
        } else {
            if (npol == 1) SDP_GW_LAUNCH(1, 256);
            else if (npol == 2) SDP_GW_LAUNCH(2, 256);
            else SDP_GW_LAUNCH(4, 256);
        }
#undef SDP_GW_LAUNCH
        SDP_HIP_CHECK(hipGetLastError());
        if (nwin)
            k_window_flush<<<(nwin + 15) / 16, kThreads, 0, st>>>(gw, nplanes, (int)nb, partial, g1);
        if (gw.mirror)
            k_mirror_fold<<<(unsigned)std::min<int64_t>((ncell + kThreads - 1) / kThreads, 16384), kThreads, 0, st>>>(gw, ncell, g1, grid);
        SDP_HIP_CHECK(hipGetLastError());
    });
}

int sdp_hip_reweight(int64_t nrow, int nchan, int npol, const double *uvw, const double *freq,
                     const double *weight, const void *flags, int flag_bytes,
                     const int32_t *vis_to_im, const double *grid_wcs, const double *grid,
                     int g_nchan, int ny, int nx, int weighting, double robust_coef,
                     const double *sumwt, int n_sumwt, double *imaging_weight, void *stream,
                     char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    using namespace sdp::weighting;
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(weighting >= 0 && weighting <= 2, "weighting must be 0 natural, 1 uniform, 2 robust");
        const Geom g = make_geom(nrow, nchan, npol, g_nchan, ny, nx, grid_wcs, flags ? flag_bytes : 0);
        if (nrow == 0) return;
        SDP_REQUIRE(weight && imaging_weight, "null pointer argument");
        SDP_REQUIRE(weighting == 0 || (uvw && freq && vis_to_im && grid), "null pointer argument");
        const hipStream_t st = as_stream(stream);
        double *f2 = nullptr;
        if (weighting == 2) {
            constexpr int kRed = 1024;
            double *part = scratch<double>("weight_reduce", 2 * kRed + 1);
            const size_t ngrid = (size_t)g_nchan * npol * ny * nx;
            const size_t nw = (size_t)nrow * nchan * npol;
            k_reduce<<<kRed, kThreads, 0, st>>>(grid, nullptr, 0, ngrid, 0, part);
            if (!sumwt)
                k_reduce<<<kRed, kThreads, 0, st>>>(weight, flags, g.flag_bytes, nw, 1, part + kRed);
            f2 = part + 2 * kRed;
            k_robust_f2<<<1, 64, 0, st>>>(part, kRed, part + kRed, kRed, sumwt, n_sumwt, robust_coef, f2);
            SDP_HIP_CHECK(hipGetLastError());
        }
        const unsigned nb = elem_blocks(g);
        if (npol == 1)
            k_reweight<1><<<nb, kThreads, 0, st>>>(g, weighting, uvw, freq, weight, flags, vis_to_im, grid, f2, imaging_weight);
        else if (npol == 2)
            k_reweight<2><<<nb, kThreads, 0, st>>>(g, weighting, uvw, freq, weight, flags, vis_to_im, grid, f2, imaging_weight);
        else
            k_reweight<4><<<nb, kThreads, 0, st>>>(g, weighting, uvw, freq, weight, flags, vis_to_im, grid, f2, imaging_weight);
        SDP_HIP_CHECK(hipGetLastError());
    });
}

int sdp_hip_taper(int64_t nrow, int nchan, int npol, const double *uvw, const double *freq,
                  const void *flags, int flag_bytes, int kind, double param,
                  double *imaging_weight, void *stream, char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    using namespace sdp::weighting;
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(kind == 0 || kind == 1, "taper kind must be 0 gaussian or 1 tukey");
        SDP_REQUIRE(nrow >= 0 && nchan > 0 && npol > 0, "bad dimensions");
        SDP_REQUIRE(flag_bytes == 0 || flag_bytes == 1 || flag_bytes == 4 || flag_bytes == 8,
                    "flag element size must be 0, 1, 4 or 8 bytes");
        if (nrow == 0) return;
        SDP_REQUIRE(uvw && freq && imaging_weight, "null pointer argument");
        const hipStream_t st = as_stream(stream);
        unsigned long long *rmax = nullptr;
        if (kind == 1) {
            rmax = scratch<unsigned long long>("taper_rmax", 1);
            SDP_HIP_CHECK(hipMemsetAsync(rmax, 0, sizeof(*rmax), st));
            const unsigned nb = (unsigned)std::min<int64_t>(1024, (nrow + kThreads - 1) / kThreads);
            k_max_radius<<<nb, kThreads, 0, st>>>(uvw, nrow, rmax);
        }
        const int64_t n = nrow * nchan;
        k_taper<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, st>>>(
            nrow, nchan, npol, kind, param, uvw, freq, flags ? flags : nullptr,
            flags ? flag_bytes : 0, rmax, imaging_weight);
        SDP_HIP_CHECK(hipGetLastError());
    });
}

}  // extern "C"
