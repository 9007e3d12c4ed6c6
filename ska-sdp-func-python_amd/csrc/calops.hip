// Calibration neighbours of StefCal for gfx950:
//   sdp_hip_point_sums   divide_visibility (src/ska_sdp_func_python/visibility/
//                        operations.py:145-189) fused with solve_gaintable's
//                        per-gain-row sums x_b, xwt_b (calibration/solvers.py:82-107),
//                        written in StefCal's canonical baseline order
//   sdp_hip_divide_vis   divide_visibility alone
//   sdp_hip_apply_gains  apply_gaintable (calibration/operations.py:23-256)
//
// All visibility-shaped arrays are the Visibility's [ntimes, nbl, nchan, npol]
// in C order.  Arithmetic follows the reference's fp64 operations: complex
// division is numpy's (Smith's algorithm, the same branches), products and
// sums in the reference's order where it is fixed; fp contraction is off.
// HBM-bound streaming kernels: one thread per output element, reads
// coalesced along (baseline, channel, pol).
#include "sdp_common.h"

#pragma clang fp contract(off)

namespace sdp {
namespace calops {

constexpr int kThreads = 256;

struct cplx {
    double re, im;
};

__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cplx cconj(cplx a) { return {a.re, -a.im}; }
__device__ __forceinline__ bool cnonzero(cplx a) { return a.re != 0.0 || a.im != 0.0; }

// numpy's complex division (umath loops: Smith's algorithm)
__device__ __forceinline__ cplx cdiv(cplx a, cplx b) {
    const double abr = fabs(b.re), abi = fabs(b.im);
    if (abr >= abi) {
        if (abr == 0.0 && abi == 0.0) return {a.re / abr, a.im / abr};
        const double rat = b.im / b.re;
        const double scl = 1.0 / (b.re + b.im * rat);
        return {(a.re + a.im * rat) * scl, (a.im - a.re * rat) * scl};
    }
    const double rat = b.re / b.im;
    const double scl = 1.0 / (b.im + b.re * rat);
    return {(a.re * rat + a.im) * scl, (a.im * rat - a.re) * scl};
}

__device__ __forceinline__ cplx load_c(const void *p, int c128, size_t i) {
    if (c128) {
        const double2 v = static_cast<const double2 *>(p)[i];
        return {v.x, v.y};
    }
    const float2 v = static_cast<const float2 *>(p)[i];
    return {(double)v.x, (double)v.y};
}

__device__ __forceinline__ void store_c(void *p, int c128, size_t i, cplx v) {
    if (c128) static_cast<double2 *>(p)[i] = make_double2(v.re, v.im);
    else static_cast<float2 *>(p)[i] = make_float2((float)v.re, (float)v.im);
}

__device__ __forceinline__ double keep_of(const void *flags, int bytes, size_t i) {
    if (!bytes) return 1.0;
    double f;
    if (bytes == 8) f = (double)static_cast<const int64_t *>(flags)[i];
    else if (bytes == 4) f = (double)static_cast<const int32_t *>(flags)[i];
    else f = (double)static_cast<const int8_t *>(flags)[i];
    return 1.0 - f;
}

// divide_visibility for one sample: x = fv / fm where xwt = |fm|^2 fw > 0;
// the model is masked with its own flags (modelvis.visibility_acc.flagged_vis)
__device__ __forceinline__ void point_sample(cplx v, cplx m, double w, double keep,
                                             double mkeep, cplx &x, double &xwt) {
    const cplx fv = {v.re * keep, v.im * keep};
    const cplx fm = {m.re * mkeep, m.im * mkeep};
    const double fw = w * keep;
    const double am = hypot(fm.re, fm.im);
    xwt = am * am * fw;
    x = xwt > 0.0 ? cdiv(fv, fm) : cplx{0.0, 0.0};
}

struct Shape {
    int64_t ntimes;
    int nbl, nchan, npol;
};

// x_b[r, j, fg, p] = sum over the row's times (and all channels when
// nchan_g == 1) of (x * xwt) * (1 - flag); xwt_b likewise of xwt * (1 - flag)
// (solvers.py:99-107); source baseline perm[j], conjugated where conj[j].
__global__ __launch_bounds__(kThreads) void k_point_sums(
    Shape s, const void *__restrict__ vis, const void *__restrict__ model, int c128,
    const double *__restrict__ weight, const void *__restrict__ flags,
    const void *__restrict__ mflags, int fbytes, int nrow_g, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ time_idx, int nchan_g,
    int nbl_out, const int32_t *__restrict__ perm, const uint8_t *__restrict__ conj, double2 *xb,
    double *xwtb) {
    const int64_t n = (int64_t)nrow_g * nbl_out * nchan_g * s.npol;
    const int64_t o = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (o >= n) return;
    const int p = (int)(o % s.npol);
    int64_t q = o / s.npol;
    const int fg = (int)(q % nchan_g);
    q /= nchan_g;
    const int j = (int)(q % nbl_out);
    const int r = (int)(q / nbl_out);
    const int b = perm ? perm[j] : j;
    const int f0 = nchan_g == 1 ? 0 : fg, f1 = nchan_g == 1 ? s.nchan : fg + 1;
    cplx acc = {0.0, 0.0};
    double accw = 0.0;
    for (int k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
        const int64_t t = time_idx[k];
        for (int f = f0; f < f1; ++f) {
            const size_t i = (((size_t)t * s.nbl + b) * s.nchan + f) * s.npol + p;
            const double keep = keep_of(flags, fbytes, i);
            const cplx v = load_c(vis, c128, i);
            const double w = weight ? weight[i] : 1.0;
            cplx x;
            double xwt;
            if (model) {
                point_sample(v, load_c(model, c128, i), w, keep,
                             mflags ? keep_of(mflags, fbytes, i) : keep, x, xwt);
            } else {
                x = v;
                xwt = w;
            }
            acc = cadd(acc, {x.re * xwt * keep, x.im * xwt * keep});
            accw += xwt * keep;
        }
    }
    if (conj && conj[j]) acc = cconj(acc);
    xb[o] = make_double2(acc.re, acc.im);
    xwtb[o] = accw;
}

__global__ __launch_bounds__(kThreads) void k_divide(int64_t n, const void *__restrict__ vis,
                                                     const void *__restrict__ model, int c128,
                                                     const double *__restrict__ weight,
                                                     const void *__restrict__ flags,
                                                     const void *__restrict__ mflags, int fbytes,
                                                     void *x_out, double *xwt_out) {
    for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads) {
        cplx x;
        double xwt;
        const double keep = keep_of(flags, fbytes, i);
        point_sample(load_c(vis, c128, i), load_c(model, c128, i), weight ? weight[i] : 1.0, keep,
                     mflags ? keep_of(mflags, fbytes, i) : keep, x, xwt);
        store_c(x_out, c128, i, x);
        xwt_out[i] = xwt;
    }
}

// ---- apply_gaintable ------------------------------------------------------
// Effective gains per (gain row, antenna, gain channel): the gain itself, or
// for inverse=True 1/g (|g| > 0, else 0) in the scalar case and the 2x2
// inverse otherwise, ok = 0 where numpy.linalg.inv raises (LAPACK's LU with
// partial pivoting meets an exactly zero pivot).
__global__ void k_gain_prep(int64_t n, int nrec, int inverse, const double2 *__restrict__ gain,
                            double2 *lg, uint8_t *ok) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int m = nrec * nrec;
    const double2 *g = gain + i * m;
    double2 *o = lg + i * m;
    if (!inverse) {
        for (int k = 0; k < m; ++k) o[k] = g[k];
        ok[i] = 1;
        return;
    }
    if (nrec == 1) {
        const cplx a = {g[0].x, g[0].y};
        const cplx inv = hypot(a.re, a.im) > 0.0 ? cdiv({1.0, 0.0}, a) : cplx{0.0, 0.0};
        o[0] = make_double2(inv.re, inv.im);
        ok[i] = 1;
        return;
    }
    // 2x2: rows swapped when |c|_1 > |a|_1 (izamax), l = r * (1/p), u22 = s - l q
    cplx a = {g[0].x, g[0].y}, b = {g[1].x, g[1].y}, c = {g[2].x, g[2].y}, d = {g[3].x, g[3].y};
    const bool swap = (fabs(c.re) + fabs(c.im)) > (fabs(a.re) + fabs(a.im));
    const cplx p = swap ? c : a, qv = swap ? d : b, r = swap ? a : c, sv = swap ? b : d;
    if (!cnonzero(p)) {
        ok[i] = 0;
        for (int k = 0; k < 4; ++k) o[k] = g[k];
        return;
    }
    const cplx l = cmul(r, cdiv({1.0, 0.0}, p));
    const cplx lq = cmul(l, qv);
    const cplx u22 = {sv.re - lq.re, sv.im - lq.im};
    if (!cnonzero(u22)) {
        ok[i] = 0;
        for (int k = 0; k < 4; ++k) o[k] = g[k];
        return;
    }
    // solve A X = I: with P A = L U, X = U^-1 L^-1 P
    // columns of P: e_swap -> rows of identity permuted
    cplx x[2][2];
    for (int col = 0; col < 2; ++col) {
        // rhs = P e_col
        cplx y0 = {0.0, 0.0}, y1 = {0.0, 0.0};
        const int row0 = swap ? 1 : 0;  // which original row sits first
        if (col == row0) y0 = {1.0, 0.0};
        else y1 = {1.0, 0.0};
        // L y = rhs (unit lower): y1 -= l y0
        const cplx ly0 = cmul(l, y0);
        y1 = {y1.re - ly0.re, y1.im - ly0.im};
        // U x = y: x1 = y1 / u22; x0 = (y0 - q x1) / p
        const cplx x1 = cdiv(y1, u22);
        const cplx qx1 = cmul(qv, x1);
        const cplx x0 = cdiv({y0.re - qx1.re, y0.im - qx1.im}, p);
        x[0][col] = x0;
        x[1][col] = x1;
    }
    o[0] = make_double2(x[0][0].re, x[0][0].im);
    o[1] = make_double2(x[0][1].re, x[0][1].im);
    o[2] = make_double2(x[1][0].re, x[1][0].im);
    o[3] = make_double2(x[1][1].re, x[1][1].im);
    ok[i] = 1;
}

// use_flags: a gain row takes the flagged vis / weights of its whole window
// when any flag there is set (operations.py:74-86)
__global__ __launch_bounds__(kThreads) void k_row_flagged(Shape s, const void *__restrict__ flags,
                                                          int fbytes,
                                                          const int32_t *__restrict__ time_row,
                                                          uint8_t *row_flag) {
    const int64_t n = s.ntimes * s.nbl * s.nchan * s.npol;
    for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads) {
        const int r = time_row[i / ((int64_t)s.nbl * s.nchan * s.npol)];
        if (r >= 0 && keep_of(flags, fbytes, (size_t)i) != 1.0 && !row_flag[r]) row_flag[r] = 1;
    }
}

__global__ __launch_bounds__(kThreads) void k_apply(Shape s, void *vis, int c128, double *weight,
                                                    const void *__restrict__ flags, int fbytes,
                                                    const int32_t *__restrict__ ant1,
                                                    const int32_t *__restrict__ ant2,
                                                    const int32_t *__restrict__ time_row,
                                                    const uint8_t *__restrict__ row_flag,
                                                    const double2 *__restrict__ lg,
                                                    const uint8_t *__restrict__ ok, int nants,
                                                    int nchan_g, int nrec, int inverse) {
    const int64_t n = s.ntimes * s.nbl * s.nchan;
    const int64_t e = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (e >= n) return;
    const int f = (int)(e % s.nchan);
    const int64_t tb = e / s.nchan;
    const int b = (int)(tb % s.nbl);
    const int64_t t = tb / s.nbl;
    const int r = time_row[t];
    if (r < 0) return;
    const size_t base = (size_t)e * s.npol;
    const bool use_fl = row_flag && row_flag[r];
    cplx v[4];
    double w[4];
    for (int p = 0; p < s.npol; ++p) {
        v[p] = load_c(vis, c128, base + p);
        w[p] = weight[base + p];
        if (use_fl) {
            const double k = keep_of(flags, fbytes, base + p);
            v[p] = {v[p].re * k, v[p].im * k};
            w[p] *= k;
        }
    }
    if (f < nchan_g) {
        const int m = nrec * nrec;
        const int64_t g1i = ((int64_t)r * nants + ant1[b]) * nchan_g + f;
        const int64_t g2i = ((int64_t)r * nants + ant2[b]) * nchan_g + f;
        const double2 *G1 = lg + g1i * m;
        const double2 *G2 = lg + g2i * m;
        if (s.npol == 1) {
            // smueller = sum_{l,m} g1[l,m] conj(g2[l,m])  (einsum ijlm,kjlm->jik)
            cplx sm = {0.0, 0.0};
            for (int k = 0; k < m; ++k)
                sm = cadd(sm, cmul({G1[k].x, G1[k].y}, cconj({G2[k].x, G2[k].y})));
            if (hypot(sm.re, sm.im) > 0.0) {
                v[0] = cmul(v[0], sm);
            } else {
                v[0] = {0.0, 0.0};
                w[0] = 0.0;
            }
        } else {
            const bool good = !inverse || (ok[g1i] && ok[g2i]);
            const cplx g1[2][2] = {{{G1[0].x, G1[0].y}, {G1[1].x, G1[1].y}},
                                   {{G1[2].x, G1[2].y}, {G1[3].x, G1[3].y}}};
            const cplx c2[2][2] = {{cconj({G2[0].x, G2[0].y}), cconj({G2[1].x, G2[1].y})},
                                   {cconj({G2[2].x, G2[2].y}), cconj({G2[3].x, G2[3].y})}};
            if (!good) {
                if (s.npol == 2) {
                    v[0] = {0.0, 0.0};
                    w[0] = 0.0;
                } else {
                    for (int p = 0; p < 4; ++p) {
                        v[p] = {0.0, 0.0};
                        w[p] = 0.0;
                    }
                }
            } else {
                cplx V[2][2];
                if (s.npol == 2) {
                    V[0][0] = v[0];
                    V[0][1] = {0.0, 0.0};
                    V[1][0] = {0.0, 0.0};
                    V[1][1] = v[1];
                } else {
                    V[0][0] = v[0];
                    V[0][1] = v[1];
                    V[1][0] = v[2];
                    V[1][1] = v[3];
                }
                // (G1 @ V) @ conj(G2), numpy's evaluation order
                cplx T[2][2], R[2][2];
                for (int i2 = 0; i2 < 2; ++i2)
                    for (int k2 = 0; k2 < 2; ++k2)
                        T[i2][k2] = cadd(cmul(g1[i2][0], V[0][k2]), cmul(g1[i2][1], V[1][k2]));
                for (int i2 = 0; i2 < 2; ++i2)
                    for (int k2 = 0; k2 < 2; ++k2)
                        R[i2][k2] = cadd(cmul(T[i2][0], c2[0][k2]), cmul(T[i2][1], c2[1][k2]));
                if (s.npol == 2) {
                    v[0] = R[0][0];
                    v[1] = R[1][1];
                } else {
                    v[0] = R[0][0];
                    v[1] = R[0][1];
                    v[2] = R[1][0];
                    v[3] = R[1][1];
                }
            }
        }
    }
    for (int p = 0; p < s.npol; ++p) {
        store_c(vis, c128, base + p, v[p]);
        weight[base + p] = w[p];
    }
}

Shape make_shape(int64_t ntimes, int nbl, int nchan, int npol) {
    SDP_REQUIRE(ntimes >= 0 && nbl >= 0 && nchan > 0, "bad visibility dimensions");
    SDP_REQUIRE(npol == 1 || npol == 2 || npol == 4, "npol must be 1, 2 or 4");
    return Shape{ntimes, nbl, nchan, npol};
}

void check_common(int vis_dtype, const void *flags, int flag_bytes) {
    SDP_REQUIRE(vis_dtype == SDP_HIP_C64 || vis_dtype == SDP_HIP_C128,
                "visibilities must be complex64 or complex128");
    SDP_REQUIRE(!flags || flag_bytes == 1 || flag_bytes == 4 || flag_bytes == 8,
                "flag element size must be 1, 4 or 8 bytes");
}

}  // namespace calops
}  // namespace sdp

extern "C" {

int sdp_hip_point_sums(int64_t ntimes, int nbl, int nchan, int npol, const void *vis,
                       const void *model, int vis_dtype, const double *weight, const void *flags,
                       const void *model_flags, int flag_bytes, int nrow_g, const int32_t *row_ptr,
                       const int32_t *time_idx, int nchan_g, int nbl_out,
                       const int32_t *bl_perm, const uint8_t *bl_conj, void *xb, double *xwt,
                       void *stream, char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    using namespace sdp::calops;
    return guarded(errbuf, errbuf_len, [&] {
        const Shape s = make_shape(ntimes, nbl, nchan, npol);
        check_common(vis_dtype, flags, flag_bytes);
        SDP_REQUIRE(nchan_g == 1 || nchan_g == nchan, "gain channels must be 1 or nchan");
        SDP_REQUIRE(nrow_g >= 0, "nrow_g must be >= 0");
        SDP_REQUIRE(bl_perm ? nbl_out >= 0 : nbl_out == nbl,
                    "nbl_out must equal nbl without a baseline permutation");
        const int64_t n = (int64_t)nrow_g * nbl_out * nchan_g * npol;
        if (n == 0) return;
        SDP_REQUIRE(vis && row_ptr && time_idx && xb && xwt, "null pointer argument");
        k_point_sums<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, as_stream(stream)>>>(
            s, vis, model, vis_dtype == SDP_HIP_C128, weight, flags, flags ? model_flags : nullptr,
            flags ? flag_bytes : 0, nrow_g, row_ptr, time_idx, nchan_g, nbl_out, bl_perm, bl_conj,
            static_cast<double2 *>(xb), xwt);
        SDP_HIP_CHECK(hipGetLastError());
    });
}

int sdp_hip_divide_vis(int64_t n, const void *vis, const void *model, int vis_dtype,
                       const double *weight, const void *flags, const void *model_flags,
                       int flag_bytes, void *x_out, double *xwt_out, void *stream, char *errbuf,
                       size_t errbuf_len) {
    using namespace sdp;
    using namespace sdp::calops;
    return guarded(errbuf, errbuf_len, [&] {
        check_common(vis_dtype, flags, flag_bytes);
        SDP_REQUIRE(n >= 0, "n must be >= 0");
        if (n == 0) return;
        SDP_REQUIRE(vis && model && x_out && xwt_out, "null pointer argument");
        const unsigned nb = (unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, 16384);
        k_divide<<<nb, kThreads, 0, as_stream(stream)>>>(n, vis, model, vis_dtype == SDP_HIP_C128,
                                                         weight, flags,
                                                         flags ? model_flags : nullptr,
                                                         flags ? flag_bytes : 0, x_out, xwt_out);
        SDP_HIP_CHECK(hipGetLastError());
    });
}

int sdp_hip_apply_gains(int64_t ntimes, int nbl, int nchan, int npol, void *vis, int vis_dtype,
                        double *weight, const void *flags, int flag_bytes, int use_flags,
                        const int32_t *ant1, const int32_t *ant2, const int32_t *time_row,
                        const void *gain, int nrow_g, int nants, int nchan_g, int nrec,
                        int inverse, void *stream, char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    using namespace sdp::calops;
    return guarded(errbuf, errbuf_len, [&] {
        const Shape s = make_shape(ntimes, nbl, nchan, npol);
        check_common(vis_dtype, flags, flag_bytes);
        SDP_REQUIRE(nrec == 1 || nrec == 2, "nrec must be 1 or 2");
        SDP_REQUIRE(npol == 1 || nrec == 2, "npol 2 and 4 need 2x2 gains");
        SDP_REQUIRE(nrow_g >= 0 && nants > 0 && nchan_g > 0, "bad gain table dimensions");
        SDP_REQUIRE(!use_flags || flags, "use_flags needs the flags");
        const int64_t n = ntimes * nbl * (int64_t)nchan;
        if (n == 0 || nrow_g == 0) return;
        SDP_REQUIRE(vis && weight && ant1 && ant2 && time_row && gain, "null pointer argument");
        const hipStream_t st = as_stream(stream);
        const int64_t ng = (int64_t)nrow_g * nants * nchan_g;
        double2 *lg = scratch<double2>("apply_lgain", (size_t)ng * nrec * nrec);
        uint8_t *ok = scratch<uint8_t>("apply_ok", (size_t)ng);
        k_gain_prep<<<(unsigned)((ng + 127) / 128), 128, 0, st>>>(
            ng, nrec, inverse, static_cast<const double2 *>(gain), lg, ok);
        uint8_t *row_flag = nullptr;
        if (use_flags) {
            row_flag = scratch<uint8_t>("apply_row_flag", (size_t)nrow_g);
            SDP_HIP_CHECK(hipMemsetAsync(row_flag, 0, (size_t)nrow_g, st));
            const int64_t nf = n * npol;
            k_row_flagged<<<(unsigned)std::min<int64_t>((nf + kThreads - 1) / kThreads, 16384),
                            kThreads, 0, st>>>(s, flags, flag_bytes, time_row, row_flag);
        }
        k_apply<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, st>>>(
            s, vis, vis_dtype == SDP_HIP_C128, weight, flags, flags ? flag_bytes : 0, ant1, ant2,
            time_row, row_flag, lg, ok, nants, nchan_g, nrec, inverse);
        SDP_HIP_CHECK(hipGetLastError());
    });
}

}  // extern "C"
