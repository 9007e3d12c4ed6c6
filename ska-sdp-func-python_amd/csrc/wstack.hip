// w-stacking / w-gridding NUFFT pair for gfx950 (MI355X): sdp_hip_ms2dirty
// and sdp_hip_dirty2ms, the drop-in for ducc0.wgridder.ms2dirty/dirty2ms as
// called by the reference's invert_ng / predict_ng
// (src/ska_sdp_func_python/imaging/ng.py:99-129, :240-289).
//
// Pipeline (one stream, two host syncs per call):
//   k_bounds       fp64 w range / uv extent over the rows
//   k_bucket<0>    per-visibility fp64 grid coordinates -> bucket key
//                  (first w plane p0, 2x2 or 16x16 uv cells) and rank in the
//                  bucket from a wave-level run-length histogram (one atomic
//                  per run of equal keys)
//   scan           hipcub exclusive sum over buckets
//   k_bucket<1>    32-byte visibility records at offs[key] + rank (no atomics)
//   k_items_*      work items = one bucket, split into <= chunk records
//   per plane chunk (all planes resident when they fit the budget):
//     k_grid       one workgroup per item owning an LDS tile of W planes
//                  x (16+W-1)^2 complex cells, planes split over its waves;
//                  per record one lane per (u,v) tap does a plain
//                  ds_read_b64/ds_write_b64 update of the wave's planes; the
//                  tile is flushed with global float atomics
//     hipFFT       batched in-place c2c over the planes
//     k_screen_fwd w-screen phase, real part, fp64 accumulate, grid correction
//   dirty2ms runs the stages in adjoint order (k_screen_adj, FFT, k_degrid).
//
// Numerics: coordinates, plane positions and phases in fp64; kernel taps and
// grid values in fp32; image accumulation and corrections in fp64.  ES kernel
// exp(beta (sqrt(1 - x^2) - 1)), beta = 2.30 W, oversampling 2 (FINUFFT
// parameter rule); the grid correction is its Fourier transform (128-point
// Gauss-Legendre quadrature on host), tabulated and interpolated on device.
#include <hipcub/hipcub.hpp>
#include <hipfft/hipfft.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <tuple>
#include <type_traits>
#include <vector>

#include "sdp_common.h"

namespace sdp {
namespace wstack {

constexpr double kCLight = 299792458.0;
constexpr int kTileCoarse = 16;  // bucket edge (cells) of the LDS-tile gridder
constexpr int kTileFine = 2;     // bucket edge (cells) of the register gridder
constexpr int kGroupFine = 4;    // fine buckets per work-item group (along y)
// invert on MFMA (k_grid_mfma): one-cell buckets ordered x-pair major
// (key tile = ((ic >> 1) * ngy + jc) * 2 + (ic & 1)), so a bucket's records
// share their footprint origin and 16 consecutive buckets form the same
// 2 x 8-cell work-item region as kGroupFine 2x2-cell buckets
constexpr int kTileCell = 1;
constexpr int kGroupCell = 16;
constexpr int64_t kMaxCellKeys = (int64_t)1 << 28;
constexpr int kGridAlign = 16;   // padded grid edges are multiples of this
// fine buckets are used while the dense (p0, 2x2-cell) histogram stays small
constexpr int64_t kMaxFineKeys = (int64_t)1 << 27;
constexpr int kChunkMin = 1024;   // records per work item: chosen per call in
constexpr int kChunkMax = 8192;   // [kChunkMin, kChunkMax] (chunk_size())
constexpr int kPitch = 24;     // LDS row pitch in complex values (b64 conflict-free)
constexpr int kMaxW = 8;
constexpr int kPhiTab = 8193;  // Phi(xi) table on xi in [0, 0.5]
constexpr int kFftBatchMax = 16;                      // planes per FFT batch
constexpr size_t kFftBatchBytes = (size_t)16 << 30;  // y-spectra buffers per batch

struct Geo {
    int W;
    float beta, inv_half_w, beta_l2e;
    int nx, ny, ngx, ngy;
    double px, py;
    int do_w, nplanes, nps;  // nps = number of distinct first planes
    double w0, dw, s0;
    int sub, nty, ntiles;  // bucket edge in cells, buckets per window column, buckets
    // bucket window: the footprint origins of all visibilities lie in cells
    // [wx0, wx0 + wnx) x [wy0, wy0 + wny) (16-aligned), so only the window's
    // buckets are histogrammed, scanned and itemised
    int wx0, wy0, wnx, wny;
    int grp;               // consecutive buckets (along y) per work-item group
    // keys per bucket (16x16-cell buckets: a power of 2 > 1): the count pass
    // spreads a bucket's histogram counter over `salt` adjacent counters by
    // row, so the uv core's hot buckets take several memory-side atomic
    // streams; the sub-buckets are adjacent, so the bucket stays contiguous
    int salt;
    int dbg;               // experiment knobs (SDP_HIP_DBG)
    double su;  // sign applied to u and w (-1 with SDP_HIP_FLIP_UW)
    int nchan;
    int64_t nrow;
};

struct __attribute__((aligned(32))) VisRec {
    float cre, cim;    // gridding: vis*wgt*exp(2 pi i w s0); degridding: wgt*exp(-2 pi i w s0)
    float fu, fv, fw;  // offset of the first tap from the exact position (cells/planes)
    uint32_t ij;       // footprint start in the centred grid: ic0 | jc0 << 16
    uint32_t p0;       // first w plane
    uint32_t idx;      // row * nchan + chan
};
static_assert(sizeof(VisRec) == 32, "record layout");

// 16-byte record of the 4-padded invert (k_grid_mfma_pad): the value and the
// footprint offsets as fixed-point fractions, e = (1 - W/2) - f in [0, 1):
// u in lo[0:21), v in lo[21:32) | hi[0:10), w in hi[10:32) (steps of 2^-21,
// 2^-21, 2^-22 cells / planes, i.e. rounding errors <= 2.4e-7 / 1.2e-7 --
// fp32 offsets near 3.5 round to 1.2e-7).  The cell and the first plane are
// those of the record's bucket, so the record does not carry them.
struct __attribute__((aligned(16))) RecC {
    float cre, cim;
    uint32_t lo, hi;
};
static_assert(sizeof(RecC) == 16, "record layout");

__device__ __forceinline__ uint32_t fix_frac(double e, int bits) {
    const double q = floor(e * (double)(1u << bits) + 0.5);
    return (uint32_t)fmin(fmax(q, 0.0), (double)((1u << bits) - 1u));
}

struct Item {
    uint32_t b, e, tile, p0;
};

// Large grids (16x16-cell buckets): work item of one group of 4 2x2-cell
// buckets (a 2 x 8-cell region) inside a sub-sorted coarse item; records
// [b, e) ordered by bucket, bucket j of the group ending at o[j] (k_subsort)
struct FineItem {
    uint32_t b, e, tile, p0;
    uint32_t o[16];  // end of bucket j of the group (2x2 buckets: j < 4; cells: j < 16)
};

// ------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------
static int env_int(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}

__device__ __forceinline__ unsigned long long ord_enc(double d) {
    long long i = __double_as_longlong(d);
    return i < 0 ? ~(unsigned long long)i : ((unsigned long long)i | 0x8000000000000000ull);
}

// ES kernel exp(beta (sqrt(1 - x^2) - 1)), x = 2t/W; `beta_l2e` = beta*log2(e)
// so the raw v_exp_f32 (2^x) and v_sqrt_f32 are used directly.
__device__ __forceinline__ float es_kernel(float t, float inv_half_w, float beta_l2e) {
    const float x = t * inv_half_w;
    const float y = 1.0f - x * x;
    const float e =
        __builtin_amdgcn_exp2f(beta_l2e * (__builtin_amdgcn_sqrtf(fmaxf(y, 0.0f)) - 1.0f));
    return y > 0.0f ? e : 0.0f;
}

// 4-point Lagrange interpolation of the tabulated Phi on [0, 0.5].
__device__ __forceinline__ double phi_lookup(const double *__restrict__ tab, double xi) {
    xi = fabs(xi);
    const double t = xi * (2.0 * (kPhiTab - 1));
    int k = (int)t;
    k = min(max(k, 1), kPhiTab - 3);
    const double f = t - k;
    const double p0 = tab[k - 1], p1 = tab[k], p2 = tab[k + 1], p3 = tab[k + 2];
    const double fm1 = f + 1.0, f1 = f - 1.0, f2 = f - 2.0;
    return -p0 * f * f1 * f2 / 6.0 + p1 * fm1 * f1 * f2 / 2.0 - p2 * fm1 * f * f2 / 2.0 +
           p3 * fm1 * f * f1 / 6.0;
}

struct Coord {
    int ic0, jc0, p0;
    float fu, fv, fw;
    double du, dv, dw;  // the same offsets in fp64 (RecC encoding)
    double w;  // w in wavelengths (sign applied)
    bool ok;
};

__device__ __forceinline__ Coord vis_coord(const Geo &g, const double *__restrict__ uvw,
                                           int64_t rs, int64_t row, double f) {
    Coord c;
    const double s = f / kCLight;
    const double u = g.su * uvw[row * rs] * s;
    const double v = uvw[row * rs + 1] * s;
    c.w = g.su * uvw[row * rs + 2] * s;
    const double a = u * g.px * g.ngx;
    const double b = v * g.py * g.ngy;
    c.ok = fabs(a) < (double)g.ngx && fabs(b) < (double)g.ngy;
    if (!c.ok) return c;
    const double fa = floor(a - 0.5 * g.W), fb = floor(b - 0.5 * g.W);
    c.du = fa + 1.0 - a;
    c.dv = fb + 1.0 - b;
    c.fu = (float)c.du;
    c.fv = (float)c.dv;
    const int ic = ((int)fa + 1 + g.ngx / 2) % g.ngx;
    const int jc = ((int)fb + 1 + g.ngy / 2) % g.ngy;
    c.ic0 = ic < 0 ? ic + g.ngx : ic;
    c.jc0 = jc < 0 ? jc + g.ngy : jc;
    if (g.do_w) {
        const double pw = (c.w - g.w0) / g.dw;
        const double fp = floor(pw - 0.5 * g.W);
        c.dw = fp + 1.0 - pw;
        c.fw = (float)c.dw;
        c.p0 = min(max((int)fp + 1, 0), g.nps - 1);
    } else {
        c.p0 = 0;
        c.fw = 0.0f;
        c.dw = 0.0;
    }
    return c;
}

// p0-major bucket keys: the items of a range of first planes are contiguous.
__device__ __forceinline__ unsigned coord_key(const Geo &g, const Coord &c, int64_t row) {
    const int ic = c.ic0 - g.wx0, jc = c.jc0 - g.wy0;
    const int tile = g.sub == kTileCell ? ((ic >> 1) * g.nty + jc) * 2 + (ic & 1)
                                        : (ic / g.sub) * g.nty + (jc / g.sub);
    return ((unsigned)c.p0 * (unsigned)g.ntiles + (unsigned)tile) * (unsigned)g.salt +
           ((unsigned)row & (unsigned)(g.salt - 1));
}

// ------------------------------------------------------------------------
// kernels: geometry and bucketing
// ------------------------------------------------------------------------
// uvw extent: per-block partials (no atomics), reduced by one block after
constexpr int kBoundsBlocks = 1024;

// raw extremes in metres (min/max of su*w, max |u|, max |v|); the host
// scales them by the frequency range (w*s is monotonic in w for s > 0)
__global__ __launch_bounds__(256) void k_bounds(const double *__restrict__ uvw, int64_t rs,
                                                int64_t nrow, double su,
                                                double *__restrict__ part) {
    __shared__ double red[4][4];
    double wmn = 1e300, wmx = -1e300, umx = 0.0, vmx = 0.0;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrow;
         r += (int64_t)gridDim.x * blockDim.x) {
        const double u = uvw[r * rs], v = uvw[r * rs + 1], w = su * uvw[r * rs + 2];
        wmn = fmin(wmn, w);
        wmx = fmax(wmx, w);
        umx = fmax(umx, fabs(u));
        vmx = fmax(vmx, fabs(v));
    }
    for (int o = 32; o > 0; o >>= 1) {
        wmn = fmin(wmn, __shfl_xor(wmn, o));
        wmx = fmax(wmx, __shfl_xor(wmx, o));
        umx = fmax(umx, __shfl_xor(umx, o));
        vmx = fmax(vmx, __shfl_xor(vmx, o));
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wv] = wmn;
        red[1][wv] = wmx;
        red[2][wv] = umx;
        red[3][wv] = vmx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k) {
            red[0][0] = fmin(red[0][0], red[0][k]);
            red[1][0] = fmax(red[1][0], red[1][k]);
            red[2][0] = fmax(red[2][0], red[2][k]);
            red[3][0] = fmax(red[3][0], red[3][k]);
        }
        for (int k = 0; k < 4; ++k) part[k * kBoundsBlocks + blockIdx.x] = red[k][0];
    }
}

// out = {min su*w, max su*w, max|u|, max|v|, min freq, max freq}
__global__ __launch_bounds__(256) void k_bounds_final(int nblocks, const double *__restrict__ part,
                                                      const double *__restrict__ freq, int nchan,
                                                      double *__restrict__ out) {
    __shared__ double red[6][256];
    double a[6] = {1e300, -1e300, 0.0, 0.0, 1e300, -1e300};
    for (int b = threadIdx.x; b < nblocks; b += 256) {
        a[0] = fmin(a[0], part[b]);
        a[1] = fmax(a[1], part[kBoundsBlocks + b]);
        a[2] = fmax(a[2], part[2 * kBoundsBlocks + b]);
        a[3] = fmax(a[3], part[3 * kBoundsBlocks + b]);
    }
    for (int c = threadIdx.x; c < nchan; c += 256) {
        a[4] = fmin(a[4], freq[c]);
        a[5] = fmax(a[5], freq[c]);
    }
    for (int k = 0; k < 6; ++k) red[k][threadIdx.x] = a[k];
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) {
            const int t = threadIdx.x;
            red[0][t] = fmin(red[0][t], red[0][t + st]);
            red[4][t] = fmin(red[4][t], red[4][t + st]);
            for (int k : {1, 2, 3, 5}) red[k][t] = fmax(red[k][t], red[k][t + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) out[threadIdx.x] = red[threadIdx.x][0];
}

// per-part plan metadata (one buffer, one D2H copy when the host needs it):
// {nbad lo, nbad hi, nrec, nitems, first item of each first-plane value
// [nps + 1]}; meta[3] is also the item count persistent launches read
__global__ void k_part_meta(const unsigned long long *__restrict__ nbad,
                            const unsigned *__restrict__ nrec, const unsigned *__restrict__ npad,
                            const unsigned *__restrict__ ioffs, int groups_per_plane, int nps,
                            unsigned *__restrict__ meta) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0) {
        meta[0] = (unsigned)(*nbad & 0xffffffffull);
        meta[1] = (unsigned)(*nbad >> 32);
        meta[2] = *nrec - (npad ? *npad : 0u);  // gridded visibilities (pads excluded)
        meta[3] = ioffs[(size_t)nps * groups_per_plane];
    }
    if (k <= nps) meta[4 + k] = ioffs[(size_t)k * groups_per_plane];
}

// Wave-level run-length aggregation: consecutive lanes with equal keys share
// one atomic on counter[key]; with kScatter each lane gets its slot.
template <bool kScatter>
__device__ __forceinline__ unsigned run_reserve(unsigned key, bool valid, unsigned *counter) {
    const int lane = threadIdx.x & 63;
    const unsigned prev = __shfl_up(key, 1);
    const bool start = (lane == 0) || (prev != key);
    const unsigned long long B = __ballot(start);
    const unsigned long long above = (lane == 63) ? 0ull : (B & ~((2ull << lane) - 1ull));
    const int end = above ? (__ffsll((long long)above) - 1) : 64;
    unsigned base = 0;
    if (valid && start) base = atomicAdd(&counter[key], (unsigned)(end - lane));
    if (!kScatter) return 0;
    const unsigned long long upto = (lane == 63) ? B : (B & ((2ull << lane) - 1ull));
    const int head = 63 - __clzll((long long)upto);
    const unsigned hb = __shfl(base, head);
    return hb + (unsigned)(lane - head);
}

// Visibility-side prologue fused into the bucketing pass (sdp_hip_ms2dirty_vis,
// SURVEY.md §8(f) rank 2): flag masking of the visibilities and weights,
// fp64 weights, the polarisation-frame conversion of the reference's
// convert_pol_frame (imaging/ng.py:193-198) as one row of its matrix, and
// the weight sum the reference takes with numpy.sum (ng.py:258, :289).
struct VisExtra {
    int64_t vps = 0;           // vis pol stride (elements); vis points at pol 0 when conv
    int npv = 1;               // vis pols combined
    bool conv = false;         // vis_eff = sum_k coef_k * vis_k * (1 - flag_k)
    double cre[4] = {1.0, 0.0, 0.0, 0.0}, cim[4] = {0.0, 0.0, 0.0, 0.0};
    int wgt_f64 = 0;           // weights are f64 (else f32)
    const void *flags = nullptr;
    int fbytes = 0;            // 1 / 4 / 8 byte integer flags at pol 0
    int64_t frs = 0, fcs = 0, fps = 0;
    int fpol = 0;              // pol whose flag masks the weight (and the vis when !conv)
    double *sumwt = nullptr;   // += sum of the effective weights (device, may be null)
    // shift_vis_to_image with tangent=True (reference imaging/base.py:48-92,
    // visibility/base.py:27-45, :60-90): phase d = uvw_lambda . (l, m, n-1)
    // in turns, folded into the record factor as exp(+2 pi i d) for invert
    // (vis * conj(phasor)) and exp(-2 pi i d) for predict (vis * phasor)
    bool shift = false;
    double sl = 0.0, sm = 0.0, sn = 0.0;
    // SDP_HIP_KEEP_BUCKETS: every in-grid visibility is bucketed (zero
    // weights add exact zeros), so the bucketing holds for any weights
    bool all = false;
};

constexpr int kSumSlots = 1024;

__device__ __forceinline__ double flag_mask(const VisExtra &x, int64_t row, int chan, int pol) {
    const int64_t i = row * x.frs + chan * x.fcs + pol * x.fps;
    double f;
    if (x.fbytes == 8) f = (double)static_cast<const int64_t *>(x.flags)[i];
    else if (x.fbytes == 4) f = (double)static_cast<const int32_t *>(x.flags)[i];
    else f = (double)static_cast<const int8_t *>(x.flags)[i];
    return 1.0 - f;
}

__device__ __forceinline__ double eff_weight(const void *wgt, int64_t wrs, int64_t wcs,
                                             const VisExtra &x, int64_t row, int chan) {
    double w = 1.0;
    if (wgt) {
        const int64_t i = row * wrs + chan * wcs;
        w = x.wgt_f64 ? static_cast<const double *>(wgt)[i]
                      : (double)static_cast<const float *>(wgt)[i];
    }
    if (x.fbytes) w *= flag_mask(x, row, chan, x.fpol);
    return w;
}

__device__ __forceinline__ double2 load_vis_d(const float2 *p) {
    const float2 v = *p;
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ double2 load_vis_d(const double2 *p) { return *p; }

__device__ __forceinline__ float2 load_vis(const float2 *p) { return *p; }
__device__ __forceinline__ float2 load_vis(const double2 *p) {
    const double2 v = *p;
    return make_float2((float)v.x, (float)v.y);
}

// Two passes over the visibilities.  Rank pass (kScatter = false): fp64
// coordinates -> bucket key, and the visibility's rank inside its bucket
// from a run-aggregated atomicAdd on the histogram; the rank is stored.
// Scatter pass: position = offs[key] + rank -- no atomics -- and the 32-byte
// record is written there.  Invalid visibilities carry key 0xffffffff.
template <class VT>
__device__ __forceinline__ float2 eff_vis(const VT *vis, int64_t vrs, int64_t vcs,
                                          const VisExtra &x, int64_t row, int chan) {
    const VT *p = vis + row * vrs + chan * vcs;
    if (!x.conv) {
        if (!x.fbytes) return load_vis(p);
        const double2 v = load_vis_d(p);
        const double m = flag_mask(x, row, chan, x.fpol);
        return make_float2((float)(v.x * m), (float)(v.y * m));
    }
    double re = 0.0, im = 0.0;
    for (int k = 0; k < x.npv; ++k) {
        if (x.cre[k] == 0.0 && x.cim[k] == 0.0) continue;
        double2 v = load_vis_d(p + k * x.vps);
        if (x.fbytes) {
            const double m = flag_mask(x, row, chan, k);
            v.x *= m;
            v.y *= m;
        }
        re += x.cre[k] * v.x - x.cim[k] * v.y;
        im += x.cre[k] * v.y + x.cim[k] * v.x;
    }
    return make_float2((float)re, (float)im);
}

template <class VT, bool kScatter, bool kGrid, bool kCompact = false>
__global__ void k_bucket(Geo g, int64_t row0, int64_t nvis, const double *__restrict__ uvw,
                         int64_t uvw_rs, const double *__restrict__ freq,
                         const VT *__restrict__ vis, int64_t vrs, int64_t vcs,
                         const void *__restrict__ wgt, int64_t wrs, int64_t wcs, VisExtra x,
                         double *sw_slots, unsigned *counter, unsigned *__restrict__ rk,
                         VisRec *__restrict__ recs, unsigned long long *nbad) {
    // v indexes the part's visibilities (rows row0...); vg the call's
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t vg = row0 * g.nchan + v;
    bool valid = v < nvis;
    int64_t row = 0;
    int chan = 0;
    float wt = 1.0f;
    Coord c;
    c.ok = false;
    unsigned mine = 0xffffffffu;  // rank in the bucket (0xffffffff: not gridded)
    if (kScatter) {
        double wd = 0.0;
        if (valid) {
            row = vg / g.nchan;
            chan = (int)(vg - row * g.nchan);
            wd = eff_weight(wgt, wrs, wcs, x, row, chan);
            wt = (float)wd;
        }
        if (sw_slots) {
            // weight sum of a reused bucketing (SDP_HIP_REUSE_BUCKETS): the
            // count pass did not run, so the value pass sums the weights
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) wd += __shfl_xor(wd, o, 64);
            if ((threadIdx.x & 63) == 0 && wd != 0.0)
                atomicAdd(&sw_slots[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) &
                                    (kSumSlots - 1)],
                          wd);
        }
        if (!valid) return;
        mine = rk[v];
        if (mine == 0xffffffffu) return;
        c = vis_coord(g, uvw, uvw_rs, row, freq[chan]);
    } else {
        double wd = 0.0;
        if (valid) {
            row = vg / g.nchan;
            chan = (int)(vg - row * g.nchan);
            wd = eff_weight(wgt, wrs, wcs, x, row, chan);
            wt = (float)wd;
            valid = x.all || (wt != 0.0f);
            if (valid) {
                c = vis_coord(g, uvw, uvw_rs, row, freq[chan]);
                if (!c.ok) {
                    valid = false;
                    atomicAdd(nbad, 1ull);
                }
            }
        }
        const unsigned key = valid ? coord_key(g, c, row) : 0xffffffffu;
        const unsigned rank = (g.dbg & 8) ? 0u : run_reserve<true>(key, valid, counter);
        // only the rank is kept: the scatter pass recomputes the key
        if (v < nvis) rk[v] = valid ? rank : 0xffffffffu;
        if (sw_slots) {
            // weight sum: wave reduction, one atomic per wave into a slot
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) wd += __shfl_xor(wd, o, 64);
            if ((threadIdx.x & 63) == 0 && wd != 0.0)
                atomicAdd(&sw_slots[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) &
                                    (kSumSlots - 1)],
                          wd);
        }
        return;
    }
    const unsigned pos = (g.dbg & 16) ? (unsigned)v : counter[coord_key(g, c, row)] + mine;
    float cr = wt, ci = 0.0f;
    if (kGrid) {
        const float2 xv = vis ? eff_vis(vis, vrs, vcs, x, row, chan) : make_float2(1.0f, 0.0f);
        cr = xv.x * wt;
        ci = xv.y * wt;
    }
    if (g.do_w || x.shift) {
        double ph = g.do_w ? c.w * g.s0 : 0.0;
        if (x.shift) {
            const double *u = uvw + row * uvw_rs;
            ph += (u[0] * x.sl + u[1] * x.sm + u[2] * x.sn) * (freq[chan] / kCLight);
        }
        ph -= rint(ph);
        float sn, cs;
        sincospif((float)(2.0 * ph), &sn, &cs);
        if (!kGrid) sn = -sn;
        const float r_ = cr * cs - ci * sn, i_ = cr * sn + ci * cs;
        cr = r_;
        ci = i_;
    }
    if (kCompact) {
        // RecC: offsets as fractions of (1 - W/2) - offset (do_w off: w = 0)
        const double base = 1.0 - 0.5 * g.W;
        const uint32_t qu = fix_frac(base - c.du, 21), qv = fix_frac(base - c.dv, 21);
        const uint32_t qw = g.do_w ? fix_frac(base - c.dw, 22) : 0u;
        RecC rc;
        rc.cre = cr;
        rc.cim = ci;
        rc.lo = qu | (qv << 21);
        rc.hi = (qv >> 11) | (qw << 10);
        reinterpret_cast<RecC *>(recs)[pos] = rc;
        return;
    }
    VisRec rec;
    rec.cre = cr;
    rec.cim = ci;
    rec.fu = c.fu;
    rec.fv = c.fv;
    rec.fw = c.fw;
    rec.ij = (uint32_t)c.ic0 | ((uint32_t)c.jc0 << 16);
    rec.p0 = (uint32_t)c.p0;
    rec.idx = (uint32_t)vg;
    recs[pos] = rec;
}

__global__ __launch_bounds__(64) void k_sum_slots(const double *__restrict__ slots, double *out) {
    double s = 0.0;
    for (int i = threadIdx.x; i < kSumSlots; i += 64) s += slots[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (threadIdx.x == 0) *out += s;
}

// work items: a group of `grp` consecutive buckets (same p0, same x) is
// split into chunks of <= chunk records
__global__ void k_items_count(int64_t ngroups, int grp, const unsigned *__restrict__ offs,
                              unsigned chunk, unsigned *nch) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k >= ngroups) return;
    const unsigned n = offs[(k + 1) * grp] - offs[k * grp];
    nch[k] = (n + chunk - 1) / chunk;
}

__global__ void k_items_fill(int64_t ngroups, int grp, int groups_per_plane,
                             const unsigned *__restrict__ offs, const unsigned *__restrict__ ioffs,
                             unsigned chunk, Item *items) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k >= ngroups) return;
    const unsigned b = offs[k * grp], e = offs[(k + 1) * grp];
    unsigned o = ioffs[k];
    const uint32_t p0 = (uint32_t)(k / groups_per_plane);
    const uint32_t tile = (uint32_t)(k - (int64_t)p0 * groups_per_plane);
    for (unsigned s = b; s < e; s += chunk) {
        Item x;
        x.b = s;
        x.e = min(e, s + chunk);
        x.tile = tile;
        x.p0 = p0;
        items[o++] = x;
    }
}

// 4-padding of the one-cell buckets for k_grid_mfma_pad: key k's records
// fill [offs[k], offs[k] + hist[k]) of a slot range rounded up to a multiple
// of 4 (the scan ran over the rounded counts); the remaining slots get
// zero-valued RecC records.  Per block the pad count is added into one of
// kSumSlots slots (k_sum_pads folds them).
__global__ __launch_bounds__(256) void k_pad_cells(unsigned nkeys,
                                                   const unsigned *__restrict__ hist,
                                                   const unsigned *__restrict__ offs,
                                                   RecC *__restrict__ recs,
                                                   unsigned *__restrict__ pad_slots) {
    __shared__ unsigned red[4];
    const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned npad = 0;
    if (k < nkeys) {
        const unsigned n = hist[k];
        if (n & 3u) {
            npad = 4u - (n & 3u);
            const unsigned base = offs[k] + n;
            RecC r;
            r.cre = r.cim = 0.0f;
            r.lo = r.hi = 0u;  // offsets 1 - W/2: in range, finite taps
            for (unsigned i = 0; i < npad; ++i) recs[base + i] = r;
        }
    }
    unsigned s = npad;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = red[0] + red[1] + red[2] + red[3];
        if (t) atomicAdd(&pad_slots[blockIdx.x & (kSumSlots - 1)], t);
    }
}

__global__ __launch_bounds__(256) void k_sum_pads(const unsigned *__restrict__ slots,
                                                  unsigned *out) {
    __shared__ unsigned red[4];
    unsigned s = 0;
    for (int i = threadIdx.x; i < kSumSlots; i += 256) s += slots[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) *out = red[0] + red[1] + red[2] + red[3];
}

struct Round4 {
    __host__ __device__ __forceinline__ unsigned operator()(unsigned n) const {
        return (n + 3u) & ~3u;
    }
};

// Large grids: the dense 2x2-cell histogram would be too large (C4: 70
// planes of 8192^2 buckets), so visibilities are bucketed by 16x16 cells and
// each coarse item's records are then re-ordered in place by 2x2-cell bucket
// -- x pair major, y pair minor, so the 4 buckets of a 2 x 8-cell group are
// consecutive -- through an LDS copy.  The item's 16 groups become register
// gridder / degridder work items (FineItem; empty groups have b == e).  One
// workgroup of kSubThreads per coarse item of <= kSubChunk records (the plan
// caps the chunk on this path); the 128 KiB staging admits one workgroup per
// CU, so it carries 16 waves.
constexpr int kSubChunk = 4096;
constexpr int kSubThreads = 1024;

// class of a record inside its 16x16-cell item: 2x2 bucket (x pair major,
// y pair minor; 64 classes) or, for the MFMA gridder, one cell in the
// x-pair-major order of kTileCell keys (256 classes)
template <bool CELLS>
__device__ __forceinline__ int sub_class(uint32_t ij) {
    const int ic = (int)(ij & 0xffffu), jc = (int)(ij >> 16);
    if (CELLS) return ((ic & 15) >> 1) * 32 + (jc & 15) * 2 + (ic & 1);
    return ((ic & 15) >> 1) * 8 + ((jc & 15) >> 1);
}

template <bool CELLS>
__global__ __launch_bounds__(kSubThreads) void k_subsort(Geo g, const Item *__restrict__ items,
                                                 VisRec *recs, FineItem *__restrict__ fitems,
                                                 unsigned *__restrict__ psize = nullptr) {
    constexpr int NC = CELLS ? 256 : 64;  // classes
    constexpr int PG = NC / 16;           // classes per fine group
    __shared__ VisRec stage[kSubChunk];
    __shared__ unsigned cur[NC], first[NC + 1];
    const Item it = items[blockIdx.x];
    const int n = (int)(it.e - it.b);
    for (int c = threadIdx.x; c < NC; c += kSubThreads) cur[c] = 0u;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kSubThreads) {
        const VisRec r = recs[it.b + i];
        stage[i] = r;
        atomicAdd(&cur[sub_class<CELLS>(r.ij)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned a = 0, pa = 0;
        for (int c = 0; c < NC; ++c) {
            first[c] = a;
            a += cur[c];
            pa += (cur[c] + 3u) & ~3u;
        }
        first[NC] = a;
        if (psize) psize[blockIdx.x] = pa;  // the item's size with every cell 4-padded
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NC; c += kSubThreads) cur[c] = first[c];
    if (threadIdx.x < 16) {
        // fine group gi = 2 * (x pair) + (y half): a 2 x 8-cell region
        const int gi = threadIdx.x, xp = gi >> 1, hf = gi & 1;
        const int c0 = CELLS ? gi * PG : xp * 8 + hf * 4;
        FineItem f;
        f.b = it.b + first[c0];
        f.e = it.b + first[c0 + PG];
#pragma unroll
        for (int j = 0; j < 16; ++j) f.o[j] = it.b + first[c0 + min(j + 1, PG)];
        const int tx = (int)it.tile / g.nty, ty = (int)it.tile - tx * g.nty;
        f.tile = (uint32_t)((tx * 8 + xp) * (g.wny / 8) + ty * 2 + hf);
        f.p0 = it.p0;
        fitems[(size_t)blockIdx.x * 16 + threadIdx.x] = f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kSubThreads) {
        const VisRec r = stage[i];
        const unsigned pos = atomicAdd(&cur[sub_class<CELLS>(r.ij)], 1u);
        recs[it.b + pos] = r;
    }
}

// Large grids, invert: the sub-sorted coarse item (cells in x-pair-major
// order, FineItem cell ends) is re-written as 16-byte RecC records with every
// cell padded to a multiple of 4 (zero-valued pads) at the item's slot of the
// padded buffer (poffs: exclusive scan of k_subsort's psize), plus FineItems
// over the padded layout -- so k_grid_mfma_pad<.., FI> runs the large grids.
__global__ __launch_bounds__(256) void k_subsort_emit(Geo g, const Item *__restrict__ items,
                                                      const VisRec *__restrict__ recs,
                                                      const FineItem *__restrict__ fitems,
                                                      const unsigned *__restrict__ poffs,
                                                      RecC *__restrict__ out,
                                                      FineItem *__restrict__ pfitems) {
    // cell c = 16 gi + j of the item (group gi, cell j): records
    // [cstart[c], cstart[c + 1]) of `recs`, padded slots from pstart[c] of `out`
    __shared__ unsigned cstart[257], pstart[256], gtot[16], gbase[16];
    const Item it = items[blockIdx.x];
    const FineItem *const fi = fitems + (size_t)blockIdx.x * 16;
    const int t = threadIdx.x;
    if (t < 16) {
        unsigned s0 = fi[t].b, ps = 0;
        for (int j = 0; j < 16; ++j) {
            const unsigned e = fi[t].o[j];
            cstart[t * 16 + j] = s0;
            pstart[t * 16 + j] = ps;  // group-relative
            ps += (e - s0 + 3u) & ~3u;
            s0 = e;
        }
        gtot[t] = ps;
        if (t == 15) cstart[256] = s0;  // = it.e
    }
    __syncthreads();
    if (t == 0) {
        unsigned b = poffs[blockIdx.x];
        for (int gi = 0; gi < 16; ++gi) {
            gbase[gi] = b;
            b += gtot[gi];
        }
    }
    __syncthreads();
    pstart[t] += gbase[t >> 4];  // blockDim.x == 256: one cell per thread
    __syncthreads();
    const int n = (int)(it.e - it.b);
    const double fb = 1.0 - 0.5 * g.W;
    for (int i = t; i < n; i += 256) {
        const VisRec r = recs[it.b + i];
        const int c = sub_class<true>(r.ij);
        const unsigned dst = pstart[c] + (it.b + (unsigned)i - cstart[c]);
        const uint32_t qu = fix_frac(fb - (double)r.fu, 21), qv = fix_frac(fb - (double)r.fv, 21);
        const uint32_t qw = g.do_w ? fix_frac(fb - (double)r.fw, 22) : 0u;
        RecC rc;
        rc.cre = r.cre;
        rc.cim = r.cim;
        rc.lo = qu | (qv << 21);
        rc.hi = (qv >> 11) | (qw << 10);
        out[dst] = rc;
    }
    {
        const unsigned cnt = cstart[t + 1] - cstart[t];
        RecC z;
        z.cre = z.cim = 0.0f;
        z.lo = z.hi = 0u;  // offsets 1 - W/2: in range, finite taps
        for (unsigned k = cnt; k < ((cnt + 3u) & ~3u); ++k) out[pstart[t] + k] = z;
    }
    if (t < 16) {
        FineItem f;
        f.b = pstart[t * 16];
        for (int j = 0; j < 16; ++j) {
            const int c = t * 16 + j;
            f.o[j] = pstart[c] + ((cstart[c + 1] - cstart[c] + 3u) & ~3u);
        }
        f.e = f.o[15];
        f.tile = fi[t].tile;
        f.p0 = fi[t].p0;
        pfitems[(size_t)blockIdx.x * 16 + t] = f;
    }
}

// ------------------------------------------------------------------------
// kernels: gridding / degridding (the hot loops)
// ------------------------------------------------------------------------
// LDS tile of an SX x SY-cell work-item region plus the W-1 footprint halo
template <int W, int SX, int SY = SX>
struct TileShape {
    static constexpr int RX = SX + W - 1, RY = SY + W - 1;
    static constexpr int R = RX;                                    // (square tiles)
    static constexpr int PITCH = SX == kTileCoarse ? kPitch : RY;  // LDS row pitch
    static constexpr int PLANE = RX * PITCH;  // complex values per plane in LDS
};

// Work items are visited in a strided order (stride coprime with the item
// count): the heavy chunks of one dense tile are spread over the launch
// instead of flushing into the same cells at the same time.
//
// A launch walks the items either one per workgroup (count known on the
// host) or persistently (count read from device memory, written by the
// bucketing of the same call -- no host round trip between the stages).
struct ItemSrc {
    const Item *items;
    uint32_t n;            // item count when ndev == nullptr
    const unsigned *ndev;  // device-side item count (persistent launches)
};

__device__ __forceinline__ uint32_t item_count(const ItemSrc &src) {
    return src.ndev ? (uint32_t)__builtin_amdgcn_readfirstlane((int)*src.ndev) : src.n;
}

__device__ __forceinline__ uint32_t item_stride(uint32_t n) {
    const uint32_t primes[5] = {7919u, 104729u, 1299709u, 15485863u, 179424673u};
    for (int k = 0; k < 5; ++k)
        if (n <= 1 || n % primes[k] != 0) return primes[k];
    return 1u;
}

__device__ __forceinline__ Item load_item(const ItemSrc &src, uint32_t w, uint32_t n,
                                          uint32_t stride) {
    const uint32_t i = (uint32_t)(((uint64_t)w * stride) % n);
    const Item raw = src.items[i];
    Item it;
    it.b = __builtin_amdgcn_readfirstlane(raw.b);
    it.e = __builtin_amdgcn_readfirstlane(raw.e);
    it.tile = __builtin_amdgcn_readfirstlane(raw.tile);
    it.p0 = __builtin_amdgcn_readfirstlane(raw.p0);
    return it;
}

template <int NO>
__device__ __forceinline__ Item load_fine_item(const FineItem *items, uint32_t w, uint32_t n,
                                               uint32_t stride, uint32_t (&fo)[NO]) {
    const uint32_t i = (uint32_t)(((uint64_t)w * stride) % n);
    const FineItem raw = items[i];
    Item it;
    it.b = __builtin_amdgcn_readfirstlane(raw.b);
    it.e = __builtin_amdgcn_readfirstlane(raw.e);
    it.tile = __builtin_amdgcn_readfirstlane(raw.tile);
    it.p0 = __builtin_amdgcn_readfirstlane(raw.p0);
#pragma unroll
    for (int j = 0; j < NO; ++j) fo[j] = __builtin_amdgcn_readfirstlane(raw.o[j]);
    return it;
}

__device__ __forceinline__ float lane_readf(float v, int src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

// Records are fetched 64 at a time, one per lane (coalesced 2 KiB), and
// broadcast to the wave with v_readlane.
struct RecRegs {
    float cre, cim, fu, fv, fw;
    uint32_t ij;
};

__device__ __forceinline__ RecRegs rec_at(const VisRec &my, int k) {
    RecRegs r;
    r.cre = lane_readf(my.cre, k);
    r.cim = lane_readf(my.cim, k);
    r.fu = lane_readf(my.fu, k);
    r.fv = lane_readf(my.fv, k);
    r.fw = lane_readf(my.fw, k);
    r.ij = (uint32_t)__builtin_amdgcn_readlane((int)my.ij, k);
    return r;
}

// Kernel taps of a 64-record batch with every lane busy: VGPR u[m] of lane
// l holds the u tap (l % 8) of record 8m + l/8 (likewise v, w), so 24 ES
// evaluations per lane cover the 64 records' 3 x 8 taps.  A record's taps
// are then fetched with one ds_bpermute (u, v: lane-dependent) or
// v_readlane (w: wave-uniform).  Taps t >= W evaluate to 0 (|x| > 1).
struct BatchTaps {
    float u[8], v[8], w[8];
};

__device__ __forceinline__ BatchTaps batch_taps(const VisRec &my, int lane, float ihw, float bl) {
    BatchTaps b;
    const float t = (float)(lane & 7);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int src = 8 * m + (lane >> 3);
        b.u[m] = es_kernel(__shfl(my.fu, src) + t, ihw, bl);
        b.v[m] = es_kernel(__shfl(my.fv, src) + t, ihw, bl);
        b.w[m] = es_kernel(__shfl(my.fw, src) + t, ihw, bl);
    }
    return b;
}

// Per-lane roles inside a wave for support W: lane = kx*W + ky is the (u,v)
// tap it accumulates; lanes [0,W) / [W,2W) / [2W,3W) evaluate the u / v / w
// 1-D taps of the current record (one ES evaluation per lane).
template <int W>
struct LaneRole {
    int kx, ky;
    bool act;
    float m0, m1, m2, toff;
    __device__ __forceinline__ explicit LaneRole(int lane) {
        kx = lane / W;
        ky = lane - kx * W;
        act = lane < W * W;
        const int set = lane / W;
        toff = (float)(lane - set * W);
        // arithmetic 0/1 selectors: a ternary chain here is lowered to scratch
        m0 = set == 0 ? 1.0f : 0.0f;
        m1 = set == 1 ? 1.0f : 0.0f;
        m2 = set == 2 ? 1.0f : 0.0f;
    }
    __device__ __forceinline__ float taps(const RecRegs &rc, float ihw, float bl) const {
        const float base = fmaf(m0, rc.fu, fmaf(m1, rc.fv, m2 * rc.fw));
        return es_kernel(base + toff, ihw, bl);
    }
};

// One workgroup of NWV waves per work item (= one (p0, tile) bucket chunk).
// The workgroup owns an LDS tile of W planes and wave wv owns planes
// [wv*NQW, (wv+1)*NQW): every wave walks all records of the item (coalesced
// 2 KiB record fetches, hits in L1/L2 after the first wave) and updates only
// its planes, so accumulation is a plain ds_read_b64/ds_write_b64
// read-modify-write with no LDS atomics (gfx950 runs ds_add_f32 at ~0.3
// lanes/clk/CU), exact fp32 sums, and in-order LDS execution
// inside each wave orders the updates of consecutive records.  Splitting the
// planes over waves raises occupancy (the 35 KiB tile is shared by NWV waves)
// to hide the LDS read->write latency of the update chain.
template <int W, bool WS, int NWV>
__global__ __launch_bounds__(64 * NWV) void k_grid_lds(Geo g, const VisRec *__restrict__ recs,
                                                       ItemSrc src, float *__restrict__ grid,
                                                       int p_lo, int p_hi) {
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int kTile = kTileCoarse;
    constexpr int R = TileShape<W, kTile>::R;
    constexpr int PS = TileShape<W, kTile>::PLANE;
    constexpr int NQ = WS ? W : 1;
    constexpr int NQW = (NQ + NWV - 1) / NWV;  // planes per wave (the last
    constexpr int NQP = NQW * NWV;             // wave may own padding planes)
    const uint32_t n_items = item_count(src);
    const uint32_t stride = item_stride(n_items);
    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        __syncthreads();  // previous item's flush reads of the LDS tile
        const Item it = load_item(src, w_it, n_items, stride);
        const int lane = threadIdx.x & 63;
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        for (int i = threadIdx.x; i < NQP * PS; i += 64 * NWV) tile[i] = make_float2(0.0f, 0.0f);
        __syncthreads();

        const int tx = (int)it.tile / g.nty, ty = (int)it.tile - tx * g.nty;
        const LaneRole<W> role(lane);
        const float ihw = g.inv_half_w, bl = g.beta_l2e;
        const int lane_off = role.kx * kPitch + role.ky - (g.wx0 + tx * kTile) * kPitch -
                             (g.wy0 + ty * kTile);
        const int q0 = wv * NQW;
        float2 *const wtile = tile + q0 * PS;

        for (uint32_t b0 = it.b; b0 < it.e; b0 += 64) {
            const int n = (int)min(64u, it.e - b0);
            const VisRec my = recs[b0 + min(lane, n - 1)];
            const BatchTaps bt = batch_taps(my, lane, ihw, bl);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int rn = min(8, n - 8 * m);  // records of this 8-record group
                for (int r = 0; r < rn; ++r) {
                    const int k = 8 * m + r;
                    const float cre = lane_readf(my.cre, k), cim = lane_readf(my.cim, k);
                    const uint32_t ij = (uint32_t)__builtin_amdgcn_readlane((int)my.ij, k);
                    const float ku = __shfl(bt.u[m], 8 * r + role.kx);
                    const float kv = __shfl(bt.v[m], 8 * r + role.ky);
                    const float kk = ku * kv;
                    const float vr = cre * kk, vi = cim * kk;
                    const int off = lane_off + (int)(ij & 0xffffu) * kPitch + (int)(ij >> 16);
                    // padding planes (q0 + q >= NQ) get a zero weight: a uniform
                    // select, so the LDS reads and writes below stay branch-free
                    float kw[NQW];
#pragma unroll
                    for (int q = 0; q < NQW; ++q) {
                        const float x = WS ? lane_readf(bt.w[m], 8 * r + min(q0 + q, NQ - 1)) : 1.0f;
                        kw[q] = (NQP == NQ || q0 + q < NQ) ? x : 0.0f;
                    }
                    if (role.act) {
                        float2 a[NQW];
#pragma unroll
                        for (int q = 0; q < NQW; ++q) a[q] = wtile[q * PS + off];
#pragma unroll
                        for (int q = 0; q < NQW; ++q) {
                            a[q].x = fmaf(vr, kw[q], a[q].x);
                            a[q].y = fmaf(vi, kw[q], a[q].y);
                            wtile[q * PS + off] = a[q];
                        }
                    }
                }
            }
        }
        __syncthreads();

        // flush: float atomics into the resident planes (the halo overlaps the
        // neighbouring tiles); zero cells are skipped.
        const int cells = R * R;
        const int64_t plane_elems = (int64_t)g.ngx * g.ngy;
        for (int c = threadIdx.x; c < NQ * cells; c += 64 * NWV) {
            const int q = c / cells;
            const int p = (int)it.p0 + q;
            if (p < p_lo || p >= p_hi) continue;
            const int rem = c - q * cells;
            const int xl = rem / R, yl = rem - (rem / R) * R;
            const float2 val = tile[q * PS + xl * kPitch + yl];
            if (val.x != 0.0f || val.y != 0.0f) {
                int gx = g.wx0 + tx * kTile + xl;
                if (gx >= g.ngx) gx -= g.ngx;
                int gy = g.wy0 + ty * kTile + yl;
                if (gy >= g.ngy) gy -= g.ngy;
                float *dst =
                    grid + ((int64_t)(p - p_lo) * plane_elems + (int64_t)gx * g.ngy + gy) * 2;
                atomicAdd(dst, val.x);
                atomicAdd(dst + 1, val.y);
            }
        }
    }
}

template <int NQ>
__device__ __forceinline__ void acc_add(float (&ar)[NQ], float (&ai)[NQ], float vr, float vi,
                                        const float (&kw)[NQ]) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        ar[q] = fmaf(vr, kw[q], ar[q]);
        ai[q] = fmaf(vi, kw[q], ai[q]);
    }
}

// Register gridder: one wave per work item = a chunk of the records of a
// group of kGroupFine consecutive 2x2-cell buckets (same first plane p0,
// same x), i.e. a 2 x 8-cell region.  Lane (kx, ky) is the (u, v) tap it
// accumulates.  Bucket by bucket, a record whose footprint starts at origin
// o in {0,1}^2 of its bucket adds vis * ku * kv * kw[q] into the VGPR
// accumulator acc[o][q] (q = w plane): per-record work is FMAs on registers,
// with no LDS traffic except two ds_bpermute for the u / v taps.  At the end
// of each bucket the <= 4 origin sets are added into the group's
// (2+W-1) x (8+W-1) x W LDS tile; the tile is flushed once per item with
// global float atomics (zero cells skipped), so neighbouring buckets share
// one flush of their overlapping halos.  Records of a bucket are consumed in
// static groups of 8 (zero-valued padding at the end of a bucket).
template <int W, bool WS, bool FI>
__global__ __launch_bounds__(64) void k_grid_reg(Geo g, const VisRec *__restrict__ recs,
                                                 ItemSrc src,
                                                 const unsigned *__restrict__ offs,
                                                 const FineItem *__restrict__ fitems,
                                                 float *__restrict__ grid, int p_lo, int p_hi,
                                                 int dbg) {
    constexpr int SUB = kTileFine;
    constexpr int GRP = kGroupFine;
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    using TS = TileShape<W, SUB, SUB * GRP>;
    constexpr int RX = TS::RX, RY = TS::RY, PS = TS::PLANE;
    constexpr int NQ = WS ? W : 1;
    constexpr int NO = SUB * SUB;
    static_assert(NO == 4, "origin select below assumes 2x2-cell buckets");
    const uint32_t n_items = item_count(src);
    const uint32_t stride = item_stride(n_items);
    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        uint32_t fo[4] = {0u, 0u, 0u, 0u};
        const Item it = FI ? load_fine_item(fitems, w_it, n_items, stride, fo)
                           : load_item(src, w_it, n_items, stride);
        if (FI && it.b >= it.e) continue;
        if (dbg & 4) {
            if (it.b == 0xfffffffeu) grid[0] = 1.0f;  // keep the item load live
            continue;
        }
        const int lane = threadIdx.x;
        const LaneRole<W> role(lane);
        const float ihw = g.inv_half_w, bl = g.beta_l2e;
        const int ntg = g.nty / GRP;
        const int sx = (int)it.tile / ntg, sg = (int)it.tile - sx * ntg;
        const int ibase = g.wx0 + sx * SUB, jbase = g.wy0 + sg * GRP * SUB;
        const int64_t key0 = (int64_t)it.p0 * g.ntiles + (int64_t)sx * g.nty + (int64_t)sg * GRP;

        for (int i = lane; i < NQ * PS; i += 64) tile[i] = make_float2(0.0f, 0.0f);

        const float tap_t = (float)(lane & 7);
        for (int j = 0; j < GRP; ++j) {
            const uint32_t rb = FI ? (j == 0 ? it.b : fo[j - 1]) : max(it.b, offs[key0 + j]);
            const uint32_t re = FI ? fo[j] : min(it.e, offs[key0 + j + 1]);
            if (rb >= re) continue;
            const int jb = jbase + j * SUB;  // bucket's first cell along y

            float acc_r[NO][NQ], acc_i[NO][NQ];
#pragma unroll
            for (int o = 0; o < NO; ++o)
#pragma unroll
                for (int q = 0; q < NQ; ++q) acc_r[o][q] = acc_i[o][q] = 0.0f;
            uint32_t used = 0;

            for (uint32_t b0 = rb; b0 < ((dbg & 2) ? rb + 1 : re); b0 += 64) {
                const int n = (int)min(64u, re - b0);
                const VisRec my = recs[b0 + min(lane, n - 1)];
                // per-lane decode of the lane's own record; lanes >= n carry
                // zero-valued padding records
                const bool live = lane < n;
                const float cre_l = live ? my.cre : 0.0f, cim_l = live ? my.cim : 0.0f;
                const int o_l = ((int)(my.ij & 0xffffu) - ibase) * SUB + ((int)(my.ij >> 16) - jb);
#pragma unroll
                for (int oo = 0; oo < NO; ++oo)
                    if (__ballot(live && o_l == oo)) used |= 1u << oo;
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    if (8 * m >= n) break;
                    // taps of this 8-record group: lane l holds tap (l % 8) of record
                    // 8m + l/8; the u tap is pre-multiplied by the record's value
                    const int src = 8 * m + (lane >> 3);
                    const float tu = es_kernel(__shfl(my.fu, src) + tap_t, ihw, bl);
                    const float tur = tu * __shfl(cre_l, src), tui = tu * __shfl(cim_l, src);
                    const float tv = es_kernel(__shfl(my.fv, src) + tap_t, ihw, bl);
                    const float tw = WS ? es_kernel(__shfl(my.fw, src) + tap_t, ihw, bl) : 1.0f;
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const int k = 8 * m + r;
                        const int o = __builtin_amdgcn_readlane(o_l, k);
                        const float kv = __shfl(tv, 8 * r + role.ky);
                        const float vr = __shfl(tur, 8 * r + role.kx) * kv;
                        const float vi = __shfl(tui, 8 * r + role.kx) * kv;
                        float kw[NQ];
#pragma unroll
                        for (int q = 0; q < NQ; ++q) kw[q] = WS ? lane_readf(tw, 8 * r + q) : 1.0f;
                        // origin select: uniform branches (one per origin set)
#pragma unroll
                        for (int oo = 0; oo < NO; ++oo)
                            if (o == oo) acc_add<NQ>(acc_r[oo], acc_i[oo], vr, vi, kw);
                    }
                }
            }

            // add the bucket's origin sets into the group tile (plain RMW: one
            // wave, in-order LDS)
#pragma unroll
            for (int oo = 0; oo < NO; ++oo) {
                if ((used >> oo) & 1u) {
                    if (role.act) {
                        const int base = (oo / SUB + role.kx) * RY + j * SUB + (oo % SUB) + role.ky;
#pragma unroll
                        for (int q = 0; q < NQ; ++q) {
                            float2 a = tile[q * PS + base];
                            a.x += acc_r[oo][q];
                            a.y += acc_i[oo][q];
                            tile[q * PS + base] = a;
                        }
                    }
                }
            }
        }

        // flush: lane f of pass i handles float (64 i + f) of each plane's
        // RX x RY complex cells (rows of RY contiguous cells, re/im interleaved);
        // zero floats are skipped.  The address of a float is the same in every
        // plane, so it is computed once.
        constexpr int FPP = RX * RY * 2;  // floats per plane
        const int64_t plane_floats = (int64_t)g.ngx * g.ngy * 2;
        const float *ftile = reinterpret_cast<const float *>(tile);
#pragma unroll
        for (int i0 = 0; i0 < FPP; i0 += 64) {
            const int f = i0 + lane;
            if (f >= FPP) break;
            const int c = f >> 1;
            const int xl = c / RY, yl = c - (c / RY) * RY;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            float *dst0 = grid + ((int64_t)gx * g.ngy + gy) * 2 + (f & 1);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int p = (int)it.p0 + q;
                const float val = ftile[q * PS * 2 + f];
                if (p >= p_lo && p < p_hi && val != 0.0f) {
                    float *dst = dst0 + (int64_t)(p - p_lo) * plane_floats;
                    if (dbg & 1) {
                        if (val == 1.2345f) dst[0] = val;  // keep the flush live, no atomics
                    } else {
                        atomicAdd(dst, val);
                    }
                }
            }
        }
    }
}

// MFMA gridder (invert): one wave per work item = a chunk of the records of
// a 2 x 8-cell region (16 one-cell buckets, same first plane p0; records
// ordered by cell).  All records of a cell share their footprint origin, so
// a cell's contribution to its W x W x W footprint is one GEMM
//     C[(kx, ky), (q, re/im)] += sum_r  tu_r[kx] tv_r[ky] * tw_r[q] c_r
// with A = the separable (u, v) taps (64 rows) and B = the w taps x value
// (8 planes x re/im = 16 columns), K = records: v_mfma_f32_16x16x4_f32
// (exact fp32 multiply-adds), 4 M-tiles of 16 taps, 4 records per K-step.
//
// Records stream through the wave 64 at a time (one per lane, one coalesced
// 2 KiB load, the next batch prefetched while this one is consumed).  Inside
// a batch the cell runs are found with ballots; a run is consumed in K-steps
// of 4 records (lanes k0..k0+3; the tail K-step of a run carries zero
// values).  In a K-step, lane l gathers the fields of record k0 + (l >> 4)
// (ds_bpermute) and evaluates its 1-D taps (l & 7) for u, v and w; the MFMA
// operands are those taps permuted inside the 16-lane record group:
// A[row][k] = tu[2t + (row >> 3)] tv[row & 7], B[k][col] = tw[col >> 1] x
// (re | im of c).  When the cell changes, the four 16 x 16 accumulators are
// added into the region's (2+W-1) x (8+W-1) x W LDS tile, which is flushed
// once per item with global float atomics (zero cells skipped), exactly as
// k_grid_reg.  Per record: one MFMA, ~8 VALU, 2.5 ds_bpermute -- versus 24
// VALU, 7.6 SALU and 4 LDS instructions in k_grid_reg.
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bperm(int byte_addr, float v) {
    return __builtin_bit_cast(float,
                              __builtin_amdgcn_ds_bpermute(byte_addr, __builtin_bit_cast(int, v)));
}

// One-wave workgroups: the LDS operations of one wavefront execute in
// program order, so a hand-off between the wave's own lanes through LDS needs
// only a compiler barrier (wavefront-scope fence), not s_barrier plus the
// s_waitcnt lgkmcnt(0) that __syncthreads() brings with it -- the wave keeps
// issuing while its writes drain.  SDP_PAD_WAVESYNC=0 restores __syncthreads
// in k_grid_mfma_pad (the gridders and degridders below all run one wave per
// workgroup).
#ifndef SDP_PAD_WAVESYNC
#define SDP_PAD_WAVESYNC 1
#endif
#ifndef SDP_PAD_UNROLL
#define SDP_PAD_UNROLL 1
#endif
__device__ __forceinline__ void wave_lds_sync() {
#if SDP_PAD_WAVESYNC
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
#else
    __syncthreads();
#endif
}

// the same hand-off in k_grid_mfma / k_degrid_mfma (SDP_MFMA_WAVESYNC=0:
// __syncthreads)
#ifndef SDP_MFMA_WAVESYNC
#define SDP_MFMA_WAVESYNC 1
#endif
__device__ __forceinline__ void wave_sync_1w() {
#if SDP_MFMA_WAVESYNC
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
#else
    __syncthreads();
#endif
}

// ES kernel for the MFMA gridder's taps: x = fu*ihw + t*ihw by one fma; for
// W = 8 every tap of the footprint lies inside the support (|x| <= 1), so
// no range select (the max() only guards rounding below zero)
template <int W>
__device__ __forceinline__ float es_tap(float f, float tihw, float ihw, float bl) {
    const float x = fmaf(f, ihw, tihw);
    const float y = fmaf(-x, x, 1.0f);
    const float e = __builtin_amdgcn_exp2f(fmaf(bl, __builtin_amdgcn_sqrtf(fmaxf(y, 0.0f)), -bl));
    return W == 8 ? e : (y > 0.0f ? e : 0.0f);
}

template <int W, bool WS, bool FI>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_grid_mfma(Geo g, const VisRec *__restrict__ recs,
                                                  ItemSrc src, const unsigned *__restrict__ offs,
                                                  const FineItem *__restrict__ fitems,
                                                  float *__restrict__ grid, int p_lo, int p_hi) {
    static_assert(W <= 8, "the MFMA tiles hold 8 taps per axis");
    // LDS: the region tile (W planes x RX x RY complex) + the staged batch
    // (64 records: fu fv fw - | cre cim - - as two float4 rows per record)
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int RX = 2 + W - 1, RY = 8 + W - 1, PS = RX * RY;
    constexpr int NQ = WS ? W : 1;
    float4 *const stage = reinterpret_cast<float4 *>(tile + NQ * PS);  // [64][2]
    (void)offs;
    const uint32_t n_items = item_count(src);
    const uint32_t stride = item_stride(n_items);
    const int lane = threadIdx.x;
    const float ihw = g.inv_half_w, bl = g.beta_l2e;
    const float tihw = (float)(lane & 7) * ihw;
    const int grp16 = lane & ~15;
    const int srcA = (grp16 | ((lane >> 3) & 1)) << 2;  // + 8 t bytes: tu tap 2t + (row >> 3)
    const int srcB = (grp16 | ((lane & 15) >> 1)) << 2;   // tw tap q = col >> 1
    const bool col_im = lane & 1;
    // accumulator element i of M-tile t: tap (2t + (lane >> 5), 4 ((lane >> 4) & 1) + i),
    // column (q, re/im) = ((lane & 15) >> 1, lane & 1)
    const int cq = (lane & 15) >> 1;
    const int ckx = lane >> 5, cky = 4 * ((lane >> 4) & 1);
    float *const ftile = reinterpret_cast<float *>(tile);

    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        Item it;
        if (FI) {
            uint32_t fo[1];
            it = load_fine_item<1>(fitems, w_it, n_items, stride, fo);
            if (it.b >= it.e) continue;
        } else {
            it = load_item(src, w_it, n_items, stride);
        }
        const int ntg = FI ? g.wny / 8 : g.nty / 8;  // groups per x pair
        const int sx = (int)it.tile / ntg, sg = (int)it.tile - sx * ntg;
        const int ibase = g.wx0 + sx * 2, jbase = g.wy0 + sg * 8;

        wave_sync_1w();
        for (int i = lane; i < NQ * PS; i += 64) tile[i] = make_float2(0.0f, 0.0f);

        floatx4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
        int cur = -1;  // cell of the accumulators (wave-uniform)
        auto flush_cell = [&]() {
            const int xo = cur & 1, yo = cur >> 1;
            if (cq < NQ) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int kx = 2 * t + ckx;
                    if (kx >= W) continue;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int ky = cky + i;
                        if (ky >= W) continue;
                        float *d = ftile + ((cq * RX + xo + kx) * RY + yo + ky) * 2 + (col_im ? 1 : 0);
                        *d += acc[t][i];
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
        };
        // one K-step: records k0 .. k0+3 of the staged batch (lane >> 4 picks
        // the record), valid below `rend`.  Phase 1 (taps): the three 1-D
        // taps (lane & 7) of the record and its value; phase 2 (gather): the
        // 5 operand values from the record group's lanes; phase 3: A, B.
        // Two K-steps are interleaved phase by phase (sched_barrier keeps
        // every ds_bpermute of both in flight before the first use).
        struct Taps {
            float tu, tv, tw, cv;
        };
        auto taps = [&](int k0, int rend) {
            const int kl = k0 + (lane >> 4);
            const float4 h = stage[2 * min(kl, 63)];      // fu fv fw -
            const float4 c = stage[2 * min(kl, 63) + 1];  // cre cim - -
            Taps r;
            r.tu = es_tap<W>(h.x, tihw, ihw, bl);
            r.tv = es_tap<W>(h.y, tihw, ihw, bl);
            r.tw = WS ? es_tap<W>(h.z, tihw, ihw, bl) : ((lane & 7) == 0 ? 1.0f : 0.0f);
            r.cv = (col_im ? c.y : c.x) * (kl < rend ? 1.0f : 0.0f);
            return r;
        };
        struct Ops {
            float u[4], w;
        };
        auto gather = [&](const Taps &r) {
            Ops o;
            o.w = bperm(srcB, r.tw);
#pragma unroll
            for (int t = 0; t < 4; ++t) o.u[t] = bperm(srcA + 8 * t, r.tu);
            return o;
        };
        auto mfma4 = [&](const Taps &r, const Ops &o) {
            const float bop = o.w * r.cv;
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(o.u[t] * r.tv, bop, acc[t], 0, 0, 0);
        };

        // batch = 64 records, lane l holds record b0 + l (staged in LDS); the
        // next batch is loaded before this one is consumed
        VisRec nx = recs[min(it.b + (uint32_t)lane, it.e - 1)];
        for (uint32_t b0 = it.b; b0 < it.e; b0 += 64) {
            const VisRec my = nx;
            if (b0 + 64 < it.e) nx = recs[min(b0 + 64 + (uint32_t)lane, it.e - 1)];
            const int nb = (int)min(64u, it.e - b0);
            const bool live = lane < nb;
            const int cj = live ? ((int)(my.ij >> 16) - jbase) * 2 + ((int)(my.ij & 0xffffu) - ibase)
                                : 16;
            wave_sync_1w();  // previous batch's stage reads
            stage[2 * lane] = make_float4(my.fu, my.fv, my.fw, 0.0f);
            stage[2 * lane + 1] = make_float4(live ? my.cre : 0.0f, live ? my.cim : 0.0f, 0.0f, 0.0f);
            wave_sync_1w();
            // run starts: lane 0, and every lane whose cell differs from the previous lane's
            const int prev = __shfl_up(cj, 1);
            uint64_t starts = __ballot(live && (lane == 0 || prev != cj));
            while (starts) {
                const int pos = __builtin_ctzll(starts);
                starts &= starts - 1;
                const int rend = starts ? __builtin_ctzll(starts) : nb;
                const int cell = __builtin_amdgcn_readlane(cj, pos);
                if (cell != cur) {
                    if (cur >= 0) flush_cell();
                    cur = cell;
                }
                int k0 = pos;
                for (; k0 + 4 < rend; k0 += 8) {  // two K-steps
                    const Taps r0 = taps(k0, rend), r1 = taps(k0 + 4, rend);
                    __builtin_amdgcn_sched_barrier(0);
                    const Ops o0 = gather(r0), o1 = gather(r1);
                    __builtin_amdgcn_sched_barrier(0);
                    mfma4(r0, o0);
                    mfma4(r1, o1);
                }
                if (k0 < rend) {  // last K-step of the run
                    const Taps r0 = taps(k0, rend);
                    __builtin_amdgcn_sched_barrier(0);
                    const Ops o0 = gather(r0);
                    __builtin_amdgcn_sched_barrier(0);
                    mfma4(r0, o0);
                }
            }
        }
        if (cur >= 0) flush_cell();
        wave_sync_1w();

        // flush: float f = i0 + lane of each plane's RX x RY complex cells,
        // buffer atomics off a per-plane descriptor (32-bit offsets), the
        // cell index advanced incrementally; zero floats are skipped
        constexpr int FPP = RX * RY * 2;
        const size_t plane_bytes = (size_t)g.ngx * g.ngy * sizeof(float2);
        int xl = (lane >> 1) / RY, yl = (lane >> 1) - xl * RY;
#pragma unroll
        for (int i0 = 0; i0 < FPP; i0 += 64) {
            const int f = i0 + lane;
            if (f >= FPP) break;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            const int voff = ((gx * g.ngy + gy) * 2 + (f & 1)) * (int)sizeof(float);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int p = (int)it.p0 + q;
                const float val = ftile[q * PS * 2 + f];
                if (p >= p_lo && p < p_hi && val != 0.0f) {
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        grid + (size_t)(p - p_lo) * (plane_bytes / sizeof(float)), 0,
                        (int)plane_bytes, 0x00020000);
                    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(val, rs, voff, 0, 0);
                }
            }
            yl += 32 % RY;
            xl += 32 / RY;
            if (yl >= RY) {
                yl -= RY;
                ++xl;
            }
        }
    }
}

// MFMA gridder on 4-padded cells (invert, one-cell buckets): the bucketing
// rounds every cell's record count up to a multiple of 4 with zero-valued
// pad records (k_pad_cells), so every K-step of 4 consecutive records
// belongs to one cell and no K-step straddles a batch or an item.  Same GEMM
// and region tile as k_grid_mfma; what changes is the work per K-step:
//  * per batch of 64 records, the 64 x 3 x 8 one-dimensional taps are
//    evaluated once with every lane busy (lane l: tap l & 7 of records
//    8m + (l >> 3), 24 ES evaluations) into an LDS tap block of one
//    kTapRec-float row per record: tu in h-major order (tu[2t + h] at
//    4h + t, so a lane's four A taps are one ds_read_b128), tv, tw, value;
//  * the 16 K-steps of a batch are unrolled with compile-time LDS offsets,
//    the operands of K-step j + 1 read before the MFMAs of K-step j issue:
//    per K-step 4 LDS reads, 5 multiplies, 4 MFMAs and a cell-change bit
//    test -- no run bookkeeping, no masking.
constexpr int kTapRec = 28;    // floats per record row of the tap block (16-B multiple)
#ifndef SDP_TAP_BATCH
#define SDP_TAP_BATCH 16
#endif
constexpr int kTapBatch = SDP_TAP_BATCH;  // records per tap block (LDS, occupancy)

template <int W, bool WS>
constexpr int mfma_tile_f2() {  // region tile, rounded to 16 B
    return (((WS ? W : 1) * (2 + W - 1) * (8 + W - 1)) + 1) & ~1;
}

// SDP_PAD_PIPE=1 (experiment, off): two tap blocks; the ES chains of block
// h + 1 issue between the MFMAs of block h (software pipeline inside each
// 64-record batch).  Measured 5.08-5.18 -> 5.58-5.70 ms on C2: the second
// tap block (12.5 KiB per wave, 13 waves per CU) and the 4-wave register cap
// (accumulators moved to VGPRs) cost more than the overlap gains.
#ifndef SDP_PAD_PIPE
#define SDP_PAD_PIPE 0
#endif
// SDP_PAD_PRIO=1: s_setprio 1 around each block's K-steps (experiment)
#ifndef SDP_PAD_PRIO
#define SDP_PAD_PRIO 0
#endif
constexpr int kTapBlocks = SDP_PAD_PIPE ? 2 : 1;

template <int W, bool WS>
constexpr size_t grid_mfma_pad_lds() {
    return (size_t)mfma_tile_f2<W, WS>() * sizeof(float2) + kTapBatch * sizeof(float4) +
           (size_t)kTapBlocks * kTapBatch * kTapRec * sizeof(float);
}

// FI: the items are FineItems of sub-sorted, 4-padded coarse buckets
// (k_subsort_emit, large grids): one 2 x 8-cell group each, cell ends in o[]
template <int W, bool WS, bool FI = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SDP_PAD_PIPE ? 4 : 1, 4))) void k_grid_mfma_pad(
    Geo g, const RecC *__restrict__ recs, ItemSrc src, const unsigned *__restrict__ offs,
    const FineItem *__restrict__ fitems, float *__restrict__ grid, int p_lo, int p_hi) {
    static_assert(W <= 8, "the MFMA tiles hold 8 taps per axis");
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int RX = 2 + W - 1, RY = 8 + W - 1, PS = RX * RY;
    constexpr int NQ = WS ? W : 1;
    float4 *const stage = reinterpret_cast<float4 *>(tile + mfma_tile_f2<W, WS>());  // fu fv fw -
    float *const blk = reinterpret_cast<float *>(stage + kTapBatch);  // [kTapBatch][kTapRec]
    const uint32_t n_items = item_count(src);
    const uint32_t stride = item_stride(n_items);
    const int lane = threadIdx.x;
    const float ihw = g.inv_half_w, bl = g.beta_l2e;
    const float fbase = 1.0f - 0.5f * (float)W;  // RecC offset origin
    // tap phase: tap t = lane & 7 of records 8m + (lane >> 3)
    const int tt = lane & 7;
    const float tihw = (float)tt * ihw;
    float *const tap_dst = blk + (lane >> 3) * kTapRec;
    const int wu = (tt & 1) * 4 + (tt >> 1), wv = 8 + tt, ww = 16 + tt;
    // K-step j: record 4j + (lane >> 4); A row lane & 15 = (tu h, tv tap),
    // B column lane & 15 = (tw tap, re / im)
    const float *const kA = blk + (lane >> 4) * kTapRec + ((lane >> 3) & 1) * 4;
    const float *const kV = blk + (lane >> 4) * kTapRec + 8 + (lane & 7);
    const float *const kW = blk + (lane >> 4) * kTapRec + 16 + ((lane & 15) >> 1);
    const float *const kC = blk + (lane >> 4) * kTapRec + 24 + (lane & 1);
    const bool col_im = lane & 1;
    // accumulator element i of M-tile t: tap (2t + (lane >> 5), 4 ((lane >> 4) & 1) + i),
    // column (q, re/im) = ((lane & 15) >> 1, lane & 1)
    const int cq = (lane & 15) >> 1;
    const int ckx = lane >> 5, cky = 4 * ((lane >> 4) & 1);
    float *const ftile = reinterpret_cast<float *>(tile);

    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        Item it;
        uint32_t bnd[kGroupCell - 1];  // ends of cells 0..14 of the group (record indices)
        if (FI) {
            uint32_t fo[kGroupCell];
            it = load_fine_item<kGroupCell>(fitems, w_it, n_items, stride, fo);
            if (it.b >= it.e) continue;
#pragma unroll
            for (int c = 0; c < kGroupCell - 1; ++c) bnd[c] = fo[c];
        } else {
            it = load_item(src, w_it, n_items, stride);
            // the group's 16 cell buckets end at ob[1..16]
            const unsigned *ob = offs + ((size_t)it.p0 * g.ntiles + (size_t)it.tile * kGroupCell);
#pragma unroll
            for (int c = 0; c < kGroupCell - 1; ++c)
                bnd[c] = __builtin_amdgcn_readfirstlane(ob[c + 1]);
        }
        const int ntg = FI ? g.wny / 8 : g.nty / 8;  // groups per x pair
        const int sx = (int)it.tile / ntg, sg = (int)it.tile - sx * ntg;
        const int ibase = g.wx0 + sx * 2, jbase = g.wy0 + sg * 8;

        wave_lds_sync();
        for (int i = lane; i < NQ * PS; i += 64) tile[i] = make_float2(0.0f, 0.0f);

        floatx4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
        int cur = -1;  // cell of the accumulators (wave-uniform)
        auto flush_cell = [&]() {
            const int xo = cur & 1, yo = cur >> 1;
            if (cq < NQ) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int kx = 2 * t + ckx;
                    if (kx >= W) continue;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int ky = cky + i;
                        if (ky >= W) continue;
                        float *d = ftile + ((cq * RX + xo + kx) * RY + yo + ky) * 2 + (col_im ? 1 : 0);
                        *d += acc[t][i];
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
        };
        struct Ops {
            floatx4 a;
            float v, w, c;
        };
        auto kload = [&](int j) {
            Ops o;
            o.a = *reinterpret_cast<const floatx4 *>(kA + 4 * j * kTapRec);
            o.v = kV[4 * j * kTapRec];
            o.w = kW[4 * j * kTapRec];
            o.c = kC[4 * j * kTapRec];
            return o;
        };
        auto kmfma = [&](const Ops &o) {
            const float b = o.w * o.c;
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(o.a[t] * o.v, b, acc[t], 0, 0, 0);
        };

        RecC nx = recs[min(it.b + (uint32_t)lane, it.e - 1)];
        for (uint32_t b0 = it.b; b0 < it.e; b0 += 64) {
            const RecC my = nx;
            if (b0 + 64 < it.e) nx = recs[min(b0 + 64 + (uint32_t)lane, it.e - 1)];
            const int nb = (int)min(64u, it.e - b0);  // a multiple of 4
            // cell (x-pair-major index in the group) of the lane's record
            const uint32_t ri = b0 + (uint32_t)lane;
            int cj = 0;
#pragma unroll
            for (int c = 0; c < kGroupCell - 1; ++c) cj += ri >= bnd[c] ? 1 : 0;
            const float fu = fbase - (float)(my.lo & 0x1fffffu) * 0x1p-21f;
            const float fv = fbase - (float)((my.lo >> 21) | ((my.hi & 0x3ffu) << 11)) * 0x1p-21f;
            const float fw = fbase - (float)(my.hi >> 10) * 0x1p-22f;
            // K-steps whose cell differs from the previous K-step's (bit 4j)
            const int prev = __shfl_up(cj, 4);
            uint64_t chg = __ballot((lane & 3) == 0 && lane >= 4 && prev != cj);
            if (__builtin_amdgcn_readfirstlane(cj) != cur) chg |= 1ull;
#if SDP_PAD_PIPE
            {
                // blocks of kTapBatch records; block hb's taps live in tap block
                // hb & 1.  Block 0's taps are evaluated up front; while block hb's
                // K-steps issue, the offsets of block hb + 1 come from their lanes
                // (ds_bpermute) and its six ES chains run between the MFMAs.
                constexpr int BS = kTapBatch * kTapRec;  // floats per tap block
                const int nblk = (nb + kTapBatch - 1) / kTapBatch;
                auto put_values = [&](int hb, float *bb) {
                    if (lane / kTapBatch == hb) {
                        const int r = lane % kTapBatch;
                        *reinterpret_cast<float2 *>(bb + r * kTapRec + 24) =
                            make_float2(lane < nb ? my.cre : 0.0f, lane < nb ? my.cim : 0.0f);
                    }
                };
                float fx[2][3];
                auto fetch = [&](int hb) {
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        const int src = kTapBatch * hb + 8 * m + (lane >> 3);
                        fx[m][0] = __shfl(fu, src);
                        fx[m][1] = __shfl(fv, src);
                        fx[m][2] = __shfl(fw, src);
                    }
                };
                auto es = [&](int m, int k) {
                    return (WS || k < 2) ? es_tap<W>(fx[m][k], tihw, ihw, bl)
                                         : (tt == 0 ? 1.0f : 0.0f);
                };
                float tv_[2][3];
                auto put_taps = [&](float *bb) {
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        float *d = bb + ((lane >> 3) + 8 * m) * kTapRec;
                        d[wu] = tv_[m][0];
                        d[wv] = tv_[m][1];
                        d[ww] = tv_[m][2];
                    }
                };
                put_values(0, blk);
                fetch(0);
#pragma unroll
                for (int m = 0; m < 2; ++m)
#pragma unroll
                    for (int k = 0; k < 3; ++k) tv_[m][k] = es(m, k);
                put_taps(blk);
                wave_lds_sync();
                for (int hb = 0; hb < nblk; ++hb) {
                    const int boff = (hb & 1) * BS;
                    float *const nbuf = blk + (BS - boff);
                    const int nk = min(kTapBatch, nb - kTapBatch * hb) >> 2;
                    const uint64_t hchg = chg >> (kTapBatch * hb);
                    Ops o[kTapBatch / 4];
#pragma unroll
                    for (int jj = 0; jj < kTapBatch / 4; ++jj) {
                        o[jj].a = *reinterpret_cast<const floatx4 *>(kA + boff + 4 * jj * kTapRec);
                        o[jj].v = kV[boff + 4 * jj * kTapRec];
                        o[jj].w = kW[boff + 4 * jj * kTapRec];
                        o[jj].c = kC[boff + 4 * jj * kTapRec];
                    }
                    const bool more = hb + 1 < nblk;  // wave-uniform
                    if (more) {
                        put_values(hb + 1, nbuf);
                        fetch(hb + 1);
                    }
                    auto kstep = [&](int jj) {
                        if (jj < nk) {
                            if ((hchg >> (4 * jj)) & 1ull) {
                                if (cur >= 0) flush_cell();
                                cur = __builtin_amdgcn_readlane(cj, kTapBatch * hb + 4 * jj);
                            }
                            kmfma(o[jj]);
                        }
                    };
                    kstep(0);
                    if (more) {
                        tv_[0][0] = es(0, 0);
                        tv_[0][1] = es(0, 1);
                    }
                    kstep(1);
                    if (more) {
                        tv_[0][2] = es(0, 2);
                        tv_[1][0] = es(1, 0);
                    }
                    kstep(2);
                    if (more) tv_[1][1] = es(1, 1);
                    kstep(3);
                    if (more) {
                        tv_[1][2] = es(1, 2);
                        put_taps(nbuf);
                    }
                    wave_lds_sync();
                }
            }
            continue;
#endif
            // two halves of kTapBatch records: taps, then their K-steps
            for (int h = 0; h < 64 / kTapBatch; ++h) {
                const int nbh = min(kTapBatch, nb - kTapBatch * h);
                if (nbh <= 0) break;
                wave_lds_sync();  // previous half's tap block reads
                if (lane / kTapBatch == h) {
                    const int r = lane % kTapBatch;
                    stage[r] = make_float4(fu, fv, fw, 0.0f);
                    *reinterpret_cast<float2 *>(blk + r * kTapRec + 24) =
                        make_float2(lane < nb ? my.cre : 0.0f, lane < nb ? my.cim : 0.0f);
                }
                wave_lds_sync();
                {
                    // both staged offsets read before any tap is written: six
                    // independent ES chains
                    float4 f[kTapBatch / 8];
#pragma unroll
                    for (int m = 0; m < kTapBatch / 8; ++m) f[m] = stage[8 * m + (lane >> 3)];
                    float tv_[kTapBatch / 8][3];
#pragma unroll
                    for (int m = 0; m < kTapBatch / 8; ++m) {
                        tv_[m][0] = es_tap<W>(f[m].x, tihw, ihw, bl);
                        tv_[m][1] = es_tap<W>(f[m].y, tihw, ihw, bl);
                        tv_[m][2] = WS ? es_tap<W>(f[m].z, tihw, ihw, bl) : (tt == 0 ? 1.0f : 0.0f);
                    }
#pragma unroll
                    for (int m = 0; m < kTapBatch / 8; ++m) {
                        float *d = tap_dst + 8 * m * kTapRec;
                        d[wu] = tv_[m][0];
                        d[wv] = tv_[m][1];
                        d[ww] = tv_[m][2];
                    }
                }
                wave_lds_sync();
                const uint64_t hchg = chg >> (kTapBatch * h);
                const int nk = nbh >> 2;
#if SDP_PAD_UNROLL
                // the block's (up to) 4 K-steps unrolled: every operand read
                // up front at compile-time offsets, a cell change (bit 4j)
                // flushes the accumulators between two K-steps
                {
                    Ops o[kTapBatch / 4];
#pragma unroll
                    for (int jj = 0; jj < kTapBatch / 4; ++jj) o[jj] = kload(jj);
#if SDP_PAD_PRIO
                    __builtin_amdgcn_s_setprio(1);  // MFMA phase first among ready waves
#endif
#pragma unroll
                    for (int jj = 0; jj < kTapBatch / 4; ++jj) {
                        if (jj < nk) {
                            if ((hchg >> (4 * jj)) & 1ull) {
                                if (cur >= 0) flush_cell();
                                cur = __builtin_amdgcn_readlane(cj, kTapBatch * h + 4 * jj);
                            }
                            kmfma(o[jj]);
                        }
                    }
#if SDP_PAD_PRIO
                    __builtin_amdgcn_s_setprio(0);
#endif
                }
                continue;
#endif
                // segments of K-steps of one cell; inside a segment the operands
                // of K-step j + 1 are read before the MFMAs of K-step j issue
                int j = 0;
                while (j < nk) {
                    if ((hchg >> (4 * j)) & 1ull) {
                        if (cur >= 0) flush_cell();
                        cur = __builtin_amdgcn_readlane(cj, kTapBatch * h + 4 * j);
                    }
                    const uint64_t rest = hchg & ~((2ull << (4 * j)) - 1ull);
                    const int je = rest ? min(nk, (int)(__builtin_ctzll(rest) >> 2)) : nk;
                    Ops o = kload(j);
                    for (++j; j < je; ++j) {
                        const Ops on = kload(j);
                        kmfma(o);
                        o = on;
                    }
                    kmfma(o);
                }
            }
        }
        if (cur >= 0) flush_cell();
        wave_lds_sync();

        // flush: float f = i0 + lane of each plane's RX x RY complex cells,
        // buffer atomics off a per-plane descriptor (32-bit offsets), the
        // cell index advanced incrementally; zero floats are skipped
        constexpr int FPP = RX * RY * 2;
        const size_t plane_bytes = (size_t)g.ngx * g.ngy * sizeof(float2);
        int xl = (lane >> 1) / RY, yl = (lane >> 1) - xl * RY;
#pragma unroll
        for (int i0 = 0; i0 < FPP; i0 += 64) {
            const int f = i0 + lane;
            if (f >= FPP) break;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            const int voff = ((gx * g.ngy + gy) * 2 + (f & 1)) * (int)sizeof(float);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int p = (int)it.p0 + q;
                const float val = ftile[q * PS * 2 + f];
                if (p >= p_lo && p < p_hi && val != 0.0f) {
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        grid + (size_t)(p - p_lo) * (plane_bytes / sizeof(float)), 0,
                        (int)plane_bytes, 0x00020000);
                    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(val, rs, voff, 0, 0);
                }
            }
            yl += 32 % RY;
            xl += 32 / RY;
            if (yl >= RY) {
                yl -= RY;
                ++xl;
            }
        }
    }
}

// Register degridder (mirror of k_grid_reg): one wave per work item = a
// chunk of a group of kGroupFine consecutive 2x2-cell buckets.  The group's
// (2+W-1) x (8+W-1) x W region is staged in LDS once; per bucket, lane
// (kx, ky) loads the W plane values of its tap cell for each of the 4
// footprint origins into VGPRs (G[o][q]).  Per record the lane forms
// kk * sum_q kw[q] G[o][q] with 8 register FMAs; the 64 lanes' partials of
// 8 records are then summed with one reduce-scatter butterfly (5 lane
// exchanges per record instead of 12).  Each record belongs to exactly one
// item, so its raw sum is added to acc[] with a plain read-modify-write; the
// record factor wgt * exp(-2 pi i w s0) is applied by k_finalize.
template <int W, bool WS, bool FI>
__global__ __launch_bounds__(64) void k_degrid_reg(Geo g, const VisRec *__restrict__ recs,
                                                   ItemSrc src,
                                                   const unsigned *__restrict__ offs,
                                                   const FineItem *__restrict__ fitems,
                                                   const float2 *__restrict__ grid, int p_lo,
                                                   int p_hi, float2 *__restrict__ acc,
                                                   float2 *__restrict__ vdirect) {
    constexpr int SUB = kTileFine;
    constexpr int GRP = kGroupFine;
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    using TS = TileShape<W, SUB, SUB * GRP>;
    constexpr int RX = TS::RX, RY = TS::RY, PS = TS::PLANE;
    constexpr int NQ = WS ? W : 1;
    constexpr int NO = SUB * SUB;
    static_assert(NO == 4, "origin select below assumes 2x2-cell buckets");
    const uint32_t n_items = item_count(src);
    const uint32_t stride = item_stride(n_items);
    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        uint32_t fo[4] = {0u, 0u, 0u, 0u};
        const Item it = FI ? load_fine_item(fitems, w_it, n_items, stride, fo)
                           : load_item(src, w_it, n_items, stride);
        if (FI && it.b >= it.e) continue;
        const int lane = threadIdx.x;
        const LaneRole<W> role(lane);
        const float ihw = g.inv_half_w, bl = g.beta_l2e;
        const int ntg = g.nty / GRP;
        const int sx = (int)it.tile / ntg, sg = (int)it.tile - sx * ntg;
        const int ibase = g.wx0 + sx * SUB, jbase = g.wy0 + sg * GRP * SUB;
        const int64_t key0 = (int64_t)it.p0 * g.ntiles + (int64_t)sx * g.nty + (int64_t)sg * GRP;
        const int64_t plane_elems = (int64_t)g.ngx * g.ngy;

        // stage the region (planes outside this pass's [p_lo, p_hi) read as 0)
        for (int i = lane; i < NQ * RX * RY; i += 64) {
            const int q = i / (RX * RY);
            const int p = (int)it.p0 + q;
            const int rem = i - q * RX * RY;
            const int xl = rem / RY, yl = rem - (rem / RY) * RY;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            tile[q * PS + xl * RY + yl] =
                (p >= p_lo && p < p_hi)
                    ? grid[(int64_t)(p - p_lo) * plane_elems + (int64_t)gx * g.ngy + gy]
                    : make_float2(0.0f, 0.0f);
        }

        const float tap_t = (float)(lane & 7);
        const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
        for (int j = 0; j < GRP; ++j) {
            const uint32_t rb = FI ? (j == 0 ? it.b : fo[j - 1]) : max(it.b, offs[key0 + j]);
            const uint32_t re = FI ? fo[j] : min(it.e, offs[key0 + j + 1]);
            if (rb >= re) continue;
            const int jb = jbase + j * SUB;

            float gr[NO][NQ], gi[NO][NQ];
#pragma unroll
            for (int o = 0; o < NO; ++o) {
                const int base = (o / SUB + role.kx) * RY + j * SUB + (o % SUB) + role.ky;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const float2 v = role.act ? tile[q * PS + base] : make_float2(0.0f, 0.0f);
                    gr[o][q] = v.x;
                    gi[o][q] = v.y;
                }
            }

            for (uint32_t b0 = rb; b0 < re; b0 += 64) {
                const int n = (int)min(64u, re - b0);
                const VisRec my = recs[b0 + min(lane, n - 1)];
                const int o_l = ((int)(my.ij & 0xffffu) - ibase) * SUB + ((int)(my.ij >> 16) - jb);
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    if (8 * m >= n) break;
                    const int src = 8 * m + (lane >> 3);
                    const float tu = es_kernel(__shfl(my.fu, src) + tap_t, ihw, bl);
                    const float tv = es_kernel(__shfl(my.fv, src) + tap_t, ihw, bl);
                    const float tw = WS ? es_kernel(__shfl(my.fw, src) + tap_t, ihw, bl) : 1.0f;
                    float pr[8], pim[8];
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const int k = 8 * m + r;
                        const int o = __builtin_amdgcn_readlane(o_l, k);
                        const float ku = __shfl(tu, 8 * r + role.kx);
                        const float kv = __shfl(tv, 8 * r + role.ky);
                        float kw[NQ];
#pragma unroll
                        for (int q = 0; q < NQ; ++q) kw[q] = WS ? lane_readf(tw, 8 * r + q) : 1.0f;
                        float sr = 0.0f, si = 0.0f;
#pragma unroll
                        for (int oo = 0; oo < NO; ++oo) {
                            if (o == oo) {
#pragma unroll
                                for (int q = 0; q < NQ; ++q) {
                                    sr = fmaf(kw[q], gr[oo][q], sr);
                                    si = fmaf(kw[q], gi[oo][q], si);
                                }
                            }
                        }
                        const float kk = ku * kv;
                        pr[r] = sr * kk;
                        pim[r] = si * kk;
                    }
                    // reduce-scatter: after the xor-32/16/8 halvings lane l holds
                    // record (l >> 3) & 7 summed over 8 lanes; xor 4/2/1 finish it
                    float a4r[4], a4i[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float sr = b5 ? pr[i] : pr[i + 4], si = b5 ? pim[i] : pim[i + 4];
                        a4r[i] = (b5 ? pr[i + 4] : pr[i]) + __shfl_xor(sr, 32);
                        a4i[i] = (b5 ? pim[i + 4] : pim[i]) + __shfl_xor(si, 32);
                    }
                    float a2r[2], a2i[2];
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const float sr = b4 ? a4r[i] : a4r[i + 2], si = b4 ? a4i[i] : a4i[i + 2];
                        a2r[i] = (b4 ? a4r[i + 2] : a4r[i]) + __shfl_xor(sr, 16);
                        a2i[i] = (b4 ? a4i[i + 2] : a4i[i]) + __shfl_xor(si, 16);
                    }
                    float tr = (b3 ? a2r[1] : a2r[0]) + __shfl_xor(b3 ? a2r[0] : a2r[1], 8);
                    float ti = (b3 ? a2i[1] : a2i[0]) + __shfl_xor(b3 ? a2i[0] : a2i[1], 8);
#pragma unroll
                    for (int msk = 4; msk > 0; msk >>= 1) {
                        tr += __shfl_xor(tr, msk);
                        ti += __shfl_xor(ti, msk);
                    }
                    const int rec = 8 * m + ((lane >> 3) & 7);
                    if (vdirect) {
                        // single pass: the record factor applied here and the
                        // visibility written in place (no acc, no k_finalize)
                        const float cr = __shfl(my.cre, rec), ci = __shfl(my.cim, rec);
                        const uint32_t ix = (uint32_t)__shfl((int)my.idx, rec);
                        if ((lane & 7) == 0 && rec < n)
                            vdirect[ix] = make_float2(cr * tr - ci * ti, cr * ti + ci * tr);
                    } else if ((lane & 7) == 0 && rec < n) {
                        float2 *dst = acc + b0 + rec;
                        float2 a = *dst;
                        a.x += tr;
                        a.y += ti;
                        *dst = a;
                    }
                }
            }
        }
    }
}

// MFMA degridder (predict) on one-cell buckets: the adjoint of
// k_grid_mfma_pad's GEMM.  All records of a cell share their footprint
// origin, so for 16 records of one cell
//   D[(q, re/im), r] = sum_(kx,ky) G[q][xo + kx][yo + ky] . tu_r[kx] tv_r[ky]
// is one 16 x 16 x 64 GEMM (16 K-steps of v_mfma_f32_16x16x4_f32, exact fp32):
// A = the cell's footprint of the W planes (row (q, re/im), held in 16
// VGPRs per lane while the cell lasts), B = the records' separable (u, v)
// taps (column = record).  K-step s covers taps (kx, ky) = (s >> 1,
// 4 (s & 1) + k), k = lane >> 4.  The w taps then weight the rows:
// V_r = sum_q tw_r[q] D[(q, .), r], a 4-lane-group reduction.  The 24 taps
// of a record are evaluated once, 6 by each of its 4 lanes (lane group k:
// tu 2k, 2k+1; tv k, k+4; tw 2k, 2k+1), the tu taps shared by ds_bpermute.
// One wave per work item (a chunk of a group of 16 cells, a 2 x 8-cell
// region whose W planes are staged in LDS once).  The record factor
// wgt * exp(-2 pi i w s0) is applied and the visibility written in place
// (vdirect), or the raw sum added to acc[record] for k_finalize.
template <int W, bool WS, bool FI>
__global__ __launch_bounds__(64) void k_degrid_mfma(Geo g, const VisRec *__restrict__ recs,
                                                    ItemSrc src, const unsigned *__restrict__ offs,
                                                    const FineItem *__restrict__ fitems,
                                                    const float2 *__restrict__ grid, int p_lo,
                                                    int p_hi, float2 *__restrict__ acc,
                                                    float2 *__restrict__ vdirect) {
    static_assert(W <= 8, "the MFMA tiles hold 8 taps per axis");
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int RX = 2 + W - 1, RY = 8 + W - 1, PS = RX * RY;
    constexpr int NQ = WS ? W : 1;
    const uint32_t n_items = item_count(src);
    const uint32_t stride = item_stride(n_items);
    const int lane = threadIdx.x;
    const int r16 = lane & 15, kg = lane >> 4;
    const float ihw = g.inv_half_w, bl = g.beta_l2e;
    const int aq = r16 >> 1, aim = r16 & 1;  // A row (q, re/im)
    const float tu0 = (float)(2 * kg) * ihw, tu1 = (float)(2 * kg + 1) * ihw;
    const float tv0 = (float)kg * ihw, tv1 = (float)(kg + 4) * ihw;
    const float *const ftile = reinterpret_cast<const float *>(tile);
    const int64_t plane_elems = (int64_t)g.ngx * g.ngy;

    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        uint32_t fo[kGroupCell];
        Item it;
        if (FI) {
            it = load_fine_item<kGroupCell>(fitems, w_it, n_items, stride, fo);
            if (it.b >= it.e) continue;
        } else {
            it = load_item(src, w_it, n_items, stride);
            const unsigned *ob = offs + ((size_t)it.p0 * g.ntiles + (size_t)it.tile * kGroupCell);
#pragma unroll
            for (int c = 0; c < kGroupCell; ++c) fo[c] = __builtin_amdgcn_readfirstlane(ob[c + 1]);
        }
        const int ntg = FI ? g.wny / 8 : g.nty / 8;  // groups per x pair
        const int sx = (int)it.tile / ntg, sg = (int)it.tile - sx * ntg;
        const int ibase = g.wx0 + sx * 2, jbase = g.wy0 + sg * 8;

        // the item's first 16 records are requested before the region is
        // staged (both depend only on the item descriptor)
        uint32_t pf = it.b;
        VisRec nxt = recs[min(pf + (uint32_t)r16, it.e - 1)];
        wave_sync_1w();  // previous item's reads of the region
        for (int i = lane; i < NQ * PS; i += 64) {
            const int q = i / PS;
            const int p = (int)it.p0 + q;
            const int rem = i - q * PS;
            const int xl = rem / RY, yl = rem - (rem / RY) * RY;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            tile[i] = (p >= p_lo && p < p_hi)
                          ? grid[(int64_t)(p - p_lo) * plane_elems + (int64_t)gx * g.ngy + gy]
                          : make_float2(0.0f, 0.0f);
        }
        wave_sync_1w();

        // the item's cells are consecutive, so the batch after [b0, b0 + 16)
        // starts at min(b0 + 16, re) -- in the next cell when this one ends;
        // its records are loaded one batch ahead (pf = the prefetched start)
        uint32_t cb = it.b;  // start of cell c's records (clipped to the item)
        for (int c = 0; c < kGroupCell; ++c) {
            const uint32_t rb = max(cb, it.b), re = min(fo[c], it.e);
            cb = fo[c];
            if (rb >= re) continue;
            const int xo = c & 1, yo = c >> 1;
            float a[16];
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const int kx = s >> 1, ky = 4 * (s & 1) + kg;
                a[s] = (aq < NQ && kx < W && ky < W)
                           ? ftile[((aq * RX + xo + kx) * RY + yo + ky) * 2 + aim]
                           : 0.0f;
            }
            for (uint32_t b0 = rb; b0 < re; b0 += 16) {
                const uint32_t ri = b0 + (uint32_t)r16;
                if (pf != b0) nxt = recs[min(ri, it.e - 1)];  // (wave-uniform; not expected)
                const VisRec rec = nxt;
                pf = min(b0 + 16, re);
                nxt = recs[min(pf + (uint32_t)r16, it.e - 1)];
                const float u0 = es_tap<W>(rec.fu, tu0, ihw, bl);
                const float u1 = es_tap<W>(rec.fu, tu1, ihw, bl);
                const float v0 = es_tap<W>(rec.fv, tv0, ihw, bl);
                const float v1 = es_tap<W>(rec.fv, tv1, ihw, bl);
                const float w0 = WS ? es_tap<W>(rec.fw, tu0, ihw, bl) : (kg == 0 ? 1.0f : 0.0f);
                const float w1 = WS ? es_tap<W>(rec.fw, tu1, ihw, bl) : 0.0f;
                float tu[8];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    tu[2 * h] = __shfl(u0, r16 + 16 * h);
                    tu[2 * h + 1] = __shfl(u1, r16 + 16 * h);
                }
                floatx4 d0 = floatx4{0.0f, 0.0f, 0.0f, 0.0f}, d1 = d0;
#pragma unroll
                for (int s = 0; s < 16; s += 2) {
                    d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], tu[s >> 1] * v0, d0, 0, 0, 0);
                    d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s + 1], tu[s >> 1] * v1, d1, 0, 0, 0);
                }
                // row 4 kg + i of D = (q = 2 kg + (i >> 1), re/im = i & 1)
                float sr = w0 * (d0[0] + d1[0]) + w1 * (d0[2] + d1[2]);
                float si = w0 * (d0[1] + d1[1]) + w1 * (d0[3] + d1[3]);
                sr += __shfl_xor(sr, 16);
                si += __shfl_xor(si, 16);
                sr += __shfl_xor(sr, 32);
                si += __shfl_xor(si, 32);
                if (kg == 0 && ri < re) {
                    if (vdirect) {
                        vdirect[rec.idx] =
                            make_float2(rec.cre * sr - rec.cim * si, rec.cre * si + rec.cim * sr);
                    } else {
                        float2 *dst = acc + ri;
                        float2 v = *dst;
                        v.x += sr;
                        v.y += si;
                        *dst = v;
                    }
                }
            }
        }
    }
}

// Degridder: one wave per work item (an SX x SY-cell region: a 16x16 tile or
// a group of kGroupFine 2x2 buckets).  The region's W planes are loaded into
// LDS; per record, lane (kx, ky) reads its tap's W plane values, and a wave
// reduction sums the footprint.
template <int W, bool WS, int SX, int SY>
__global__ __launch_bounds__(64) void k_degrid(Geo g, const VisRec *__restrict__ recs,
                                               ItemSrc src,
                                               const float2 *__restrict__ grid, int p_lo,
                                               int p_hi, float2 *acc) {
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    using TS = TileShape<W, SX, SY>;
    constexpr int RX = TS::RX, RY = TS::RY, PS = TS::PLANE, PITCH = TS::PITCH;
    constexpr int NQ = WS ? W : 1;
    const uint32_t n_items = item_count(src);
    const uint32_t stride = item_stride(n_items);
    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        const Item it = load_item(src, w_it, n_items, stride);
        const int ntg = g.nty / g.grp;
        const int tx = (int)it.tile / ntg, tg = (int)it.tile - tx * ntg;
        const int ibase = g.wx0 + tx * SX, jbase = g.wy0 + tg * SY;
        const int64_t plane_elems = (int64_t)g.ngx * g.ngy;
        const int lane = threadIdx.x;
        for (int i = lane; i < NQ * RX * RY; i += 64) {
            const int q = i / (RX * RY);
            const int p = (int)it.p0 + q;
            const int rem = i - q * RX * RY;
            const int xl = rem / RY, yl = rem - (rem / RY) * RY;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            tile[q * PS + xl * PITCH + yl] =
                (p >= p_lo && p < p_hi)
                    ? grid[(int64_t)(p - p_lo) * plane_elems + (int64_t)gx * g.ngy + gy]
                    : make_float2(0.0f, 0.0f);
        }

        const LaneRole<W> role(lane);
        const float ihw = g.inv_half_w, bl = g.beta_l2e;
        const int lane_off = role.kx * PITCH + role.ky - ibase * PITCH - jbase;
        for (uint32_t b0 = it.b; b0 < it.e; b0 += 64) {
            const int n = (int)min(64u, it.e - b0);
            const VisRec my = recs[b0 + min(lane, n - 1)];
            float mine_r = 0.0f, mine_i = 0.0f;
            for (int k = 0; k < n; ++k) {
                const RecRegs rc = rec_at(my, k);
                const float kval = role.taps(rc, ihw, bl);
                const float ku = __shfl(kval, role.kx);
                const float kv = __shfl(kval, W + role.ky);
                const int off = lane_off + (int)(rc.ij & 0xffffu) * PITCH + (int)(rc.ij >> 16);
                float kw[NQ];
#pragma unroll
                for (int q = 0; q < NQ; ++q) kw[q] = WS ? lane_readf(kval, 2 * W + q) : 1.0f;
                float sr = 0.0f, si = 0.0f;
                if (role.act) {
                    float2 a[NQ];
#pragma unroll
                    for (int q = 0; q < NQ; ++q) a[q] = tile[q * PS + off];
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        sr = fmaf(kw[q], a[q].x, sr);
                        si = fmaf(kw[q], a[q].y, si);
                    }
                }
                const float kk = role.act ? ku * kv : 0.0f;
                sr *= kk;
                si *= kk;
                for (int o = 32; o > 0; o >>= 1) {
                    sr += __shfl_xor(sr, o);
                    si += __shfl_xor(si, o);
                }
                if (k == lane) {
                    mine_r = sr;
                    mine_i = si;
                }
            }
            if (lane < n) {
                atomicAdd(&acc[b0 + lane].x, mine_r);
                atomicAdd(&acc[b0 + lane].y, mine_i);
            }
        }
    }
}

// ------------------------------------------------------------------------
// kernels: image-domain w screens and grid correction
// ------------------------------------------------------------------------
struct PixelGeom {
    int gx, gy;
    double corr, s;
    bool inside;
};

__device__ __forceinline__ PixelGeom pixel_geom(const Geo &g, int ix, int iy,
                                                const double *__restrict__ tab) {
    PixelGeom p;
    const int X = ix - g.nx / 2, Y = iy - g.ny / 2;
    p.gx = X < 0 ? X + g.ngx : X;
    p.gy = Y < 0 ? Y + g.ngy : Y;
    const double l = X * g.px, m = Y * g.py;
    const double r2 = l * l + m * m;
    p.inside = !g.do_w || r2 < 1.0;
    p.corr = 1.0 / (phi_lookup(tab, (double)X / g.ngx) * phi_lookup(tab, (double)Y / g.ngy));
    p.s = 0.0;
    if (g.do_w && p.inside) {
        const double nm1 = -r2 / (sqrt(1.0 - r2) + 1.0);
        p.s = -nm1 - g.s0;
        p.corr /= phi_lookup(tab, g.dw * p.s) * (nm1 + 1.0);
    }
    if ((X + Y) & 1) p.corr = -p.corr;  // centred-grid storage
    return p;
}

// ---- transposed y-spectrum layout for the pruned 2-D FFT -------------
// T[q][iy][kx] (iy = image row index 0..ny-1, i.e. ky = (iy - ny/2) mod ngy;
// kx = 0..ngx-1) holds, per plane, the needed y-frequency columns of the grid
// transposed so the x-direction transform runs over contiguous rows.
constexpr int kTr = 64;      // transpose tile edge
constexpr int kTrRows = 4;   // threads along the tile's second axis (64 x 4 = 256)

// grid[q][x][ky(iy)] -> T[q][iy][x] for the rows x in [row_lo, row_hi); the
// rest of each T row is kept zero by the caller (persistent zeros)
__global__ __launch_bounds__(256) void k_tr_grid_to_t(Geo g, const float2 *__restrict__ grid,
                                                      float2 *__restrict__ t, int row_lo,
                                                      int row_hi) {
    __shared__ float2 sm[kTr][kTr + 1];
    const int x0 = row_lo + blockIdx.x * kTr, i0 = blockIdx.y * kTr, q = blockIdx.z;
    const int64_t plane = (int64_t)g.ngx * g.ngy, tplane = (int64_t)g.ny * g.ngx;
    for (int r = threadIdx.y; r < kTr; r += kTrRows) {
        const int x = x0 + r, iy = i0 + threadIdx.x;
        float2 v = make_float2(0.0f, 0.0f);
        if (x < row_hi && iy < g.ny) {
            const int Y = iy - g.ny / 2;
            const int ky = Y < 0 ? Y + g.ngy : Y;
            v = grid[q * plane + (int64_t)x * g.ngy + ky];
        }
        sm[r][threadIdx.x] = v;
    }
    __syncthreads();
    for (int r = threadIdx.y; r < kTr; r += kTrRows) {
        const int iy = i0 + r, x = x0 + threadIdx.x;
        if (iy < g.ny && x < row_hi) t[q * tplane + (int64_t)iy * g.ngx + x] = sm[threadIdx.x][r];
    }
}

// T[q][iy][x] -> grid[q][x][ky(iy)] for the rows x in [row_lo, row_hi)
__global__ __launch_bounds__(256) void k_tr_t_to_grid(Geo g, const float2 *__restrict__ t,
                                                      float2 *__restrict__ grid, int row_lo,
                                                      int row_hi) {
    __shared__ float2 sm[kTr][kTr + 1];
    const int x0 = row_lo + blockIdx.x * kTr, i0 = blockIdx.y * kTr, q = blockIdx.z;
    const int64_t plane = (int64_t)g.ngx * g.ngy, tplane = (int64_t)g.ny * g.ngx;
    for (int r = threadIdx.y; r < kTr; r += kTrRows) {
        const int iy = i0 + r, x = x0 + threadIdx.x;
        sm[r][threadIdx.x] = (iy < g.ny && x < row_hi) ? t[q * tplane + (int64_t)iy * g.ngx + x]
                                                       : make_float2(0.0f, 0.0f);
    }
    __syncthreads();
    for (int r = threadIdx.y; r < kTr; r += kTrRows) {
        const int x = x0 + r, iy = i0 + threadIdx.x;
        if (x < row_hi && iy < g.ny) {
            const int Y = iy - g.ny / 2;
            const int ky = Y < 0 ? Y + g.ngy : Y;
            grid[q * plane + (int64_t)x * g.ngy + ky] = sm[threadIdx.x][r];
        }
    }
}

// w screens + grid correction reading the transposed spectrum (ix fastest:
// coalesced T reads; RASCIL's transposed output (sx = 1) is coalesced too)
__global__ void k_screen_fwd_t(Geo g, const float2 *__restrict__ t, int p_begin, int np,
                               double *dirty, int64_t sx, int64_t sy, int accumulate,
                               const double *__restrict__ tab) {
    const int ix = blockIdx.x * blockDim.x + threadIdx.x;
    const int iy = blockIdx.y;
    if (ix >= g.nx) return;
    const PixelGeom p = pixel_geom(g, ix, iy, tab);
    double res = 0.0;
    if (p.inside) {
        const int64_t tplane = (int64_t)g.ny * g.ngx;
        const float2 *src = t + (int64_t)iy * g.ngx + p.gx;
        if (g.do_w) {
            double acc = 0.0;
            for (int q = 0; q < np; ++q) {
                const float2 h = src[q * tplane];
                double ph = (g.w0 + (p_begin + q) * g.dw) * p.s;
                ph -= rint(ph);
                float sn, cs;
                sincospif((float)(2.0 * ph), &sn, &cs);
                acc += (double)h.x * cs - (double)h.y * sn;
            }
            res = acc * p.corr;
        } else {
            res = (double)src[0].x * p.corr;
        }
    }
    double *o = dirty + ix * sx + iy * sy;
    *o = accumulate ? *o + res : res;
}

// adjoint: T[q][iy][kx] = screen(q) * corr * dirty for kx in the image's
// x-frequencies, 0 for the other kx (full rows are written)
__global__ void k_screen_adj_t(Geo g, const double *__restrict__ dirty, int64_t sx, int64_t sy,
                               int p_begin, int np, float2 *__restrict__ t,
                               const double *__restrict__ tab) {
    const int kx = blockIdx.x * blockDim.x + threadIdx.x;
    const int iy = blockIdx.y;
    if (kx >= g.ngx) return;
    const int X = kx < g.ngx / 2 ? kx : kx - g.ngx;
    const int ix = X + g.nx / 2;
    const int64_t tplane = (int64_t)g.ny * g.ngx;
    float2 *dst = t + (int64_t)iy * g.ngx + kx;
    if (ix < 0 || ix >= g.nx) {
        for (int q = 0; q < np; ++q) dst[q * tplane] = make_float2(0.0f, 0.0f);
        return;
    }
    const PixelGeom p = pixel_geom(g, ix, iy, tab);
    const double val = p.inside ? dirty[ix * sx + iy * sy] * p.corr : 0.0;
    if (g.do_w) {
        for (int q = 0; q < np; ++q) {
            double ph = (g.w0 + (p_begin + q) * g.dw) * p.s;
            ph -= rint(ph);
            float sn, cs;
            sincospif((float)(2.0 * ph), &sn, &cs);
            dst[q * tplane] = make_float2((float)(val * cs), (float)(-val * sn));
        }
    } else {
        dst[0] = make_float2((float)val, 0.0f);
    }
}

__device__ __forceinline__ void store_vis(float2 *p, float2 v, int accumulate) {
    if (accumulate) {
        const float2 o = *p;
        v.x += o.x;
        v.y += o.y;
    }
    *p = v;
}
__device__ __forceinline__ void store_vis(double2 *p, float2 v, int accumulate) {
    double2 w = make_double2(v.x, v.y);
    if (accumulate) {
        const double2 o = *p;
        w.x += o.x;
        w.y += o.y;
    }
    *p = w;
}
__device__ __forceinline__ void store_vis_d(float2 *p, double xr, double xi, int accumulate) {
    float2 w = make_float2((float)xr, (float)xi);
    if (accumulate) {
        const float2 o = *p;
        w.x += o.x;
        w.y += o.y;
    }
    *p = w;
}
__device__ __forceinline__ void store_vis_d(double2 *p, double xr, double xi, int accumulate) {
    double2 w = make_double2(xr, xi);
    if (accumulate) {
        const double2 o = *p;
        w.x += o.x;
        w.y += o.y;
    }
    *p = w;
}

// Predict-side pol conversion (sdp_hip_dirty2ms_vis, reference
// imaging/ng.py:131-136): the degridded image-pol visibility x goes to every
// output pol v as coef_v * x.  Disabled (npv 1, coef 1) for sdp_hip_dirty2ms.
struct OutConv {
    int npv = 1;
    int64_t vps = 0;
    double cre[4] = {1.0, 0.0, 0.0, 0.0}, cim[4] = {0.0, 0.0, 0.0, 0.0};
};

template <class VT>
__global__ void k_zero_vis(int64_t nrow, int nchan, VT *vis, int64_t vrs, int64_t vcs,
                           OutConv oc) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= nrow * nchan) return;
    const int64_t row = v / nchan;
    const int chan = (int)(v - row * nchan);
    VT z;
    z.x = 0;
    z.y = 0;
    for (int k = 0; k < oc.npv; ++k) vis[row * vrs + chan * vcs + k * oc.vps] = z;
}

// record factor and scatter back to visibility order; the record count is
// read from device memory when `ndev` is given (pipelined plans)
template <class VT>
__global__ void k_finalize(int64_t nrec, const unsigned *__restrict__ ndev, int nchan,
                           const VisRec *__restrict__ recs, const float2 *__restrict__ acc, VT *vis,
                           int64_t vrs, int64_t vcs, int accumulate, OutConv oc) {
    const int64_t n = ndev ? (int64_t)*ndev : nrec;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const VisRec rc = recs[r];
        const float2 a = acc[r];
        const float2 v = make_float2(rc.cre * a.x - rc.cim * a.y, rc.cre * a.y + rc.cim * a.x);
        const int64_t row = rc.idx / (uint32_t)nchan;
        const int chan = (int)(rc.idx - row * nchan);
        VT *p = vis + row * vrs + chan * vcs;
        if (oc.npv == 1 && oc.cre[0] == 1.0 && oc.cim[0] == 0.0) {
            store_vis(p, v, accumulate);
            continue;
        }
        for (int k = 0; k < oc.npv; ++k) {
            if (oc.cre[k] == 0.0 && oc.cim[k] == 0.0) continue;
            const double xr = oc.cre[k] * v.x - oc.cim[k] * v.y;
            const double xi = oc.cre[k] * v.y + oc.cim[k] * v.x;
            store_vis_d(p + k * oc.vps, xr, xi, accumulate);
        }
    }
}

// ------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------
static double es_kernel_host(double t, int W, double beta) {
    const double x = 2.0 * t / W;
    const double y = 1.0 - x * x;
    return y > 0.0 ? std::exp(beta * (std::sqrt(y) - 1.0)) : 0.0;
}

static void gauss_legendre(int n, std::vector<double> &x, std::vector<double> &w) {
    x.resize(n);
    w.resize(n);
    for (int i = 0; i < n; ++i) {
        double z = std::cos(M_PI * (i + 0.75) / (n + 0.5));
        double dp = 1.0;
        for (int it = 0; it < 100; ++it) {
            double p0 = 1.0, p1 = 0.0;
            for (int k = 1; k <= n; ++k) {
                const double p2 = p1;
                p1 = p0;
                p0 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p2) / k;
            }
            dp = n * (z * p0 - p1) / (z * z - 1.0);
            const double dz = p0 / dp;
            z -= dz;
            if (std::fabs(dz) < 1e-16) break;
        }
        x[i] = z;
        w[i] = 2.0 / ((1.0 - z * z) * dp * dp);
    }
}

// Phi(xi) = int_{-W/2}^{W/2} phi(t) cos(2 pi t xi) dt on xi in [0, 0.5].
static const double *phi_table(int W, double beta, hipStream_t stream) {
    static std::mutex mu;
    static std::map<int, std::vector<double>> cache;
    const std::vector<double> *tab;
    {
        std::lock_guard<std::mutex> lk(mu);
        std::vector<double> &t = cache[W];
        if (t.empty()) {
            std::vector<double> z, wq;
            gauss_legendre(128, z, wq);
            t.resize(kPhiTab);
            for (int k = 0; k < kPhiTab; ++k) {
                const double xi = 0.5 * k / (kPhiTab - 1);
                double s = 0.0;
                for (int i = 0; i < 128; ++i) {
                    const double tt = 0.25 * W * (z[i] + 1.0);
                    s += 0.25 * W * wq[i] * es_kernel_host(tt, W, beta) *
                         std::cos(2.0 * M_PI * tt * xi);
                }
                t[k] = 2.0 * s;
            }
        }
        tab = &t;
    }
    double *d = scratch<double>("phi_tab_W" + std::to_string(W), kPhiTab);
    SDP_HIP_CHECK(hipMemcpyAsync(d, tab->data(), kPhiTab * sizeof(double),
                                 hipMemcpyHostToDevice, stream));
    return d;
}

// Cached hipFFT plans: 1-D c2c of length n over `batch` transforms whose
// elements are `stride` apart and whose starts are `dist` apart.
static hipfftHandle fft_plan_1d(int n, int stride, int dist, int batch, hipStream_t stream) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, int, int>, hipfftHandle> plans;
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_tuple(dev, n, stride, dist, batch);
    auto itp = plans.find(key);
    hipfftHandle h;
    if (itp == plans.end()) {
        int nn[1] = {n};
        if (hipfftPlanMany(&h, 1, nn, nn, stride, dist, nn, stride, dist, HIPFFT_C2C, batch) !=
            HIPFFT_SUCCESS)
            throw Error(SDP_HIP_ERR_RUNTIME, "hipfftPlanMany failed");
        plans[key] = h;
    } else {
        h = itp->second;
    }
    if (hipfftSetStream(h, stream) != HIPFFT_SUCCESS)
        throw Error(SDP_HIP_ERR_RUNTIME, "hipfftSetStream failed");
    return h;
}

static double ord_dec(unsigned long long u) {
    const long long i = (u & 0x8000000000000000ull) ? (long long)(u & 0x7fffffffffffffffull)
                                                    : (long long)~u;
    double d;
    std::memcpy(&d, &i, sizeof(d));
    return d;
}

static int kernel_support(double epsilon) {
    const double eps = std::max(epsilon, 1.0e-7);
    const int W = (int)std::ceil(-std::log10(eps / 10.0) - 1e-9);
    return std::min(std::max(W, 2), kMaxW);
}

// Pinned host staging for the plan's small device->host reads (pageable
// destinations go through a slow staging copy).  Byte offset `off` into a
// per-device 1 MiB buffer; the plan uses [0, 64) and [64, ...).
template <class T>
static T *pinned_host(size_t off, size_t count) {
    static std::mutex mu;
    static std::map<int, char *> bufs;
    constexpr size_t kBytes = 1 << 20;
    SDP_REQUIRE(off + count * sizeof(T) <= kBytes, "plan metadata too large");
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    char *&b = bufs[dev];
    if (!b) SDP_HIP_CHECK(hipHostMalloc((void **)&b, kBytes, hipHostMallocDefault));
    return reinterpret_cast<T *>(b + off);
}

static bool g_stage_timing = false;

struct StageTimer {
    hipStream_t s;
    bool on;
    hipEvent_t ev[8];
    int n = 0;
    explicit StageTimer(hipStream_t st) : s(st), on(g_stage_timing) {
        if (on)
            for (auto &e : ev) SDP_HIP_CHECK(hipEventCreate(&e));
    }
    void mark() {
        if (on && n < 8) SDP_HIP_CHECK(hipEventRecord(ev[n++], s));
    }
    float ms(int a, int b) {
        if (!on || b >= n) return 0.0f;
        float t = 0.0f;
        SDP_HIP_CHECK(hipEventSynchronize(ev[b]));
        SDP_HIP_CHECK(hipEventElapsedTime(&t, ev[a], ev[b]));
        return t;
    }
    ~StageTimer() {
        if (on)
            for (auto &e : ev) (void)hipEventDestroy(e);
    }
};

// One visibility part: a contiguous row range with its own buckets and work
// items.  Its records occupy recs[vbase, vbase + nvis) of the call's record
// array (positions are part-local offsets).
struct Part {
    int64_t r0 = 0, r1 = 0, vbase = 0, nvis = 0;
    unsigned *hist = nullptr, *offs = nullptr, *nch = nullptr, *ioffs = nullptr;
    unsigned long long *nbad = nullptr;
    unsigned *npad = nullptr;  // pad records of a 4-padded plan (device)
    Item *items = nullptr;
    FineItem *fitems = nullptr;  // 16 per item when sub-sorted (k_subsort)
    RecC *precs = nullptr;       // sub-sorted, 4-padded 16-B records (subpad plans)
    FineItem *pfitems = nullptr;  // FineItems over precs
    unsigned *meta = nullptr;  // device: see k_part_meta
    // host copies (filled by read_part_meta; synchronous plans only)
    int64_t nrec = 0, nitems = 0;
    std::vector<unsigned> p0_items;
};

struct Plan {
    Geo g;
    VisRec *recs = nullptr;
    std::vector<Part> parts;
    bool pipelined = false;          // row parts, persistent launches, no host syncs
    bool aux_bucketing = false;      // bucketing on the auxiliary stream
    bool subsort = false;            // 16x16 buckets re-ordered to 2x2 (register kernels)
    bool cells = false;              // invert on k_grid_mfma: one-cell buckets / sub-sort
    bool pad4 = false;               // one-cell buckets padded to 4 records (k_grid_mfma_pad)
    bool subpad = false;             // sub-sorted coarse items re-written 4-padded (k_grid_mfma_pad FI)
    float2 *vdirect = nullptr;       // dirty2ms: register degridders write c64 vis in place
    int chunk_planes = 1;            // planes resident per pass
    int fft_planes = 1;              // planes per FFT / screen batch (spec, spec_in)
    int row_lo = 0, row_hi = 0;      // grid rows (x) the visibilities reach
    unsigned chunk = kChunkMin;      // max records per work item
    int64_t nrec = 0, nitems = 0;    // totals
    float2 *grid = nullptr;
    float2 *spec = nullptr;     // T[q][iy][kx]: transposed y-spectra (pruned FFT)
    float2 *spec_in = nullptr;  // band-only input of the backward x-FFT (zeros elsewhere)
};

struct Inputs {
    const double *uvw;
    int64_t uvw_rs;
    const double *freq;
    int nchan;
    int64_t nrow;
    const void *vis;
    int vis_dtype;
    int64_t vrs, vcs;
    const void *wgt;  // f32, or f64 when x.wgt_f64
    int64_t wrs, wcs;
    int nx, ny;
    double px, py;
    double eps;
    int do_w;
    unsigned flags;
    VisExtra x{};
    // batched invert (sdp_hip_ms2dirty_batch): host {min w, max w, max |u|,
    // max |v|} in metres (uvw as given, before FLIP_UW) and {fmin, fmax} of
    // every batch of the sequence, so all batches share one plane layout
    const double *bounds = nullptr;
};

// Bytes of w planes kept resident per pass: SDP_HIP_GRID_BUDGET_GB if set,
// else the device memory this call can still use -- free memory plus what the
// workspace already holds for the planes and the records, less the records
// and key/rank arrays still to be allocated (`need_other`) and a reserve of
// 6 GiB.  A C2 invert keeps its 9 planes resident, and so does a C4 shard
// (70 planes of 16384^2, 150 GB) on a 288 GB MI355X, gridding every record
// once instead of once per plane chunk.
static size_t grid_budget_bytes(size_t need_other) {
    const char *e = std::getenv("SDP_HIP_GRID_BUDGET_GB");
    if (e && std::atof(e) > 0) return (size_t)(std::atof(e) * 1073741824.0);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b == 0) return (size_t)8 << 30;
    Workspace &ws = Workspace::get();
    const size_t held_planes = ws.held("grid") + ws.held("spec") + ws.held("spec_in");
    const size_t held_other = ws.held("recs") + ws.held("key_rank") + ws.held("degrid_acc") +
                              ws.held("precs#0") + ws.held("pfitems#0");
    const size_t avail = free_b + held_planes + held_other;
    const size_t reserve = (size_t)6 << 30;
    const size_t need = need_other + reserve;
    return avail > need ? avail - need : (size_t)1 << 30;
}

// SDP_HIP_PIPELINE: 0 (default) = bucket on the caller's stream; 1 = dirty2ms
// buckets on an auxiliary stream under its screen + FFT; 2 = additionally
// split the rows in two parts bucketed on the auxiliary stream while the
// previous part (de)grids, with persistent launches reading the device-side
// item counts.  Both overlaps measured slower on C2: the
// bucketing is memory/atomic bound and contends with the FFT, and the row
// halves add 24% work items.
constexpr int kPipelineParts = 2;

static hipStream_t aux_stream() {
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    auto it = streams.find(dev);
    if (it != streams.end()) return it->second;
    hipStream_t s;
    SDP_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    streams[dev] = s;
    return s;
}

// The backward x-FFT input T_in holds the transposed band [row_lo, row_hi)
// of every T row and zeros elsewhere.  The transpose writes only the band,
// so the zeros are kept across calls: the buffer is cleared only when it is
// (re)allocated or the band / shape changes.
struct BandState {
    float2 *ptr = nullptr;
    size_t elems = 0;
    int lo = -1, hi = -1, ny = 0, ngx = 0;
};

static float2 *band_input(const Plan &P, hipStream_t st) {
    static std::mutex mu;
    static std::map<int, BandState> states;
    const Geo &g = P.g;
    const size_t elems = (size_t)P.fft_planes * g.ny * g.ngx;
    float2 *buf = scratch<float2>("spec_in", elems);
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    BandState &b = states[dev];
    if (b.ptr != buf || b.elems < elems || b.lo != P.row_lo || b.hi != P.row_hi || b.ny != g.ny ||
        b.ngx != g.ngx) {
        SDP_HIP_CHECK(hipMemsetAsync(buf, 0, elems * sizeof(float2), st));
        b = BandState{buf, elems, P.row_lo, P.row_hi, g.ny, g.ngx};
    }
    return buf;
}

// Bucketing kept by an SDP_HIP_KEEP_BUCKETS invert for SDP_HIP_REUSE_BUCKETS
// calls (invert_ng's other polarisations): the plan (its scratch pointers and
// host metadata), the workspace generation it is valid under, and the
// arguments the bucketing depends on.  Every fresh plan drops it.
struct KeptBuckets {
    bool valid = false;
    uint64_t gen = 0;
    const double *uvw = nullptr, *freq = nullptr;
    int64_t uvw_rs = 0, nrow = 0;
    int nchan = 0, nx = 0, ny = 0, do_w = 0;
    double px = 0, py = 0, eps = 0;
    unsigned flip = 0;
    Plan P;
};

static std::mutex g_kept_mu;
static std::map<int, KeptBuckets> g_kept;

static KeptBuckets &kept_buckets() {
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    return g_kept[dev];
}

static void drop_kept_buckets() {
    std::lock_guard<std::mutex> lk(g_kept_mu);
    kept_buckets().valid = false;
}

static void keep_buckets(const Plan &P, const Inputs &in) {
    std::lock_guard<std::mutex> lk(g_kept_mu);
    KeptBuckets &k = kept_buckets();
    k.valid = true;
    k.gen = Workspace::get().generation();
    k.uvw = in.uvw;
    k.freq = in.freq;
    k.uvw_rs = in.uvw_rs;
    k.nrow = in.nrow;
    k.nchan = in.nchan;
    k.nx = in.nx;
    k.ny = in.ny;
    k.do_w = in.do_w;
    k.px = in.px;
    k.py = in.py;
    k.eps = in.eps;
    k.flip = in.flags & SDP_HIP_FLIP_UW;
    k.P = P;
}

static Plan reuse_buckets(const Inputs &in) {
    std::lock_guard<std::mutex> lk(g_kept_mu);
    const KeptBuckets &k = kept_buckets();
    SDP_REQUIRE(k.valid && k.gen == Workspace::get().generation(),
                "SDP_HIP_REUSE_BUCKETS: no kept bucketing (another wstack call or a workspace "
                "release came in between)");
    SDP_REQUIRE(k.uvw == in.uvw && k.freq == in.freq && k.uvw_rs == in.uvw_rs &&
                    k.nrow == in.nrow && k.nchan == in.nchan && k.nx == in.nx &&
                    k.ny == in.ny && k.do_w == in.do_w && k.px == in.px && k.py == in.py &&
                    k.eps == in.eps && k.flip == (in.flags & SDP_HIP_FLIP_UW),
                "SDP_HIP_REUSE_BUCKETS: uvw, freq and the geometry must be those of the "
                "SDP_HIP_KEEP_BUCKETS call");
    return k.P;
}

// Geometry shared by both directions: kernel, padded grid, w planes, bucket
// granularity, row band, plane chunking, part split.  One host sync (uvw and
// frequency extremes).
static Plan plan_geometry(const Inputs &in, bool grid_mode, hipStream_t st) {
    SDP_REQUIRE(in.nx > 0 && in.ny > 0 && in.nx % 2 == 0 && in.ny % 2 == 0,
                "npix_x and npix_y must be positive and even");
    SDP_REQUIRE(in.px > 0 && in.py > 0, "pixel sizes must be positive");
    SDP_REQUIRE(in.nchan > 0 && in.nrow >= 0, "nchan must be positive");
    SDP_REQUIRE(in.nrow * (int64_t)in.nchan < (int64_t)0xffffffffll,
                "more than 2^32 visibilities per call");
    drop_kept_buckets();  // a fresh plan re-uses the bucketing scratch
    Plan P;
    Geo &g = P.g;
    g.W = kernel_support(in.eps);
    g.beta = (float)(2.30 * g.W);
    g.inv_half_w = 2.0f / (float)g.W;
    g.beta_l2e = (float)(2.30 * g.W * 1.4426950408889634);
    g.nx = in.nx;
    g.ny = in.ny;
    g.ngx = ((2 * in.nx + kGridAlign - 1) / kGridAlign) * kGridAlign;
    g.ngy = ((2 * in.ny + kGridAlign - 1) / kGridAlign) * kGridAlign;
    SDP_REQUIRE(g.ngx <= 65535 && g.ngy <= 65535, "image too large (padded grid > 65535)");
    g.px = in.px;
    g.py = in.py;
    g.su = (in.flags & SDP_HIP_FLIP_UW) ? -1.0 : 1.0;
    g.nchan = in.nchan;
    g.nrow = in.nrow;
    g.dbg = std::getenv("SDP_HIP_DBG") ? std::atoi(std::getenv("SDP_HIP_DBG")) : 0;

    // uvw and frequency extremes (device) -> host, or the batch sequence's
    double *hb = pinned_host<double>(0, 6);
    if (in.bounds) {
        const double *b = in.bounds;
        SDP_REQUIRE(b[0] <= b[1] && b[2] >= 0 && b[3] >= 0 && b[4] > 0 && b[4] <= b[5],
                    "bounds must be {wmin <= wmax, umax >= 0, vmax >= 0, 0 < fmin <= fmax}");
        hb[0] = g.su > 0 ? b[0] : -b[1];  // extremes of su * w
        hb[1] = g.su > 0 ? b[1] : -b[0];
        hb[2] = b[2];
        hb[3] = b[3];
        hb[4] = b[4];
        hb[5] = b[5];
    } else {
        auto *part = scratch<double>("bounds_part", 4 * kBoundsBlocks);
        auto *bnd = scratch<double>("bounds", 6);
        const int nb = (int)std::max<int64_t>(
            1, std::min<int64_t>(grid1d(in.nrow, 256), kBoundsBlocks));
        k_bounds<<<nb, 256, 0, st>>>(in.uvw, in.uvw_rs, in.nrow, g.su, part);
        k_bounds_final<<<1, 256, 0, st>>>(nb, part, in.freq, in.nchan, bnd);
        SDP_HIP_CHECK(hipMemcpyAsync(hb, bnd, 6 * sizeof(double), hipMemcpyDeviceToHost, st));
        SDP_HIP_CHECK(hipStreamSynchronize(st));
    }
    const double fmin_ = hb[4], fmax_ = hb[5];
    SDP_REQUIRE(fmin_ > 0, "frequencies must be positive");
    const double slo = fmin_ / kCLight, shi = fmax_ / kCLight;
    const bool any = in.nrow > 0 || in.bounds;
    const double wmin = any ? std::min(hb[0] * slo, hb[0] * shi) : 0.0;
    const double wmax = any ? std::max(hb[1] * slo, hb[1] * shi) : 0.0;
    const double umax = hb[2] * shi, vmax = hb[3] * shi;
    SDP_REQUIRE(std::isfinite(wmin) && std::isfinite(wmax) && std::isfinite(umax) &&
                    std::isfinite(vmax),
                "non-finite uvw coordinates");
    SDP_REQUIRE(umax * in.px < 0.5 && vmax * in.py < 0.5,
                "some uvw coordinates exceed the image's Nyquist limit (|u|*pixsize >= 0.5)");

    const double lmax = (in.nx / 2) * in.px, mmax = (in.ny / 2) * in.py;
    const double r2 = std::min(lmax * lmax + mmax * mmax, 1.0);
    const double tmax = 1.0 - std::sqrt(1.0 - r2);
    g.do_w = (in.do_w && tmax > 0.0) ? 1 : 0;
    if (g.do_w) {
        g.s0 = 0.5 * tmax;
        g.dw = 1.0 / (2.0 * tmax);
        g.w0 = wmin - (0.5 * g.W - 0.5) * g.dw;
        const double pwmax = (wmax - g.w0) / g.dw;
        g.nplanes = (int)std::floor(pwmax - 0.5 * g.W) + 1 + g.W;
        g.nps = g.nplanes - g.W + 1;
    } else {
        g.s0 = 0.0;
        g.dw = 1.0;
        g.w0 = 0.0;
        g.nplanes = 1;
        g.nps = 1;
    }
    // bucket window (origins only: the footprints' halo may leave it)
    {
        const double amax = umax * in.px * g.ngx, bmax = vmax * in.py * g.ngy;
        auto window = [&](double m, int ng, int &w0, int &wn) {
            const int reach = (int)std::ceil(m + 0.5 * g.W) + 2;
            int lo = (ng / 2 - reach) & ~(kGridAlign - 1);
            int hi = ((ng / 2 + reach + kGridAlign - 1) / kGridAlign) * kGridAlign;
            if (lo <= 0 || hi >= ng || env_int("SDP_HIP_NO_WINDOW", 0)) {
                lo = 0;
                hi = ng;
            }
            w0 = lo;
            wn = hi - lo;
        };
        // x (rows) only: the y stride stays ngy, since a compacted y range
        // packs the hot histogram counters of the uv core closer together
        // and measured 2x slower count-pass atomics on C2
        (void)bmax;
        window(amax, g.ngx, g.wx0, g.wnx);
        g.wy0 = 0;
        g.wny = g.ngy;
    }
    // bucket granularity.  Invert: one-cell buckets for the MFMA gridder
    // while the dense (first plane, cell) histogram stays below kMaxCellKeys
    // (SDP_HIP_MFMA=0: the register gridder's 2x2-cell buckets).  Predict:
    // 2x2-cell buckets for the register degridder below kMaxFineKeys.  Else
    // 16x16-cell buckets (sub-sorted to cells / 2x2 buckets below, or the
    // LDS-tile kernels).
    {
        const char *e = std::getenv("SDP_HIP_BUCKET");
        const char *m = std::getenv("SDP_HIP_MFMA");
        // predict: SDP_HIP_MFMA_DEGRID=0 keeps the register degridder
        P.cells = !(m && std::atoi(m) == 0) &&
                  (grid_mode || env_int("SDP_HIP_MFMA_DEGRID", 1) != 0);
        const int64_t cell = (int64_t)g.wnx * g.wny * g.nps;
        const int64_t fine = (int64_t)(g.wnx / kTileFine) * (g.wny / kTileFine) * g.nps;
        if (P.cells) g.sub = cell <= kMaxCellKeys ? kTileCell : kTileCoarse;
        else g.sub = fine <= kMaxFineKeys ? kTileFine : kTileCoarse;
        if (e && std::atoi(e) == kTileCoarse) g.sub = kTileCoarse;
    }
    g.nty = g.wny / g.sub;
    g.ntiles = (g.wnx / g.sub) * g.nty;
    g.grp = g.sub == kTileCell ? kGroupCell : (g.sub == kTileFine ? kGroupFine : 1);
    g.salt = 1;
    if (g.sub == kTileCoarse) {
        const int sv = env_int("SDP_HIP_SALT", 4);
        g.salt = (sv >= 1 && sv <= 64 && (sv & (sv - 1)) == 0) ? sv : 4;
        while (g.salt > 1 && (double)g.ntiles * g.nps * g.salt >= 1.0e9) g.salt >>= 1;
    }
    SDP_REQUIRE((double)g.ntiles * g.nps * g.salt < 4.0e9, "too many (plane, tile) buckets");

    // grid rows reached by any footprint (centred storage)
    {
        const double amax = umax * in.px * g.ngx;
        const int reach = (int)std::ceil(amax) + g.W + 1;
        P.row_lo = std::max(0, g.ngx / 2 - reach);
        P.row_hi = std::min(g.ngx, g.ngx / 2 + reach);
        if (2 * reach >= g.ngx) {
            P.row_lo = 0;
            P.row_hi = g.ngx;
        }
    }

    // plane chunking against the grid memory budget.  The y-spectra buffers
    // (spec, spec_in: ny x ngx per plane) serve batches of fft_planes planes,
    // so the resident planes cost one grid each (C4: 70 planes of 16384^2)
    const size_t grid_plane = (size_t)g.ngx * g.ngy * sizeof(float2);
    const size_t spec_plane = 2 * (size_t)g.ny * g.ngx * sizeof(float2);
    P.fft_planes = (int)std::max<size_t>(
        1, std::min<size_t>(kFftBatchMax, kFftBatchBytes / spec_plane));
    if (const char *e = std::getenv("SDP_HIP_FFT_PLANES"))  // tests: force small batches
        if (std::atoi(e) > 0) P.fft_planes = std::atoi(e);
    P.fft_planes = std::min(P.fft_planes, g.nplanes);
    const int64_t nvis_all = in.nrow * (int64_t)in.nchan;
    const size_t need_other =
        (size_t)nvis_all * (sizeof(VisRec) + sizeof(unsigned) + (grid_mode ? 0 : sizeof(float2))) +
        (size_t)g.ntiles * g.nps * g.salt * 2 * sizeof(unsigned) +
        (size_t)P.fft_planes * spec_plane;
    int cp = (int)std::max<size_t>(1, grid_budget_bytes(need_other) / grid_plane);
    // large-grid inverts: the sub-sorted records re-written 4-padded as 16-B
    // records (~21 B per visibility with the pads) when that costs no plane
    // residency (SDP_HIP_SUBSORT_PAD=0: never)
    if (grid_mode && P.cells && g.sub == kTileCoarse && env_int("SDP_HIP_SUBSORT_PAD", 0) != 0 &&
        !P.aux_bucketing) {
        const size_t need_pad = need_other + (size_t)nvis_all * 21;
        const int cpp = (int)std::max<size_t>(1, grid_budget_bytes(need_pad) / grid_plane);
        if (std::min(cpp, g.nplanes) >= std::min(cp, g.nplanes)) P.subpad = true;
    }
    P.chunk_planes = std::min(cp, g.nplanes);
    P.fft_planes = std::min(P.fft_planes, P.chunk_planes);
    P.grid = scratch<float2>("grid", (size_t)P.chunk_planes * g.ngx * g.ngy);
    P.spec = scratch<float2>("spec", (size_t)P.fft_planes * g.ny * g.ngx);
    if (grid_mode) P.spec_in = band_input(P, st);

    // records per item: large enough to amortise the tile flush over dense
    // tiles, small enough to leave >= ~16k items for the 256 CUs
    const int64_t nvis = in.nrow * (int64_t)in.nchan;
    P.chunk = (unsigned)std::min<int64_t>(kChunkMax, std::max<int64_t>(kChunkMin, nvis / 16384));
    if (const char *e = std::getenv("SDP_HIP_CHUNK"))
        if (std::atoi(e) >= 64) P.chunk = (unsigned)std::atoi(e);

    // part split
    const char *pe = std::getenv("SDP_HIP_PIPELINE");
    const int pmode = pe ? std::atoi(pe) : 0;
    P.pipelined = pmode == 2 && (g.sub == kTileFine || g.sub == kTileCell) &&
                  P.chunk_planes == g.nplanes && in.nrow >= 2 &&
                  !(in.flags & SDP_HIP_KEEP_BUCKETS);
    P.aux_bucketing = P.pipelined || (pmode == 1 && !grid_mode);
    const int nparts = P.pipelined ? kPipelineParts : 1;
    for (int i = 0; i < nparts; ++i) {
        Part pt;
        pt.r0 = in.nrow * i / nparts;
        pt.r1 = in.nrow * (i + 1) / nparts;
        pt.vbase = pt.r0 * in.nchan;
        pt.nvis = (pt.r1 - pt.r0) * in.nchan;
        P.parts.push_back(pt);
    }
    // large grids: re-order the 16x16 buckets by 2x2 bucket for the register
    // kernels (SDP_HIP_SUBSORT=0 keeps the LDS-tile kernels)
    {
        const char *e = std::getenv("SDP_HIP_SUBSORT");
        P.subsort = g.sub == kTileCoarse && !P.aux_bucketing && !(e && std::atoi(e) == 0);
        if (P.subsort) P.chunk = std::min<unsigned>(P.chunk, kSubChunk);
        P.subpad = P.subpad && P.subsort;
    }
    // one-cell buckets padded to multiples of 4 records (k_grid_mfma_pad);
    // SDP_HIP_PAD4=0 keeps the unpadded run-walking k_grid_mfma.  The padded
    // record count is read back before the scatter (one host sync), so the
    // host-sync-free pipelined plans stay unpadded.
    P.pad4 = grid_mode && P.cells && g.sub == kTileCell && !P.aux_bucketing &&
             env_int("SDP_HIP_PAD4", 1) != 0;
    P.chunk &= ~63u;  // items start on 64-record batches (and 4-record K-steps)
    P.recs = scratch<VisRec>("recs", std::max<int64_t>(nvis, 1));
    return P;
}

// Bucketing of one part on stream `st` (no host sync): histogram with ranks,
// scan, scatter of the 32-byte records, work items, part metadata.
static void bucket_part(Plan &P, int ip, const Inputs &in, bool grid_mode, hipStream_t st,
                        bool values_only = false) {
    const Geo &g = P.g;
    Part &pt = P.parts[ip];
    const std::string sfx = "#" + std::to_string(ip);
    const size_t nkeys = (size_t)g.ntiles * g.nps * g.salt;
    const int kpg = g.grp * g.salt;  // keys per work-item group
    const int64_t ngroups = (int64_t)nkeys / kpg;
    const int gpp = g.ntiles / g.grp;  // groups per first-plane value
    pt.hist = scratch<unsigned>("hist" + sfx, nkeys + 1);
    pt.offs = scratch<unsigned>("offs" + sfx, nkeys + 1);
    pt.nch = scratch<unsigned>("nch" + sfx, ngroups + 1);
    pt.ioffs = scratch<unsigned>("ioffs" + sfx, ngroups + 1);
    pt.nbad = scratch<unsigned long long>("nbad" + sfx, 1);
    pt.meta = scratch<unsigned>("meta" + sfx, g.nps + 5);
    const int64_t icap = std::min<int64_t>(ngroups, pt.nvis) + pt.nvis / P.chunk + 1;
    pt.items = scratch<Item>("items" + sfx, icap);
    unsigned *kr = scratch<unsigned>("key_rank", std::max<int64_t>(in.nrow * (int64_t)in.nchan, 1)) +
                pt.vbase;
    if (!values_only) SDP_HIP_CHECK(hipMemsetAsync(pt.hist, 0, (nkeys + 1) * sizeof(unsigned), st));
    if (!values_only) {
        SDP_HIP_CHECK(hipMemsetAsync(pt.nbad, 0, sizeof(unsigned long long), st));
        SDP_HIP_CHECK(hipMemsetAsync(pt.nch + ngroups, 0, sizeof(unsigned), st));
    }

    const unsigned nb = grid1d(std::max<int64_t>(pt.nvis, 1), 256);
    double *slots = in.x.sumwt ? scratch<double>("sumwt_slots", kSumSlots) : nullptr;
    // weight sums: in the count pass, or in the value pass of a reused plan
    auto launch_bucket = [&](auto scatter_tag, unsigned *counter) {
        constexpr bool S = decltype(scatter_tag)::value;
        VisRec *out = S ? P.recs + pt.vbase : nullptr;
        double *sl = S == values_only ? slots : nullptr;
        if (in.vis_dtype == SDP_HIP_C128) {
            if (grid_mode && S && P.pad4)  // 16-byte RecC records
                k_bucket<double2, S, true, true><<<nb, 256, 0, st>>>(
                    g, pt.r0, pt.nvis, in.uvw, in.uvw_rs, in.freq, (const double2 *)in.vis,
                    in.vrs, in.vcs, in.wgt, in.wrs, in.wcs, in.x, sl, counter, kr, out, pt.nbad);
            else if (grid_mode)
                k_bucket<double2, S, true><<<nb, 256, 0, st>>>(
                    g, pt.r0, pt.nvis, in.uvw, in.uvw_rs, in.freq, (const double2 *)in.vis,
                    in.vrs, in.vcs, in.wgt, in.wrs, in.wcs, in.x, sl, counter, kr, out, pt.nbad);
            else
                k_bucket<double2, S, false><<<nb, 256, 0, st>>>(
                    g, pt.r0, pt.nvis, in.uvw, in.uvw_rs, in.freq, nullptr, 0, 0, in.wgt, in.wrs,
                    in.wcs, in.x, sl, counter, kr, out, pt.nbad);
        } else {
            if (grid_mode && S && P.pad4)  // 16-byte RecC records
                k_bucket<float2, S, true, true><<<nb, 256, 0, st>>>(
                    g, pt.r0, pt.nvis, in.uvw, in.uvw_rs, in.freq, (const float2 *)in.vis,
                    in.vrs, in.vcs, in.wgt, in.wrs, in.wcs, in.x, sl, counter, kr, out, pt.nbad);
            else if (grid_mode)
                k_bucket<float2, S, true><<<nb, 256, 0, st>>>(
                    g, pt.r0, pt.nvis, in.uvw, in.uvw_rs, in.freq, (const float2 *)in.vis,
                    in.vrs, in.vcs, in.wgt, in.wrs, in.wcs, in.x, sl, counter, kr, out, pt.nbad);
            else
                k_bucket<float2, S, false><<<nb, 256, 0, st>>>(
                    g, pt.r0, pt.nvis, in.uvw, in.uvw_rs, in.freq, nullptr, 0, 0, in.wgt, in.wrs,
                    in.wcs, in.x, sl, counter, kr, out, pt.nbad);
        }
    };
    if (values_only) {  // SDP_HIP_REUSE_BUCKETS: keys, ranks, offsets, items kept
        if (pt.nvis > 0) launch_bucket(std::true_type{}, pt.offs);
        SDP_HIP_CHECK(hipGetLastError());
        return;
    }
    if (pt.nvis > 0) launch_bucket(std::false_type{}, pt.hist);
    size_t tmp_bytes = 0;
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, pt.hist, pt.offs,
                                                   (int)(nkeys + 1), st));
    void *tmp = scratch<char>("scan_tmp" + sfx, tmp_bytes + 16);
    size_t tb = tmp_bytes + 16;
    if (P.pad4) {
        // scan of the counts rounded up to 4, then the padded total sizes
        // the record array (one host sync)
        hipcub::TransformInputIterator<unsigned, Round4, const unsigned *> r4(pt.hist, Round4{});
        size_t need = 0;
        SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, r4, pt.offs,
                                                       (int)(nkeys + 1), st));
        if (need > tmp_bytes) {
            tmp_bytes = need;
            tmp = scratch<char>("scan_tmp" + sfx, tmp_bytes + 16);
        }
        tb = tmp_bytes + 16;
        SDP_HIP_CHECK(
            hipcub::DeviceScan::ExclusiveSum(tmp, tb, r4, pt.offs, (int)(nkeys + 1), st));
        unsigned *htot = pinned_host<unsigned>(48, 1);
        SDP_HIP_CHECK(hipMemcpyAsync(htot, pt.offs + nkeys, sizeof(unsigned),
                                     hipMemcpyDeviceToHost, st));
        SDP_HIP_CHECK(hipStreamSynchronize(st));
        SDP_REQUIRE(P.parts.size() == 1, "4-padded bucketing runs on one part");
        P.recs = scratch<VisRec>("recs", ((int64_t)*htot + 1) / 2 + 1);  // RecC records
    } else {
        SDP_HIP_CHECK(
            hipcub::DeviceScan::ExclusiveSum(tmp, tb, pt.hist, pt.offs, (int)(nkeys + 1), st));
    }
    if (pt.nvis > 0) launch_bucket(std::true_type{}, pt.offs);
    if (P.pad4) {
        unsigned *pslots = scratch<unsigned>("pad_slots", kSumSlots);
        pt.npad = scratch<unsigned>("npad" + sfx, 1);
        SDP_HIP_CHECK(hipMemsetAsync(pslots, 0, kSumSlots * sizeof(unsigned), st));
        k_pad_cells<<<grid1d((int64_t)nkeys, 256), 256, 0, st>>>(
            (unsigned)nkeys, pt.hist, pt.offs, reinterpret_cast<RecC *>(P.recs), pslots);
        k_sum_pads<<<1, 256, 0, st>>>(pslots, pt.npad);
    }

    // work items (p0-major, so a first-plane range is a contiguous item range)
    k_items_count<<<grid1d(ngroups, 256), 256, 0, st>>>(ngroups, kpg, pt.offs, P.chunk, pt.nch);
    tb = tmp_bytes + 16;
    SDP_HIP_CHECK(
        hipcub::DeviceScan::ExclusiveSum(tmp, tb, pt.nch, pt.ioffs, (int)(ngroups + 1), st));
    k_items_fill<<<grid1d(ngroups, 256), 256, 0, st>>>(ngroups, kpg, gpp, pt.offs, pt.ioffs,
                                                       P.chunk, pt.items);
    k_part_meta<<<grid1d(g.nps + 1, 64), 64, 0, st>>>(pt.nbad, pt.offs + nkeys, pt.npad, pt.ioffs, gpp,
                                                      g.nps, pt.meta);
    SDP_HIP_CHECK(hipGetLastError());
}

// Host copy of every part's metadata (one sync): counts, the first-plane item
// offsets (plane-chunked launches need them) and the out-of-grid check.
static void read_part_meta(Plan &P, hipStream_t st) {
    const int nps = P.g.nps;
    const size_t per = (size_t)nps + 5;
    unsigned *hm = pinned_host<unsigned>(64, per * P.parts.size());
    for (size_t i = 0; i < P.parts.size(); ++i)
        SDP_HIP_CHECK(hipMemcpyAsync(hm + i * per, P.parts[i].meta, per * sizeof(unsigned),
                                     hipMemcpyDeviceToHost, st));
    SDP_HIP_CHECK(hipStreamSynchronize(st));
    P.nrec = P.nitems = 0;
    for (size_t i = 0; i < P.parts.size(); ++i) {
        const unsigned *m = hm + i * per;
        const unsigned long long nbad = (unsigned long long)m[0] | ((unsigned long long)m[1] << 32);
        SDP_REQUIRE(nbad == 0, "visibilities outside the padded grid");
        Part &pt = P.parts[i];
        pt.nrec = m[2];
        pt.nitems = m[3];
        pt.p0_items.assign(m + 4, m + 4 + nps + 1);
        P.nrec += pt.nrec;
        P.nitems += pt.nitems;
    }
}

// Item range of a part whose W-plane windows intersect planes [p_lo, p_hi).
static std::pair<unsigned, unsigned> chunk_items(const Plan &P, const Part &pt, int p_lo,
                                                 int p_hi) {
    const int a = std::max(0, p_lo - (P.g.do_w ? P.g.W : 1) + 1);
    const int b = std::min(P.g.nps - 1, p_hi - 1);
    if (a > b) return {0u, 0u};
    return {pt.p0_items[a], pt.p0_items[b + 1]};
}

// Launch shape of one gridding pass over a part: one workgroup per item when
// the host knows the range, else a persistent grid reading the count.
struct Launch {
    ItemSrc src;
    unsigned blocks;
};

static unsigned persistent_blocks(const void *fn, int threads, size_t lds) {
    static std::mutex mu;
    static std::map<std::pair<const void *, size_t>, unsigned> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair(fn, lds);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int dev = 0, ncu = 0, per = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    SDP_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    SDP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, threads, lds));
    unsigned nb = (unsigned)std::max(1, ncu * std::max(1, per));
    if (const char *e = std::getenv("SDP_HIP_PBLOCKS")) nb = (unsigned)std::max(1, std::atoi(e));
    else nb *= 8;  // several workgroups per slot: the hardware balances the uneven items
    cache[key] = nb;
    return nb;
}

static Launch part_launch(const Plan &P, const Part &pt, int p_lo, int p_hi, const void *fn,
                          int threads, size_t lds) {
    Launch L;
    if (P.pipelined) {
        L.src = ItemSrc{pt.items, 0u, pt.meta + 3};
        L.blocks = persistent_blocks(fn, threads, lds);
    } else {
        const auto r = chunk_items(P, pt, p_lo, p_hi);
        L.src = ItemSrc{pt.items + r.first, r.second - r.first, nullptr};
        L.blocks = r.second - r.first;
    }
    return L;
}

static void allow_lds(const void *fn, size_t bytes) {
    if (bytes > 65536)
        SDP_HIP_CHECK(
            hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

// waves per gridding workgroup (planes split across them); SDP_HIP_GRID_WAVES
// overrides the default for experiments
static int grid_waves(int W, bool do_w) {
    if (!do_w) return 1;
    const char *e = std::getenv("SDP_HIP_GRID_WAVES");
    const int v = e ? std::atoi(e) : 2;
    return (v == 1 || v == 2 || v == 4) && v <= W ? v : 2;
}

template <int W, bool WS, int NWV>
static void launch_grid_n(const Plan &P, const Part &pt, int p_lo, int p_hi, hipStream_t st) {
    constexpr int NQ = WS ? W : 1;
    const size_t lds = (size_t)((NQ + NWV - 1) / NWV * NWV) *
                       TileShape<W, kTileCoarse>::PLANE * sizeof(float2);
    const void *fn = (const void *)k_grid_lds<W, WS, NWV>;
    allow_lds(fn, lds);
    const Launch L = part_launch(P, pt, p_lo, p_hi, fn, 64 * NWV, lds);
    if (L.blocks == 0) return;
    k_grid_lds<W, WS, NWV><<<L.blocks, 64 * NWV, lds, st>>>(P.g, P.recs + pt.vbase, L.src,
                                                          (float *)P.grid, p_lo, p_hi);
}

template <int W, bool WS>
static void launch_grid_reg(const Plan &P, const Part &pt, int p_lo, int p_hi, hipStream_t st) {
    const size_t lds = (size_t)(WS ? W : 1) *
                       TileShape<W, kTileFine, kTileFine * kGroupFine>::PLANE * sizeof(float2);
    const void *fn = (const void *)k_grid_reg<W, WS, false>;
    const Launch L = part_launch(P, pt, p_lo, p_hi, fn, 64, lds);
    if (L.blocks == 0) return;
    k_grid_reg<W, WS, false><<<L.blocks, 64, lds, st>>>(P.g, P.recs + pt.vbase, L.src, pt.offs,
                                                       nullptr, (float *)P.grid, p_lo, p_hi,
                                                       P.g.dbg);
}

// The register kernels' view of a sub-sorted coarse plan: 2x2-cell buckets
// in groups of kGroupFine (the work items carry their bucket offsets).
static Geo fine_view(const Geo &g) {
    Geo f = g;
    f.sub = kTileFine;
    f.nty = g.wny / kTileFine;
    f.ntiles = (g.wnx / kTileFine) * f.nty;
    f.grp = kGroupFine;
    return f;
}

template <int W, bool WS>
static void launch_grid_fine_items(const Plan &P, const Part &pt, int p_lo, int p_hi,
                                   hipStream_t st) {
    const size_t lds = (size_t)(WS ? W : 1) *
                       TileShape<W, kTileFine, kTileFine * kGroupFine>::PLANE * sizeof(float2);
    const auto r = chunk_items(P, pt, p_lo, p_hi);
    const unsigned n = 16u * (r.second - r.first);
    if (n == 0) return;
    k_grid_reg<W, WS, true><<<n, 64, lds, st>>>(fine_view(P.g), P.recs + pt.vbase,
                                                ItemSrc{nullptr, n, nullptr}, nullptr,
                                                pt.fitems + 16 * (size_t)r.first, (float *)P.grid,
                                                p_lo, p_hi, P.g.dbg);
}

template <int W, bool WS>
static void launch_degrid_fine_items(const Plan &P, const Part &pt, int p_lo, int p_hi,
                                     float2 *acc, hipStream_t st) {
    const size_t lds = (size_t)(WS ? W : 1) *
                       TileShape<W, kTileFine, kTileFine * kGroupFine>::PLANE * sizeof(float2);
    const auto r = chunk_items(P, pt, p_lo, p_hi);
    const unsigned n = 16u * (r.second - r.first);
    if (n == 0) return;
    k_degrid_reg<W, WS, true><<<n, 64, lds, st>>>(fine_view(P.g), P.recs + pt.vbase,
                                                  ItemSrc{nullptr, n, nullptr}, nullptr,
                                                  pt.fitems + 16 * (size_t)r.first, P.grid, p_lo,
                                                  p_hi, acc + pt.vbase, P.vdirect);
}

template <int W, bool WS>
static void launch_grid_mfma(const Plan &P, const Part &pt, int p_lo, int p_hi, hipStream_t st) {
    const size_t lds = (size_t)(WS ? W : 1) * (2 + W - 1) * (8 + W - 1) * sizeof(float2) +
                       128 * sizeof(float4);
    if (P.subsort) {
        const auto r = chunk_items(P, pt, p_lo, p_hi);
        const unsigned n = 16u * (r.second - r.first);
        if (n == 0) return;
        k_grid_mfma<W, WS, true><<<n, 64, lds, st>>>(P.g, P.recs + pt.vbase,
                                                     ItemSrc{nullptr, n, nullptr}, nullptr,
                                                     pt.fitems + 16 * (size_t)r.first,
                                                     (float *)P.grid, p_lo, p_hi);
        return;
    }
    const void *fn = (const void *)k_grid_mfma<W, WS, false>;
    const Launch L = part_launch(P, pt, p_lo, p_hi, fn, 64, lds);
    if (L.blocks == 0) return;
    // SDP_HIP_DBG & 32 (timing experiment): an empty plane range skips the flush
    const int ph = (P.g.dbg & 32) ? p_lo : p_hi;
    k_grid_mfma<W, WS, false><<<L.blocks, 64, lds, st>>>(P.g, P.recs + pt.vbase, L.src, pt.offs,
                                                        nullptr, (float *)P.grid, p_lo, ph);
}

template <int W, bool WS>
static void launch_grid_mfma_pad(const Plan &P, const Part &pt, int p_lo, int p_hi,
                                 hipStream_t st) {
    constexpr size_t lds = grid_mfma_pad_lds<W, WS>();
    const void *fn = (const void *)k_grid_mfma_pad<W, WS>;
    Launch L = part_launch(P, pt, p_lo, p_hi, fn, 64, lds);
    if (L.blocks == 0) return;
    const int ph = (P.g.dbg & 32) ? p_lo : p_hi;  // SDP_HIP_DBG & 32: no flush (timing)
    k_grid_mfma_pad<W, WS><<<L.blocks, 64, lds, st>>>(
        P.g, reinterpret_cast<const RecC *>(P.recs) + pt.vbase, L.src, pt.offs, nullptr,
        (float *)P.grid, p_lo, ph);
}

template <int W, bool WS>
static void launch_grid_mfma_pad_fi(const Plan &P, const Part &pt, int p_lo, int p_hi,
                                    hipStream_t st) {
    constexpr size_t lds = grid_mfma_pad_lds<W, WS>();
    const auto r = chunk_items(P, pt, p_lo, p_hi);
    const unsigned n = 16u * (r.second - r.first);
    if (n == 0) return;
    k_grid_mfma_pad<W, WS, true><<<n, 64, lds, st>>>(
        P.g, pt.precs, ItemSrc{nullptr, n, nullptr}, nullptr, pt.pfitems + 16 * (size_t)r.first,
        (float *)P.grid, p_lo, p_hi);
}

template <int W>
static void launch_grid(const Plan &P, const Part &pt, int p_lo, int p_hi, hipStream_t st) {
    if (P.subpad) {
        if (P.g.do_w) return launch_grid_mfma_pad_fi<W, true>(P, pt, p_lo, p_hi, st);
        return launch_grid_mfma_pad_fi<W, false>(P, pt, p_lo, p_hi, st);
    }
    if (P.pad4) {
        if (P.g.do_w) return launch_grid_mfma_pad<W, true>(P, pt, p_lo, p_hi, st);
        return launch_grid_mfma_pad<W, false>(P, pt, p_lo, p_hi, st);
    }
    if (P.cells && (P.subsort || P.g.sub == kTileCell)) {
        if (P.g.do_w) return launch_grid_mfma<W, true>(P, pt, p_lo, p_hi, st);
        return launch_grid_mfma<W, false>(P, pt, p_lo, p_hi, st);
    }
    if (P.subsort) {
        if (P.g.do_w) return launch_grid_fine_items<W, true>(P, pt, p_lo, p_hi, st);
        return launch_grid_fine_items<W, false>(P, pt, p_lo, p_hi, st);
    }
    if (P.g.sub == kTileFine) {
        if (P.g.do_w) return launch_grid_reg<W, true>(P, pt, p_lo, p_hi, st);
        return launch_grid_reg<W, false>(P, pt, p_lo, p_hi, st);
    }
    if (!P.g.do_w) return launch_grid_n<W, false, 1>(P, pt, p_lo, p_hi, st);
    switch (grid_waves(W, true)) {
        case 1: return launch_grid_n<W, true, 1>(P, pt, p_lo, p_hi, st);
        case 4: return launch_grid_n<W, true, (W >= 4 ? 4 : 2)>(P, pt, p_lo, p_hi, st);
        default: return launch_grid_n<W, true, 2>(P, pt, p_lo, p_hi, st);
    }
}

template <int W, bool WS, int SX, int SY>
static void launch_degrid_n(const Plan &P, const Part &pt, int p_lo, int p_hi, float2 *acc,
                            hipStream_t st) {
    const size_t lds = (size_t)(WS ? W : 1) * TileShape<W, SX, SY>::PLANE * sizeof(float2);
    const void *fn = (const void *)k_degrid<W, WS, SX, SY>;
    allow_lds(fn, lds);
    const Launch L = part_launch(P, pt, p_lo, p_hi, fn, 64, lds);
    if (L.blocks == 0) return;
    k_degrid<W, WS, SX, SY><<<L.blocks, 64, lds, st>>>(P.g, P.recs + pt.vbase, L.src, P.grid,
                                                      p_lo, p_hi, acc + pt.vbase);
}

template <int W, bool WS>
static void launch_degrid_reg(const Plan &P, const Part &pt, int p_lo, int p_hi, float2 *acc,
                              hipStream_t st) {
    const size_t lds = (size_t)(WS ? W : 1) *
                       TileShape<W, kTileFine, kTileFine * kGroupFine>::PLANE * sizeof(float2);
    const void *fn = (const void *)k_degrid_reg<W, WS, false>;
    const Launch L = part_launch(P, pt, p_lo, p_hi, fn, 64, lds);
    if (L.blocks == 0) return;
    k_degrid_reg<W, WS, false><<<L.blocks, 64, lds, st>>>(P.g, P.recs + pt.vbase, L.src, pt.offs,
                                                         nullptr, P.grid, p_lo, p_hi,
                                                         acc + pt.vbase, P.vdirect);
}

template <int W, bool WS>
static void launch_degrid_mfma(const Plan &P, const Part &pt, int p_lo, int p_hi, float2 *acc,
                               hipStream_t st) {
    const size_t lds = (size_t)(WS ? W : 1) * (2 + W - 1) * (8 + W - 1) * sizeof(float2);
    if (P.subsort) {
        const auto r = chunk_items(P, pt, p_lo, p_hi);
        const unsigned n = 16u * (r.second - r.first);
        if (n == 0) return;
        k_degrid_mfma<W, WS, true><<<n, 64, lds, st>>>(
            P.g, P.recs + pt.vbase, ItemSrc{nullptr, n, nullptr}, nullptr,
            pt.fitems + 16 * (size_t)r.first, P.grid, p_lo, p_hi, acc ? acc + pt.vbase : nullptr,
            P.vdirect);
        return;
    }
    const void *fn = (const void *)k_degrid_mfma<W, WS, false>;
    const Launch L = part_launch(P, pt, p_lo, p_hi, fn, 64, lds);
    if (L.blocks == 0) return;
    k_degrid_mfma<W, WS, false><<<L.blocks, 64, lds, st>>>(
        P.g, P.recs + pt.vbase, L.src, pt.offs, nullptr, P.grid, p_lo, p_hi,
        acc ? acc + pt.vbase : nullptr, P.vdirect);
}

template <int W>
static void launch_degrid(const Plan &P, const Part &pt, int p_lo, int p_hi, float2 *acc,
                          hipStream_t st) {
    if (P.cells && (P.subsort || P.g.sub == kTileCell)) {
        if (P.g.do_w) return launch_degrid_mfma<W, true>(P, pt, p_lo, p_hi, acc, st);
        return launch_degrid_mfma<W, false>(P, pt, p_lo, p_hi, acc, st);
    }
    if (P.subsort) {
        if (P.g.do_w) return launch_degrid_fine_items<W, true>(P, pt, p_lo, p_hi, acc, st);
        return launch_degrid_fine_items<W, false>(P, pt, p_lo, p_hi, acc, st);
    }
    if (P.g.sub == kTileFine) {
        if (P.g.do_w) return launch_degrid_reg<W, true>(P, pt, p_lo, p_hi, acc, st);
        return launch_degrid_reg<W, false>(P, pt, p_lo, p_hi, acc, st);
    }
    if (P.g.do_w)
        return launch_degrid_n<W, true, kTileCoarse, kTileCoarse>(P, pt, p_lo, p_hi, acc, st);
    return launch_degrid_n<W, false, kTileCoarse, kTileCoarse>(P, pt, p_lo, p_hi, acc, st);
}

#define SDP_W_DISPATCH(W, CALL) \
    switch (W) {                \
        case 2: CALL(2); break; \
        case 3: CALL(3); break; \
        case 4: CALL(4); break; \
        case 5: CALL(5); break; \
        case 6: CALL(6); break; \
        case 7: CALL(7); break; \
        default: CALL(8); break; \
    }

static void fill_info(const Plan &P, sdp_hip_wgrid_info *info) {
    if (!info) return;
    info->support = P.g.W;
    info->beta = P.g.beta;
    info->ngrid_x = P.g.ngx;
    info->ngrid_y = P.g.ngy;
    info->nplanes = P.g.nplanes;
    info->w0 = P.g.w0;
    info->dw = P.g.dw;
    info->nvis_used = P.nrec;
    info->nitems = P.nitems;
    info->plane_chunk = P.chunk_planes;
    info->bucket = P.g.sub;
    info->grid_launches = (int)P.parts.size() *
                          ((P.g.nplanes + P.chunk_planes - 1) / P.chunk_planes);
}

// Pruned 2-D FFT of each resident plane.  The uv grid is non-zero only in
// the row band [row_lo, row_hi) the visibilities reach (with cell < Nyquist
// that band is a fraction of the padded grid), and only the ny columns
// ky = (iy - ny/2) mod ngy of the y transform feed the image.  Strided
// column transforms are slow in hipFFT, so the x transform runs on the
// transposed layout T[q][iy][kx] (contiguous rows):
//   backward: y-FFT of the band rows (in place, per plane) -> transpose the
//             needed columns into T -> x-FFT of T rows (one batched call)
//   forward:  x-FFT of T rows -> transpose back into the band rows of the
//             (zeroed) grid -> y-FFT of the band rows
static void exec_fft(hipfftHandle h, float2 *p, int direction) {
    if (hipfftExecC2C(h, (hipfftComplex *)p, (hipfftComplex *)p, direction) != HIPFFT_SUCCESS)
        throw Error(SDP_HIP_ERR_RUNTIME, "hipfftExecC2C failed");
}

static void fft_rows_y(const Plan &P, int q0, int np, int direction, hipStream_t st) {
    const Geo &g = P.g;
    const int nrow = P.row_hi - P.row_lo;
    if (nrow <= 0) return;
    hipfftHandle hr = fft_plan_1d(g.ngy, 1, g.ngy, nrow, st);
    for (int q = q0; q < q0 + np; ++q)
        exec_fft(hr, P.grid + (size_t)q * g.ngx * g.ngy + (size_t)P.row_lo * g.ngy, direction);
}

// x transforms of the T rows into P.spec, in place or from `in`
static void fft_rows_x(const Plan &P, int np, int direction, hipStream_t st,
                       float2 *in = nullptr) {
    const Geo &g = P.g;
    hipfftHandle hc = fft_plan_1d(g.ngx, 1, g.ngx, np * g.ny, st);
    if (!in) return exec_fft(hc, P.spec, direction);
    if (hipfftExecC2C(hc, (hipfftComplex *)in, (hipfftComplex *)P.spec, direction) !=
        HIPFFT_SUCCESS)
        throw Error(SDP_HIP_ERR_RUNTIME, "hipfftExecC2C failed");
}

// Only the row band [row_lo, row_hi) of a plane is ever written or read.
static void zero_band(const Plan &P, int np, hipStream_t st) {
    const Geo &g = P.g;
    if (P.row_hi <= P.row_lo || np <= 0) return;
    const size_t width = (size_t)(P.row_hi - P.row_lo) * g.ngy * sizeof(float2);
    for (int q = 0; q < np; ++q)
        SDP_HIP_CHECK(hipMemsetAsync(
            P.grid + (size_t)q * g.ngx * g.ngy + (size_t)P.row_lo * g.ngy, 0, width, st));
}

static dim3 tr_grid(const Geo &g, int xrows, int np) {
    return dim3((unsigned)((xrows + kTr - 1) / kTr), (unsigned)((g.ny + kTr - 1) / kTr),
                (unsigned)np);
}

// Bucket every part.  Synchronous plans bucket on `st` and read the
// metadata back (plane-chunked launches need the item offsets).  Pipelined
// plans bucket on the auxiliary stream after an event on `st` (inputs ready)
// and record one event per part for the consumer launches to wait on.
static std::vector<hipEvent_t> bucket_parts(Plan &P, const Inputs &in, bool grid_mode,
                                            hipStream_t st) {
    std::vector<hipEvent_t> ev;
    // weight sum of the fused prologue: slots zeroed before the parts' count
    // passes, folded into *sumwt after the first part (all parts share slots)
    double *slots = in.x.sumwt ? scratch<double>("sumwt_slots", kSumSlots) : nullptr;
    auto sum_end = [&](hipStream_t s) {
        if (slots) k_sum_slots<<<1, 64, 0, s>>>(slots, in.x.sumwt);
    };
    if (!P.aux_bucketing) {
        if (slots) SDP_HIP_CHECK(hipMemsetAsync(slots, 0, kSumSlots * sizeof(double), st));
        for (size_t i = 0; i < P.parts.size(); ++i) bucket_part(P, (int)i, in, grid_mode, st);
        sum_end(st);
        read_part_meta(P, st);
        return ev;
    }
    hipStream_t aux = aux_stream();
    hipEvent_t ready;
    SDP_HIP_CHECK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    SDP_HIP_CHECK(hipEventRecord(ready, st));
    SDP_HIP_CHECK(hipStreamWaitEvent(aux, ready, 0));
    SDP_HIP_CHECK(hipEventDestroy(ready));
    if (slots) SDP_HIP_CHECK(hipMemsetAsync(slots, 0, kSumSlots * sizeof(double), aux));
    for (size_t i = 0; i < P.parts.size(); ++i) {
        bucket_part(P, (int)i, in, grid_mode, aux);
        if (i + 1 == P.parts.size()) sum_end(aux);
        hipEvent_t e;
        SDP_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(e, aux));
        ev.push_back(e);
    }
    return ev;
}

// Sub-sort of every part's coarse items (synchronous plans: the item counts
// are on the host)
static void subsort_parts(Plan &P, hipStream_t st) {
    for (size_t i = 0; i < P.parts.size(); ++i) {
        Part &pt = P.parts[i];
        if (pt.nitems == 0) continue;
        const std::string sfx = "#" + std::to_string(i);
        pt.fitems = scratch<FineItem>("fitems" + sfx, (size_t)pt.nitems * 16);
        if (P.cells && P.subpad) {
            // sub-sort, padded sizes, their scan (one host read of the total),
            // then the 4-padded 16-B re-write with FineItems over it
            unsigned *psize = scratch<unsigned>("psize" + sfx, (size_t)pt.nitems + 1);
            unsigned *poffs = scratch<unsigned>("poffs" + sfx, (size_t)pt.nitems + 1);
            SDP_HIP_CHECK(hipMemsetAsync(psize + pt.nitems, 0, sizeof(unsigned), st));
            k_subsort<true><<<(unsigned)pt.nitems, kSubThreads, 0, st>>>(
                P.g, pt.items, P.recs + pt.vbase, pt.fitems, psize);
            SDP_HIP_CHECK(hipGetLastError());
            size_t tb = 0;
            SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, psize, poffs,
                                                           (int)(pt.nitems + 1), st));
            void *tmp = scratch<char>("pscan_tmp" + sfx, tb + 16);
            SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, psize, poffs,
                                                           (int)(pt.nitems + 1), st));
            unsigned total = 0;
            SDP_HIP_CHECK(hipMemcpyAsync(&total, poffs + pt.nitems, sizeof(unsigned),
                                         hipMemcpyDeviceToHost, st));
            SDP_HIP_CHECK(hipStreamSynchronize(st));
            pt.precs = scratch<RecC>("precs" + sfx, std::max<size_t>(total, 1));
            pt.pfitems = scratch<FineItem>("pfitems" + sfx, (size_t)pt.nitems * 16);
            k_subsort_emit<<<(unsigned)pt.nitems, 256, 0, st>>>(
                P.g, pt.items, P.recs + pt.vbase, pt.fitems, poffs, pt.precs, pt.pfitems);
            SDP_HIP_CHECK(hipGetLastError());
            continue;
        }
        if (P.cells)
            k_subsort<true><<<(unsigned)pt.nitems, kSubThreads, 0, st>>>(
                P.g, pt.items, P.recs + pt.vbase, pt.fitems);
        else
            k_subsort<false><<<(unsigned)pt.nitems, kSubThreads, 0, st>>>(
                P.g, pt.items, P.recs + pt.vbase, pt.fitems);
        SDP_HIP_CHECK(hipGetLastError());
    }
}

static void release_events(std::vector<hipEvent_t> &ev) {
    for (auto e : ev) (void)hipEventDestroy(e);
    ev.clear();
}

static void ms2dirty(const Inputs &in, double *dirty, int64_t sx, int64_t sy,
                     sdp_hip_wgrid_info *info, hipStream_t st) {
    SDP_REQUIRE(in.vis == nullptr || in.vis_dtype == SDP_HIP_C64 ||
                    in.vis_dtype == SDP_HIP_C128,
                "vis must be complex64 or complex128");
    StageTimer tm(st);
    tm.mark();
    const bool keep = in.flags & SDP_HIP_KEEP_BUCKETS, reuse = in.flags & SDP_HIP_REUSE_BUCKETS;
    SDP_REQUIRE(!(keep && reuse), "SDP_HIP_KEEP_BUCKETS and SDP_HIP_REUSE_BUCKETS exclude each other");
    SDP_REQUIRE(in.bounds == nullptr || !(keep || reuse),
                "batched inverts do not keep or reuse bucketings");
    Inputs inx = in;
    inx.x.all = keep;
    Plan P = reuse ? reuse_buckets(in) : plan_geometry(inx, true, st);
    const Geo &g = P.g;
    // batched invert: planes zeroed by the first batch, FFT + screens by the
    // last; in between they stay resident in the workspace
    const bool batched = in.bounds != nullptr;
    const bool first = !batched || (in.flags & SDP_HIP_BATCH_FIRST);
    const bool last = !batched || (in.flags & SDP_HIP_BATCH_LAST);
    if (batched) {
        SDP_REQUIRE(P.chunk_planes == g.nplanes,
                    "batched invert: the w planes do not all fit in device memory");
    }
    const double *tab = phi_table(g.W, g.beta, st);
    // the band zeroing of the first plane chunk (HBM writes) overlaps the
    // bucketing (bound by memory-side atomics): it runs on the auxiliary
    // stream after the call's earlier work on `st`; the gridding waits for it
    hipEvent_t zdone = nullptr;
    // (single calls only: on C4's streamed batches it measured 1-2 % slower)
    if (first && !batched && !P.aux_bucketing && env_int("SDP_HIP_ZERO_OVERLAP", 1) != 0) {
        hipStream_t aux = aux_stream();
        hipEvent_t ready;
        SDP_HIP_CHECK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(ready, st));
        SDP_HIP_CHECK(hipStreamWaitEvent(aux, ready, 0));
        SDP_HIP_CHECK(hipEventDestroy(ready));
        zero_band(P, std::min(g.nplanes, P.chunk_planes), aux);
        SDP_HIP_CHECK(hipEventCreateWithFlags(&zdone, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(zdone, aux));
    }
    std::vector<hipEvent_t> ev;
    if (reuse) {
        // value pass only (weight sums included), then the kept sub-sort
        double *slots = in.x.sumwt ? scratch<double>("sumwt_slots", kSumSlots) : nullptr;
        if (slots) SDP_HIP_CHECK(hipMemsetAsync(slots, 0, kSumSlots * sizeof(double), st));
        for (size_t i = 0; i < P.parts.size(); ++i) bucket_part(P, (int)i, inx, true, st, true);
        if (slots) k_sum_slots<<<1, 64, 0, st>>>(slots, in.x.sumwt);
    } else {
        ev = bucket_parts(P, inx, true, st);
    }
    if (P.subsort) subsort_parts(P, st);
    if (keep) keep_buckets(P, in);
    const int accumulate = (in.flags & SDP_HIP_ACCUMULATE) ? 1 : 0;
    float tprep = 0, tgrid = 0, tfft = 0, tscr = 0;
    for (int p_lo = 0; p_lo < g.nplanes; p_lo += P.chunk_planes) {
        const int p_hi = std::min(g.nplanes, p_lo + P.chunk_planes);
        const int np = p_hi - p_lo;
        if (zdone) {
            SDP_HIP_CHECK(hipStreamWaitEvent(st, zdone, 0));
            SDP_HIP_CHECK(hipEventDestroy(zdone));
            zdone = nullptr;
        } else if (first) {
            zero_band(P, np, st);
        }
        for (size_t i = 0; i < P.parts.size(); ++i) {
            if (!ev.empty()) SDP_HIP_CHECK(hipStreamWaitEvent(st, ev[i], 0));
            StageTimer tg(st);
            tg.mark();
#define SDP_LAUNCH_GRID(WW) launch_grid<WW>(P, P.parts[i], p_lo, p_hi, st)
            SDP_W_DISPATCH(g.W, SDP_LAUNCH_GRID);
#undef SDP_LAUNCH_GRID
            SDP_HIP_CHECK(hipGetLastError());
            tg.mark();
            tgrid += tg.ms(0, 1);
        }
        for (int sb = 0; last && sb < np; sb += P.fft_planes) {
            const int nb = std::min(P.fft_planes, np - sb);
            StageTimer t2(st);
            t2.mark();
            fft_rows_y(P, sb, nb, HIPFFT_BACKWARD, st);
            if (P.row_hi > P.row_lo)
                k_tr_grid_to_t<<<tr_grid(g, P.row_hi - P.row_lo, nb), dim3(kTr, kTrRows), 0,
                                 st>>>(g, P.grid + (size_t)sb * g.ngx * g.ngy, P.spec_in,
                                       P.row_lo, P.row_hi);
            SDP_HIP_CHECK(hipGetLastError());
            fft_rows_x(P, nb, HIPFFT_BACKWARD, st, P.spec_in);
            t2.mark();
            const dim3 grd(grid1d(g.nx, 256), g.ny);
            k_screen_fwd_t<<<grd, 256, 0, st>>>(g, P.spec, p_lo + sb, nb, dirty, sx, sy,
                                                (accumulate || p_lo + sb > 0) ? 1 : 0, tab);
            SDP_HIP_CHECK(hipGetLastError());
            t2.mark();
            tfft += t2.ms(0, 1);
            tscr += t2.ms(1, 2);
        }
    }
    tm.mark();
    if (P.pipelined) read_part_meta(P, st);
    release_events(ev);
    fill_info(P, info);
    if (info) {
        // everything on the call's stream that is not gridding, FFT or screen:
        // geometry, bucketing not hidden behind gridding, band zeroing
        tprep = tm.ms(0, 1) - tgrid - tfft - tscr;
        info->ms_prep = tm.on ? tprep : 0.0f;
        info->ms_grid = tgrid;
        info->ms_fft = tfft;
        info->ms_screen = tscr;
    }
}

static void dirty2ms(const Inputs &in, const double *dirty, int64_t sx, int64_t sy, void *vis,
                     sdp_hip_wgrid_info *info, hipStream_t st, const OutConv &oc = OutConv{}) {
    SDP_REQUIRE(in.vis_dtype == SDP_HIP_C64 || in.vis_dtype == SDP_HIP_C128,
                "vis must be complex64 or complex128");
    StageTimer tm(st);
    tm.mark();
    Plan P = plan_geometry(in, false, st);
    const Geo &g = P.g;
    const double *tab = phi_table(g.W, g.beta, st);
    const int accumulate = (in.flags & SDP_HIP_ACCUMULATE) ? 1 : 0;
    const int64_t nvis = in.nrow * (int64_t)in.nchan;
    // the output zeroing and the first plane chunk's band zeroing (HBM
    // writes) overlap the bucketing (memory-side atomics; it reads uvw and
    // weights only) on the auxiliary stream, after the call's earlier work
    hipEvent_t zdone = nullptr;
    if (!P.aux_bucketing && env_int("SDP_HIP_ZERO_OVERLAP", 1) != 0) {
        hipStream_t aux = aux_stream();
        hipEvent_t ready;
        SDP_HIP_CHECK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(ready, st));
        SDP_HIP_CHECK(hipStreamWaitEvent(aux, ready, 0));
        SDP_HIP_CHECK(hipEventDestroy(ready));
        if (!accumulate && nvis > 0) {
            if (in.vis_dtype == SDP_HIP_C128)
                k_zero_vis<double2><<<grid1d(nvis, 256), 256, 0, aux>>>(
                    in.nrow, in.nchan, (double2 *)vis, in.vrs, in.vcs, oc);
            else
                k_zero_vis<float2><<<grid1d(nvis, 256), 256, 0, aux>>>(
                    in.nrow, in.nchan, (float2 *)vis, in.vrs, in.vcs, oc);
            SDP_HIP_CHECK(hipGetLastError());
        }
        zero_band(P, std::min(g.nplanes, P.chunk_planes), aux);
        SDP_HIP_CHECK(hipEventCreateWithFlags(&zdone, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(zdone, aux));
    }
    // the bucketing runs on the aux stream under the screen + FFT
    std::vector<hipEvent_t> ev = bucket_parts(P, in, false, st);
    if (P.subsort) subsort_parts(P, st);
    if (!zdone && !accumulate && nvis > 0) {
        if (in.vis_dtype == SDP_HIP_C128)
            k_zero_vis<double2><<<grid1d(nvis, 256), 256, 0, st>>>(
                in.nrow, in.nchan, (double2 *)vis, in.vrs, in.vcs, oc);
        else
            k_zero_vis<float2><<<grid1d(nvis, 256), 256, 0, st>>>(
                in.nrow, in.nchan, (float2 *)vis, in.vrs, in.vcs, oc);
    }
    // all planes in one pass into plain contiguous c64 visibilities: the
    // register degridders apply the record factor and write each visibility
    // once (k_zero_vis above covers the ones with no record)
    const bool trivial_oc = oc.npv == 1 && oc.cre[0] == 1.0 && oc.cim[0] == 0.0;
    if (P.chunk_planes == g.nplanes && !accumulate && in.vis_dtype != SDP_HIP_C128 && trivial_oc &&
        in.vcs == 1 && in.vrs == in.nchan &&
        (P.subsort || g.sub == kTileFine || g.sub == kTileCell) &&
        !std::getenv("SDP_HIP_NO_DIRECT"))
        P.vdirect = static_cast<float2 *>(vis);
    float2 *acc = P.vdirect ? nullptr : scratch<float2>("degrid_acc", std::max<int64_t>(nvis, 1));
    if (acc)
        SDP_HIP_CHECK(hipMemsetAsync(acc, 0, std::max<int64_t>(nvis, 1) * sizeof(float2), st));
    float tgrid = 0, tfft = 0, tscr = 0;
    bool waited = false;
    for (int p_lo = 0; p_lo < g.nplanes; p_lo += P.chunk_planes) {
        const int p_hi = std::min(g.nplanes, p_lo + P.chunk_planes);
        const int np = p_hi - p_lo;
        if (zdone) {
            SDP_HIP_CHECK(hipStreamWaitEvent(st, zdone, 0));
            SDP_HIP_CHECK(hipEventDestroy(zdone));
            zdone = nullptr;
        } else {
            zero_band(P, np, st);
        }
        for (int sb = 0; sb < np; sb += P.fft_planes) {
            const int nb = std::min(P.fft_planes, np - sb);
            StageTimer t2(st);
            t2.mark();
            const dim3 grd(grid1d(g.ngx, 256), g.ny);
            k_screen_adj_t<<<grd, 256, 0, st>>>(g, dirty, sx, sy, p_lo + sb, nb, P.spec, tab);
            SDP_HIP_CHECK(hipGetLastError());
            t2.mark();
            fft_rows_x(P, nb, HIPFFT_FORWARD, st);
            if (P.row_hi > P.row_lo)
                k_tr_t_to_grid<<<tr_grid(g, P.row_hi - P.row_lo, nb), dim3(kTr, kTrRows), 0,
                                 st>>>(g, P.spec, P.grid + (size_t)sb * g.ngx * g.ngy, P.row_lo,
                                       P.row_hi);
            SDP_HIP_CHECK(hipGetLastError());
            fft_rows_y(P, sb, nb, HIPFFT_FORWARD, st);
            t2.mark();
            tscr += t2.ms(0, 1);
            tfft += t2.ms(1, 2);
        }
        if (P.aux_bucketing && !P.pipelined && !waited)
            read_part_meta(P, aux_stream());  // host waits for the bucketing only
        for (size_t i = 0; i < P.parts.size(); ++i) {
            if (!ev.empty() && !waited) SDP_HIP_CHECK(hipStreamWaitEvent(st, ev[i], 0));
            StageTimer tg(st);
            tg.mark();
#define SDP_LAUNCH_DEGRID(WW) launch_degrid<WW>(P, P.parts[i], p_lo, p_hi, acc, st)
            SDP_W_DISPATCH(g.W, SDP_LAUNCH_DEGRID);
#undef SDP_LAUNCH_DEGRID
            SDP_HIP_CHECK(hipGetLastError());
            tg.mark();
            tgrid += tg.ms(0, 1);
        }
        waited = true;
    }
    if (zdone) {  // (no plane pass ran)
        SDP_HIP_CHECK(hipStreamWaitEvent(st, zdone, 0));
        SDP_HIP_CHECK(hipEventDestroy(zdone));
    }
    for (size_t i = 0; i < P.parts.size() && !P.vdirect; ++i) {
        const Part &pt = P.parts[i];
        if (pt.nvis == 0) continue;
        const unsigned *ndev = P.pipelined ? pt.meta + 2 : nullptr;
        const unsigned nb = std::min<unsigned>(grid1d(pt.nvis, 256), 16384);
        if (in.vis_dtype == SDP_HIP_C128)
            k_finalize<double2><<<nb, 256, 0, st>>>(pt.nrec, ndev, in.nchan, P.recs + pt.vbase,
                                                    acc + pt.vbase, (double2 *)vis, in.vrs,
                                                    in.vcs, accumulate, oc);
        else
            k_finalize<float2><<<nb, 256, 0, st>>>(pt.nrec, ndev, in.nchan, P.recs + pt.vbase,
                                                   acc + pt.vbase, (float2 *)vis, in.vrs, in.vcs,
                                                   accumulate, oc);
        SDP_HIP_CHECK(hipGetLastError());
    }
    tm.mark();
    if (P.pipelined) read_part_meta(P, st);
    release_events(ev);
    fill_info(P, info);
    if (info) {
        info->ms_prep = tm.on ? tm.ms(0, 1) - tgrid - tfft - tscr : 0.0f;
        info->ms_grid = tgrid;
        info->ms_fft = tfft;
        info->ms_screen = tscr;
    }
}

}  // namespace wstack
}  // namespace sdp

using namespace sdp;

extern "C" {

int sdp_hip_version(void) { return 1; }

int sdp_hip_set_stage_timing(int enable) {
    wstack::g_stage_timing = enable != 0;
    return SDP_HIP_OK;
}

int sdp_hip_device_count(int *count, char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) {
            (void)hipGetLastError();
            n = 0;
        }
        if (count) *count = n;
    });
}

int sdp_hip_release_workspace(char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] { Workspace::get().release(); });
}

int sdp_hip_ms2dirty(const double *uvw, int64_t uvw_row_stride, const double *freq, int nchan,
                     int64_t nrow, const void *vis, int vis_dtype, int64_t vis_row_stride,
                     int64_t vis_chan_stride, const float *wgt, int64_t wgt_row_stride,
                     int64_t wgt_chan_stride, int npix_x, int npix_y, double pixsize_x,
                     double pixsize_y, double epsilon, int do_wstacking, unsigned flags,
                     double *dirty, int64_t dirty_stride_x, int64_t dirty_stride_y, void *stream,
                     sdp_hip_wgrid_info *info, char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        const wstack::Inputs in{uvw,         uvw_row_stride,  freq,           nchan,
                                nrow,        vis,             vis_dtype,      vis_row_stride,
                                vis_chan_stride, wgt,         wgt_row_stride, wgt_chan_stride,
                                npix_x,      npix_y,          pixsize_x,      pixsize_y,
                                epsilon,     do_wstacking,    flags};
        wstack::ms2dirty(in, dirty, dirty_stride_x, dirty_stride_y, info, as_stream(stream));
    });
}

int sdp_hip_ms2dirty_batch(const double *uvw, int64_t uvw_row_stride, const double *freq,
                           int nchan, int64_t nrow, const void *vis, int vis_dtype,
                           int64_t vis_row_stride, int64_t vis_chan_stride, const float *wgt,
                           int64_t wgt_row_stride, int64_t wgt_chan_stride, int npix_x,
                           int npix_y, double pixsize_x, double pixsize_y, double epsilon,
                           int do_wstacking, unsigned flags, const double *bounds,
                           double *dirty, int64_t dirty_stride_x, int64_t dirty_stride_y,
                           void *stream, sdp_hip_wgrid_info *info, char *errbuf,
                           size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(freq != nullptr && (uvw != nullptr || nrow == 0) && bounds != nullptr,
                    "null pointer argument");
        SDP_REQUIRE(dirty != nullptr || !(flags & SDP_HIP_BATCH_LAST),
                    "the last batch needs the dirty image");
        wstack::Inputs in{uvw,         uvw_row_stride,  freq,           nchan,
                          nrow,        vis,             vis_dtype,      vis_row_stride,
                          vis_chan_stride, wgt,         wgt_row_stride, wgt_chan_stride,
                          npix_x,      npix_y,          pixsize_x,      pixsize_y,
                          epsilon,     do_wstacking,    flags};
        in.bounds = bounds;
        wstack::ms2dirty(in, dirty, dirty_stride_x, dirty_stride_y, info, as_stream(stream));
    });
}

int sdp_hip_ms2dirty_vis(const double *uvw, int64_t uvw_row_stride, const double *freq, int nchan,
                         int64_t nrow, const void *vis, int vis_dtype, int64_t vis_row_stride,
                         int64_t vis_chan_stride, int64_t vis_pol_stride, int npol_vis,
                         const double *pol_coeff, const void *wgt, int wgt_dtype,
                         int64_t wgt_row_stride, int64_t wgt_chan_stride, const void *vis_flags,
                         int flag_bytes, int64_t flag_row_stride, int64_t flag_chan_stride,
                         int64_t flag_pol_stride, int pol, int npix_x, int npix_y,
                         double pixsize_x, double pixsize_y, double epsilon, int do_wstacking,
                         unsigned flags, double *dirty, int64_t dirty_stride_x,
                         int64_t dirty_stride_y, double *sumwt, const double *shift_lmn,
                         void *stream, sdp_hip_wgrid_info *info, char *errbuf,
                         size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        SDP_REQUIRE(npol_vis >= 1 && npol_vis <= 4, "npol_vis must be 1..4");
        SDP_REQUIRE(pol >= 0 && pol < npol_vis, "pol out of range");
        SDP_REQUIRE(wgt_dtype == SDP_HIP_F32 || wgt_dtype == SDP_HIP_F64,
                    "weights must be f32 or f64");
        SDP_REQUIRE(vis_flags == nullptr || flag_bytes == 1 || flag_bytes == 4 || flag_bytes == 8,
                    "flag element size must be 1, 4 or 8 bytes");
        wstack::Inputs in{uvw,         uvw_row_stride,  freq,           nchan,
                          nrow,        vis,             vis_dtype,      vis_row_stride,
                          vis_chan_stride, wgt,         wgt_row_stride, wgt_chan_stride,
                          npix_x,      npix_y,          pixsize_x,      pixsize_y,
                          epsilon,     do_wstacking,    flags};
        wstack::VisExtra &x = in.x;
        x.vps = vis_pol_stride;
        x.npv = npol_vis;
        x.wgt_f64 = wgt_dtype == SDP_HIP_F64;
        x.flags = vis_flags;
        x.fbytes = vis_flags ? flag_bytes : 0;
        x.frs = flag_row_stride;
        x.fcs = flag_chan_stride;
        x.fps = flag_pol_stride;
        x.fpol = pol;
        x.sumwt = sumwt;
        if (shift_lmn) {
            x.shift = true;
            x.sl = shift_lmn[0];
            x.sm = shift_lmn[1];
            x.sn = shift_lmn[2];
        }
        if (pol_coeff) {
            x.conv = true;
            for (int k = 0; k < npol_vis; ++k) {
                x.cre[k] = pol_coeff[2 * k];
                x.cim[k] = pol_coeff[2 * k + 1];
            }
        } else if (vis) {
            // no conversion: the image pol is the vis pol `pol`
            in.vis = static_cast<const char *>(vis) +
                     pol * vis_pol_stride * (vis_dtype == SDP_HIP_C128 ? 16 : 8);
        }
        wstack::ms2dirty(in, dirty, dirty_stride_x, dirty_stride_y, info, as_stream(stream));
    });
}

int sdp_hip_dirty2ms(const double *uvw, int64_t uvw_row_stride, const double *freq, int nchan,
                     int64_t nrow, const double *dirty, int64_t dirty_stride_x,
                     int64_t dirty_stride_y, int npix_x, int npix_y, double pixsize_x,
                     double pixsize_y, const float *wgt, int64_t wgt_row_stride,
                     int64_t wgt_chan_stride, double epsilon, int do_wstacking, unsigned flags,
                     void *vis, int vis_dtype, int64_t vis_row_stride, int64_t vis_chan_stride,
                     void *stream, sdp_hip_wgrid_info *info, char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && vis != nullptr &&
                        (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        const wstack::Inputs in{uvw,         uvw_row_stride,  freq,           nchan,
                                nrow,        nullptr,         vis_dtype,      vis_row_stride,
                                vis_chan_stride, wgt,         wgt_row_stride, wgt_chan_stride,
                                npix_x,      npix_y,          pixsize_x,      pixsize_y,
                                epsilon,     do_wstacking,    flags};
        wstack::dirty2ms(in, dirty, dirty_stride_x, dirty_stride_y, vis, info,
                         as_stream(stream));
    });
}

int sdp_hip_dirty2ms_vis(const double *uvw, int64_t uvw_row_stride, const double *freq, int nchan,
                         int64_t nrow, const double *dirty, int64_t dirty_stride_x,
                         int64_t dirty_stride_y, int npix_x, int npix_y, double pixsize_x,
                         double pixsize_y, double epsilon, int do_wstacking, unsigned flags,
                         void *vis, int vis_dtype, int64_t vis_row_stride, int64_t vis_chan_stride,
                         int64_t vis_pol_stride, int npol_vis, const double *pol_coeff,
                         const double *shift_lmn, void *stream, sdp_hip_wgrid_info *info,
                         char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && vis != nullptr &&
                        (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        SDP_REQUIRE(npol_vis >= 1 && npol_vis <= 4, "npol_vis must be 1..4");
        wstack::Inputs in{uvw,         uvw_row_stride,  freq,           nchan,
                          nrow,        nullptr,         vis_dtype,      vis_row_stride,
                          vis_chan_stride, nullptr,     0,              0,
                          npix_x,      npix_y,          pixsize_x,      pixsize_y,
                          epsilon,     do_wstacking,    flags};
        if (shift_lmn) {
            in.x.shift = true;
            in.x.sl = shift_lmn[0];
            in.x.sm = shift_lmn[1];
            in.x.sn = shift_lmn[2];
        }
        wstack::OutConv oc;
        oc.npv = npol_vis;
        oc.vps = vis_pol_stride;
        for (int k = 0; k < npol_vis; ++k) {
            oc.cre[k] = pol_coeff ? pol_coeff[2 * k] : (k == 0 ? 1.0 : 0.0);
            oc.cim[k] = pol_coeff ? pol_coeff[2 * k + 1] : 0.0;
        }
        wstack::dirty2ms(in, dirty, dirty_stride_x, dirty_stride_y, vis, info, as_stream(stream),
                         oc);
    });
}

}  // extern "C"
