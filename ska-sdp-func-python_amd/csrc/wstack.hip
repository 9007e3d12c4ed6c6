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
#include <functional>
#include <memory>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <vector>

#include "sdp_common.h"

namespace sdp {
namespace wstack {

constexpr double kCLight = 299792458.0;
constexpr int kTileCoarse = 16;  // bucket edge (cells) of large grids (sub-sorted by cell)
// one-cell buckets ordered x-pair major (key tile = ((ic >> 1) * ngy + jc) *
// 2 + (ic & 1)), so a bucket's records share their footprint origin and 16
// consecutive buckets form one 2 x 8-cell work-item region
constexpr int kTileCell = 1;
constexpr int kGroupCell = 16;
constexpr int64_t kMaxCellKeys = (int64_t)1 << 28;
constexpr int kGridAlign = 16;   // padded grid edges are multiples of this
constexpr int kChunkMin = 1024;   // records per work item: chosen per call in
constexpr int kChunkMax = 8192;   // [kChunkMin, kChunkMax] (chunk_size())
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
    double su;  // sign applied to u and w (-1 with SDP_HIP_FLIP_UW)
    int nchan;
    int64_t nrow;
    // one-cell keys: blocks of bx x 8 cells (bx = 2, 4 or 8; bxs = log2 bx),
    // each bx / 2 groups of 2 x 8 cells, consecutive in the key order
    int bx, bxs;
    // w slab (SDP_HIP_W_SLAB): this call grids only the visibilities whose
    // first plane lies in [slab_lo, slab_lo + nps) of the sequence's layout of
    // nps_all first planes; w0 is then the slab's first plane, and the others
    // are skipped without being counted as out of bounds
    int slab, slab_lo, nps_all;
    // two-level bucketing of one-cell keys (tiled = 1): the window is cut into
    // tlx x tly bins of 64 x 64 cells per first plane (nbins in all); the
    // keys of a bin are contiguous (bin-major, 4096 per bin)
    int tiled, tlx, tly, nbins;
    double inv_nchan;  // 1 / nchan (the two-level passes' row = v / nchan)
    // folded per-visibility factors (geo_factors): a = u_m s kax, b = v_m s
    // kby, fractional plane pw = w_m s kpw - kpw0 of the FULL layout (a w
    // slab subtracts its first plane as an integer, so slabs partition the
    // visibilities exactly) -- no fp64 division per visibility
    double kax, kby, kpw, kpw0;
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
    bool skip = false;  // w slab: inside the sequence's layout, outside this slab
};

// the visibility's grid coordinates from its row's uvw (metres) and its
// frequency
__device__ __forceinline__ Coord vis_coord_v(const Geo &g, double um, double vm, double wm,
                                             double s) {
    Coord c;
    const double ws = wm * s;
    c.w = g.su * ws;
    const double a = (um * s) * g.kax;
    const double b = (vm * s) * g.kby;
    c.ok = fabs(a) < (double)g.ngx && fabs(b) < (double)g.ngy;
    if (!c.ok) return c;
    const double fa = floor(a - 0.5 * g.W), fb = floor(b - 0.5 * g.W);
    c.du = fa + 1.0 - a;
    c.dv = fb + 1.0 - b;
    c.fu = (float)c.du;
    c.fv = (float)c.dv;
    // (fa + 1 + ng/2) mod ng: |a| < ng puts it in (-ng, 2 ng), so one
    // conditional add or subtract is the modulo (no integer division)
    int ic = (int)fa + 1 + g.ngx / 2, jc = (int)fb + 1 + g.ngy / 2;
    ic = ic >= g.ngx ? ic - g.ngx : (ic < 0 ? ic + g.ngx : ic);
    jc = jc >= g.ngy ? jc - g.ngy : (jc < 0 ? jc + g.ngy : jc);
    c.ic0 = ic;
    c.jc0 = jc;
    // the footprint origin must lie in the bucket window and the first plane
    // in [0, nps): always so when the geometry comes from these
    // visibilities' own extremes (a margin of >= 2 cells / half a plane), but
    // a batch of a batched invert is checked against the bounds its caller
    // gave (out of them it would index outside the histogram or the planes)
    c.ok = (unsigned)(c.ic0 - g.wx0) < (unsigned)g.wnx &&
           (unsigned)(c.jc0 - g.wy0) < (unsigned)g.wny;
    if (g.do_w) {
        const double pw = fma(ws, g.kpw, -g.kpw0);
        const double fp = floor(fmin(fmax(pw - 0.5 * g.W, -2.0), 2.0e9));
        c.dw = fp + 1.0 - pw;
        c.fw = (float)c.dw;
        c.p0 = (int)fp + 1 - g.slab_lo;
        const bool in_slab = c.p0 >= 0 && c.p0 < g.nps;
        c.ok = c.ok && in_slab;
        if (g.slab) c.skip = !in_slab && (unsigned)(c.p0 + g.slab_lo) < (unsigned)g.nps_all;
        c.p0 = min(max(c.p0, 0), g.nps - 1);
    } else {
        c.p0 = 0;
        c.fw = 0.0f;
        c.dw = 0.0;
    }
    return c;
}

__device__ __forceinline__ Coord vis_coord(const Geo &g, const double *__restrict__ uvw,
                                           int64_t rs, int64_t row, double f) {
    return vis_coord_v(g, uvw[row * rs], uvw[row * rs + 1], uvw[row * rs + 2], f / kCLight);
}

// w slab: the visibility's first plane (computed exactly as vis_coord does)
// lies in the sequence's layout but outside this call's slab -- tested before
// anything else of the visibility is read
__device__ __forceinline__ bool slab_out_v(const Geo &g, double wm, double s) {
    const double pw = fma(wm * s, g.kpw, -g.kpw0);
    const int p0 = (int)floor(fmin(fmax(pw - 0.5 * g.W, -2.0), 2.0e9)) + 1 - g.slab_lo;
    return (p0 < 0 || p0 >= g.nps) && (unsigned)(p0 + g.slab_lo) < (unsigned)g.nps_all;
}

__device__ __forceinline__ bool slab_out(const Geo &g, const double *__restrict__ uvw, int64_t rs,
                                         int64_t row, double f) {
    return slab_out_v(g, uvw[row * rs + 2], f / kCLight);
}

// p0-major bucket keys: the items of a range of first planes are contiguous.
// One-cell keys inside a plane: block (x-major), x pair in the block, y, x
// parity -- 16 consecutive keys are a group of 2 x 8 cells.
// Two-level (tiled) one-cell keys: bin = (first plane, 64 x 64-cell tile of
// the window), then inside the bin: x pair (32), y block of 8 (8), and the
// cell of the 2 x 8-cell group, (y & 7) * 2 + (x & 1) -- 16 consecutive keys
// are again one group, 256 groups per bin.
constexpr int kTile = 64;
constexpr int kBinCells = kTile * kTile;
__device__ __forceinline__ unsigned tiled_key(const Geo &g, const Coord &c) {
    const int ic = c.ic0 - g.wx0, jc = c.jc0 - g.wy0;
    const int tile = (ic >> 6) * g.tly + (jc >> 6);
    const int lx = ic & 63, ly = jc & 63;
    const unsigned local = ((unsigned)(((lx >> 1) << 3) | (ly >> 3)) << 4) |
                           (unsigned)((ly & 7) << 1) | (unsigned)(lx & 1);
    return ((unsigned)c.p0 * (unsigned)(g.tlx * g.tly) + (unsigned)tile) * (unsigned)kBinCells +
           local;
}

__device__ __forceinline__ unsigned coord_key(const Geo &g, const Coord &c, int64_t row) {
    if (g.tiled) return tiled_key(g, c);
    const int ic = c.ic0 - g.wx0, jc = c.jc0 - g.wy0;
    const int tile =
        g.sub == kTileCell
            ? ((((ic >> g.bxs) * (g.wny >> 3) + (jc >> 3)) << (g.bxs - 1)) + ((ic & (g.bx - 1)) >> 1)) *
                      16 + (jc & 7) * 2 + (ic & 1)
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
    // select, not multiply: a flagged sample's weight is an exact zero even
    // when the stored weight is NaN or Inf (ducc0 skips zero-weight samples)
    if (x.fbytes) {
        const double m = flag_mask(x, row, chan, x.fpol);
        w = m == 0.0 ? 0.0 : w * m;
    }
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
    // flagged pols contribute exact zeros (select, not multiply: a NaN in a
    // flagged visibility must not reach the image)
    if (!x.conv) {
        if (!x.fbytes) return load_vis(p);
        const double m = flag_mask(x, row, chan, x.fpol);
        if (m == 0.0) return make_float2(0.0f, 0.0f);
        const double2 v = load_vis_d(p);
        return make_float2((float)(v.x * m), (float)(v.y * m));
    }
    double re = 0.0, im = 0.0;
    for (int k = 0; k < x.npv; ++k) {
        if (x.cre[k] == 0.0 && x.cim[k] == 0.0) continue;
        double m = 1.0;
        if (x.fbytes) {
            m = flag_mask(x, row, chan, k);
            if (m == 0.0) continue;
        }
        double2 v = load_vis_d(p + k * x.vps);
        v.x *= m;
        v.y *= m;
        re += x.cre[k] * v.x - x.cim[k] * v.y;
        im += x.cre[k] * v.y + x.cim[k] * v.x;
    }
    return make_float2((float)re, (float)im);
}

template <class T>
struct TypeTag {
    using type = T;
};

template <class VT>
__device__ __forceinline__ double2 eff_vis_d(const VT *vis, int64_t vrs, int64_t vcs,
                                             const VisExtra &x, int64_t row, int chan) {
    const VT *p = vis + row * vrs + chan * vcs;
    if (!x.conv) {
        if (!x.fbytes) return load_vis_d(p);
        const double m = flag_mask(x, row, chan, x.fpol);
        if (m == 0.0) return make_double2(0.0, 0.0);
        const double2 v = load_vis_d(p);
        return make_double2(v.x * m, v.y * m);
    }
    double re = 0.0, im = 0.0;
    for (int k = 0; k < x.npv; ++k) {
        if (x.cre[k] == 0.0 && x.cim[k] == 0.0) continue;
        double m = 1.0;
        if (x.fbytes) {
            m = flag_mask(x, row, chan, k);
            if (m == 0.0) continue;
        }
        double2 v = load_vis_d(p + k * x.vps);
        v.x *= m;
        v.y *= m;
        re += x.cre[k] * v.x - x.cim[k] * v.y;
        im += x.cre[k] * v.y + x.cim[k] * v.x;
    }
    return make_double2(re, im);
}

struct TLoad {
    uint32_t row, chan;
    double um, vm, wm, s, wd;  // s = frequency / c (fsc[chan]: the same division as vis_coord)
    double keep;               // 1 - flag of the weight's pol (1 without flags)
    bool live;
};

// The weight and flag element types are compile-time in the bucketing
// passes -- WT: 4 = f32, 8 = f64 (no weights: a device 1.0f with zero
// strides); FB: 0 = no flags, 1 = int8, 8 = int64 flags (int32 flags are
// widened to int64 first, k_widen_flags) -- and a lane's visibilities load
// from clamped, in-bounds indices with no branch before their first use:
// all of a lane's visibilities' loads (uvw, frequency scale, weight, flag,
// and in the value pass the visibility) are in flight together.  A runtime switch on the
// types, with each load behind its own branch and a `live` test, had put a
// wait for every load before the next one issued (C2 count pass: ~200
// instructions and four serialised memory round trips per visibility).
template <int WT, int FB>
__device__ __forceinline__ TLoad t_load(const Geo &g, int64_t v, int64_t vend,
                                        const double *__restrict__ uvw, int64_t rs,
                                        const double *__restrict__ fsc,
                                        const void *__restrict__ wgt, int64_t wrs, int64_t wcs,
                                        const VisExtra &x) {
    TLoad L;
    L.live = v < vend;
    const uint32_t v32 = (uint32_t)(L.live ? v : vend - 1), nc = (uint32_t)g.nchan;
    // row = v / nchan through the fp64 reciprocal (exact to one step, then
    // corrected), not an integer division
    uint32_t r32 = (uint32_t)((double)v32 * g.inv_nchan);
    if ((uint64_t)r32 * nc > v32) --r32;
    else if ((uint64_t)(r32 + 1u) * nc <= v32) ++r32;
    L.row = r32;
    L.chan = v32 - r32 * nc;
    const double *p = uvw + (int64_t)L.row * rs;
    L.um = p[0];
    L.vm = p[1];
    L.wm = p[2];
    L.s = fsc[L.chan];
    double w;
    const int64_t wi = (int64_t)L.row * wrs + (int64_t)L.chan * wcs;
    if constexpr (WT == 8) w = static_cast<const double *>(wgt)[wi];
    else w = (double)static_cast<const float *>(wgt)[wi];
    L.keep = 1.0;
    if constexpr (FB != 0) {
        using FT = typename std::conditional<FB == 8, int64_t, int8_t>::type;
        L.keep = 1.0 - (double)static_cast<const FT *>(
                           x.flags)[(int64_t)L.row * x.frs + (int64_t)L.chan * x.fcs + x.fpol * x.fps];
        // select, not multiply: a flagged sample's weight is an exact zero
        // even when the stored weight is NaN or Inf
        w = L.keep == 0.0 ? 0.0 : w * L.keep;
    }
    L.wd = L.live ? w : 0.0;
    return L;
}

// int32 flags of a two-level pass as int64 (FB = 8): a contiguous
// [nrow, nchan, npol] copy (one element for a zero-stride broadcast)
__device__ float g_unit_weight = 1.0f;  // the weights of a call without weights
template <class FT>
__global__ void k_widen_flags(const FT *__restrict__ src, int64_t frs, int64_t fcs, int64_t fps,
                              int64_t nrow, int nchan, int npol, int64_t *__restrict__ dst) {
    const int64_t n = nrow * nchan * (int64_t)npol;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t rc = i / npol, row = rc / nchan;
        const int pol = (int)(i - rc * npol), chan = (int)(rc - row * nchan);
        dst[i] = (int64_t)src[row * frs + chan * fcs + pol * fps];
    }
}

// A pol conversion's visibility (x.conv) for the typed passes: every used
// pol's value and flag are loaded before any is combined.  The generic
// eff_vis / eff_vis_d load a pol's flag, branch on it and only then load its
// value, pol after pol -- serialised memory round trips (the 4-pol MFS value
// pass ran at 1.5 TB/s).  Coefficients are uniform, flags selected, not
// multiplied: a NaN in a flagged pol must not reach the image.
template <class VT, int FB>
__device__ __forceinline__ double2 conv_vis(const VT *vis, int64_t vrs, int64_t vcs,
                                            const VisExtra &x, uint32_t row, uint32_t chan) {
    using FT = typename std::conditional<FB == 8, int64_t, int8_t>::type;
    const VT *p = vis + (int64_t)row * vrs + (int64_t)chan * vcs;
    VT v[4];
    FT f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = VT{};
        f[k] = 0;
        if (k < x.npv && (x.cre[k] != 0.0 || x.cim[k] != 0.0)) {
            v[k] = p[k * x.vps];
            if constexpr (FB != 0)
                f[k] = static_cast<const FT *>(
                    x.flags)[(int64_t)row * x.frs + (int64_t)chan * x.fcs + k * x.fps];
        }
    }
    double re = 0.0, im = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < x.npv && (x.cre[k] != 0.0 || x.cim[k] != 0.0)) {
            const double m = 1.0 - (double)f[k];
            const double vx = m == 0.0 ? 0.0 : (double)v[k].x * m;
            const double vy = m == 0.0 ? 0.0 : (double)v[k].y * m;
            re += x.cre[k] * vx - x.cim[k] * vy;
            im += x.cre[k] * vy + x.cim[k] * vx;
        }
    }
    return make_double2(re, im);
}

// the visibility's value in two phases: `load` issues the loads (the
// visibility from clamped indices, beside the lane's other loads), `value`
// combines them after every load is in flight.  Without a pol conversion the
// weight pol's flag (TLoad::keep) masks it; a pol conversion (x.conv, the
// 4-pol frames) reads its pols and flags in `value`.
template <class VT, int KIND, bool kGrid, int FB>
struct TVal {
    using type = typename std::conditional<KIND >= 2, double2, float2>::type;
    __device__ static __forceinline__ VT load(const VT *vis, int64_t vrs, int64_t vcs,
                                              const VisExtra &x, const TLoad &L) {
        VT raw{};
        if constexpr (kGrid)
            if (vis && !x.conv) raw = vis[(int64_t)L.row * vrs + (int64_t)L.chan * vcs];
        return raw;
    }
    __device__ static __forceinline__ type value(const VT *vis, int64_t vrs, int64_t vcs,
                                                 const VisExtra &x, const TLoad &L, VT raw) {
        type xv;
        xv.x = 1;
        xv.y = 0;
        if constexpr (kGrid) {
            if (!vis) return xv;  // (unit visibilities: the PSF)
            if (x.conv) {
                const double2 d = conv_vis<VT, FB>(vis, vrs, vcs, x, L.row, L.chan);
                xv.x = d.x;
                xv.y = d.y;
                return xv;
            }
            const double2 v = make_double2((double)raw.x, (double)raw.y);
            if constexpr (FB == 0) {
                xv.x = v.x;
                xv.y = v.y;
            } else {
                // select, not multiply: a NaN in a flagged visibility must not
                // reach the image
                const double m = L.keep;
                xv.x = m == 0.0 ? 0.0 : v.x * m;
                xv.y = m == 0.0 ? 0.0 : v.y * m;
            }
        }
        return xv;
    }
};

// One visibility of k_bucket (single-level bucketing: the fp32 predict, kept
// buckets, large grids).  Its loads -- uvw, frequency scale, weight, flag,
// and in the value pass its rank and visibility -- are issued together from
// clamped indices (t_load<WT, FB>, TVal), before any of them is used.
template <class VT, bool kScatter, bool kGrid, bool kCompact, int WT, int FB>
__device__ __forceinline__ void bucket_one(const Geo &g, int64_t v, int64_t nvis,
                                           const double *__restrict__ uvw, int64_t uvw_rs,
                                           const double *__restrict__ fsc,
                                           const VT *__restrict__ vis, int64_t vrs, int64_t vcs,
                                           const void *__restrict__ wgt, int64_t wrs,
                                           int64_t wcs, const VisExtra &x, double *sw_slots,
                                           unsigned *counter, unsigned *__restrict__ rk,
                                           VisRec *__restrict__ recs, unsigned long long *nbad,
                                           uint8_t *__restrict__ cls, float2 *__restrict__ zout) {
    using V = TVal<VT, kCompact ? 0 : 1, kGrid, FB>;
    const TLoad L = t_load<WT, FB>(g, v, nvis, uvw, uvw_rs, fsc, wgt, wrs, wcs, x);
    const int64_t vg = (int64_t)L.row * g.nchan + L.chan;  // row * nchan + chan
    // (a w-slab call's outsiders: no rank stored, no weight summed)
    const bool outside = L.live && g.slab && slab_out_v(g, L.wm, L.s);
    const double wd = outside ? 0.0 : L.wd;
    const float wt = (float)wd;
    if (kScatter) {
        const unsigned mine = rk[vg];
        const VT raw = V::load(vis, vrs, vcs, x, L);
        if (sw_slots) {
            // weight sum of a reused bucketing (SDP_HIP_REUSE_BUCKETS): the
            // count pass did not run, so the value pass sums the weights
            double ws = wd;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o, 64);
            if ((threadIdx.x & 63) == 0 && ws != 0.0)
                atomicAdd(&sw_slots[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) &
                                    (kSumSlots - 1)],
                          ws);
        }
        if (!L.live || outside || mine == 0xffffffffu) return;
        const Coord c = vis_coord_v(g, L.um, L.vm, L.wm, L.s);
        const unsigned pos = counter[coord_key(g, c, L.row)] + mine;
        float cr = wt, ci = 0.0f;
        if (kGrid) {
            // a zero-weight sample (bucketed only by a SDP_HIP_KEEP_BUCKETS
            // plan, for the other pols) is an exact zero whatever its
            // visibility holds
            const float2 xv = V::value(vis, vrs, vcs, x, L, raw);
            cr = wt != 0.0f ? xv.x * wt : 0.0f;
            ci = wt != 0.0f ? xv.y * wt : 0.0f;
        }
        if (g.do_w || x.shift) {
            double ph = g.do_w ? c.w * g.s0 : 0.0;
            if (x.shift) ph += (L.um * x.sl + L.vm * x.sm + L.wm * x.sn) * L.s;
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
            // large grids (16x16-cell buckets): the record's cell in its
            // bucket, for the padded sub-sort (k_subsort_pad)
            if (cls) cls[pos] = (uint8_t)(((c.ic0 & 15) >> 1) * 32 + (c.jc0 & 15) * 2 + (c.ic0 & 1));
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
        return;
    }
    // rank pass
    bool valid = L.live && !outside && (x.all || wt != 0.0f);
    Coord c;
    c.ok = false;
    if (valid) {
        c = vis_coord_v(g, L.um, L.vm, L.wm, L.s);
        if (!c.ok) {
            valid = false;
            if (!c.skip) atomicAdd(nbad, 1ull);
        }
    }
    const unsigned key = valid ? coord_key(g, c, L.row) : 0xffffffffu;
    const unsigned rank = run_reserve<true>(key, valid, counter);
    // only the rank is kept: the scatter pass recomputes the key
    if (L.live && !outside) rk[vg] = valid ? rank : 0xffffffffu;
    // a predict writing its visibilities in place zeroes the ones no record
    // reaches here (the degridder writes every other one)
    if (zout && L.live && !valid) zout[vg] = make_float2(0.0f, 0.0f);
    if (sw_slots) {
        // weight sum: wave reduction, one atomic per wave into a slot
        double ws = wd;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o, 64);
        if ((threadIdx.x & 63) == 0 && ws != 0.0)
            atomicAdd(&sw_slots[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) &
                                (kSumSlots - 1)],
                      ws);
    }
}

template <class VT, bool kScatter, bool kGrid, bool kCompact, int WT, int FB>
__global__ void k_bucket(Geo g, int64_t nvis, const double *__restrict__ uvw, int64_t uvw_rs,
                         const double *__restrict__ fsc, const VT *__restrict__ vis, int64_t vrs,
                         int64_t vcs, const void *__restrict__ wgt, int64_t wrs, int64_t wcs,
                         VisExtra x, double *sw_slots, unsigned *counter, unsigned *__restrict__ rk,
                         VisRec *__restrict__ recs, unsigned long long *nbad,
                         uint8_t *__restrict__ cls, float2 *__restrict__ zout) {
    bucket_one<VT, kScatter, kGrid, kCompact, WT, FB>(
        g, blockIdx.x * (int64_t)blockDim.x + threadIdx.x, nvis, uvw, uvw_rs, fsc, vis, vrs, vcs,
        wgt, wrs, wcs, x, sw_slots, counter, rk, recs, nbad, cls, zout);
}

// The image pols of one invert_ng call sharing one bucketing
// (sdp_hip_ms2dirty_vis_pols): image pol q takes row q of the conversion
// matrix over the visibility pols, the weights of pol q masked by the flags
// of pol q, and its own record array.
struct PolsSpec {
    int npo = 0;                              // image pols (<= 4)
    double cre[4][4] = {}, cim[4][4] = {};    // [image pol][vis pol]
    const void *wgt = nullptr;                // weights [row, chan, pol]
    int64_t wrs = 0, wcs = 0, wps = 0;
    RecC *recs[4] = {};
    double *slots[4] = {};                    // weight-sum slots per image pol, or null
};

// The value pass of all image pols at once (one-cell 4-padded plans): each
// visibility's pols, flags and weights are read once and the npo records
// written at the one position the shared bucketing gives it.  One pass per
// image pol read the pol-interleaved visibilities, flags and weights whole
// every time (their cache lines) -- the 4-pol MFS value passes ran 5.7 ms
// each on C2.  The values are those of the per-pol pass bit for bit: the
// conversion sum in fp64 rounded to fp32, times the fp32 masked weight, then
// the record factor.
template <class VT, int WT, int FB, int NPO>
__global__ __launch_bounds__(256) void k_bucket_pols(Geo g, int64_t nvis,
                                                     const double *__restrict__ uvw,
                                                     int64_t uvw_rs,
                                                     const double *__restrict__ fsc,
                                                     const VT *__restrict__ vis, int64_t vrs,
                                                     int64_t vcs, VisExtra x, PolsSpec ps,
                                                     const unsigned *__restrict__ counter,
                                                     const unsigned *__restrict__ rk) {
    using FT = typename std::conditional<FB == 8, int64_t, int8_t>::type;
    using WTT = typename std::conditional<WT == 8, double, float>::type;
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    // (t_load's weight and flag are pol 0's; the loop below reads every pol's)
    const TLoad L = t_load<WT, FB>(g, v, nvis, uvw, uvw_rs, fsc, ps.wgt, ps.wrs, ps.wcs, x);
    const int64_t vg = (int64_t)L.row * g.nchan + L.chan;
    const bool outside = L.live && g.slab && slab_out_v(g, L.wm, L.s);
    // every load of the visibility before any use
    const unsigned mine = rk[vg];
    const VT *pv = vis + (int64_t)L.row * vrs + (int64_t)L.chan * vcs;
    VT vv[4];
    FT ff[4];
    WTT ww[NPO];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        vv[k] = VT{};
        ff[k] = 0;
        if (k < x.npv) {
            vv[k] = pv[k * x.vps];
            if constexpr (FB != 0)
                ff[k] = static_cast<const FT *>(
                    x.flags)[(int64_t)L.row * x.frs + (int64_t)L.chan * x.fcs + k * x.fps];
        }
    }
#pragma unroll
    for (int q = 0; q < NPO; ++q)
        ww[q] = static_cast<const WTT *>(
            ps.wgt)[(int64_t)L.row * ps.wrs + (int64_t)L.chan * ps.wcs + q * ps.wps];
    // the masked weights (select: a flagged sample's weight is an exact zero
    // even when the stored weight is NaN or Inf) and their sums
    double wd[NPO];
#pragma unroll
    for (int q = 0; q < NPO; ++q) {
        double w = (double)ww[q];
        if constexpr (FB != 0) {
            const double keep = 1.0 - (double)ff[q];
            w = keep == 0.0 ? 0.0 : w * keep;
        }
        wd[q] = (L.live && !outside) ? w : 0.0;
        if (ps.slots[q]) {
            double ws = wd[q];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o, 64);
            if ((threadIdx.x & 63) == 0 && ws != 0.0)
                atomicAdd(&ps.slots[q][(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) &
                                       (kSumSlots - 1)],
                          ws);
        }
    }
    if (!L.live || outside || mine == 0xffffffffu) return;
    const Coord c = vis_coord_v(g, L.um, L.vm, L.wm, L.s);
    const unsigned pos = counter[coord_key(g, c, L.row)] + mine;
    float sn = 0.0f, cs = 1.0f;
    const bool rot = g.do_w || x.shift;
    if (rot) {
        double ph = g.do_w ? c.w * g.s0 : 0.0;
        if (x.shift) ph += (L.um * x.sl + L.vm * x.sm + L.wm * x.sn) * L.s;
        ph -= rint(ph);
        sincospif((float)(2.0 * ph), &sn, &cs);
    }
    const double base = 1.0 - 0.5 * g.W;
    const uint32_t qu = fix_frac(base - c.du, 21), qv = fix_frac(base - c.dv, 21);
    const uint32_t qw = g.do_w ? fix_frac(base - c.dw, 22) : 0u;
#pragma unroll
    for (int q = 0; q < NPO; ++q) {
        double re = 0.0, im = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < x.npv && (ps.cre[q][k] != 0.0 || ps.cim[q][k] != 0.0)) {
                double m = 1.0;
                if constexpr (FB != 0) m = 1.0 - (double)ff[k];
                const double vx = m == 0.0 ? 0.0 : (double)vv[k].x * m;
                const double vy = m == 0.0 ? 0.0 : (double)vv[k].y * m;
                re += ps.cre[q][k] * vx - ps.cim[q][k] * vy;
                im += ps.cre[q][k] * vy + ps.cim[q][k] * vx;
            }
        }
        const float wt = (float)wd[q];
        const float xr = (float)re, xi = (float)im;
        const float cr = wt != 0.0f ? xr * wt : 0.0f, ci = wt != 0.0f ? xi * wt : 0.0f;
        RecC rc;
        rc.cre = rot ? cr * cs - ci * sn : cr;
        rc.cim = rot ? cr * sn + ci * cs : ci;
        rc.lo = qu | (qv << 21);
        rc.hi = (qv >> 11) | (qw << 10);
        ps.recs[q][pos] = rc;
    }
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

// One-cell plans: the offsets, pads and work items come from two passes over
// units of `ucells` consecutive cells (the groups of kGroupCell cells whose
// FineItem work items carry the 16 cell ends) instead of a scan over every
// cell.  k_group_sums: per unit its record total (each cell rounded up to a
// multiple of 4 when PAD) and work-item count, packed as (records << 32) |
// items so one 64-bit exclusive scan over the units yields both bases (the
// totals stay below 2^32, so the low half never carries); the pad count is
// added per block into one of kSumSlots slots.
template <bool PAD>
__global__ __launch_bounds__(256) void k_group_sums(int64_t nunits, int ucells,
                                                    const unsigned *__restrict__ hist,
                                                    unsigned chunk,
                                                    unsigned long long *__restrict__ gsum,
                                                    unsigned *__restrict__ pad_slots) {
    __shared__ unsigned red[4];
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    unsigned npad = 0;
    if (k < nunits) {
        const uint4 *h = reinterpret_cast<const uint4 *>(hist + k * ucells);
        unsigned tot = 0;
        for (int q = 0; q < ucells / 4; ++q) {
            const uint4 v = h[q];
            const unsigned n[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const unsigned r = PAD ? (n[j] + 3u) & ~3u : n[j];
                tot += r;
                npad += r - n[j];
            }
        }
        gsum[k] = ((unsigned long long)tot << 32) | (unsigned long long)((tot + chunk - 1) / chunk);
    }
    if (!PAD) return;
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

// k_group_fill: from the scanned unit bases, the cells' record offsets
// (offs[key], what the scatter adds the ranks to; offs[nkeys] = total), the
// zero-valued pad records of the 4-padded cells (RecC, offsets 1 - W/2: in
// range, finite taps; they sit behind each cell's records, where the
// scatter never writes), the units' item bases (ioffs) and their FineItem
// work items.
// the other image pols' record arrays of a pols call (k_bucket_pols): pads too
struct PadMore {
    RecC *r[3] = {nullptr, nullptr, nullptr};
};

template <bool PAD>
__global__ __launch_bounds__(256) void k_group_fill(int64_t nunits, int units_per_plane,
                                                    int ucells,
                                                    const unsigned *__restrict__ hist,
                                                    const unsigned long long *__restrict__ gofs,
                                                    unsigned chunk, unsigned *__restrict__ offs,
                                                    unsigned *__restrict__ ioffs,
                                                    RecC *__restrict__ recs, void *items,
                                                    PadMore more = PadMore{}) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k > nunits) return;
    const unsigned long long go = gofs[k];
    const unsigned base = (unsigned)(go >> 32), ib = (unsigned)go;
    ioffs[k] = ib;
    if (k == nunits) {
        offs[k * ucells] = base;
        return;
    }
    const uint4 *h = reinterpret_cast<const uint4 *>(hist + k * ucells);
    uint4 *of = reinterpret_cast<uint4 *>(offs + k * ucells);
    FineItem x;
    unsigned run = base;
    for (int q = 0; q < ucells / 4; ++q) {
        const uint4 v = h[q];
        const unsigned n[4] = {v.x, v.y, v.z, v.w};
        unsigned st[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            st[j] = run;
            const unsigned r = PAD ? (n[j] + 3u) & ~3u : n[j];
            if (PAD && r != n[j]) {
                RecC z;
                z.cre = z.cim = 0.0f;
                z.lo = z.hi = 0u;
                for (unsigned i = run + n[j]; i < run + r; ++i) {
                    recs[i] = z;
#pragma unroll
                    for (int m = 0; m < 3; ++m)
                        if (more.r[m]) more.r[m][i] = z;
                }
            }
            run += r;
            x.o[(q * 4 + j) & (kGroupCell - 1)] = run;
        }
        of[q] = make_uint4(st[0], st[1], st[2], st[3]);
    }
    x.p0 = (uint32_t)(k / units_per_plane);
    x.tile = (uint32_t)(k - (int64_t)x.p0 * units_per_plane);
    unsigned o = ib;
    FineItem *fi = static_cast<FineItem *>(items);
    for (unsigned s = base; s < run; s += chunk) {
        x.b = s;
        x.e = min(run, s + chunk);
        fi[o++] = x;
    }
}

// the pad count of a 4-padded plan (k_group_sums' per-block slots)
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
                                                 VisRec *recs, FineItem *__restrict__ fitems) {
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
        unsigned a = 0;
        for (int c = 0; c < NC; ++c) {
            first[c] = a;
            a += cur[c];
        }
        first[NC] = a;
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

// Large-grid gridding (invert) on 4-padded cells: the value pass wrote
// 16-byte RecC records in 16x16-cell bucket order plus each record's cell
// class (sub_class<true>, one byte).  k_sub_count: per coarse item its
// record count with every cell rounded up to a multiple of 4 (the scan of
// these places the items' padded records);  k_subsort_pad: the item's
// records staged in LDS, ordered by cell into the padded layout (zero pad
// records, offsets 1 - W/2), and its 16 FineItems (2 x 8-cell groups; empty
// groups have b == e) for k_grid_mfma_pad.
__global__ __launch_bounds__(256) void k_sub_count(const Item *__restrict__ items,
                                                   const uint8_t *__restrict__ cls,
                                                   unsigned *__restrict__ pcnt) {
    __shared__ unsigned h[256];
    __shared__ unsigned red[4];
    const Item it = items[blockIdx.x];
    h[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t i = it.b + threadIdx.x; i < it.e; i += 256) atomicAdd(&h[cls[i]], 1u);
    __syncthreads();
    unsigned r = (h[threadIdx.x] + 3u) & ~3u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = r;
    __syncthreads();
    if (threadIdx.x == 0) pcnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// one workgroup: 64-bit sum of n 32-bit counts
__global__ __launch_bounds__(1024) void k_sum_u32(const unsigned *__restrict__ c, unsigned n,
                                                  unsigned long long *__restrict__ out) {
    __shared__ unsigned long long red[16];
    unsigned long long s = 0;
    for (unsigned i = threadIdx.x; i < n; i += 1024) s += c[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < 16; ++i) t += red[i];
        *out = t;
    }
}

__global__ __launch_bounds__(kSubThreads) void k_subsort_pad(Geo g, const Item *__restrict__ items,
                                                             const RecC *__restrict__ in,
                                                             const uint8_t *__restrict__ cls,
                                                             const unsigned *__restrict__ pbase,
                                                             RecC *__restrict__ out,
                                                             FineItem *__restrict__ fitems) {
    constexpr int NC = 256, PG = 16;
    __shared__ RecC stage[kSubChunk];
    __shared__ uint8_t scls[kSubChunk];
    __shared__ unsigned cnt[NC], first[NC + 1], cur[NC];
    const Item it = items[blockIdx.x];
    const int n = (int)(it.e - it.b);
    const unsigned pb = pbase[blockIdx.x];
    for (int c = threadIdx.x; c < NC; c += kSubThreads) cnt[c] = 0u;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kSubThreads) {
        stage[i] = in[it.b + i];
        const uint8_t k = cls[it.b + i];
        scls[i] = k;
        atomicAdd(&cnt[k], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        // padded exclusive prefix over the 256 cells: 4 per lane, then a
        // wave scan of the lane sums
        const int l = threadIdx.x;
        unsigned r[4], t = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            r[j] = (cnt[4 * l + j] + 3u) & ~3u;
            t += r[j];
        }
        unsigned incl = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(incl, o, 64);
            if (l >= o) incl += y;
        }
        unsigned a = incl - t;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            first[4 * l + j] = a;
            cur[4 * l + j] = a;
            a += r[j];
        }
        if (l == 63) first[NC] = a;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        // fine group gi = 2 * (x pair) + (y half): a 2 x 8-cell region
        const int gi = threadIdx.x, xp = gi >> 1, hf = gi & 1;
        const int c0 = gi * PG;
        FineItem f;
        f.b = pb + first[c0];
        f.e = pb + first[c0 + PG];
#pragma unroll
        for (int j = 0; j < 16; ++j) f.o[j] = pb + first[c0 + j + 1];
        const int tx = (int)it.tile / g.nty, ty = (int)it.tile - tx * g.nty;
        f.tile = (uint32_t)((tx * 8 + xp) * (g.wny / 8) + ty * 2 + hf);
        f.p0 = it.p0;
        fitems[(size_t)blockIdx.x * 16 + threadIdx.x] = f;
    }
    // zero pad records behind each cell's records
    for (int c = threadIdx.x; c < NC; c += kSubThreads) {
        const unsigned e = first[c] + cnt[c], pe = first[c + 1];
        RecC z;
        z.cre = z.cim = 0.0f;
        z.lo = z.hi = 0u;
        for (unsigned i = e; i < pe; ++i) out[pb + i] = z;
    }
    for (int i = threadIdx.x; i < n; i += kSubThreads) {
        const unsigned pos = atomicAdd(&cur[scls[i]], 1u);
        out[pb + pos] = stage[i];
    }
}

// ------------------------------------------------------------------------
// kernels: gridding / degridding (the hot loops)
// ------------------------------------------------------------------------
// first cell (centred grid) of 16-key group `gi` (index inside its first
// plane) of a one-cell plan: block gi / (bx / 2), x pair gi % (bx / 2)
__device__ __forceinline__ void group_origin(const Geo &g, int gi, int &ib, int &jb) {
    if (g.tiled) {  // bin-major: 256 groups per 64 x 64-cell tile, x pair major
        const int tile = gi >> 8, gt = gi & 255;
        const int tx = tile / g.tly, ty = tile - tx * g.tly;
        ib = g.wx0 + tx * kTile + 2 * (gt >> 3);
        jb = g.wy0 + ty * kTile + 8 * (gt & 7);
        return;
    }
    const int ppb = g.bx >> 1;
    const int blk = gi / ppb, xp = gi - blk * ppb;
    const int nby = g.wny >> 3;
    const int bxi = blk / nby, byi = blk - bxi * nby;
    ib = g.wx0 + bxi * g.bx + 2 * xp;
    jb = g.wy0 + byi * 8;
}
// Work items are visited transposed: workgroup w = q m + r (m = n / K)
// takes item r K + q, so the consecutive items of one dense tile (the chunks
// of a heavy cell group) go to workgroups m apart -- spread over the launch
// instead of flushing into the same grid cells at the same time (visiting
// them a few workgroups apart made C2 gridding 5x slower on atomic
// contention), and consecutive workgroups take items K apart.  32-bit
// scalar arithmetic (the previous 64-bit "w * prime % n" cost ~100 SALU per
// item).
constexpr uint32_t kItemSpread = 64;
__device__ __forceinline__ uint32_t item_index(uint32_t w, uint32_t n) {
    const uint32_t m = n / kItemSpread;
    if (w >= kItemSpread * m) return w;
    const uint32_t q = w / m, r = w - q * m;
    return r * kItemSpread + q;
}

__device__ __forceinline__ Item load_item(const Item *items, uint32_t w, uint32_t n) {
    const Item raw = items[item_index(w, n)];
    Item it;
    it.b = __builtin_amdgcn_readfirstlane(raw.b);
    it.e = __builtin_amdgcn_readfirstlane(raw.e);
    it.tile = __builtin_amdgcn_readfirstlane(raw.tile);
    it.p0 = __builtin_amdgcn_readfirstlane(raw.p0);
    return it;
}

// natural: item w itself -- the degridders only read the grid, so they visit
// items in order and neighbouring items' overlapping regions are L2 hits (C2
// k_degrid_mfma 5.55 -> 5.09 ms); the gridders keep the transposed order for
// their atomics
template <int NO>
__device__ __forceinline__ Item load_fine_item(const FineItem *items, uint32_t w, uint32_t n,
                                               uint32_t (&fo)[NO], bool natural = false) {
    const FineItem raw = items[natural ? w : item_index(w, n)];
    Item it;
    it.b = __builtin_amdgcn_readfirstlane(raw.b);
    it.e = __builtin_amdgcn_readfirstlane(raw.e);
    it.tile = __builtin_amdgcn_readfirstlane(raw.tile);
    it.p0 = __builtin_amdgcn_readfirstlane(raw.p0);
#pragma unroll
    for (int j = 0; j < NO; ++j) fo[j] = __builtin_amdgcn_readfirstlane(raw.o[j]);
    return it;
}


// MFMA kernels' operand types and wave-level helpers
typedef float floatx4 __attribute__((ext_vector_type(4)));

// One-wave workgroups: the LDS operations of one wavefront execute in
// program order, so a hand-off between the wave's own lanes through LDS needs
// only a compiler barrier (wavefront-scope fence), not s_barrier plus the
// s_waitcnt lgkmcnt(0) that __syncthreads() brings with it -- the wave keeps
// issuing while its writes drain (C2 gridding 5.26 -> 5.09 ms,
// profiles/r02_pad_ab.txt).  Every gridder / degridder below runs one wave
// per workgroup.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ES kernel for the MFMA gridder's taps: x = fu*ihw + t*ihw by one fma.  For
// W = 8 every tap of the footprint lies inside the support: the first tap's
// offset f is in [-4, -3] and ihw = 1/4 scales exactly, so x = (f + t) / 4 in
// [-1, 1] and y = 1 - x^2 >= 0 with no range select and no clamp (for other
// W, 2/W rounds, so y is clamped and taps outside the support are zeroed)
template <int W>
__device__ __forceinline__ float es_tap(float f, float tihw, float ihw, float bl) {
    const float x = fmaf(f, ihw, tihw);
    const float y = fmaf(-x, x, 1.0f);
    const float e = __builtin_amdgcn_exp2f(
        fmaf(bl, __builtin_amdgcn_sqrtf(W == 8 ? y : fmaxf(y, 0.0f)), -bl));
    return W == 8 ? e : (y > 0.0f ? e : 0.0f);
}

// MFMA gridder on 4-padded cells (invert, one-cell buckets).  The bucketing
// rounds every cell's record count up to a multiple of 4 with zero-valued
// pad records (k_group_fill), so every K-step of 4 consecutive records belongs
// to one cell.  A cell's contribution to its W x W x W footprint is one GEMM
//     C[(q, re/im), (kx, ky)] += sum_r  tw_r[q] c_r  *  tu_r[kx] tv_r[ky]
// on v_mfma_f32_16x16x4_f32 (exact fp32 multiply-adds): A = the w taps x
// value (16 rows: 8 planes x re/im), B = the separable (u, v) taps (4 N-tiles
// of 16 columns), K = 4 records per K-step.
//
// Region-resident accumulation.  With (q, re/im) on the rows, lane l holds
// element i of N-tile t at plane q = 2 (l >> 4) + (i >> 1), component i & 1,
// tap (kx, ky) = (2t + ((l & 15) >> 3), l & 7): its 4 values are 4
// consecutive floats of the footprint cell (xo + kx, yo + ky) when the LDS
// region tile stores each cell's 8 planes x re/im as 16 consecutive floats
// ([x][y][q][re/im], 64 B per cell).  So a cell's accumulators are LOADED
// from the region tile when the cell starts (4 ds_read_b128), the MFMAs add
// on top, and they are STORED back when it ends (4 ds_write_b128): no
// zeroing, no read-add-write per element (the previous layout spent ~80
// VALU + LDS instructions per cell change on that).  A cell's footprint
// overlaps its neighbours', and one wave's LDS operations execute in
// program order, so the store of a cell always precedes the load of the next.
//
// Taps: per block of 16 records the 16 x 3 x 8 one-dimensional taps are
// evaluated once with every lane busy (lane l: tap l & 7 of records
// 8m + (l >> 3)) into an LDS tap block of one 24-float row per record (tu in
// h-major order so a lane's four B taps are one ds_read_b128, tv, tw) and a
// 2-float value row; the 24-float pitch (24 mod 32 banks) makes the tap
// writes and the operand reads bank-conflict-free (the 28-float pitch cost
// 88 % of the LDS cycles in conflicts, profiles/r02_k_grid_mfma_pad_pmc.json).
// The block's (up to) 4 K-steps are unrolled with compile-time LDS offsets.
// The region tile is flushed once per item with buffer float atomics.
// buffer offset past any plane (planes are < 2^32 - 16 bytes): an atomic
// issued there is dropped by the buffer range check
constexpr int kDropOff = -16;
constexpr int kTapRec = 24;    // floats per record row of the tap block
constexpr int kTapBatch = 16;  // records per tap block
constexpr int kRegCell = 16;  // floats per region cell: 8 planes x re/im
// 16-B chunk (plane pair k) of region row y: XOR-swizzled by (y >> 1) & 3
__device__ __forceinline__ int reg_chunk(int k, int y) { return k ^ ((y >> 1) & 3); }

// Work unit of NG groups: 1 (one-cell plans: a chunk of one 2 x 8-cell
// group) or 4 (large grids: 2 x pairs x both y halves of a sub-sorted
// 16 x 16-cell coarse item, gridded into one 11 x 23-cell region -- half
// the flushed atomics of 4 separate 9 x 15-cell regions; C4's sparse groups,
// ~120 records each, flushed 121 GB of atomics per 1.67 Gvis one by one).
template <int NG>
struct PadUnit {
    // NG = 1: one 2 x 8-cell group; NG >= 2: NG / 2 x pairs of a sub-sorted
    // 16x16-cell item, both y halves (groups gi = 2 x pair + y half)
    static constexpr int TX = NG == 1 ? 2 : NG, TY = NG == 1 ? 8 : 16;  // cells
    static constexpr int RGX = TX + 7, RGY = TY + 7;                    // region cells
};

template <int NG>
constexpr size_t grid_mfma_pad_lds() {
    return (size_t)PadUnit<NG>::RGX * PadUnit<NG>::RGY * kRegCell * sizeof(float) +
           kTapBatch * sizeof(float4) + (size_t)kTapBatch * kTapRec * sizeof(float) +
           kTapBatch * sizeof(float2);
}

// The dense uv core's cells take 10^6-10^7 flushed additions per invert (C4's
// whole band: 13.4 Gvis into 71 planes), whose fp32 rounding grows with the
// count and varies with the atomics' order.  A work item whose whole region
// lies in the core window [x0, x0 + nx) x [y0, y0 + ny) therefore flushes into
// c128 companion planes with fp64 atomics; the companion is added to the fp32
// planes once, before the FFT (k_core_merge).  C4 full band against exact
// sums at 64 pixels: 1.9e-6 - 2.8e-6 -> 0.91e-6 - 0.96e-6 relative RMS with a
// 128-cell window (time within 0.3 %; 256 cells: the same error, +0.4 %;
// 512: the same error, +2 %: more items pay fp64 atomics) (scripts/
// c4_precision.py, profiles/r05_c4_precision.jsonl).  Capping
// a cell's fp32 MFMA chain at 64 records (partial sums added to the region
// per batch) changed nothing measurable there and cost C2 4 % of its
// gridding, so the in-item accumulation stays one chain.  p == nullptr: no
// companion.
struct CoreAcc {
    double *p;
    int x0, nx, y0, ny;
};

// Flush of a k_grid_mfma_pad region tile into the planes: the waves of the
// workgroup (wave wv of nwv) take every nwv-th 64-float slice of each plane.
template <int W, bool WS, int NG>
__device__ __forceinline__ void region_flush(const Geo &g, const float *reg, int ibase, int jbase,
                                             uint32_t p0, int p_lo, int p_hi, const CoreAcc &core,
                                             float *__restrict__ grid, int lane, int wv, int nwv) {
    constexpr int NQ = WS ? W : 1;
    constexpr int kRegY = PadUnit<NG>::RGY;
    constexpr int RX = PadUnit<NG>::TX + W - 1, RY = PadUnit<NG>::TY + W - 1;
    // flush: lane l takes float f = i0 + l of a plane's RX x RY cells in
    // the grid's order (x rows of RY cells, re/im interleaved), i.e.
    // region float (x * kRegY + y) * 16 + 4 reg_chunk(q >> 1, y) +
    // 2 (q & 1) + (f & 1); the NQ planes' values are read before any
    // atomic is issued (one LDS wait per 64 floats, not one per plane);
    // buffer atomics off a per-plane descriptor (32-bit offsets); zero
    // floats are dropped by the range check
    constexpr int FPP = RX * RY * 2;
    if (core.p != nullptr && ibase >= core.x0 && ibase + RX <= core.x0 + core.nx &&
        jbase >= core.y0 && jbase + RY <= core.y0 + core.ny) {
        // the whole region lies in the core window: fp64 atomics into the
        // companion planes [p - p_lo][x - x0][y - y0] (c128)
        for (int i0 = 64 * wv; i0 < FPP; i0 += 64 * nwv) {
            const int f = i0 + lane;
            if (f >= FPP) break;
            const int c = f >> 1, xl = c / RY, yl = c - xl * RY;
            const size_t cell = (size_t)(ibase + xl - core.x0) * core.ny + (jbase + yl - core.y0);
            const float *src = reg + (xl * kRegY + yl) * kRegCell + (f & 1);
            float vals[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) vals[q] = src[4 * reg_chunk(q >> 1, yl) + 2 * (q & 1)];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int p = (int)p0 + q;
                if (vals[q] != 0.0f && p >= p_lo && p < p_hi)
                    unsafeAtomicAdd(core.p + ((size_t)(p - p_lo) * core.nx * core.ny + cell) * 2 +
                                        (f & 1),
                                    (double)vals[q]);
            }
        }
        return;
    }
    const size_t plane_bytes = (size_t)g.ngx * g.ngy * sizeof(float2);
    // one buffer descriptor per plane (scalar registers); a plane outside
    // [p_lo, p_hi) gets an empty range, and a zero float an offset past
    // the plane, so the buffer range check drops those atomics: no branch
    __amdgpu_buffer_rsrc_t prs[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int p = (int)p0 + q;
        const bool in = p >= p_lo && p < p_hi;
        prs[q] = __builtin_amdgcn_make_buffer_rsrc(
            in ? grid + (size_t)(p - p_lo) * (plane_bytes / sizeof(float)) : grid, 0,
            in ? (int)plane_bytes : 0, 0x00020000);
    }
#pragma unroll
    for (int i0 = 64 * wv; i0 < FPP; i0 += 64 * nwv) {
        const int f = i0 + lane;
        if (f >= FPP) break;
        const int c = f >> 1, xl = c / RY, yl = c - xl * RY;
        int gx = ibase + xl;
        if (gx >= g.ngx) gx -= g.ngx;
        int gy = jbase + yl;
        if (gy >= g.ngy) gy -= g.ngy;
        const int voff = ((gx * g.ngy + gy) * 2 + (f & 1)) * (int)sizeof(float);
        const float *src = reg + (xl * kRegY + yl) * kRegCell + (f & 1);
        float vals[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) vals[q] = src[4 * reg_chunk(q >> 1, yl) + 2 * (q & 1)];
#pragma unroll
        for (int q = 0; q < NQ; ++q)
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(
                vals[q], prs[q], vals[q] != 0.0f ? voff : kDropOff, 0, 0);
    }
}

template <int W, bool WS, int NG>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_grid_mfma_pad(
    Geo g, const RecC *__restrict__ recs, const FineItem *__restrict__ items, uint32_t n_items,
    float *__restrict__ grid, int p_lo, int p_hi, CoreAcc core) {
    static_assert(W <= 8, "the MFMA tiles hold 8 taps per axis");
    static_assert(NG == 1 || NG == 2 || NG == 4 || NG == 8 || NG == 16, "units of 1-16 groups");
    // (NG = 2, 8, 16 are valid but measured slower on C4; only 1 and 4 are launched)
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int NQ = WS ? W : 1;
    constexpr int kRegX = PadUnit<NG>::RGX, kRegY = PadUnit<NG>::RGY;
    // cells a footprint of the unit reaches
    constexpr int RX = PadUnit<NG>::TX + W - 1, RY = PadUnit<NG>::TY + W - 1;
    float *const reg = reinterpret_cast<float *>(tile);  // [kRegX][kRegY][16]
    float4 *const stage = reinterpret_cast<float4 *>(reg + kRegX * kRegY * kRegCell);
    float *const blk = reinterpret_cast<float *>(stage + kTapBatch);  // [kTapBatch][kTapRec]
    float2 *const cval = reinterpret_cast<float2 *>(blk + kTapBatch * kTapRec);
    const int lane = threadIdx.x;
    const float ihw = g.inv_half_w, bl = g.beta_l2e;
    const float fbase = 1.0f - 0.5f * (float)W;  // RecC offset origin
    // tap phase: tap t = lane & 7 of records 8m + (lane >> 3)
    const int tt = lane & 7;
    const float tihw = (float)tt * ihw;
    float *const tap_dst = blk + (lane >> 3) * kTapRec;
    const int wu = (tt & 1) * 4 + (tt >> 1), wv = 8 + tt, ww = 16 + tt;
    // K-step j: record 4j + (lane >> 4).  B column lane & 15 = (tu h, tv
    // tap); A row lane & 15 = (tw tap, re / im)
    const float *const kB = blk + (lane >> 4) * kTapRec + ((lane >> 3) & 1) * 4;
    const float *const kV = blk + (lane >> 4) * kTapRec + 8 + (lane & 7);
    const float *const kW = blk + (lane >> 4) * kTapRec + 16 + ((lane & 15) >> 1);
    const float *const kC = reinterpret_cast<const float *>(cval) + (lane >> 4) * 2 + (lane & 1);
    // this lane's accumulator slot in a footprint cell (xo, yo) + (kx, ky):
    // region cell (X, Y) = (xo + 2t + h, yo + (l & 7)), float offset
    // (X kRegY + Y) 16 + 4 reg_chunk(l >> 4, Y) -- the 16-B chunk of plane pair
    // k sits at k ^ ((Y >> 1) & 3), so the 8 lanes of a ds_write_b128 group
    // (consecutive Y) cover all 32 banks (unswizzled: 4-way conflicts, and
    // 8-way in the flush reads; profiles/r03_k_grid_mfma_pad_v2_pmc.json)
    const int acc_lane = (((lane & 15) >> 3) * kRegY) * kRegCell;
    const int acc_y = lane & 7, acc_k = lane >> 4;
    constexpr int acc_t = 2 * kRegY * kRegCell;  // + t N-tiles (two x rows each)

    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        // the unit's first group: its origin is the unit's; for NG = 1 the
        // item and the ends of its group's 16 cells (one 80-byte
        // descriptor, scalar loads)
        const uint32_t u = NG == 1 ? w_it : item_index(w_it, n_items);
        uint32_t bnd[kGroupCell];
        Item it = NG == 1 ? load_fine_item<kGroupCell>(items, w_it, n_items, bnd)
                          : load_fine_item<kGroupCell>(items + (size_t)u * NG, 0, 1, bnd);
        if (NG == 1 && it.b >= it.e) continue;
        int ibase, jbase;
        group_origin(g, (int)it.tile, ibase, jbase);
        const uint32_t p0 = it.p0;
        // the first group's first 64 records are requested before the region
        // is zeroed (the load's latency under the LDS stores)
        RecC nx;
        if (it.b < it.e) nx = recs[min(it.b + (uint32_t)lane, it.e - 1)];

        wave_lds_sync();  // the previous item's flush reads of the region
        {
            constexpr int kZ = kRegX * kRegY * kRegCell / 4;  // float4s
            float4 *r4 = reinterpret_cast<float4 *>(reg);
#pragma unroll
            for (int i = 0; i < kZ / 64; ++i) r4[lane + 64 * i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (kZ % 64 && lane < kZ % 64)
                r4[lane + 64 * (kZ / 64)] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }

        // the accumulators and their base offset (floats) in the region: they
        // start as zeros bound to a (zero) region slot of this lane, so the
        // store before every cell's load needs no "first cell" test (a group
        // that follows re-stores the previous group's last cell: the same values
        // to the same slot)
        floatx4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
        int cbase = acc_y * kRegCell + acc_lane + 4 * reg_chunk(acc_k, acc_y);
        auto store_cell = [&]() {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                *reinterpret_cast<floatx4 *>(reg + cbase + t * acc_t) = acc[t];
        };
        struct Ops {
            floatx4 b;
            float v, w, c;
        };
        auto kload = [&](int j) {
            Ops o;
            o.b = *reinterpret_cast<const floatx4 *>(kB + 4 * j * kTapRec);
            o.v = kV[4 * j * kTapRec];
            o.w = kW[4 * j * kTapRec];
            o.c = kC[8 * j];
            return o;
        };
        auto kmfma = [&](const Ops &o) {
            // all five operand products first: no VALU-write -> MFMA-read
            // wait states between the four MFMAs
            const float a = o.w * o.c;
            float bt[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) bt[t] = o.b[t] * o.v;
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bt[t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x0002, 5, 0);  // the 5 VALU products
            __builtin_amdgcn_sched_group_barrier(0x0008, 4, 0);  // then the 4 MFMAs
        };

        for (int gi = 0; gi < NG; ++gi) {
            if (NG > 1 && gi > 0) it = load_fine_item<kGroupCell>(items + (size_t)u * NG + gi, 0, 1, bnd);
            const uint32_t rb = it.b, re = it.e;
            if (rb >= re) continue;  // (empty groups of a sub-sorted coarse item)
            // the group's first cell in the unit: x pair gi >> 1, y half gi & 1
            const int gxo = NG == 1 ? 0 : 2 * (gi >> 1), gyo = NG == 1 ? 0 : 8 * (gi & 1);
            int cur = -1;  // cell of the accumulators (wave-uniform)
            auto load_cell = [&](int cell) {
                const int xo = gxo + (cell & 1), y = gyo + (cell >> 1) + acc_y;
                cbase = (xo * kRegY + y) * kRegCell + acc_lane + 4 * reg_chunk(acc_k, y);
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    acc[t] = *reinterpret_cast<const floatx4 *>(reg + cbase + t * acc_t);
            };

            if (gi > 0) nx = recs[min(rb + (uint32_t)lane, re - 1)];  // (group 0: above)
            for (uint32_t b0 = rb; b0 < re; b0 += 64) {
                const RecC my = nx;
                if (b0 + 64 < re) nx = recs[min(b0 + 64 + (uint32_t)lane, re - 1)];
                const int nb = (int)min(64u, re - b0);  // a multiple of 4
                // cell (x-pair-major index in the group) of the lane's record
                const uint32_t ri = b0 + (uint32_t)lane;
                int cj = 0;
#pragma unroll
                for (int c = 0; c < kGroupCell - 1; ++c) cj += ri >= bnd[c] ? 1 : 0;
                const float fu = fbase - (float)(my.lo & 0x1fffffu) * 0x1p-21f;
                const float fv =
                    fbase - (float)((my.lo >> 21) | ((my.hi & 0x3ffu) << 11)) * 0x1p-21f;
                const float fw = fbase - (float)(my.hi >> 10) * 0x1p-22f;
                // K-steps whose cell differs from the previous K-step's (bit 4j)
                const int prev = __shfl_up(cj, 4);
                uint64_t chg = __ballot((lane & 3) == 0 && lane >= 4 && prev != cj);
                if (__builtin_amdgcn_readfirstlane(cj) != cur) chg |= 1ull;
                // blocks of kTapBatch records: taps, then their K-steps
                for (int h = 0; h < 64 / kTapBatch; ++h) {
                    const int nbh = min(kTapBatch, nb - kTapBatch * h);
                    if (nbh <= 0) break;
                    wave_lds_sync();  // the previous block's tap reads
                    if (lane / kTapBatch == h) {
                        const int r = lane % kTapBatch;
                        stage[r] = make_float4(fu, fv, fw, 0.0f);
                        cval[r] =
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
                            tv_[m][2] =
                                WS ? es_tap<W>(f[m].z, tihw, ihw, bl) : (tt == 0 ? 1.0f : 0.0f);
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
                    // the block's (up to) 4 K-steps unrolled: every operand read
                    // up front at compile-time offsets; a cell change (bit 4j)
                    // stores the accumulators and loads the next cell's
                    Ops o[kTapBatch / 4];
#pragma unroll
                    for (int jj = 0; jj < kTapBatch / 4; ++jj) o[jj] = kload(jj);
#pragma unroll
                    for (int jj = 0; jj < kTapBatch / 4; ++jj) {
                        if (jj < nk) {
                            if ((hchg >> (4 * jj)) & 1ull) {
                                store_cell();
                                cur = __builtin_amdgcn_readlane(cj, kTapBatch * h + 4 * jj);
                                load_cell(cur);
                            }
                            kmfma(o[jj]);
                        }
                    }
                }
            }
            store_cell();
        }
        wave_lds_sync();

        region_flush<W, WS, NG>(g, reg, ibase, jbase, p0, p_lo, p_hi, core, grid, lane, 0, 1);
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
// tu 2k, 2k+1; tv k, k+4; tw 2k, 2k+1), the tu taps shared by ds_bpermute
// (each lane evaluating its group's 4 x 4 tap block itself, with no
// broadcast, measured 5.40 vs 4.69 ms on C2: the transcendentals cost more).
// One wave per work item (a chunk of a group of 16 cells, a 2 x 8-cell
// region), items in their natural order (the grid is only read, so
// neighbouring items' overlapping regions hit L2).  The region's W planes
// are copied into LDS by LDS-DMA, 16-byte cell pairs in rows of 16 cells:
// no staging registers, one round trip per item.  The item's batches (16
// records of one cell; a cell's last batch may be short) run in one flat
// loop: a batch's cell and end come from a ballot over the 16 cell ends (lane
// j holds cell j's), the next batch's records are loaded while this one is
// computed, and the A operands are reloaded only when the cell changes (the
// per-cell loop nest this replaced waited for the prefetched records at every
// cell change: C2 5.05 -> 4.69 ms).  The record factor wgt * exp(-2 pi i w s0)
// is applied and the visibility written in place (VD: out = the
// visibilities), or the raw sum added to out[record] for k_finalize.  Every
// lane stores, without a branch: lanes past the batch's records write to a
// per-block slot of `sink` (a skipped store left the record wait behind the
// previous batch's store), and the 4 lanes of a record write the same value.
// Those duplicate and sink stores cost no HBM traffic: with one lane group
// storing (the others into the sink) WRITE_SIZE stays 2.74 GB per C2 launch
// (2.72 now) for 0.99 GB of visibilities, and a masked store (no sink) gives
// 2.38 GB but 5.09 vs 4.85 ms (profiles/r06_degrid_store_ab.txt): the write
// amplification is the scattered 8-byte visibility stores themselves.
constexpr int kDegridSinkBlocks = 4096;  // sink slots (x 64 lanes)
__device__ float4 g_zero16[1];            // 16 zero bytes (never written)
template <int W, bool WS>
constexpr int degrid_lds_bytes() {  // 16-byte pieces of the region, whole waves of them
    return (((WS ? W : 1) * (W + 1) * 8 + 63) / 64) * 64 * 16;
}
struct DgBatch {
    uint32_t b, ce;  // start, end of its cell's records (clipped to the item)
    int c;           // cell
};
template <int W, bool WS, bool VD>
__global__ __launch_bounds__(64) void k_degrid_mfma(Geo g, const VisRec *__restrict__ recs,
                                                    uint32_t n_items,
                                                    const FineItem *__restrict__ fitems,
                                                    const float2 *__restrict__ grid, int p_lo,
                                                    int p_hi, float2 *__restrict__ out,
                                                    float2 *__restrict__ sink) {
    static_assert(W <= 8, "the MFMA tiles hold 8 taps per axis");
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int RX = 2 + W - 1, RY = 16;  // LDS rows of 16 cells (8 + W - 1 used)
    constexpr int NQ = WS ? W : 1;
    const int lane = threadIdx.x;
    const int r16 = lane & 15, kg = lane >> 4;
    const float ihw = g.inv_half_w, bl = g.beta_l2e;
    const int aq = r16 >> 1, aim = r16 & 1;  // A row (q, re/im)
    const float tu0 = (float)(2 * kg) * ihw, tu1 = (float)(2 * kg + 1) * ihw;
    const float tv0 = (float)kg * ihw, tv1 = (float)(kg + 4) * ihw;
    const float *const ftile = reinterpret_cast<const float *>(tile);
    const int64_t plane_elems = (int64_t)g.ngx * g.ngy;
    float2 *const dump = sink + (blockIdx.x & (kDegridSinkBlocks - 1)) * 64 + lane;

    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        uint32_t fo[kGroupCell];
        const Item it = load_fine_item<kGroupCell>(fitems, w_it, n_items, fo, true);
        if (it.b >= it.e) continue;
        const uint32_t ie = it.e;
        const uint32_t fol = fitems[w_it].o[r16];  // lane j < 16: end of cell j's records
        // the batch starting at record x: the first cell whose end exceeds x
        auto locate = [&](uint32_t x) {
            DgBatch s;
            s.b = x;
            const uint64_t m = __ballot(fol > x) & 0xffffull;
            s.c = m ? (int)__builtin_ctzll(m) : kGroupCell;
            s.ce = min(m ? (uint32_t)__builtin_amdgcn_readlane((int)fol, s.c) : ie, ie);
            return s;
        };
        // the next batch: the rest of this cell, else the next non-empty cell
        auto advance = [&](const DgBatch &s) {
            const uint32_t nb = min(s.b + 16u, s.ce);
            if (nb < s.ce || nb >= ie) {
                DgBatch t = s;
                t.b = nb;
                return t;
            }
            return locate(nb);
        };
        int ibase, jbase;
        group_origin(g, (int)it.tile, ibase, jbase);

        DgBatch s0 = locate(it.b);
        DgBatch s1 = advance(s0);
        // the first batch's records are requested before the region
        VisRec nxt = recs[min(s0.b + (uint32_t)r16, ie - 1)];
        wave_lds_sync();  // previous item's reads of the region
        {
            // piece i: plane q, row xl, cell pair m (jbase and ngy are even, so
            // a pair never straddles the y wrap); planes outside the call's
            // range (and the pieces past the region) read 16 zero bytes
            constexpr int NPC = RX * 8, NGL = degrid_lds_bytes<W, WS>() / 1024;
#pragma unroll
            for (int k = 0; k < NGL; ++k) {
                const int i = lane + 64 * k;
                const int q = i / NPC, rem = i - q * NPC, xl = rem >> 3, m = rem & 7;
                const int p = (int)it.p0 + q;
                int gx = ibase + xl;
                if (gx >= g.ngx) gx -= g.ngx;
                int gy = jbase + 2 * m;
                if (gy >= g.ngy) gy -= g.ngy;
                const void *src = (q < NQ && p >= p_lo && p < p_hi)
                                      ? (const void *)(grid + (int64_t)(p - p_lo) * plane_elems +
                                                       (int64_t)gx * g.ngy + gy)
                                      : (const void *)g_zero16;
                __builtin_amdgcn_global_load_lds(
                    src,
                    (__attribute__((address_space(3))) void *)(
                        (__attribute__((address_space(3))) char *)tile + 1024 * k),
                    16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }

        int acell = -1;
        float a[16];
        while (s0.b < ie) {
            if (s0.c != acell) {
                acell = s0.c;
                const int xo = acell & 1, yo = acell >> 1;
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    const int kx = s >> 1, ky = 4 * (s & 1) + kg;
                    a[s] = (aq < NQ && kx < W && ky < W)
                               ? ftile[((aq * RX + xo + kx) * RY + yo + ky) * 2 + aim]
                               : 0.0f;
                }
            }
            const float fu = nxt.fu, fv = nxt.fv, fw = nxt.fw, cre = nxt.cre, cim = nxt.cim;
            const uint32_t idx = nxt.idx;
            const uint32_t ri = s0.b + (uint32_t)r16;
            const bool valid = ri < s0.ce;
            nxt = recs[min(s1.b + (uint32_t)r16, ie - 1)];
            // (the next batch's loads issue first, a whole batch ahead of use)
            __builtin_amdgcn_sched_barrier(0);
            const float u0 = es_tap<W>(fu, tu0, ihw, bl);
            const float u1 = es_tap<W>(fu, tu1, ihw, bl);
            float tu[8];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                tu[2 * h] = __shfl(u0, r16 + 16 * h);
                tu[2 * h + 1] = __shfl(u1, r16 + 16 * h);
            }
            // all 8 tap broadcasts in flight before the v / w taps are
            // evaluated under them
            __builtin_amdgcn_sched_barrier(0);
            const float v0 = es_tap<W>(fv, tv0, ihw, bl);
            const float v1 = es_tap<W>(fv, tv1, ihw, bl);
            const float w0 = WS ? es_tap<W>(fw, tu0, ihw, bl) : (kg == 0 ? 1.0f : 0.0f);
            const float w1 = WS ? es_tap<W>(fw, tu1, ihw, bl) : 0.0f;
            floatx4 d0 = floatx4{0.0f, 0.0f, 0.0f, 0.0f}, d1 = d0;
#pragma unroll
            for (int s = 0; s < 16; s += 2) {
                d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], tu[s >> 1] * v0, d0, 0, 0, 0);
                d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s + 1], tu[s >> 1] * v1, d1, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            // row 4 kg + i of D = (q = 2 kg + (i >> 1), re/im = i & 1)
            float sr = w0 * (d0[0] + d1[0]) + w1 * (d0[2] + d1[2]);
            float si = w0 * (d0[1] + d1[1]) + w1 * (d0[3] + d1[3]);
            sr += __shfl_xor(sr, 16);
            si += __shfl_xor(si, 16);
            sr += __shfl_xor(sr, 32);
            si += __shfl_xor(si, 32);
            if constexpr (VD) {
                float2 *const dst = valid ? out + idx : dump;
                *dst = make_float2(cre * sr - cim * si, cre * si + cim * sr);
            } else {
                float2 *const dst = valid ? out + ri : dump;
                float2 v = *dst;
                v.x += sr;
                v.y += si;
                *dst = v;
            }
            s0 = s1;
            s1 = advance(s1);
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

// complex element of the planes: float2 (fp32 path) or double2 (fp64 path)
template <class T>
__device__ __forceinline__ T cplx(double re, double im) {
    T v;
    v.x = re;
    v.y = im;
    return v;
}
template <class T>
__device__ __forceinline__ void sincospi_t(double x, double *sn, double *cs) {
    if constexpr (std::is_same<T, double2>::value) {
        sincospi(x, sn, cs);
    } else {
        float s_, c_;
        sincospif((float)x, &s_, &c_);
        *sn = s_;
        *cs = c_;
    }
}

// ---- transposed y-spectrum layout for the pruned 2-D FFT -------------
// T[q][iy][kx] (iy = image row index 0..ny-1, i.e. ky = (iy - ny/2) mod ngy;
// kx = 0..ngx-1) holds, per plane, the needed y-frequency columns of the grid
// transposed so the x-direction transform runs over contiguous rows.
constexpr int kTr = 64;      // transpose tile edge
constexpr int kTrRows = 4;   // threads along the tile's second axis (64 x 4 = 256)

// grid[q][x][ky(iy)] -> T[q][iy][x] for the rows x in [row_lo, row_hi); the
// rest of each T row is kept zero by the caller (persistent zeros)
template <class T>
__global__ __launch_bounds__(256) void k_tr_grid_to_t(Geo g, const T *__restrict__ grid,
                                                      T *__restrict__ t, int row_lo, int row_hi) {
    __shared__ T sm[kTr][kTr + 1];
    const int x0 = row_lo + blockIdx.x * kTr, i0 = blockIdx.y * kTr, q = blockIdx.z;
    const int64_t plane = (int64_t)g.ngx * g.ngy, tplane = (int64_t)g.ny * g.ngx;
    for (int r = threadIdx.y; r < kTr; r += kTrRows) {
        const int x = x0 + r, iy = i0 + threadIdx.x;
        T v = cplx<T>(0.0, 0.0);
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
template <class T>
__global__ __launch_bounds__(256) void k_tr_t_to_grid(Geo g, const T *__restrict__ t,
                                                      T *__restrict__ grid, int row_lo, int row_hi) {
    __shared__ T sm[kTr][kTr + 1];
    const int x0 = row_lo + blockIdx.x * kTr, i0 = blockIdx.y * kTr, q = blockIdx.z;
    const int64_t plane = (int64_t)g.ngx * g.ngy, tplane = (int64_t)g.ny * g.ngx;
    for (int r = threadIdx.y; r < kTr; r += kTrRows) {
        const int iy = i0 + r, x = x0 + threadIdx.x;
        sm[r][threadIdx.x] = (iy < g.ny && x < row_hi) ? t[q * tplane + (int64_t)iy * g.ngx + x]
                                                       : cplx<T>(0.0, 0.0);
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

// c64 planes with ny % 4 == 0: the same transposes with 16-byte accesses (two
// complex per lane; image rows come in even pairs, so a pair never straddles
// the ky wrap) over tiles aligned to 64 grid rows.  grid -> T writes the
// whole aligned tile: its rows below row_lo read as zeros, which T holds
// there anyway.
__global__ __launch_bounds__(256) void k_tr_grid_to_t16(Geo g, const float2 *__restrict__ grid,
                                                        float2 *__restrict__ t, int row_lo,
                                                        int row_hi) {
    __shared__ float2 sm[kTr][kTr + 1];
    const int x0 = (row_lo & ~(kTr - 1)) + blockIdx.x * kTr, i0 = blockIdx.y * kTr, q = blockIdx.z;
    const int64_t plane = (int64_t)g.ngx * g.ngy, tplane = (int64_t)g.ny * g.ngx;
    const int tid = threadIdx.y * kTr + threadIdx.x, c2 = tid & 31, rr = tid >> 5;
    {
        const int iy = i0 + 2 * c2;
        const int Y = iy - g.ny / 2;
        const int ky = Y < 0 ? Y + g.ngy : Y;
#pragma unroll
        for (int r = rr; r < kTr; r += 8) {
            const int x = x0 + r;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (x >= row_lo && x < row_hi && iy < g.ny)
                v = *reinterpret_cast<const float4 *>(grid + q * plane + (int64_t)x * g.ngy + ky);
            sm[r][2 * c2] = make_float2(v.x, v.y);
            sm[r][2 * c2 + 1] = make_float2(v.z, v.w);
        }
    }
    __syncthreads();
    const int x = x0 + 2 * c2;
#pragma unroll
    for (int r = rr; r < kTr; r += 8) {
        const int iy = i0 + r;
        if (iy < g.ny && x < g.ngx) {
            const float2 a = sm[2 * c2][r], b = sm[2 * c2 + 1][r];
            *reinterpret_cast<float4 *>(t + q * tplane + (int64_t)iy * g.ngx + x) =
                make_float4(a.x, a.y, b.x, b.y);
        }
    }
}

__global__ __launch_bounds__(256) void k_tr_t_to_grid16(Geo g, const float2 *__restrict__ t,
                                                        float2 *__restrict__ grid, int row_lo,
                                                        int row_hi) {
    __shared__ float2 sm[kTr][kTr + 1];
    const int x0 = (row_lo & ~(kTr - 1)) + blockIdx.x * kTr, i0 = blockIdx.y * kTr, q = blockIdx.z;
    const int64_t plane = (int64_t)g.ngx * g.ngy, tplane = (int64_t)g.ny * g.ngx;
    const int tid = threadIdx.y * kTr + threadIdx.x, c2 = tid & 31, rr = tid >> 5;
    {
        const int x = x0 + 2 * c2;
#pragma unroll
        for (int r = rr; r < kTr; r += 8) {
            const int iy = i0 + r;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (iy < g.ny && x < g.ngx)
                v = *reinterpret_cast<const float4 *>(t + q * tplane + (int64_t)iy * g.ngx + x);
            sm[2 * c2][r] = make_float2(v.x, v.y);
            sm[2 * c2 + 1][r] = make_float2(v.z, v.w);
        }
    }
    __syncthreads();
    const int iy = i0 + 2 * c2;
    const int Y = iy - g.ny / 2;
    const int ky = Y < 0 ? Y + g.ngy : Y;
#pragma unroll
    for (int r = rr; r < kTr; r += 8) {
        const int x = x0 + r;
        if (x >= row_lo && x < row_hi && iy < g.ny) {
            const float2 a = sm[r][2 * c2], b = sm[r][2 * c2 + 1];
            *reinterpret_cast<float4 *>(grid + q * plane + (int64_t)x * g.ngy + ky) =
                make_float4(a.x, a.y, b.x, b.y);
        }
    }
}

// w screens + grid correction reading the transposed spectrum (ix fastest:
// coalesced T reads; RASCIL's transposed output (sx = 1) is coalesced too)
template <class T>
__global__ void k_screen_fwd_t(Geo g, const T *__restrict__ t, int p_begin, int np,
                               double *dirty, int64_t sx, int64_t sy, int accumulate,
                               const double *__restrict__ tab) {
    const int ix = blockIdx.x * blockDim.x + threadIdx.x;
    const int iy = blockIdx.y;
    if (ix >= g.nx) return;
    const PixelGeom p = pixel_geom(g, ix, iy, tab);
    double res = 0.0;
    if (p.inside) {
        const int64_t tplane = (int64_t)g.ny * g.ngx;
        const T *src = t + (int64_t)iy * g.ngx + p.gx;
        if (g.do_w) {
            double acc = 0.0;
            for (int q = 0; q < np; ++q) {
                const T h = src[q * tplane];
                double ph = (g.w0 + (p_begin + q) * g.dw) * p.s;
                ph -= rint(ph);
                double sn, cs;
                sincospi_t<T>(2.0 * ph, &sn, &cs);
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

// adjoint: T[q][iy][kx] = screen(q) * corr * dirty for the kx of the image's
// x-frequencies (thread ix: kx = (ix - nx/2) mod ngx); the other kx of the
// forward x-FFT's input stay zero across calls (adj_input)
template <class T>
__global__ void k_screen_adj_t(Geo g, const double *__restrict__ dirty, int64_t sx, int64_t sy,
                               int p_begin, int np, T *__restrict__ t,
                               const double *__restrict__ tab) {
    const int ix = blockIdx.x * blockDim.x + threadIdx.x;
    const int iy = blockIdx.y;
    if (ix >= g.nx) return;
    const int X = ix - g.nx / 2;
    const int kx = X < 0 ? X + g.ngx : X;
    const int64_t tplane = (int64_t)g.ny * g.ngx;
    T *dst = t + (int64_t)iy * g.ngx + kx;
    const PixelGeom p = pixel_geom(g, ix, iy, tab);
    const double val = p.inside ? dirty[ix * sx + iy * sy] * p.corr : 0.0;
    if (g.do_w) {
        for (int q = 0; q < np; ++q) {
            double ph = (g.w0 + (p_begin + q) * g.dw) * p.s;
            ph -= rint(ph);
            double sn, cs;
            sincospi_t<T>(2.0 * ph, &sn, &cs);
            dst[q * tplane] = cplx<T>(val * cs, -val * sn);
        }
    } else {
        dst[0] = cplx<T>(val, 0.0);
    }
}

// ---- fused x-FFT + w screens (fp32 planes, power-of-two ngx) ------------
// One workgroup per image row iy.  Per plane of the batch the T row (c64,
// N = ngx points) is transformed in LDS by a Stockham mixed-radix FFT: N / 16
// threads hold 16 points each, radix-16 passes and at most one radix-2/4/8
// pass (natural-order output, no bit reversal), LDS padded by one element
// per 16 so the strided pass-0 writes are conflict-free.  The twiddles do not
// depend on the plane: each thread's w, w^2, w^4, w^8 per pass are computed
// once by sincospif (exact fractions) and the other powers by at most three
// products.  The invert screens the FFT's image columns straight from LDS
// into fp64 registers (the x-spectra are never written), the predict
// screens the image into the FFT's input in LDS (the zero-filled x-FFT input
// is never written or read).
__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// e^{SG 2 pi i m / 16} (SG = +1: backward, -1: forward), m a constant
template <int SG>
__device__ __forceinline__ float2 root16(int m) {
    constexpr float c16[16] = {1.0f,
                               0.92387953251128673848f,
                               0.70710678118654752440f,
                               0.38268343236508978178f,
                               0.0f,
                               -0.38268343236508978178f,
                               -0.70710678118654752440f,
                               -0.92387953251128673848f,
                               -1.0f,
                               -0.92387953251128673848f,
                               -0.70710678118654752440f,
                               -0.38268343236508978178f,
                               0.0f,
                               0.38268343236508978178f,
                               0.70710678118654752440f,
                               0.92387953251128673848f};
    m &= 15;
    return make_float2(c16[m], SG * c16[(m + 12) & 15]);  // sin = cos(. - pi/2)
}

// R-point DFT (R = 2, 4, 8, 16) of v[0..R) in registers, radix-2
// decimation in frequency: the result leaves bit-reversed (out[bitrev(r)] =
// v[r]); the callers index it through fx_brev
template <int R, int SG>
__device__ __forceinline__ void fx_dft(float2 *v) {
#pragma unroll
    for (int L = R; L >= 2; L >>= 1) {
        const int h = L >> 1;
#pragma unroll
        for (int s = 0; s < R; s += L) {
#pragma unroll
            for (int k = 0; k < h; ++k) {
                const float2 a = v[s + k], b = v[s + k + h];
                v[s + k] = make_float2(a.x + b.x, a.y + b.y);
                const float2 d = make_float2(a.x - b.x, a.y - b.y);
                v[s + k + h] = k == 0 ? d : cmulf(d, root16<SG>(k * (16 / L)));
            }
        }
    }
}

template <int R>
__device__ __forceinline__ constexpr int fx_brev(int r) {
    int o = 0;
    for (int b = 1, t = R >> 1; b < R; b <<= 1, t >>= 1)
        if (r & b) o |= t;
    return o;
}

__device__ __forceinline__ int fx_pad(int i) { return i + (i >> 4); }
// fx_pad(t + c), pt = fx_pad(t), c a multiple of T: for T % 16 == 0 it is
// pt + 17 c / 16 (an immediate offset from one base)
template <int T>
__device__ __forceinline__ int fx_padc(int t, int pt, int c) {
    if constexpr (T % 16 == 0) return pt + (c / 16) * 17;
    else return fx_pad(t + c);
}

// the 15 twiddles w^r, r = 1..15, from w, w^2, w^4, w^8
__device__ __forceinline__ void fx_powers(const float2 (&b)[4], float2 *w) {
    w[1] = b[0];
    w[2] = b[1];
    w[3] = cmulf(b[1], b[0]);
    w[4] = b[2];
    w[5] = cmulf(b[2], b[0]);
    w[6] = cmulf(b[2], b[1]);
    w[7] = cmulf(b[2], w[3]);
#pragma unroll
    for (int r = 1; r < 8; ++r) w[8 + r] = cmulf(b[3], w[r]);
    w[8] = b[3];
}

template <int LOGN>
struct FxShape {
    static constexpr int N = 1 << LOGN;
    static constexpr int T = N / 16;          // threads
    static constexpr int P16 = LOGN / 4;      // radix-16 passes
    static constexpr int RR = 1 << (LOGN % 4);  // last pass radix (1: none)
    static constexpr int LDS = N + N / 16;    // padded float2 elements
    // twiddle table (fx_twiddles), copied into LDS behind the data by each
    // workgroup: radix-16 pass p >= 1 at tw_off(p), w and w^4 per k < 16^p;
    // the last pass's e^{2 pi i t / N} at tw_off(P16)
    static constexpr int tw_off(int p) { return p <= 1 ? 0 : tw_off(p - 1) + 2 * (1 << (4 * (p - 1))); }
    static constexpr int TW = tw_off(P16) + T;
    static constexpr size_t lds_bytes() { return (size_t)(LDS + TW) * 8; }
};

// the transform of the row held as v[r] = X[t + r T] (pass 0's inputs) into
// buf (natural order, padded); ends with the workgroup synchronised
template <int LOGN, int SG>
__device__ __forceinline__ void fx_fft(float2 (&v)[16], float2 *buf, const float2 *__restrict__ twt,
                                       int t) {
    using S = FxShape<LOGN>;
    // pass 0 (Ns = 1): no twiddles, outputs to 16 t + r
    fx_dft<16, SG>(v);
    {
        float2 *const o = buf + 17 * t;  // fx_pad(16 t + r) = 17 t + r
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] = v[fx_brev<16>(r)];
    }
    __syncthreads();
    const int pt = fx_pad(t);
    int ns = 16;
#pragma unroll
    for (int p = 1; p < S::P16; ++p) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = buf[fx_padc<S::T>(t, pt, r * S::T)];
        __syncthreads();
        // twiddles w^r, w = e^{SG 2 pi i k / (16 Ns)}, k = t mod Ns
        const int k = t % ns, d = (t / ns) * ns * 16 + k;
        {
            // (kk opaque: the twiddles are loaded and multiplied out per
            // transform, not hoisted out of the caller's plane loop, where
            // they held ~60 VGPRs)
            int kk = k;
            asm volatile("" : "+v"(kk));
            float2 b[4], w[16];
            const float4 q0 = *reinterpret_cast<const float4 *>(twt + S::tw_off(p) + 2 * kk);
            b[0] = make_float2(q0.x, SG * q0.y);
            b[2] = make_float2(q0.z, SG * q0.w);
            b[1] = cmulf(b[0], b[0]);
            b[3] = cmulf(b[2], b[2]);
            fx_powers(b, w);
#pragma unroll
            for (int r = 1; r < 16; ++r) v[r] = cmulf(v[r], w[r]);
        }
        fx_dft<16, SG>(v);
        const int pd = fx_pad(d);  // (ns >= 16: r ns is a multiple of 16)
#pragma unroll
        for (int r = 0; r < 16; ++r) buf[pd + r * ns + ((r * ns) >> 4)] = v[fx_brev<16>(r)];
        __syncthreads();
        ns *= 16;
    }
    if constexpr (S::RR > 1) {
        // last pass, Ns = N / RR: butterfly j = t + T m reads and writes
        // X[j + r N / RR] in place (no hazard across threads)
        constexpr int RR = S::RR, NB = 16 / RR, STR = S::N / RR;
        int tt = t;
        asm volatile("" : "+v"(tt));
        const float2 l0 = twt[S::tw_off(S::P16) + tt], last = make_float2(l0.x, SG * l0.y);
#pragma unroll
        for (int m = 0; m < NB; ++m) {
            float2 u[RR];
            const int j = t + S::T * m;
#pragma unroll
            for (int r = 0; r < RR; ++r) u[r] = buf[fx_padc<S::T>(t, pt, S::T * m + r * STR)];
            // twiddle w_j^r, w_j = e^{SG 2 pi i j / N} = last * e^{SG 2 pi i m / 16}
            const float2 wj = m == 0 ? last : cmulf(last, root16<SG>(m));
            float2 wr = wj;
#pragma unroll
            for (int r = 1; r < RR; ++r) {
                u[r] = cmulf(u[r], wr);
                if (r + 1 < RR) wr = cmulf(wr, wj);
            }
            fx_dft<RR, SG>(u);
#pragma unroll
            for (int r = 0; r < RR; ++r) buf[fx_padc<S::T>(t, pt, S::T * m + r * STR)] = u[fx_brev<RR>(r)];
        }
        __syncthreads();
    }
}

// the workgroup's LDS copy of the twiddle table (behind the data buffer)
template <int LOGN>
__device__ __forceinline__ float2 *fx_twl(float2 *fbuf, const float2 *__restrict__ twg, int t) {
    using S = FxShape<LOGN>;
    float2 *const twl = fbuf + S::LDS;
    for (int i = t; i < S::TW; i += S::T) twl[i] = twg[i];
    __syncthreads();
    return twl;
}

// pass 0's inputs v[r] = X[t + r T] of one T row; the columns outside the
// band [lo, hi) are zeros in the buffer and are not read
template <int LOGN>
__device__ __forceinline__ void fx_load_row(float2 (&v)[16], const float2 *__restrict__ row, int t,
                                            int lo, int hi) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int i = t + r * FxShape<LOGN>::T;
        v[r] = (i >= lo && i < hi) ? row[i] : make_float2(0.0f, 0.0f);
    }
}

// invert: dirty(ix, iy) (+)= corr * sum_q Re(FFT_x(T_in[q][iy])[gx] e^{2 pi i w_q s})
template <int LOGN>
__global__ __launch_bounds__(FxShape<LOGN>::T) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_xfft_screen_fwd(
    Geo g, const float2 *__restrict__ tin, int row_lo, int row_hi, int p_begin, int np,
    double *dirty, int64_t sx, int64_t sy, int accumulate, const double *__restrict__ tab,
    const float2 *__restrict__ twg) {
    using S = FxShape<LOGN>;
    constexpr int PX = 8;  // pixels per thread: nx <= N / 2 = 8 T
    extern __shared__ float2 fbuf[];
    const int t = threadIdx.x, iy = blockIdx.x;
    float2 *const twl = fx_twl<LOGN>(fbuf, twg, t);
    // (each pixel's s is recomputed per plane, as pixel_geom does: 16 VGPRs of
    // stored s pushed the kernel past 128 VGPRs into scratch)
    double acc[PX];
#pragma unroll
    for (int m = 0; m < PX; ++m) acc[m] = 0.0;
    const double mm = (iy - g.ny / 2) * g.py, m2 = mm * mm;
    const int64_t tplane = (int64_t)g.ny * g.ngx;
    const float2 *row = tin + (int64_t)iy * g.ngx;
    float2 v[16];
    fx_load_row<LOGN>(v, row, t, row_lo, row_hi);
    for (int q = 0; q < np; ++q) {
        fx_fft<LOGN, 1>(v, fbuf, twl, t);
        if (q + 1 < np) fx_load_row<LOGN>(v, row + (q + 1) * tplane, t, row_lo, row_hi);  // (in flight under the screens)
        const double wq = g.w0 + (p_begin + q) * g.dw;
        int tt = t;  // (opaque: the pixels' LDS addresses are not hoisted out of the plane loop)
        asm volatile("" : "+v"(tt));
#pragma unroll
        for (int m = 0; m < PX; ++m) {
            const int ix = tt + m * S::T;
            if (ix < g.nx) {
                const int X = ix - g.nx / 2;
                const float2 h = fbuf[fx_pad(X < 0 ? X + g.ngx : X)];
                if (g.do_w) {
                    const double l = X * g.px, r2 = l * l + m2;
                    const double sp = r2 < 1.0 ? r2 / (sqrt(1.0 - r2) + 1.0) - g.s0 : 0.0;
                    double ph = wq * sp;
                    ph -= rint(ph);
                    double sn, cs;
                    sincospi_t<float2>(2.0 * ph, &sn, &cs);
                    acc[m] += (double)h.x * cs - (double)h.y * sn;
                } else {
                    acc[m] += (double)h.x;
                }
            }
        }
        __syncthreads();  // (the next plane's pass 0 overwrites the buffer)
    }
#pragma unroll
    for (int m = 0; m < PX; ++m) {
        const int ix = t + m * S::T;
        if (ix < g.nx) {
            const PixelGeom p = pixel_geom(g, ix, iy, tab);
            const double res = p.inside ? acc[m] * p.corr : 0.0;
            double *o = dirty + ix * sx + iy * sy;
            *o = accumulate ? *o + res : res;
        }
    }
}

// predict: spec[q][iy][k] = FFT_x forward of the row whose image kx columns
// hold corr * dirty(ix, iy) * e^{-2 pi i w_q s} (zeros elsewhere), the input
// built in registers per thread (its 16 positions t + r T) -- the separate
// screen pass and the zero-filled x-FFT input are not needed
template <int LOGN>
__global__ __launch_bounds__(FxShape<LOGN>::T) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_screen_adj_xfft(Geo g, const double *__restrict__ dirty, int64_t sx, int64_t sy, int p_begin,
                  int np, float2 *__restrict__ spec, const double *__restrict__ tab,
                  const float2 *__restrict__ twg) {
    using S = FxShape<LOGN>;
    extern __shared__ float2 fbuf[];
    const int t = threadIdx.x, iy = blockIdx.x;
    float2 *const twl = fx_twl<LOGN>(fbuf, twg, t);
    // the corrected image value at the thread's x positions t + r T that can
    // hold a pixel (fp32, as the spectrum stores it; 0 where none maps): with
    // nx <= N / 2 only r < 4 and r >= 12 can (|X| <= N / 4 = 4 T)
    float val[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int r = e < 4 ? e : e + 8;
        const int i = t + r * S::T;
        const int X = i < g.ngx / 2 ? i : i - g.ngx, ix = X + g.nx / 2;
        val[e] = 0.0f;
        if (ix >= 0 && ix < g.nx) {
            const PixelGeom p = pixel_geom(g, ix, iy, tab);
            val[e] = p.inside ? (float)(dirty[ix * sx + iy * sy] * p.corr) : 0.0f;
        }
    }
    const double mm = (iy - g.ny / 2) * g.py, m2 = mm * mm;
    const int64_t tplane = (int64_t)g.ny * g.ngx;
    const int pt = fx_pad(t);
    for (int q = 0; q < np; ++q) {
        const double wq = g.w0 + (p_begin + q) * g.dw;
        int tt = t;  // (opaque, as in k_xfft_screen_fwd)
        asm volatile("" : "+v"(tt));
        float2 v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = make_float2(0.0f, 0.0f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int r = e < 4 ? e : e + 8;
            const int i = tt + r * S::T;
            const int X = i < g.ngx / 2 ? i : i - g.ngx;
            if (val[e] != 0.0f) {
                if (g.do_w) {
                    const double l = X * g.px, r2 = l * l + m2;
                    const double sp = r2 / (sqrt(1.0 - r2) + 1.0) - g.s0;
                    double ph = wq * sp;
                    ph -= rint(ph);
                    double sn, cs;
                    sincospi_t<float2>(2.0 * ph, &sn, &cs);
                    v[r] = make_float2((float)(val[e] * cs), (float)(-val[e] * sn));
                } else {
                    v[r] = make_float2(val[e], 0.0f);
                }
            }
        }
        fx_fft<LOGN, -1>(v, fbuf, twl, t);
        float2 *o = spec + q * tplane + (int64_t)iy * g.ngx;
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t + r * S::T] = fbuf[fx_padc<S::T>(t, pt, r * S::T)];
        __syncthreads();  // (the next plane's pass 0 overwrites the buffer)
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

// record factor and scatter back to visibility order
template <class VT>
__global__ void k_finalize(int64_t n, int nchan,
                           const VisRec *__restrict__ recs, const float2 *__restrict__ acc, VT *vis,
                           int64_t vrs, int64_t vcs, int accumulate, OutConv oc) {
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

// The image pols of one predict in one write-back (sdp_hip_dirty2ms_vis_pols):
// each record's NPO degridded sums are combined into every visibility pol
// through the conversion matrix's columns (fp64) and the visibility written
// once, where one finalize per image pol read-modified-wrote every pol of it.
struct PolAccs {
    const float2 *a[4] = {};
    OutConv oc[4];
};
template <class VT, int NPO>
__global__ void k_finalize_pols(int64_t n, int nchan, const VisRec *__restrict__ recs,
                                PolAccs pa, VT *vis, int64_t vrs, int64_t vcs, int accumulate) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const VisRec rc = recs[r];
        float2 v[NPO];
#pragma unroll
        for (int q = 0; q < NPO; ++q) {
            const float2 a = pa.a[q][r];
            v[q] = make_float2(rc.cre * a.x - rc.cim * a.y, rc.cre * a.y + rc.cim * a.x);
        }
        const int64_t row = rc.idx / (uint32_t)nchan;
        const int chan = (int)(rc.idx - row * nchan);
        VT *p = vis + row * vrs + chan * vcs;
        for (int k = 0; k < pa.oc[0].npv; ++k) {
            double xr = 0.0, xi = 0.0;
            bool any = false;
#pragma unroll
            for (int q = 0; q < NPO; ++q) {
                const double cr = pa.oc[q].cre[k], ci = pa.oc[q].cim[k];
                if (cr == 0.0 && ci == 0.0) continue;
                any = true;
                xr += cr * v[q].x - ci * v[q].y;
                xi += cr * v[q].y + ci * v[q].x;
            }
            if (any) store_vis_d(p + k * pa.oc[0].vps, xr, xi, accumulate);
        }
    }
}

// ------------------------------------------------------------------------
// kernels: the fp64 NUFFT (epsilon < 1e-7, the reference's default 1e-12)
// ------------------------------------------------------------------------
// ducc0 computes in fp64 (ng.py:251-254, double_precision_accumulation), so
// a request below the fp32 floor runs this path: W = ceil(-log10(eps/10)) in
// [9, 16], fp64 coordinates, taps, records, grid planes (c128), FFT (Z2Z)
// and screens.  One-cell buckets (no padding) and FineItem work items as in
// fp32; the gridder/degridder are VALU (fp64 FMA; the fp64 matrix rate of
// gfx950 equals its vector rate, and W = 13 does not tile the 16x16x4 shape).
constexpr int kMinW64 = 9, kMaxW64 = 16;
constexpr int kTap64 = 16;  // records per tap block

struct __attribute__((aligned(16))) VisRec64 {
    double cre, cim;    // gridding: vis*wgt*exp(2 pi i w s0); degridding: wgt*exp(-2 pi i w s0)
    double du, dv, dw;  // offset of the first tap from the exact position (cells / planes)
    uint32_t ij, p0, idx, pad;
};
static_assert(sizeof(VisRec64) == 64, "record layout");

// The 48-byte fp64 record of the two-level bucketing for the MFMA kernels:
// VisRec64 without the cell / first plane (the bucket's) -- the value pass
// writes, the final move moves and the kernels read 48 instead of 64 bytes.
// A 32-byte record with 42-bit fixed-point offsets halved the moves (C2 eps
// 1e-12 invert prep 11.1 -> 7.6 ms) but its decode cost the gridder +1.9 ms
// and the degridder +1.0 ms (each of a gridder workgroup's four waves decodes
// every record of a block).
struct __attribute__((aligned(16))) Rec64 {
    double cre, cim;
    double du, dv, dw;
    uint32_t idx, pad;
};
static_assert(sizeof(Rec64) == 48, "record layout");

// tap t of offset f: exp(beta (sqrt(1 - x^2) - 1)), x = (f + t) 2 / W
__device__ __forceinline__ double es_tap64(double f, int t, double ihw, double beta) {
    const double x = (f + (double)t) * ihw;
    const double y = 1.0 - x * x;
    return y > 0.0 ? exp(beta * (sqrt(y) - 1.0)) : 0.0;
}

// value pass of the fp64 path (the count pass is k_bucket's): VisRec64 at
// offs[key] + rank, value and phase factor in fp64
template <class VT, bool kGrid>
__global__ void k_bucket_f64(Geo g, int64_t nvis, const double *__restrict__ uvw, int64_t uvw_rs,
                             const double *__restrict__ freq, const VT *__restrict__ vis,
                             int64_t vrs, int64_t vcs, const void *__restrict__ wgt, int64_t wrs,
                             int64_t wcs, VisExtra x, double *sw_slots,
                             const unsigned *__restrict__ counter,
                             const unsigned *__restrict__ rk, VisRec64 *__restrict__ recs) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const bool valid = v < nvis;
    int64_t row = 0;
    int chan = 0;
    double wd = 0.0;
    if (valid) {
        row = v / g.nchan;
        chan = (int)(v - row * g.nchan);
        wd = eff_weight(wgt, wrs, wcs, x, row, chan);
    }
    if (sw_slots) {  // (a reused bucketing: the count pass did not sum the weights)
        double ws = wd;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o, 64);
        if ((threadIdx.x & 63) == 0 && ws != 0.0)
            atomicAdd(&sw_slots[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) &
                                (kSumSlots - 1)],
                      ws);
    }
    if (!valid) return;
    const unsigned mine = rk[v];
    if (mine == 0xffffffffu) return;
    const Coord c = vis_coord(g, uvw, uvw_rs, row, freq[chan]);
    const unsigned pos = counter[coord_key(g, c, row)] + mine;
    double cr = wd, ci = 0.0;
    if (kGrid) {
        const double2 xv = (vis && wd != 0.0) ? eff_vis_d(vis, vrs, vcs, x, row, chan)
                                              : make_double2(1.0, 0.0);
        cr = wd != 0.0 ? xv.x * wd : 0.0;
        ci = wd != 0.0 ? xv.y * wd : 0.0;
    }
    if (g.do_w || x.shift) {
        double ph = g.do_w ? c.w * g.s0 : 0.0;
        if (x.shift) {
            const double *u = uvw + row * uvw_rs;
            ph += (u[0] * x.sl + u[1] * x.sm + u[2] * x.sn) * (freq[chan] / kCLight);
        }
        ph -= rint(ph);
        double sn, cs;
        sincospi(2.0 * ph, &sn, &cs);
        if (!kGrid) sn = -sn;
        const double r_ = cr * cs - ci * sn, i_ = cr * sn + ci * cs;
        cr = r_;
        ci = i_;
    }
    VisRec64 rec;
    rec.cre = cr;
    rec.cim = ci;
    rec.du = c.du;
    rec.dv = c.dv;
    rec.dw = c.dw;
    rec.ij = (uint32_t)c.ic0 | ((uint32_t)c.jc0 << 16);
    rec.p0 = (uint32_t)c.p0;
    rec.idx = (uint32_t)v;
    rec.pad = 0u;
    recs[pos] = rec;
}

// ------------------------------------------------------------------------
// Two-level bucketing of one-cell plans (Geo::tiled).  The one-cell
// histogram of the single-level path takes one returning global atomic per
// run of equal cells (C2: 60 M for 123.6 M visibilities, serialised on the
// uv core's hot cells).  Here no per-cell global atomic exists:
//   k_t_count     per workgroup (a contiguous range of visibilities) an LDS
//                 histogram over the nbins 64 x 64-cell bins; one returning
//                 atomic per (workgroup, non-empty bin) reserves the
//                 workgroup's slice of each bin
//   k_t_bins      one workgroup: bin bases (scan), the bins' chunks of
//                 kTChunk records, segments of kTSeg chunks, and the
//                 non-empty bin list
//   k_t_scatter   the value pass: the record (RecC / VisRec / VisRec64) and
//                 its cell in the bin (u16) written in bin order, ranks from
//                 LDS cursors (one LDS atomic per run of equal bins)
//   k_t_cellcount per chunk an LDS histogram over the bin's 4096 cells
//   k_t_segscan   per (segment, cell): the count prefix over the segment's
//                 chunks (in place) and the segment total
//   k_t_cellcol   per (bin, cell): the prefix over the bin's segments (in
//                 place), the total, and the bin's padded-record / item sums
//                 (packed, one 64-bit atomic per 256 cells)
//   k_t_binscan   one workgroup: record and item bases of the bins, the
//                 metadata the host reads (the only host sync)
//   k_t_cellfin   per bin: cell bases, pad records, FineItem work items
//   k_t_final_s   per chunk: records moved to their cell (LDS cursors
//                 seeded with the cell base + the chunk's prefix)
// The writes of the two scatter passes land in runs inside the few bins /
// cells a workgroup touches at a time, not at random addresses.
constexpr int kMaxBins = 16384;    // LDS histogram of the first level (64 KiB)
constexpr int kTThreads = 1024;     // second-level kernels, bin scans
constexpr int kT1Threads = 512;     // count and value passes (VGPR-limited occupancy)
constexpr unsigned kTChunk = 131072;  // records per second-level chunk
constexpr unsigned kTSeg = 16;       // chunks per segment of the cells' column prefix
// visibilities per lane in flight in the value pass: 1 (C2: 1.10 ms, against
// 1.21 for 2 and 1.10 for 4; profiles/r06_sort_tu_ab.txt)
constexpr int kTU = 1;
constexpr int kTUc = 2;  // the same for the count pass (C2: 0.66 ms, 0.69 for 4)
constexpr int kTU2 = 4;              // records per lane in flight (cell count / final move)

struct TChunk {
    uint32_t bin, b, e, seg;  // records [b, e) of `bin`; `seg`: its prefix segment
};
struct TSeg {
    uint32_t c0, nc, pad0, pad1;  // chunks [c0, c0 + nc) of one bin
};

// consecutive lanes with equal `key` form a run; its head lane adds the run
// length to ctr[key] (LDS); with kRet every lane of a valid run gets its slot
template <bool kRet>
__device__ __forceinline__ unsigned lds_run_add(unsigned key, bool valid, unsigned *ctr) {
    const int lane = threadIdx.x & 63;
    const unsigned k = valid ? key : 0xffffffffu;
    const unsigned prev = __shfl_up(k, 1);
    const bool start = (lane == 0) || (prev != k);
    const unsigned long long B = __ballot(start);
    const unsigned long long above = (lane == 63) ? 0ull : (B & ~((2ull << lane) - 1ull));
    const int end = above ? (__ffsll((long long)above) - 1) : 64;
    unsigned base = 0;
    if (valid && start) base = atomicAdd(&ctr[k], (unsigned)(end - lane));
    if (!kRet) return 0;
    const unsigned long long upto = (lane == 63) ? B : (B & ((2ull << lane) - 1ull));
    const int head = 63 - __clzll((long long)upto);
    const unsigned hb = __shfl(base, head);
    return hb + (unsigned)(lane - head);
}

// A visibility of the two-level passes in two phases, so that a lane's kTU
// visibilities issue all their loads before any of them is used: t_load
// (above: uvw of the row, frequency, flag-masked weight) and t_classify
// (in-slab test, fp64 coordinates, bucketed or not) -- bit-identical in the
// count and the value pass.  v < 2^32 (the plan refuses larger calls).

// frequency / c per channel (the division vis_coord performs per visibility)
__global__ void k_fscale(const double *__restrict__ freq, int nchan, double *__restrict__ fsc) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < nchan) fsc[c] = freq[c] / kCLight;
}

struct TPoint {
    int64_t row;
    int chan;
    double wd;  // effective weight (0 outside the call's w slab)
    Coord c;
    bool in;
};

template <bool kCount>
__device__ __forceinline__ TPoint t_classify(const Geo &g, const TLoad &L, const VisExtra &x,
                                             unsigned long long *nbad) {
    TPoint p;
    p.in = false;
    p.wd = 0.0;
    p.row = L.row;
    p.chan = (int)L.chan;
    p.c.ok = false;
    if (!L.live) return p;
    if (g.slab && slab_out_v(g, L.wm, L.s)) return p;
    p.wd = L.wd;
    if (!(x.all || (float)p.wd != 0.0f)) return p;
    p.c = vis_coord_v(g, L.um, L.vm, L.wm, L.s);
    if (!p.c.ok) {
        if (kCount && !p.c.skip) atomicAdd(nbad, 1ull);
        return p;
    }
    p.in = true;
    return p;
}

// weight sum of the workgroup's visibilities: wave reduction, one fp64
// atomic per wave into the call's slots (k_sum_slots folds them)
__device__ __forceinline__ void t_weight_sum(double ws, double *sw_slots) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ws += __shfl_xor(ws, o, 64);
    if ((threadIdx.x & 63) == 0 && ws != 0.0)
        atomicAdd(&sw_slots[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) &
                            (kSumSlots - 1)],
                  ws);
}

template <int WT, int FB>
__global__ __launch_bounds__(kT1Threads) void k_t_count(Geo g, int64_t nvis, int64_t vpw,
                                                       const double *__restrict__ uvw, int64_t rs,
                                                       const double *__restrict__ fsc,
                                                       const void *__restrict__ wgt, int64_t wrs,
                                                       int64_t wcs, VisExtra x, double *sw_slots,
                                                       unsigned *__restrict__ binc,
                                                       unsigned *__restrict__ m1,
                                                       unsigned long long *nbad) {
    extern __shared__ unsigned hist[];
    const int nb = g.nbins;
    for (int b = threadIdx.x; b < nb; b += kT1Threads) hist[b] = 0u;
    __syncthreads();
    const int64_t v0 = (int64_t)blockIdx.x * vpw, v1 = min(nvis, v0 + vpw);
    double ws = 0.0;
    for (int64_t base = v0; base < v1; base += (int64_t)kT1Threads * kTUc) {
        TLoad L[kTUc];
#pragma unroll
        for (int u = 0; u < kTUc; ++u)
            L[u] = t_load<WT, FB>(g, base + u * kT1Threads + threadIdx.x, v1, uvw, rs, fsc, wgt,
                                  wrs, wcs, x);
#pragma unroll
        for (int u = 0; u < kTUc; ++u) {
            const TPoint p = t_classify<true>(g, L[u], x, nbad);
            ws += p.wd;
            lds_run_add<false>(p.in ? tiled_key(g, p.c) >> 12 : 0u, p.in, hist);
        }
    }
    if (sw_slots) t_weight_sum(ws, sw_slots);
    __syncthreads();
    // the workgroup's slice of every non-empty bin (its offset inside the bin)
    unsigned *row = m1 + (size_t)blockIdx.x * nb;
    for (int b = threadIdx.x; b < nb; b += kT1Threads) {
        const unsigned c = hist[b];
        row[b] = c ? atomicAdd(&binc[b], c) : 0u;
    }
}

// 1024-thread exclusive scan helper (hipcub block scan)
template <class T>
using TBlockScan = hipcub::BlockScan<T, kTThreads>;

// one workgroup: bin bases, the bins' chunks of kTChunk records and their
// prefix segments of kTSeg chunks, the non-empty bins.  Thread t owns bins
// [t * per, t * per + per).  binbase[nb] = total records; nbl[0] = number of
// non-empty bins, nbl[1 + k] = the k-th; meta_ch = {chunks, segments}.
__global__ __launch_bounds__(kTThreads) void k_t_bins(int nb, const unsigned *__restrict__ binc,
                                                      unsigned *__restrict__ binbase,
                                                      unsigned *__restrict__ segb,
                                                      unsigned *__restrict__ nsegb,
                                                      unsigned *__restrict__ nbl,
                                                      TChunk *__restrict__ chunks,
                                                      TSeg *__restrict__ segs,
                                                      unsigned *__restrict__ meta_ch) {
    __shared__ typename TBlockScan<unsigned>::TempStorage tmp;
    const int per = (nb + kTThreads - 1) / kTThreads;
    const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    unsigned rec = 0, nch = 0, nsg = 0, nne = 0;
    for (int b = b0; b < b1; ++b) {
        const unsigned n = binc[b];
        rec += n;
        const unsigned k = (n + kTChunk - 1) / kTChunk;
        nch += k;
        nsg += (k + kTSeg - 1) / kTSeg;
        nne += n ? 1u : 0u;
    }
    unsigned rec_x, nch_x, nsg_x, nne_x, rec_t, nch_t, nsg_t, nne_t;
    TBlockScan<unsigned>(tmp).ExclusiveSum(rec, rec_x, rec_t);
    __syncthreads();
    TBlockScan<unsigned>(tmp).ExclusiveSum(nch, nch_x, nch_t);
    __syncthreads();
    TBlockScan<unsigned>(tmp).ExclusiveSum(nsg, nsg_x, nsg_t);
    __syncthreads();
    TBlockScan<unsigned>(tmp).ExclusiveSum(nne, nne_x, nne_t);
    for (int b = b0; b < b1; ++b) {
        const unsigned n = binc[b];
        const unsigned k = (n + kTChunk - 1) / kTChunk, ks = (k + kTSeg - 1) / kTSeg;
        binbase[b] = rec_x;
        segb[b] = nsg_x;
        nsegb[b] = ks;
        for (unsigned j = 0; j < k; ++j) {
            TChunk t;
            t.bin = (uint32_t)b;
            t.b = rec_x + j * kTChunk;
            t.e = rec_x + min(n, (j + 1) * kTChunk);
            t.seg = nsg_x + j / kTSeg;
            chunks[nch_x + j] = t;
        }
        for (unsigned j = 0; j < ks; ++j) {
            TSeg sg;
            sg.c0 = nch_x + j * kTSeg;
            sg.nc = min(k - j * kTSeg, kTSeg);
            sg.pad0 = sg.pad1 = 0u;
            segs[nsg_x + j] = sg;
        }
        if (n) nbl[1 + nne_x++] = (unsigned)b;
        rec_x += n;
        nch_x += k;
        nsg_x += ks;
    }
    if (threadIdx.x == kTThreads - 1) {
        binbase[nb] = rec_t;
        nbl[0] = nne_t;
        meta_ch[0] = nch_t;
        meta_ch[1] = nsg_t;
    }
}

// KIND 0: RecC (4-padded invert), 1: VisRec (fp32 predict), 3: Rec64 (the
// fp64 MFMA kernels)
template <int KIND>
struct TRec;
template <>
struct TRec<0> {
    using type = RecC;
};
template <>
struct TRec<1> {
    using type = VisRec;
};
template <>
struct TRec<3> {
    using type = Rec64;
};

// Record writers of the value pass: the fields bucket_one / k_bucket_f64
// write for the single-level path, computed the same way.
template <int KIND, bool kGrid, class XV>
__device__ __forceinline__ void t_write(const Geo &g, const VisExtra &x, const TLoad &L,
                                        const TPoint &p, XV xv, void *out, unsigned pos) {
    double ph = 0.0;
    const bool rot = g.do_w || x.shift;
    if (rot) {
        ph = g.do_w ? p.c.w * g.s0 : 0.0;
        if (x.shift) ph += (L.um * x.sl + L.vm * x.sm + L.wm * x.sn) * L.s;
        ph -= rint(ph);
    }
    if constexpr (KIND >= 2) {
        double cr = p.wd, ci = 0.0;
        if (kGrid) {
            cr = p.wd != 0.0 ? xv.x * p.wd : 0.0;
            ci = p.wd != 0.0 ? xv.y * p.wd : 0.0;
        }
        if (rot) {
            double sn, cs;
            sincospi(2.0 * ph, &sn, &cs);
            if (!kGrid) sn = -sn;
            const double r_ = cr * cs - ci * sn, i_ = cr * sn + ci * cs;
            cr = r_;
            ci = i_;
        }
        Rec64 rec;
        rec.cre = cr;
        rec.cim = ci;
        rec.du = p.c.du;
        rec.dv = p.c.dv;
        rec.dw = p.c.dw;
        rec.idx = (uint32_t)(L.row * (uint32_t)g.nchan + L.chan);
        rec.pad = 0u;
        static_cast<Rec64 *>(out)[pos] = rec;
    } else {
        const float wt = (float)p.wd;
        float cr = wt, ci = 0.0f;
        if (kGrid) {
            cr = wt != 0.0f ? xv.x * wt : 0.0f;
            ci = wt != 0.0f ? xv.y * wt : 0.0f;
        }
        if (rot) {
            float sn, cs;
            sincospif((float)(2.0 * ph), &sn, &cs);
            if (!kGrid) sn = -sn;
            const float r_ = cr * cs - ci * sn, i_ = cr * sn + ci * cs;
            cr = r_;
            ci = i_;
        }
        if constexpr (KIND == 0) {
            const double base = 1.0 - 0.5 * g.W;
            const uint32_t qu = fix_frac(base - p.c.du, 21), qv = fix_frac(base - p.c.dv, 21);
            const uint32_t qw = g.do_w ? fix_frac(base - p.c.dw, 22) : 0u;
            RecC rc;
            rc.cre = cr;
            rc.cim = ci;
            rc.lo = qu | (qv << 21);
            rc.hi = (qv >> 11) | (qw << 10);
            static_cast<RecC *>(out)[pos] = rc;
        } else {
            VisRec rec;
            rec.cre = cr;
            rec.cim = ci;
            rec.fu = p.c.fu;
            rec.fv = p.c.fv;
            rec.fw = p.c.fw;
            rec.ij = (uint32_t)p.c.ic0 | ((uint32_t)p.c.jc0 << 16);
            rec.p0 = (uint32_t)p.c.p0;
            rec.idx = L.row * (uint32_t)g.nchan + L.chan;
            static_cast<VisRec *>(out)[pos] = rec;
        }
    }
}

template <class VT, int KIND, bool kGrid, int WT, int FB>
__global__ __launch_bounds__(kT1Threads) void k_t_scatter(
    Geo g, int64_t nvis, int64_t vpw, const double *__restrict__ uvw, int64_t rs,
    const double *__restrict__ fsc, const VT *__restrict__ vis, int64_t vrs, int64_t vcs,
    const void *__restrict__ wgt, int64_t wrs, int64_t wcs, VisExtra x, double *sw_slots,
    const unsigned *__restrict__ binbase, const unsigned *__restrict__ m1, void *__restrict__ out,
    uint16_t *__restrict__ lkey) {
    using V = TVal<VT, KIND, kGrid, FB>;
    extern __shared__ unsigned cur[];
    const int nb = g.nbins;
    const unsigned *row = m1 + (size_t)blockIdx.x * nb;
    for (int b = threadIdx.x; b < nb; b += kT1Threads) cur[b] = binbase[b] + row[b];
    __syncthreads();
    const int64_t v0 = (int64_t)blockIdx.x * vpw, v1 = min(nvis, v0 + vpw);
    double ws = 0.0;
    for (int64_t base = v0; base < v1; base += (int64_t)kT1Threads * kTU) {
        TLoad L[kTU];
        VT raw[kTU];
#pragma unroll
        for (int u = 0; u < kTU; ++u) {
            L[u] = t_load<WT, FB>(g, base + u * kT1Threads + threadIdx.x, v1, uvw, rs, fsc, wgt,
                                  wrs, wcs, x);
            raw[u] = V::load(vis, vrs, vcs, x, L[u]);
        }
#pragma unroll
        for (int u = 0; u < kTU; ++u) {
            const typename V::type xv = V::value(vis, vrs, vcs, x, L[u], raw[u]);
            const TPoint p = t_classify<false>(g, L[u], x, nullptr);
            ws += p.wd;
            const unsigned key = p.in ? tiled_key(g, p.c) : 0u;
            const unsigned pos = lds_run_add<true>(key >> 12, p.in, cur);
            if (p.in) {
                t_write<KIND, kGrid>(g, x, L[u], p, xv, out, pos);
                lkey[pos] = (uint16_t)(key & (kBinCells - 1));
            }
        }
    }
    if (sw_slots) t_weight_sum(ws, sw_slots);
}

// per chunk: its records' cell histogram (M2 row of kBinCells counts)
__global__ __launch_bounds__(kTThreads) void k_t_cellcount(const TChunk *__restrict__ chunks,
                                                           const unsigned *__restrict__ meta_ch,
                                                           const uint16_t *__restrict__ lkey,
                                                           unsigned *__restrict__ m2) {
    __shared__ unsigned h[kBinCells];
    const unsigned n = meta_ch[0];
    for (unsigned c = blockIdx.x; c < n; c += gridDim.x) {
        for (int i = threadIdx.x; i < kBinCells; i += kTThreads) h[i] = 0u;
        __syncthreads();
        const TChunk t = chunks[c];
        for (uint32_t i0 = t.b; i0 < t.e; i0 += kTThreads * kTU2) {
            unsigned k[kTU2];
#pragma unroll
            for (int u = 0; u < kTU2; ++u) {
                const uint32_t i = i0 + u * kTThreads + threadIdx.x;
                k[u] = i < t.e ? (unsigned)lkey[i] : 0xffffu;
            }
#pragma unroll
            for (int u = 0; u < kTU2; ++u) lds_run_add<false>(k[u], k[u] != 0xffffu, h);
        }
        __syncthreads();
        uint4 *dst = reinterpret_cast<uint4 *>(m2 + (size_t)c * kBinCells);
        const uint4 *src = reinterpret_cast<const uint4 *>(h);
        for (int i = threadIdx.x; i < kBinCells / 4; i += kTThreads) dst[i] = src[i];
        __syncthreads();
    }
}

// per (segment of <= kTSeg chunks of one bin, 256-cell slice), one thread
// per cell: the exclusive prefix of the cell's counts over the segment's
// chunks (in place in M2) and the segment total (S)
__global__ __launch_bounds__(256) void k_t_segscan(const TSeg *__restrict__ segs,
                                                   const unsigned *__restrict__ meta_ch,
                                                   unsigned *__restrict__ m2,
                                                   unsigned *__restrict__ stot) {
    const unsigned nwork = meta_ch[1] * (kBinCells / 256);
    for (unsigned w = blockIdx.x; w < nwork; w += gridDim.x) {
        const unsigned sg = w / (kBinCells / 256);
        const int cell = (int)(w % (kBinCells / 256)) * 256 + threadIdx.x;
        const TSeg t = segs[sg];
        unsigned *q = m2 + (size_t)t.c0 * kBinCells + cell;
        unsigned v[kTSeg];
#pragma unroll
        for (unsigned j = 0; j < kTSeg; ++j) v[j] = j < t.nc ? q[(size_t)j * kBinCells] : 0u;
        unsigned run = 0;
#pragma unroll
        for (unsigned j = 0; j < kTSeg; ++j) {
            if (j < t.nc) q[(size_t)j * kBinCells] = run;
            run += v[j];
        }
        stot[(size_t)sg * kBinCells + cell] = run;
    }
}

// per (non-empty bin, 256-cell slice), one thread per cell: the exclusive
// prefix of the segment totals over the bin's segments (in place in S), the
// cell total T, and into binsum[bin] the slice's (padded records << 32 |
// items) -- a group of 16 cells is 16 consecutive lanes; its items are its
// padded records in chunks of `chunk`
template <bool PAD>
__global__ __launch_bounds__(256) void k_t_cellcol(const unsigned *__restrict__ nbl,
                                                   const unsigned *__restrict__ segb,
                                                   const unsigned *__restrict__ nsegb,
                                                   unsigned *__restrict__ stot,
                                                   unsigned *__restrict__ tot, unsigned chunk,
                                                   unsigned long long *__restrict__ binsum) {
    __shared__ unsigned long long red[4];
    const unsigned nwork = nbl[0] * (kBinCells / 256);
    for (unsigned w = blockIdx.x; w < nwork; w += gridDim.x) {
        const unsigned b = nbl[1 + w / (kBinCells / 256)];
        const int cell = (int)(w % (kBinCells / 256)) * 256 + threadIdx.x;
        const unsigned s0 = segb[b], ns = nsegb[b];
        unsigned *q = stot + (size_t)s0 * kBinCells + cell;
        unsigned run = 0;
        unsigned k = 0;
        for (; k + 8 <= ns; k += 8) {
            unsigned v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = q[(size_t)(k + j) * kBinCells];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                q[(size_t)(k + j) * kBinCells] = run;
                run += v[j];
            }
        }
        for (; k < ns; ++k) {
            const unsigned v = q[(size_t)k * kBinCells];
            q[(size_t)k * kBinCells] = run;
            run += v;
        }
        tot[(size_t)b * kBinCells + cell] = run;
        const unsigned pd = PAD ? (run + 3u) & ~3u : run;
        unsigned gt = pd;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) gt += __shfl_xor(gt, o, 64);
        unsigned long long r =
            ((unsigned long long)pd << 32) |
            (unsigned long long)((threadIdx.x & 15) == 0 ? (gt + chunk - 1) / chunk : 0u);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = r;
        __syncthreads();
        if (threadIdx.x == 0) {
            // (one atomic per 256 cells of a bin: the padded total needs no
            // chip-wide counter -- same-address atomics serialise at ~10 ns)
            const unsigned long long t = red[0] + red[1] + red[2] + red[3];
            if (t) atomicAdd(&binsum[b], t);
        }
        __syncthreads();
    }
}

// one workgroup: exclusive scan of the bins' (padded records << 32 | items)
// -> bofs; the metadata the host reads: {nbad lo, nbad hi, gridded records,
// items, first item of each first plane [nps + 1], padded records}
__global__ __launch_bounds__(kTThreads) void k_t_binscan(
    int nb, int bins_per_plane, int nps, const unsigned long long *__restrict__ binsum,
    const unsigned *__restrict__ binbase, const unsigned long long *__restrict__ nbad,
    unsigned long long *__restrict__ bofs, unsigned *__restrict__ meta) {
    __shared__ typename TBlockScan<unsigned long long>::TempStorage tmp;
    const int per = (nb + kTThreads - 1) / kTThreads;
    const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    unsigned long long s = 0;
    for (int b = b0; b < b1; ++b) s += binsum[b];
    unsigned long long x, t;
    TBlockScan<unsigned long long>(tmp).ExclusiveSum(s, x, t);
    for (int b = b0; b < b1; ++b) {
        bofs[b] = x;
        x += binsum[b];
    }
    if (threadIdx.x == kTThreads - 1) bofs[nb] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        meta[0] = (unsigned)(*nbad & 0xffffffffull);
        meta[1] = (unsigned)(*nbad >> 32);
        meta[2] = binbase[nb];
        meta[3] = (unsigned)(t & 0xffffffffull);
        meta[5 + nps] = (unsigned)(t >> 32);
    }
    for (int p = threadIdx.x; p <= nps; p += kTThreads)
        meta[4 + p] = (unsigned)((p < nps ? bofs[(size_t)p * bins_per_plane] : t) & 0xffffffffull);
}

// per non-empty bin, thread = one of its 256 groups of 16 cells: cell bases
// (cbase, absolute record index), zero pad records behind each cell's
// records (RecC, PAD), and the group's FineItems (chunks of `chunk` padded
// records, each with the 16 cell ends)
template <bool PAD, int KIND>
__global__ __launch_bounds__(256) void k_t_cellfin(const Geo g, const unsigned *__restrict__ nbl,
                                                   const unsigned *__restrict__ tot,
                                                   const unsigned long long *__restrict__ bofs,
                                                   unsigned chunk, unsigned *__restrict__ cbase,
                                                   void *__restrict__ recs,
                                                   FineItem *__restrict__ items) {
    __shared__ typename hipcub::BlockScan<unsigned long long, 256>::TempStorage tmp;
    const unsigned nne = nbl[0];
    const int tpp = g.tlx * g.tly;
    for (unsigned w = blockIdx.x; w < nne; w += gridDim.x) {
        const unsigned b = nbl[1 + w];
        const int gi = threadIdx.x;
        const uint4 *t4 = reinterpret_cast<const uint4 *>(tot + (size_t)b * kBinCells + gi * 16);
        unsigned n[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = t4[q];
            n[4 * q] = v.x;
            n[4 * q + 1] = v.y;
            n[4 * q + 2] = v.z;
            n[4 * q + 3] = v.w;
        }
        unsigned G = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) G += PAD ? (n[j] + 3u) & ~3u : n[j];
        const unsigned it = (G + chunk - 1) / chunk;
        unsigned long long x;
        hipcub::BlockScan<unsigned long long, 256>(tmp).ExclusiveSum(
            ((unsigned long long)G << 32) | it, x);
        const unsigned long long bo = bofs[b];
        const unsigned base = (unsigned)(bo >> 32) + (unsigned)(x >> 32);
        const unsigned ib = (unsigned)bo + (unsigned)x;
        FineItem f;
        unsigned run = base;
        unsigned st[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            st[j] = run;
            const unsigned r = PAD ? (n[j] + 3u) & ~3u : n[j];
            if (PAD && r != n[j]) {
                // zero-valued pads with in-range offsets (finite taps): RecC
                // fractions 0 (offset 1 - W/2), or VisRec64 offsets 1 - W/2
                if constexpr (KIND == 3) {
                    Rec64 z;
                    z.cre = z.cim = 0.0;
                    z.du = z.dv = z.dw = 1.0 - 0.5 * g.W;
                    z.idx = z.pad = 0u;
                    for (unsigned i = run + n[j]; i < run + r; ++i) static_cast<Rec64 *>(recs)[i] = z;
                } else {
                    RecC z;
                    z.cre = z.cim = 0.0f;
                    z.lo = z.hi = 0u;
                    for (unsigned i = run + n[j]; i < run + r; ++i) static_cast<RecC *>(recs)[i] = z;
                }
            }
            run += r;
            f.o[j] = run;
        }
        uint4 *cb = reinterpret_cast<uint4 *>(cbase + (size_t)b * kBinCells + gi * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            cb[q] = make_uint4(st[4 * q], st[4 * q + 1], st[4 * q + 2], st[4 * q + 3]);
        f.p0 = b / (unsigned)tpp;
        f.tile = (b - f.p0 * (unsigned)tpp) * 256u + (unsigned)gi;
        for (unsigned s = 0; s < it; ++s) {
            f.b = base + s * chunk;
            f.e = min(run, f.b + chunk);
            items[ib + s] = f;
        }
        __syncthreads();  // (tmp reused by the next bin)
    }
}

// k_t_final_s, the final move of the two-level sort: each batch of NB records is
// counting-sorted by cell in LDS (batch histogram, block scan, staging), then
// written out in that order, so a cell's records of the batch leave as one
// contiguous run instead of lane-scattered 16-byte stores.  LDS: cursors and
// batch counts (kBinCells each), the staged records and their destinations.
template <int KIND, int NB>
constexpr size_t t_final_lds() {
    return (size_t)2 * kBinCells * sizeof(unsigned) + (size_t)NB * sizeof(unsigned) +
           (size_t)NB * sizeof(typename TRec<KIND>::type);
}

template <int KIND, int NB>
__global__ __launch_bounds__(kTThreads) void k_t_final_s(const TChunk *__restrict__ chunks,
                                                         const unsigned *__restrict__ meta_ch,
                                                         const uint16_t *__restrict__ lkey,
                                                         const unsigned *__restrict__ m2,
                                                         const unsigned *__restrict__ stot,
                                                         const unsigned *__restrict__ cbase,
                                                         const void *__restrict__ in,
                                                         void *__restrict__ out, int xmap) {
    using R = typename TRec<KIND>::type;
    constexpr int NW = (int)(sizeof(R) / sizeof(uint4));
    constexpr int U = NB / kTThreads;
    constexpr int CPT = kBinCells / kTThreads;  // cells per thread (4)
    static_assert(NB % kTThreads == 0 && CPT == 4, "k_t_final_s batch shape");
    __shared__ typename TBlockScan<unsigned>::TempStorage tmp;
    extern __shared__ __attribute__((aligned(16))) unsigned fsm[];
    unsigned *const cur = fsm;
    unsigned *const cnt = fsm + kBinCells;
    unsigned *const sdst = cnt + kBinCells;
    uint4 *const stg = reinterpret_cast<uint4 *>(sdst + NB);
    const unsigned n = meta_ch[0];
    const uint4 *src = reinterpret_cast<const uint4 *>(in);
    uint4 *dst = reinterpret_cast<uint4 *>(out);
    const int c0 = threadIdx.x * CPT;
    for (int j = 0; j < CPT; ++j) cnt[c0 + j] = 0u;
    // xmap: the workgroups resident on one XCD (blockIdx mod 8) take
    // consecutive chunks -- of one bin, mostly -- whose writes to a cell's
    // run fall into the same lines of that XCD's L2
    const unsigned G = gridDim.x,
                   off = xmap ? (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    for (unsigned c = off; c < n; c += G) {
        const TChunk t = chunks[c];
        {
            const uint4 pv = reinterpret_cast<const uint4 *>(m2 + (size_t)c * kBinCells)[threadIdx.x];
            const uint4 sv =
                reinterpret_cast<const uint4 *>(stot + (size_t)t.seg * kBinCells)[threadIdx.x];
            const uint4 bv =
                reinterpret_cast<const uint4 *>(cbase + (size_t)t.bin * kBinCells)[threadIdx.x];
            reinterpret_cast<uint4 *>(cur)[threadIdx.x] =
                make_uint4(pv.x + sv.x + bv.x, pv.y + sv.y + bv.y, pv.z + sv.z + bv.z,
                           pv.w + sv.w + bv.w);
        }
        __syncthreads();
        for (uint32_t i0 = t.b; i0 < t.e; i0 += NB) {
            // the records as scalars: held as uint4 arrays the compiler kept
            // them in scratch between the load and the staging loop
            unsigned r[U][4 * NW];
            unsigned k[U], rk[U];
            // clamped-index loads: behind `if (i < t.e)` the compiler kept the
            // records in scratch between the two loops
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * kTThreads + threadIdx.x, ic = min(i, t.e - 1u);
                k[u] = lkey[ic];
                if (i >= t.e) k[u] = 0xffffu;
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    const uint4 v = src[(size_t)ic * NW + q];
                    r[u][4 * q] = v.x;
                    r[u][4 * q + 1] = v.y;
                    r[u][4 * q + 2] = v.z;
                    r[u][4 * q + 3] = v.w;
                }
            }
            // rank of each record among the batch's records of its cell
#pragma unroll
            for (int u = 0; u < U; ++u) rk[u] = lds_run_add<true>(k[u], k[u] != 0xffffu, cnt);
            __syncthreads();
            unsigned h[CPT], s = 0;
#pragma unroll
            for (int j = 0; j < CPT; ++j) {
                h[j] = cnt[c0 + j];
                s += h[j];
            }
            unsigned x;
            TBlockScan<unsigned>(tmp).ExclusiveSum(s, x);
#pragma unroll
            for (int j = 0; j < CPT; ++j) {
                cnt[c0 + j] = x;  // the cell's first staging slot
                x += h[j];
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (k[u] != 0xffffu) {
                    const unsigned slot = cnt[k[u]] + rk[u];
                    sdst[slot] = cur[k[u]] + rk[u];
#pragma unroll
                    for (int q = 0; q < NW; ++q)
                        stg[slot * NW + q] =
                            make_uint4(r[u][4 * q], r[u][4 * q + 1], r[u][4 * q + 2], r[u][4 * q + 3]);
                }
            }
            __syncthreads();
            const int nb = (int)min((uint32_t)NB, t.e - i0);
            for (int j = threadIdx.x; j < nb * NW; j += kTThreads) {
                const int rec = j / NW, q = j - rec * NW;
                dst[(size_t)sdst[rec] * NW + q] = stg[j];
            }
#pragma unroll
            for (int j = 0; j < CPT; ++j) {
                cur[c0 + j] += h[j];
                cnt[c0 + j] = 0u;
            }
            __syncthreads();
        }
    }
}

template <int W, bool WS>
constexpr size_t grid_f64_lds() {
    return (size_t)(WS ? W : 1) * (W + 1) * (W + 7) * sizeof(double2) +
           (size_t)kTap64 * (3 * W * sizeof(double) + sizeof(double2));
}

// The taps of up to kTap64 records into LDS ([record][u | v | w][W]) and
// their values (cv), every lane busy; returns the record count.
template <int W, bool WS>
__device__ __forceinline__ int stage_taps64(const VisRec64 *__restrict__ recs, uint32_t b0,
                                            uint32_t e, double *tap, double2 *cv, double ihw,
                                            double beta) {
    constexpr int TR = 3 * W;
    const int nb = (int)min((uint32_t)kTap64, e - b0);
    for (int t = threadIdx.x; t < nb * TR; t += 64) {
        const int r = t / TR, k = t - r * TR, ax = k / W, j = k - ax * W;
        const VisRec64 *R = recs + b0 + r;
        double tv;
        if (ax == 2 && !WS) tv = j == 0 ? 1.0 : 0.0;
        else tv = es_tap64(ax == 0 ? R->du : (ax == 1 ? R->dv : R->dw), j, ihw, beta);
        tap[t] = tv;
    }
    if ((int)threadIdx.x < nb)
        cv[threadIdx.x] = make_double2(recs[b0 + threadIdx.x].cre, recs[b0 + threadIdx.x].cim);
    return nb;
}

// fp64 gridder: one wave per FineItem (a chunk of a 2 x 8-cell group's
// records, ordered by cell).  Lane l owns the footprint taps (kx, ky) =
// divmod(l + 64 i, W) and accumulates, per cell, c tw[q] tu[kx] tv[ky] for
// every plane q in registers; a cell change adds them into the region's
// (2 + W - 1) x (8 + W - 1) x W c128 LDS tile, flushed once per item with
// fp64 global atomics (zeros skipped).
template <int W, bool WS>
__global__ __launch_bounds__(64) void k_grid_f64(Geo g, const VisRec64 *__restrict__ recs,
                                                 const FineItem *__restrict__ items,
                                                 uint32_t n_items, double *__restrict__ grid,
                                                 int p_lo, int p_hi) {
    constexpr int NQ = WS ? W : 1;
    constexpr int RX = W + 1, RY = W + 7, NP = (W * W + 63) / 64, TR = 3 * W;
    extern __shared__ __attribute__((aligned(16))) double2 sm64[];
    double2 *const reg = sm64;  // [NQ][RX][RY]
    double *const tap = reinterpret_cast<double *>(reg + NQ * RX * RY);
    double2 *const cv = reinterpret_cast<double2 *>(tap + kTap64 * TR);
    const int lane = threadIdx.x;
    const double ihw = 2.0 / W, beta = (double)g.beta;
    int px[NP], py[NP];
    bool pv[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int pp = lane + 64 * i;
        pv[i] = pp < W * W;
        px[i] = pv[i] ? pp / W : 0;
        py[i] = pv[i] ? pp % W : 0;
    }
    const size_t plane_elems = (size_t)g.ngx * g.ngy;
    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        uint32_t bnd[kGroupCell];
        const Item it = load_fine_item<kGroupCell>(items, w_it, n_items, bnd);
        if (it.b >= it.e) continue;
        int ibase, jbase;
        group_origin(g, (int)it.tile, ibase, jbase);
        wave_lds_sync();  // the previous item's flush reads of the region
        for (int i = lane; i < NQ * RX * RY; i += 64) reg[i] = make_double2(0.0, 0.0);
        double2 acc[NP][NQ];
#pragma unroll
        for (int i = 0; i < NP; ++i)
#pragma unroll
            for (int q = 0; q < NQ; ++q) acc[i][q] = make_double2(0.0, 0.0);
        int cur = -1;
        auto flush_acc = [&]() {
            const int xo = cur & 1, yo = cur >> 1;
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                if (!pv[i]) continue;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    double2 *d = reg + (q * RX + xo + px[i]) * RY + yo + py[i];
                    double2 o = *d;
                    o.x += acc[i][q].x;
                    o.y += acc[i][q].y;
                    *d = o;
                    acc[i][q] = make_double2(0.0, 0.0);
                }
            }
        };
        for (uint32_t b0 = it.b; b0 < it.e; b0 += kTap64) {
            wave_lds_sync();  // the previous block's tap reads
            const int nb = stage_taps64<W, WS>(recs, b0, it.e, tap, cv, ihw, beta);
            wave_lds_sync();
            for (int r = 0; r < nb; ++r) {
                const uint32_t ri = b0 + (uint32_t)r;
                int cell = 0;
#pragma unroll
                for (int c = 0; c < kGroupCell - 1; ++c) cell += ri >= bnd[c] ? 1 : 0;
                if (cell != cur) {
                    if (cur >= 0) flush_acc();
                    cur = cell;
                }
                const double *T = tap + r * TR;
                const double2 c = cv[r];
                double2 ctw[NQ];
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const double tw = T[2 * W + q];
                    ctw[q] = make_double2(c.x * tw, c.y * tw);
                }
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const double t = T[px[i]] * T[W + py[i]];
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        acc[i][q].x = fma(t, ctw[q].x, acc[i][q].x);
                        acc[i][q].y = fma(t, ctw[q].y, acc[i][q].y);
                    }
                }
            }
        }
        if (cur >= 0) flush_acc();
        wave_lds_sync();
        for (int i = lane; i < NQ * RX * RY; i += 64) {
            const int q = i / (RX * RY), rem = i - q * (RX * RY);
            const int p = (int)it.p0 + q;
            if (p < p_lo || p >= p_hi) continue;
            const double2 v = reg[i];
            if (v.x == 0.0 && v.y == 0.0) continue;
            const int xl = rem / RY, yl = rem - xl * RY;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            double *dst = grid + 2 * ((size_t)(p - p_lo) * plane_elems + (size_t)gx * g.ngy + gy);
            if (v.x != 0.0) atomicAdd(dst, v.x);
            if (v.y != 0.0) atomicAdd(dst + 1, v.y);
        }
    }
}

// fp64 MFMA kernels (epsilon < 1e-7, W <= 16) on one-cell buckets.
//
// Taps.  The ES kernel's W taps of an offset f (s = f + W/2 in (0, 1]) are
// evaluated as W polynomials of degree kPoly64 in t = 2 s - 1 (Horner; the
// coefficients, uniform across lanes, fitted on the host at Chebyshev nodes,
// es_poly64_table, and copied to LDS per workgroup).  Interior taps are
// within ~1e-14 of the kernel; the two edge taps, where sqrt(1 - x^2) is not
// analytic, within ~1.5 e^-beta, about 0.15 of the epsilon W is chosen for
// (W = 9: 1.5e-9, W = 13: 1.6e-13, W = 16: 7e-15; the fp64 exp they
// replace kept a dozen constants live in registers across the kernel).  One
// lane computes all taps of one (record, axis) pair of a 16-record block.
constexpr int kPoly64 = 12;
constexpr int kPolyStride = 16;  // table [kPoly64 + 1][kPolyStride]
constexpr int kBlk64 = 16;       // records per tap block

constexpr int kPolyN = (kPoly64 + 1) * kPolyStride;  // doubles of the table

// taps J0 .. J1 - 1 of the pair's offset f into dst[j]: Horner over the
// degrees (outer) for all the taps at once (inner), the coefficients read
// from the workgroup's LDS copy of the table (uniform addresses: broadcast
// reads; as scalar loads the whole table stayed live in SGPRs and spilled)
template <int W, int J0, int J1>
__device__ __forceinline__ void es_taps_poly(double f, const double *cl, double ihw, double beta,
                                             double *dst) {
    constexpr int NJ = J1 - J0;
    const double t = 2.0 * (f + 0.5 * W) - 1.0;
    // one degree's coefficients in registers at a time: each row's reads
    // take their offset through an empty asm statement, so the compiler can
    // neither hoist the table out of the caller's loops (it did: 169 doubles
    // live, scratch spills) nor batch every row up front; the next row's
    // reads are issued before this row's FMAs
    int zo = 0;
    asm volatile("" : "+v"(zo));
    double v[NJ], c[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) v[j] = cl[zo + kPoly64 * kPolyStride + J0 + j];
#pragma unroll
    for (int j = 0; j < NJ; ++j) c[j] = cl[zo + (kPoly64 - 1) * kPolyStride + J0 + j];
#pragma unroll
    for (int d = kPoly64 - 1; d >= 0; --d) {
        // row d - 1's reads hang on an offset that the previous row's FMA
        // results fed (one row of lookahead, never the whole table)
        double cn[NJ];
        if (d > 0) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) cn[j] = cl[zo + (d - 1) * kPolyStride + J0 + j];
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) v[j] = fma(v[j], t, c[j]);
        asm volatile("" : "+v"(zo) : "v"(v[0]));
        if (d > 0) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) c[j] = cn[j];
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) dst[J0 + j] = v[j];
}

// The tap block of nb <= kBlk64 records (b0 ..): [record][tu | tv | tw |
// cre, cim] rows of TR = 3 W + 2 doubles, in two phases so that a block's
// record loads can be issued a block ahead: stage64_load (lane < 48: the
// offset of pair (record lane / 3, axis lane % 3); lanes 48..63: the value of
// record lane - 48; lane < 16: the output index of record lane) and
// stage64_write (the taps: `part` / `nparts` is this wave's share of each
// pair's taps -- the gridder's two waves split them in halves).
struct Stage64 {
    double a, b;   // pair offset, or (cre, cim)
    uint32_t idx;  // output index (degridder)
};

template <class RT>  // VisRec64 or Rec64
__device__ __forceinline__ Stage64 stage64_load(const RT *__restrict__ recs, uint32_t b0, int nb,
                                                int lane) {
    Stage64 s;
    s.a = s.b = 0.0;
    s.idx = 0u;
    if (nb <= 0) return s;
    if (lane < 3 * kBlk64) {
        const int r = lane / 3, ax = lane - 3 * r;
        if (r < nb) {
            const RT *R = recs + b0 + r;
            s.a = ax == 0 ? R->du : (ax == 1 ? R->dv : R->dw);
        }
    } else if (lane - 3 * kBlk64 < nb) {
        const RT *R = recs + b0 + (lane - 3 * kBlk64);
        s.a = R->cre;
        s.b = R->cim;
    }
    if (lane < nb) s.idx = recs[b0 + lane].idx;
    return s;
}

template <int W, bool WS, int J0, int J1>
__device__ __forceinline__ void stage64_write(const Stage64 &s, int nb, double *tap, const double *cl,
                                              double ihw, double beta, int lane, bool vals) {
    constexpr int TR = 3 * W + 2;
    if (lane < 3 * kBlk64) {
        const int r = lane / 3, ax = lane - 3 * r;
        if (r < nb) {
            double *dst = tap + r * TR + ax * W;
            if (ax == 2 && !WS) {
#pragma unroll
                for (int j = J0; j < J1; ++j) dst[j] = j == 0 ? 1.0 : 0.0;
            } else {
                es_taps_poly<W, J0, J1>(s.a, cl, ihw, beta, dst);
            }
        }
    } else if (vals && lane - 3 * kBlk64 < nb) {
        const int r = lane - 3 * kBlk64;
        tap[r * TR + 3 * W] = s.a;
        tap[r * TR + 3 * W + 1] = s.b;
    }
}

// fp64 MFMA gridder (invert) on 4-padded cells (the two-level bucketing pads
// VisRec64 cells to a multiple of 4 records, SDP_HIP_F64_MFMA).  A cell's
// records share their footprint origin, so its contribution is one GEMM on
// v_mfma_f64_16x16x4_f64 (exact fp64 FMAs):
//     C[(kx, ky), (q, re/im)] += sum_r tu_r[kx] tv_r[ky] * tw_r[q] c_r
// M-tile kx (W tiles) holds the rows ky = 0..15 (ky >= W: A = 0), N = the
// 2 NQ (q, re/im) columns (one 16-column tile per wave), K = 4 records of
// the cell.  Lane (row (lane >> 4) + 4 i, column lane & 15) of tile kx sits
// in the item's LDS region [x][y][column] at a compile-time offset from one
// per-lane base, so a cell change is 4 W stores and 4 W loads with
// immediate offsets.  Rows ky >= W add exact zeros to region cells of the
// same wave's columns (an identity update: the region is RY = 8 + 15 rows
// deep); columns >= 2 NQ are never stored.  The region is zeroed per item
// and flushed once with fp64 global atomics (zeros skipped) in plane order.
template <int W, bool WS>
constexpr int f64m_ntiles() {  // 16-column N-tiles of the 2 NQ (q, re/im) columns
    return (2 * (WS ? W : 1) + 15) / 16;
}
template <int W, bool WS>
constexpr int f64m_waves() {  // one wave per (N-tile, half of the kx M-tiles)
    return 2 * f64m_ntiles<W, WS>();
}
template <int W, bool WS>
constexpr int f64m_ry() {  // rows a cell's footprint reaches (rows ky >= W are never stored)
    return 8 + W - 1;
}
// records per tap block of k_grid_f64_mfma, in 16-record parts (C2 eps 1e-12 gridding: 16 -> 60.8,
// 32 -> 59.4, 48 -> 58.7 ms; 48 is the most whose LDS still fits two workgroups per CU)
constexpr int kBlkG64 = 48;
// region rows: each kx half of the waves owns a slab of the region, rows
// x + kx of its own tiles (lower half KH + 1 rows, upper W - KH + 1; the row
// where they meet is held twice and flushed from both)
template <int W>
constexpr int f64m_rows() {
    return ((W + 1) / 2 + 1) + (W - (W + 1) / 2 + 1);
}
template <int W, bool WS>
constexpr size_t grid_f64m_lds() {
    return (size_t)f64m_rows<W>() * f64m_ry<W, WS>() * 2 * (WS ? W : 1) * sizeof(double) +
           (size_t)kBlkG64 * (3 * W + 2) * sizeof(double) + kPolyN * sizeof(double);
}
typedef double doublex4 __attribute__((ext_vector_type(4)));

// taps [J0, J1) of wave P of NP: the W taps in NP near-equal parts
template <int W, bool WS, int NP>
__device__ __forceinline__ void stage64_part(int part, const Stage64 &s, int nb, double *tap,
                                             const double *cl, double ihw, double beta, int lane) {
    static_assert(NP >= 1 && NP <= 4, "up to four parts");
    switch (part) {
        case 0: stage64_write<W, WS, 0, W / NP>(s, nb, tap, cl, ihw, beta, lane, true); break;
        case 1:
            if constexpr (NP > 1)
                stage64_write<W, WS, W / NP, 2 * W / NP>(s, nb, tap, cl, ihw, beta, lane, false);
            break;
        case 2:
            if constexpr (NP > 2)
                stage64_write<W, WS, 2 * W / NP, 3 * W / NP>(s, nb, tap, cl, ihw, beta, lane, false);
            break;
        default:
            if constexpr (NP > 3)
                stage64_write<W, WS, 3 * W / NP, W>(s, nb, tap, cl, ihw, beta, lane, false);
            break;
    }
}

template <int W, bool WS>
__global__ __attribute__((amdgpu_flat_work_group_size(64, 256))) void k_grid_f64_mfma(
    Geo g, const Rec64 *__restrict__ recs, const FineItem *__restrict__ items,
    uint32_t n_items, double *__restrict__ grid, int p_lo, int p_hi,
    const double *__restrict__ pc) {
    static_assert(W <= 16, "one M-tile of 16 rows per kx");
    constexpr int NQ = WS ? W : 1, NC = 2 * NQ, NT = f64m_ntiles<W, WS>(), NW = f64m_waves<W, WS>();
    constexpr int RX = f64m_rows<W>(), RY = f64m_ry<W, WS>(), RS = RX * RY * NC;
    constexpr int TR = 3 * W + 2, NTH = 64 * NW;
    constexpr int KH = (W + 1) / 2;  // kx M-tiles per wave
    extern __shared__ __attribute__((aligned(16))) double smd[];
    double *const reg = smd;       // [RX][RY][NC]: the lower slab's rows, then the upper's
    double *const tap = smd + RS;  // [kBlkG64][TR]
    double *const cl = tap + kBlkG64 * TR;  // the tap polynomials
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const double ihw = 2.0 / W, beta = (double)g.beta;
    for (int i = threadIdx.x; i < kPolyN; i += NTH) cl[i] = pc[i];
    // wave (N-tile wv % NT, kx half wv / NT): 4 waves for W > 8 with
    // w-stacking, two per SIMD at two workgroups per CU
    const int kx0 = (wv / NT) * KH;
    const int col = (wv % NT) * 16 + (lane & 15);
    const bool colok = col < NC;
    // B operand: tw[q] c[re/im] of record (lane >> 4); A: tu[kx] tv[ky]
    const int bq = 2 * W + (colok ? col >> 1 : 0), bc = 3 * W + (col & 1);
    const int ky = lane & 15;
    // rows ky >= W take A = 0: a clamped read times a 0 / 1 factor (no exec
    // masking in the K-step)
    const int kyc = min(ky, W - 1);
    const double kym = ky < W ? 1.0 : 0.0;
    const int rk = lane >> 4;
    const bool lower = kx0 == 0;  // this wave's kx tiles: KH (lower half) or W - KH
    // accumulator (k, i) = tap row (kx0 + k, rk + 4 i) of a cell at region
    // cell (cx, cy): element ((cx + kx0 + k) RY + cy + rk + 4 i) NC + col
    // (the upper half's slab starts at row KH + 1 of reg: its row x + k is
    // region row KH + x + k)
    const int lbase = (kx0 == 0 ? 0 : (KH + 1) * RY * NC) + rk * NC + col;
    const size_t plane_elems = (size_t)g.ngx * g.ngy;
    // the item loop on two code paths, the wave's kx tile count NK a
    // compile-time constant on each (KH for the lower half, W - KH for the
    // upper): a runtime guard `k < nkx` became an exec-mask branch around
    // every MFMA, and a per-K-step branch between two tile counts gave the
    // accumulators two register sets (24 v_mov_b64 per K-step); both paths
    // meet the same barriers in the same order
    auto run = [&](auto nk_tag) {
        for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
            uint32_t bnd[kGroupCell];
            const Item it = load_fine_item<kGroupCell>(items, w_it, n_items, bnd);
            if (it.b >= it.e) continue;
            int ibase, jbase;
            group_origin(g, (int)it.tile, ibase, jbase);
            __syncthreads();  // the previous item's flush reads of the region
            for (int i = threadIdx.x; i < RS; i += NTH) reg[i] = 0.0;
            doublex4 acc[KH];
#pragma unroll
            for (int k = 0; k < KH; ++k) acc[k] = doublex4{0.0, 0.0, 0.0, 0.0};
            int cur = -1, cb = 0;
            uint32_t cend = 0;  // end of the current cell's records
            // rows ky = rk + 4 i >= W hold exact zeros (A = 0 there): never
            // stored or loaded, so the region is only 8 + W - 1 rows deep
            auto store_n = [&](auto nt) {
                constexpr int NK = decltype(nt)::value;
                if (colok) {
                    double *d = reg + cb + lbase;
#pragma unroll
                    for (int k = 0; k < NK; ++k)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (4 * i + 3 < W || rk + 4 * i < W) d[k * RY * NC + 4 * i * NC] = acc[k][i];
                }
            };
            auto load_n = [&](auto nt) {
                constexpr int NK = decltype(nt)::value;
                const double *s = reg + cb + lbase;
#pragma unroll
                for (int k = 0; k < NK; ++k)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        acc[k][i] = (4 * i + 3 < W || rk + 4 * i < W) ? s[k * RY * NC + 4 * i * NC] : 0.0;
            };
            auto store_cell = [&]() { store_n(nk_tag); };
            auto load_cell = [&](int cell) {
                cb = ((cell & 1) * RY + (cell >> 1)) * NC;
                load_n(nk_tag);
            };
            auto kstep = [&](auto nt, const double *T) {
                constexpr int NK = decltype(nt)::value;
                const double bop = T[bq] * T[bc];
                const double tv = T[W + kyc] * kym;
                double aop[NK];
#pragma unroll
                for (int k = 0; k < NK; ++k) aop[k] = T[kx0 + k] * tv;
#pragma unroll
                for (int k = 0; k < NK; ++k)
                    acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(aop[k], bop, acc[k], 0, 0, 0);
            };
            // a block = 16-record parts (stage64_* handle 16 records)
            auto half_n = [&](uint32_t b, int h) {
                return (int)min((uint32_t)kBlk64, b + h * kBlk64 < it.e ? it.e - b - h * kBlk64 : 0u);
            };
            constexpr int NH = kBlkG64 / kBlk64;
            Stage64 nx[NH];
#pragma unroll
            for (int h = 0; h < NH; ++h) nx[h] = stage64_load(recs, it.b + h * kBlk64, half_n(it.b, h), lane);
            for (uint32_t b0 = it.b; b0 < it.e; b0 += kBlkG64) {
                __syncthreads();  // the region zeroing / previous block's tap reads
                const int nb = (int)min((uint32_t)kBlkG64, it.e - b0);  // (a multiple of 4)
#pragma unroll
                for (int h = 0; h < NH; ++h)
                    if (nb > h * kBlk64)
                        stage64_part<W, WS, NW>(wv, nx[h], min(nb - h * kBlk64, kBlk64), tap + h * kBlk64 * TR,
                                                cl, ihw, beta, lane);
                // the next block's records, in flight during this block's K-steps
                // (three blocks of 16 ahead, in three unrolled register sets,
                // measured the same: 61.3 ms)
                if (b0 + kBlkG64 < it.e) {
#pragma unroll
                    for (int h = 0; h < NH; ++h)
                        nx[h] = stage64_load(recs, b0 + kBlkG64 + h * kBlk64, half_n(b0 + kBlkG64, h),
                                             lane);
                }
                __syncthreads();
                // (K-steps not unrolled: unrolled, the register allocator gave
                // the accumulators two register sets and copied all 104 doubles
                // on every K-step without a cell change, behind the MFMAs)
#pragma unroll 1
                for (int kk = 0; kk < kBlkG64 / 4; ++kk) {
                    if (4 * kk >= nb) break;
                    const uint32_t ri = b0 + 4u * (uint32_t)kk;
                    // one scalar compare per K-step against the current cell's
                    // end; the 15 compares of the cell search only at a change
                    // (the compare chain per K-step was ~45 of the kernel's
                    // ~340 SALU per block and wave)
                    if (ri >= cend) {  // (workgroup-uniform)
                        int cell = 0;
                        uint32_t e = bnd[kGroupCell - 1];
#pragma unroll
                        for (int c = 0; c < kGroupCell - 1; ++c) {
                            cell += ri >= bnd[c] ? 1 : 0;
                            e = (ri < bnd[c] && bnd[c] < e) ? bnd[c] : e;
                        }
                        cend = e;
                        if (cur >= 0) store_cell();
                        // (no barrier: the two kx halves accumulate into slabs of
                        // their own, and the two column tiles of a half touch
                        // disjoint columns; a barrier here with the shared region
                        // stopped all four waves at every cell change)
                        cur = cell;
                        load_cell(cur);
                    }
                    const double *T = tap + (4 * kk + rk) * TR;
                    kstep(nk_tag, T);
                }
            }
            if (cur >= 0) store_cell();
            __syncthreads();
            // flush in the planes' own order: consecutive lanes take consecutive
            // doubles of one plane's region rows (re/im interleaved), so a wave's
            // atomics cover a few contiguous segments
            constexpr int RYV = 8 + W - 1;  // rows a footprint reaches
            constexpr int FPP = RX * RYV * 2;  // doubles per plane of the region
            for (int i = threadIdx.x; i < NQ * FPP; i += NTH) {
                const int q = i / FPP, f = i - q * FPP, cell = f >> 1;
                const int xl = cell / RYV, yl = cell - xl * RYV;
                const double v = reg[(xl * RY + yl) * NC + 2 * q + (f & 1)];
                const int p = (int)it.p0 + q;
                if (v == 0.0 || p < p_lo || p >= p_hi) continue;
                // slab row -> region row (the upper slab starts at KH)
                int gx = ibase + (xl <= KH ? xl : xl - 1);
                if (gx >= g.ngx) gx -= g.ngx;
                int gy = jbase + yl;
                if (gy >= g.ngy) gy -= g.ngy;
                atomicAdd(grid + 2 * ((size_t)(p - p_lo) * plane_elems + (size_t)gx * g.ngy + gy) + (f & 1),
                          v);
            }
        }
    };
    if (lower) run(std::integral_constant<int, KH>{});
    else run(std::integral_constant<int, W - KH>{});
}

// fp64 MFMA degridder (predict), the adjoint GEMM per block of <= 16
// records of one cell:
//     P[(q, re/im), r] = sum_(kx, ky) G[(kx, ky), (q, re/im)] tu_r[kx] tv_r[ky]
// M = the 2 NQ (q, re/im) rows (<= 2 tiles), N = 16 records, K = the taps
// in steps of 4 rows ky (ky >= W: B = 0), then V_r = c_r sum_q tw_r[q]
// P[q, r] (lane-local plus two cross-lane adds).  The item's region of the
// planes is staged in LDS once ([x][y][(q, re/im)], rows ky >= W zero) and
// shared read-only by the workgroup's waves, each of which takes every NW-th
// 16-record block of the item's cells (no barriers between blocks).
constexpr int kDeg64Waves = 8;
// blocks of one item: chunk / 16 + one partial block per cell (plan_geometry
// caps a k_degrid_f64_mfma plan's chunk to fit)
constexpr int kMaxBlk64 = 1024;
template <int W, bool WS>
constexpr size_t degrid_f64m_lds() {
    return (size_t)(W + 1) * 23 * 2 * (WS ? W : 1) * sizeof(double) +
           (size_t)kDeg64Waves * kBlk64 * (3 * W + 2) * sizeof(double) + kPolyN * sizeof(double) +
           (size_t)(2 * kMaxBlk64 + 1) * sizeof(uint32_t);
}

template <int W, bool WS, class VT, class R>
__global__ __launch_bounds__(64 * kDeg64Waves) void k_degrid_f64_mfma(
    Geo g, const R *__restrict__ recs, const FineItem *__restrict__ items,
    uint32_t n_items, const double2 *__restrict__ grid, int p_lo, int p_hi, VT *vis, int64_t vrs,
    int64_t vcs, int accumulate, OutConv oc, const double *__restrict__ pc) {
    static_assert(W <= 16, "K-steps of 4 rows ky < 16");
    constexpr int NQ = WS ? W : 1, NC = 2 * NQ, MT = (NC + 15) / 16;
    constexpr int RX = W + 1, RY = 23, RS = RX * RY * NC, TR = 3 * W + 2;
    constexpr int NTH = 64 * kDeg64Waves;
    constexpr int RYV = 8 + W - 1;                          // region rows footprints reach
    constexpr int NLD = (NQ * RX * RYV + NTH - 1) / NTH;  // c128 loads per thread
    extern __shared__ __attribute__((aligned(16))) double smd[];
    double *const reg = smd;  // [RX][RY][NC]
    // rows RYV .. RY - 1 are read by K-steps whose B is zero: they must hold
    // finite values, so they are zeroed once (the item loads never write them)
    for (int i = threadIdx.x; i < RS; i += NTH) reg[i] = 0.0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double *const tap = smd + RS + wv * kBlk64 * TR;  // this wave's tap block
    double *const cl = smd + RS + kDeg64Waves * kBlk64 * TR;  // the tap polynomials
    for (int i = threadIdx.x; i < kPolyN; i += NTH) cl[i] = pc[i];
    // tap rows past a block's records are read (times 0) by its K-steps: they
    // start finite
    for (int i = threadIdx.x; i < kDeg64Waves * kBlk64 * TR; i += NTH) smd[RS + i] = 0.0;
    uint32_t *const bcel = reinterpret_cast<uint32_t *>(cl + kPolyN);  // block: cell | records << 8
    uint32_t *const btab = bcel + kMaxBlk64;                            // block: first record (+ count)
    const double ihw = 2.0 / W, beta = (double)g.beta;
    const int rn = lane & 15, gk = lane >> 4;  // B column (record), K row
    const size_t plane_elems = (size_t)g.ngx * g.ngy;
    const bool plain = oc.npv == 1 && oc.cre[0] == 1.0 && oc.cim[0] == 0.0;
    // A operand of M-tile m at tap (kx, 4 s + gk): region element
    // (kx RY + cy + 4 s + gk) NC + 16 m + rn of the cell's origin (cx, cy)
    for (uint32_t w_it = blockIdx.x; w_it < n_items; w_it += gridDim.x) {
        uint32_t bnd[kGroupCell];
        const Item it = load_fine_item<kGroupCell>(items, w_it, n_items, bnd, true);
        if (it.b >= it.e) continue;
        int ibase, jbase;
        group_origin(g, (int)it.tile, ibase, jbase);
        // the region's planes: consecutive threads take consecutive y of one
        // plane row (16-B c128 loads, coalesced), all loads issued before
        // any LDS store; planes outside [p_lo, p_hi) are zeros
        // (the thread index through an empty asm statement: the index math
        // is redone per item instead of being hoisted and kept live -- it
        // was, 8 x 5 registers spilled to scratch)
        int tid = (int)threadIdx.x;
        asm volatile("" : "+v"(tid));
        double2 gv[NLD];
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int i = tid + k * NTH;
            const int q = i / (RX * RYV), rem = i - q * (RX * RYV);
            const int xl = rem / RYV, yl = rem - xl * RYV;
            const int p = (int)it.p0 + q;
            const bool ok = i < NQ * RX * RYV && p >= p_lo && p < p_hi;
            int gx = ibase + xl;
            if (gx >= g.ngx) gx -= g.ngx;
            int gy = jbase + yl;
            if (gy >= g.ngy) gy -= g.ngy;
            const double2 *src = grid + (size_t)(ok ? p - p_lo : 0) * plane_elems +
                                 (ok ? (size_t)gx * g.ngy + gy : 0);
            gv[k] = *src;
            if (!ok) gv[k] = make_double2(0.0, 0.0);
        }
        __syncthreads();  // the previous item's region reads
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int i = tid + k * NTH;
            if (i < NQ * RX * RYV) {
                const int q = i / (RX * RYV), rem = i - q * (RX * RYV);
                const int xl = rem / RYV, yl = rem - xl * RYV;
                *reinterpret_cast<double2 *>(reg + (xl * RY + yl) * NC + 2 * q) = gv[k];
            }
        }
        // the item's blocks (cell c's records [cs, ce) in blocks of 16) as a
        // table in LDS: lane c of wave 0 counts its cell's blocks, a wave
        // prefix sum places them (a scalar walk of the cells per block cost
        // ~400 SALU per block and wave)
        if (wv == 0) {
            const int c = lane & 15;
            const FineItem *F = items + w_it;  // (load_fine_item's, natural order)
            const uint32_t o_prev = c == 0 ? (uint32_t)it.b : F->o[c - 1];
            const uint32_t o_c = c == kGroupCell - 1 ? (uint32_t)it.e : F->o[c];
            const uint32_t cs = min(max(o_prev, (uint32_t)it.b), (uint32_t)it.e);
            const uint32_t ce = min(max(o_c, cs), (uint32_t)it.e);
            const uint32_t nbk = lane < kGroupCell ? (ce - cs + kBlk64 - 1) / kBlk64 : 0u;
            uint32_t x = nbk;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if ((lane & 15) >= o) x += y;
            }
            const uint32_t off = x - nbk;  // exclusive prefix
            if (lane == 15) btab[kMaxBlk64] = x;  // the block count
            if (lane < kGroupCell)
                for (uint32_t j = 0; j < nbk && off + j < kMaxBlk64; ++j) {
                    const uint32_t b0 = cs + j * kBlk64;
                    btab[off + j] = b0;
                    bcel[off + j] = (uint32_t)c | (min((uint32_t)kBlk64, ce - b0) << 8);
                }
        }
        __syncthreads();
        const uint32_t nblk = min(btab[kMaxBlk64], (uint32_t)kMaxBlk64);
        uint32_t kb = (uint32_t)wv;
        Stage64 nxt =
            kb < nblk ? stage64_load(recs, btab[kb], (int)(bcel[kb] >> 8), lane) : Stage64{};
        for (; kb < nblk; kb += kDeg64Waves) {
            {
                const uint32_t b0 = btab[kb], cn = bcel[kb];
                const int c = (int)(cn & 15u);
                const int nb = (int)(cn >> 8);
                const Stage64 cur_s = nxt;
                // (in two halves of the taps: half the Horner registers live)
                stage64_write<W, WS, 0, W / 2>(cur_s, nb, tap, cl, ihw, beta, lane, true);
                stage64_write<W, WS, W / 2, W>(cur_s, nb, tap, cl, ihw, beta, lane, false);
                if (kb + kDeg64Waves < nblk)
                    nxt = stage64_load(recs, btab[kb + kDeg64Waves],
                                       (int)(bcel[kb + kDeg64Waves] >> 8), lane);
                wave_lds_sync();
                const double *T = tap + rn * TR;  // this lane's record (B column)
                const bool rok = rn < nb;
                const double *G = reg + ((c & 1) * RY + (c >> 1)) * NC + gk * NC + rn;
                doublex4 acc[MT];
#pragma unroll
                for (int m = 0; m < MT; ++m) acc[m] = doublex4{0.0, 0.0, 0.0, 0.0};
                // the four tv taps of this lane's K rows (the same for every
                // kx), zero for rows ky >= W; lanes past the block's records
                // take tu = 0 by a factor, not an exec-masked read
                double tvk[4];
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int ky = 4 * s + gk;
                    tvk[s] = ky < W ? T[W + min(ky, W - 1)] : 0.0;
                }
                const double rokf = rok ? 1.0 : 0.0;
                // (kx not unrolled: unrolled, the compiler hoists every K-step's
                // LDS reads to the top, 256 registers and scratch spills); one
                // kx's 4 MT A operands are all read before its MFMAs
#pragma unroll 1
                for (int kx = 0; kx < W; ++kx) {
                    const double tu = T[kx] * rokf;
                    double gvs[4][MT];
#pragma unroll
                    for (int s = 0; s < 4; ++s)
#pragma unroll
                        // (rows (q, re/im) >= NC read the next region cell's
                        // values: finite, and those rows of D are never used)
                        for (int m = 0; m < MT; ++m) gvs[s][m] = G[(kx * RY + 4 * s) * NC + 16 * m];
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        const double bop = tu * tvk[s];
#pragma unroll
                        for (int m = 0; m < MT; ++m)
                            acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(gvs[s][m], bop, acc[m], 0, 0, 0);
                    }
                    // the LDS reads first, then the products, then the MFMAs
                    // (left to itself the scheduler waited on each read right
                    // before its MFMA)
                    __builtin_amdgcn_sched_group_barrier(0x0100, 4 * MT + 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x0002, 5, 0);
                    __builtin_amdgcn_sched_group_barrier(0x0008, 4 * MT, 0);
                }
                // lane holds rows 16 m + gk + 4 i of column rn: (q, re/im) =
                // ((16 m + gk + 4 i) >> 1, gk & 1)
                double part = 0.0;
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = 16 * m + gk + 4 * i;
                        if (row < NC) part = fma(acc[m][i], T[2 * W + (row >> 1)], part);
                    }
                part += __shfl_xor(part, 32, 64);  // gk and gk ^ 2: the same component
                const double pim = __shfl_xor(part, 16, 64);
                if (gk == 0 && rok) {
                    const double sr = part, si = pim;
                    const double cr = T[3 * W], ci = T[3 * W + 1];
                    const double xr = cr * sr - ci * si, xi = cr * si + ci * sr;
                    const uint32_t idx = cur_s.idx;  // (lane rn < 16: record rn)
                    const int64_t row = idx / (uint32_t)g.nchan;
                    const int chan = (int)(idx - row * g.nchan);
                    VT *pv_ = vis + row * vrs + chan * vcs;
                    if (plain) {
                        store_vis_d(pv_, xr, xi, accumulate);
                    } else {
                        for (int k = 0; k < oc.npv; ++k) {
                            if (oc.cre[k] == 0.0 && oc.cim[k] == 0.0) continue;
                            store_vis_d(pv_ + k * oc.vps, oc.cre[k] * xr - oc.cim[k] * xi,
                                        oc.cre[k] * xi + oc.cim[k] * xr, accumulate);
                        }
                    }
                }
                wave_lds_sync();  // the block's tap reads before the next staging
            }
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
static hipfftHandle fft_plan_1d(int n, int stride, int dist, int batch, hipStream_t stream,
                               bool f64 = false) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, int, int, int, int>, hipfftHandle> plans;
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    // (one plan per workspace slot: a plan's stream and work area are its own)
    const auto key = std::make_tuple(dev, n, stride, dist, batch, f64 ? 1 : 0, ws_slot());
    auto itp = plans.find(key);
    hipfftHandle h;
    if (itp == plans.end()) {
        int nn[1] = {n};
        if (hipfftPlanMany(&h, 1, nn, nn, stride, dist, nn, stride, dist,
                           f64 ? HIPFFT_Z2Z : HIPFFT_C2C, batch) != HIPFFT_SUCCESS)
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

// fp64 path: epsilon below the fp32 floor, W in [kMinW64, kMaxW64]
static int kernel_support64(double epsilon) {
    const int W = (int)std::ceil(-std::log10(std::max(epsilon, 1e-15) / 10.0) - 1e-9);
    return std::min(std::max(W, kMinW64), kMaxW64);
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
    char *&b = bufs[2 * dev + ws_slot()];  // one per workspace slot
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

// The visibilities' bucketing: histogram, offsets, work items and the
// per-call metadata read back by the host.  Records occupy recs[0, nrec).
struct Part {
    int64_t nvis = 0;
    unsigned *hist = nullptr, *offs = nullptr, *nch = nullptr, *ioffs = nullptr;
    unsigned long long *nbad = nullptr;
    unsigned *npad = nullptr;  // pad records of a 4-padded plan (device)
    Item *items = nullptr;       // coarse (16x16-cell) plans
    FineItem *fitems = nullptr;  // one-cell plans: one per item; coarse plans: 16 per
                                 // item after the sub-sort (k_subsort)
    unsigned *meta = nullptr;    // device: see k_part_meta
    // host copies (read_part_meta)
    int64_t nrec = 0, nitems = 0;
    std::vector<unsigned> p0_items;
    // two-level (tiled) plans: see k_t_count .. k_t_final_s
    int t_g1 = 0;          // workgroups of the count / value passes
    int64_t t_vpw = 0;     // visibilities per such workgroup
    unsigned t_maxch = 0;  // bound on the second-level chunks
    unsigned t_maxseg = 0;  // bound on their prefix segments
    unsigned *t_binc = nullptr, *t_binbase = nullptr, *t_segb = nullptr, *t_nsegb = nullptr;
    unsigned *t_nbl = nullptr, *t_m1 = nullptr, *t_m2 = nullptr, *t_tot = nullptr;
    unsigned *t_cbase = nullptr, *t_meta_ch = nullptr, *t_stot = nullptr;
    TChunk *t_chunks = nullptr;
    TSeg *t_segs = nullptr;
    unsigned long long *t_binsum = nullptr, *t_bofs = nullptr;
    uint16_t *t_lkey = nullptr;
    double *t_fsc = nullptr;  // frequency / c per channel
    void *t_a = nullptr;  // records in bin order (the value pass's output)
};

struct Plan {
    Geo g;
    VisRec *recs = nullptr;
    Part pt;
    bool f64 = false;                // fp64 NUFFT (epsilon < 1e-7): VisRec64, c128 planes
    bool subsort = false;            // 16x16-cell buckets re-ordered by cell (k_subsort)
    bool subpad = false;             // ... into 4-padded RecC cells (invert: k_subsort_pad)
    uint8_t *cls = nullptr;          // subpad: each RecC record's cell in its bucket
    RecC *recs_pad = nullptr;        // subpad: the 4-padded, cell-ordered records
    bool pad4 = false;               // one-cell buckets padded to 4 records (k_grid_mfma_pad)
    bool pad64 = false;              // fp64 invert: VisRec64 cells padded to 4 (k_grid_f64_mfma)
    bool mfma64 = false;             // fp64 predict on k_degrid_f64_mfma (one-cell buckets)
    float2 *vdirect = nullptr;       // dirty2ms: the degridder writes c64 vis in place
    float2 *zout = nullptr;          // ... and the rank pass zeroes the ones with no record
    int chunk_planes = 1;            // planes resident per pass
    int fft_planes = 1;              // planes per FFT / screen batch (spec, spec_in)
    int row_lo = 0, row_hi = 0;      // grid rows (x) the visibilities reach
    unsigned chunk = kChunkMin;      // max records per work item
    float2 *grid = nullptr;
    float2 *spec = nullptr;     // T[q][iy][kx]: transposed y-spectra (pruned FFT)
    float2 *spec_in = nullptr;  // band-only input of the backward x-FFT (zeros elsewhere)
    float2 *spec_adj = nullptr;  // forward x-FFT input: the image's kx columns (zeros elsewhere)
    CoreAcc core{nullptr, 0, 0, 0, 0};  // fp32 invert: fp64 companion of the uv core
};

// the element size of the planes and spectra: c64, or c128 on the fp64 path
static size_t cbytes(const Plan &P) { return P.f64 ? sizeof(double2) : sizeof(float2); }

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
// and key/rank arrays still to be allocated (`need_other`) and a reserve for
// the caller: max(6 GiB, 1/16 of the device, 18 GB on a 288 GB MI355X), so
// that the output arrays of the caller's next calls still fit beside the
// planes the workspace keeps cached (a C4 shard keeps 150 GB of planes).  A
// C2 invert keeps its 9 planes resident, and so does a C4 shard (70 planes of
// 16384^2) on a 288 GB MI355X, gridding every record once instead of once
// per plane chunk.
static size_t grid_budget_bytes(size_t need_other) {
    const char *e = std::getenv("SDP_HIP_GRID_BUDGET_GB");
    if (e && std::atof(e) > 0) return (size_t)(std::atof(e) * 1073741824.0);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b == 0) return (size_t)8 << 30;
    Workspace &ws = Workspace::get();
    const size_t held_planes =
        ws.held(ws_name("grid")) + ws.held(ws_name("spec")) + ws.held(ws_name("spec_in")) +
        ws.held(ws_name("spec_adj"));
    const size_t held_other = ws.held(ws_name("recs")) + ws.held(ws_name("key_rank")) +
                              ws.held(ws_name("degrid_acc")) + ws.held(ws_name("recs_pad")) +
                              ws.held(ws_name("rec_cls")) + ws.held(ws_name("recs_a")) +
                              ws.held(ws_name("rec_lkey")) + ws.held(ws_name("t_m2"));
    const size_t avail = free_b + held_planes + held_other;
    const size_t reserve = std::max<size_t>((size_t)6 << 30, total_b / 16);
    const size_t need = need_other + reserve;
    return avail > need ? avail - need : (size_t)1 << 30;
}

static hipStream_t aux_stream() {
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    dev = 2 * dev + ws_slot();  // one per workspace slot
    std::lock_guard<std::mutex> lk(mu);
    auto it = streams.find(dev);
    if (it != streams.end()) return it->second;
    hipStream_t s;
    SDP_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    streams[dev] = s;
    return s;
}

// The backward x-FFT input T_in holds the transposed band [row_lo, row_hi)
// of every T row and zeros elsewhere.  The transposes write only the band
// (the 16-byte one also the zeros around it in its 64-row aligned tiles),
// so the zeros are kept across calls: the buffer is cleared only when it is
// (re)allocated or the band / shape changes.
struct BandState {
    uint64_t epoch = 0;  // the allocation (Workspace epoch) the zeros were written to
    size_t elems = 0;
    int lo = -1, hi = -1, ny = 0, ngx = 0;
    int cb = 0;  // element bytes (8: c64, 16: c128): a c128 band read as c64 is not zero
};

static float2 *band_input(const Plan &P, hipStream_t st) {
    static std::mutex mu;
    static std::map<int, BandState> states;
    const Geo &g = P.g;
    const size_t elems = (size_t)P.fft_planes * g.ny * g.ngx * (cbytes(P) / sizeof(float2));
    float2 *buf = scratch<float2>("spec_in", elems);
    // the buffer's allocation identity, not its address: a release and a
    // new allocation at the same address leaves unzeroed memory behind
    const uint64_t ep = Workspace::get().epoch(ws_name("spec_in"));
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    BandState &b = states[2 * dev + ws_slot()];
    if (b.epoch != ep || b.elems < elems || b.lo != P.row_lo || b.hi != P.row_hi || b.ny != g.ny ||
        b.ngx != g.ngx || b.cb != (int)cbytes(P)) {
        SDP_HIP_CHECK(hipMemsetAsync(buf, 0, elems * sizeof(float2), st));
        b = BandState{ep, elems, P.row_lo, P.row_hi, g.ny, g.ngx, (int)cbytes(P)};
    }
    return buf;
}

// The forward x-FFT input of the predict holds the screened image in the
// kx columns of the image's x-frequencies and zeros in the others; the
// screens write only those columns, so the zeros are kept across calls (a
// separate buffer: the invert's x-FFT output overwrites whole rows of spec)
struct AdjState {
    uint64_t epoch = 0;
    size_t elems = 0;
    int nx = 0, ny = 0, ngx = 0, cb = 0;  // (cb: element bytes, as BandState)
};

static float2 *adj_input(const Plan &P, hipStream_t st) {
    static std::mutex mu;
    static std::map<int, AdjState> states;
    const Geo &g = P.g;
    const size_t elems = (size_t)P.fft_planes * g.ny * g.ngx * (cbytes(P) / sizeof(float2));
    float2 *buf = scratch<float2>("spec_adj", elems);
    const uint64_t ep = Workspace::get().epoch(ws_name("spec_adj"));
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    AdjState &b = states[2 * dev + ws_slot()];
    if (b.epoch != ep || b.elems < elems || b.nx != g.nx || b.ny != g.ny || b.ngx != g.ngx ||
        b.cb != (int)cbytes(P)) {
        SDP_HIP_CHECK(hipMemsetAsync(buf, 0, elems * sizeof(float2), st));
        b = AdjState{ep, elems, g.nx, g.ny, g.ngx, (int)cbytes(P)};
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

// The resident planes of a batched invert between its FIRST and LAST batch:
// the plane buffer they live in (its workspace epoch: any reallocation or
// release changes it), the geometry and the bounds.  A later batch must match it; any other wstack call (a fresh
// non-batched plan) or a workspace release invalidates it, so a batch that
// would accumulate into planes another call has overwritten or freed is
// refused instead of gridding into them.
struct BatchSeq {
    bool valid = false;
    uint64_t epoch = 0;
    const void *grid = nullptr;
    int nx = 0, ny = 0, do_w = 0, nplanes = 0;
    double px = 0, py = 0, eps = 0;
    unsigned flip = 0;
    double b[8] = {0, 0, 0, 0, 0, 0, -1, -1};  // bounds (+ the w slab)
};

static std::mutex g_kept_mu;
static std::map<int, KeptBuckets> g_kept;
static std::map<int, BatchSeq> g_batch;

static int cur_device() {
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    return dev;
}

static void drop_kept_buckets() {
    std::lock_guard<std::mutex> lk(g_kept_mu);
    g_kept[cur_device()].valid = false;
}

static void drop_batch_seq() {
    std::lock_guard<std::mutex> lk(g_kept_mu);
    g_batch[cur_device()].valid = false;
}

static void keep_buckets(const Plan &P, const Inputs &in) {
    std::lock_guard<std::mutex> lk(g_kept_mu);
    KeptBuckets &k = g_kept[cur_device()];
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
    const KeptBuckets &k = g_kept[cur_device()];
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

static BatchSeq batch_token(const Plan &P, const Inputs &in) {
    BatchSeq s;
    s.valid = true;
    s.epoch = Workspace::get().epoch(ws_name("grid"));
    s.grid = P.grid;
    s.nx = in.nx;
    s.ny = in.ny;
    s.do_w = in.do_w;
    s.nplanes = P.g.nplanes;
    s.px = in.px;
    s.py = in.py;
    s.eps = in.eps;
    s.flip = in.flags & SDP_HIP_FLIP_UW;
    for (int k = 0; k < 6; ++k) s.b[k] = in.bounds[k];
    if (in.flags & SDP_HIP_W_SLAB) {
        s.b[6] = in.bounds[6];
        s.b[7] = in.bounds[7];
    }
    return s;
}

static void check_batch_seq(const Plan &P, const Inputs &in, bool first) {
    std::lock_guard<std::mutex> lk(g_kept_mu);
    BatchSeq &cur = g_batch[cur_device()];
    const BatchSeq t = batch_token(P, in);
    if (first) {
        cur = t;
        return;
    }
    SDP_REQUIRE(cur.valid && cur.epoch == t.epoch && cur.grid == t.grid,
                "batched invert: no resident planes of this sequence (its first batch did not "
                "run, or another wstack call or a workspace release came in between)");
    bool same = cur.nx == t.nx && cur.ny == t.ny && cur.do_w == t.do_w &&
                cur.nplanes == t.nplanes && cur.px == t.px && cur.py == t.py &&
                cur.eps == t.eps && cur.flip == t.flip;
    for (int k = 0; k < 8; ++k) same = same && cur.b[k] == t.b[k];
    SDP_REQUIRE(same, "batched invert: every batch of a sequence needs the geometry, epsilon, "
                      "flags and bounds of its first batch");
}

// w-plane layout of an invert / predict (ducc0's w-stacking geometry): plane
// spacing dw = 1 / (2 tmax) from the image's largest n - 1, first plane w0 a
// half support below the smallest w, nplanes covering the largest; nps =
// distinct first planes.  Shared by plan_geometry and sdp_hip_wstack_layout.
static void w_layout(const Inputs &in, double wmin, double wmax, Geo &g) {
    const double lmax = (in.nx / 2) * in.px, mmax = (in.ny / 2) * in.py;
    const double r2 = std::min(lmax * lmax + mmax * mmax, 1.0);
    const double tmax = 1.0 - std::sqrt(1.0 - r2);
    g.do_w = (in.do_w && tmax > 0.0) ? 1 : 0;
    if (g.do_w) {
        g.s0 = 0.5 * tmax;
        g.dw = 1.0 / (2.0 * tmax);
        g.w0 = wmin - (0.5 * g.W - 0.5) * g.dw;
        const double pwmax = std::fma(wmax, 1.0 / g.dw, -(g.w0 * (1.0 / g.dw)));
        g.nplanes = (int)std::floor(pwmax - 0.5 * g.W) + 1 + g.W;
        g.nps = g.nplanes - g.W + 1;
    } else {
        g.s0 = 0.0;
        g.dw = 1.0;
        g.w0 = 0.0;
        g.nplanes = 1;
        g.nps = 1;
    }
}

// the folded per-visibility factors of vis_coord_v (the full layout's
// plane origin: call before a w slab moves w0)
static void geo_factors(Geo &g) {
    const double idw = 1.0 / g.dw;
    g.kax = g.su * g.px * g.ngx;
    g.kby = g.py * g.ngy;
    g.kpw = g.su * idw;
    g.kpw0 = g.w0 * idw;
}

// Geometry shared by both directions: kernel, padded grid, w planes, bucket
// granularity, row band, plane chunking.  One host sync (uvw and frequency
// extremes) unless the bounds are given.
static Plan plan_geometry(const Inputs &in, bool grid_mode, hipStream_t st) {
    SDP_REQUIRE(in.nx > 0 && in.ny > 0 && in.nx % 2 == 0 && in.ny % 2 == 0,
                "npix_x and npix_y must be positive and even");
    SDP_REQUIRE(in.px > 0 && in.py > 0, "pixel sizes must be positive");
    SDP_REQUIRE(in.nchan > 0 && in.nrow >= 0, "nchan must be positive");
    SDP_REQUIRE(in.nrow * (int64_t)in.nchan < (int64_t)0xffffffffll,
                "more than 2^32 visibilities per call");
    // a fresh plan re-uses the bucketing scratch and may overwrite a batch
    // sequence's planes -- those of its own slot: kept buckets and batch
    // sequences exist in slot 0 only, and a slot-1 plan uses the '#1'
    // buffers, so it leaves them valid
    if (ws_slot() == 0) {
        drop_kept_buckets();
        if (!in.bounds) drop_batch_seq();
    }
    Plan P;
    Geo &g = P.g;
    P.f64 = in.eps < 1.0e-7 && !(in.flags & SDP_HIP_FP32);
    g.W = P.f64 ? kernel_support64(in.eps) : kernel_support(in.eps);
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
    g.inv_nchan = 1.0 / in.nchan;
    g.nrow = in.nrow;

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

    w_layout(in, wmin, wmax, g);
    geo_factors(g);
    // w slab of the sequence's plane layout (bounds[6], bounds[7]: first
    // planes [lo, hi)): this call's planes are lo .. hi + W - 2 and its w0 the
    // slab's first plane, so records, keys, FFTs and screens see only the slab
    g.slab = 0;
    g.slab_lo = 0;
    g.nps_all = g.nps;
    if (in.flags & SDP_HIP_W_SLAB) {
        SDP_REQUIRE(in.bounds != nullptr, "SDP_HIP_W_SLAB needs the batch bounds (8 doubles)");
        SDP_REQUIRE(g.do_w, "SDP_HIP_W_SLAB needs w-stacking");
        SDP_REQUIRE(grid_mode && !P.f64, "SDP_HIP_W_SLAB is an fp32 invert option");
        const double lo_d = in.bounds[6], hi_d = in.bounds[7];
        SDP_REQUIRE(lo_d >= 0.0 && lo_d < hi_d && lo_d == std::floor(lo_d) &&
                        hi_d == std::floor(hi_d) && lo_d < (double)g.nps,
                    "w slab: first planes [lo, hi) must be integers with 0 <= lo < hi and lo "
                    "below the layout's first-plane count");
        const int lo = (int)lo_d, hi = (int)std::min<double>(hi_d, (double)g.nps);
        g.slab = 1;
        g.slab_lo = lo;
        g.w0 += lo * g.dw;
        g.nps = hi - lo;
        g.nplanes = g.nps + g.W - 1;
    }
    // bucket window (origins only: the footprints' halo may leave it): the
    // `al`-aligned cell range [ng/2 - reach, ng/2 + reach), or the whole
    // (al-rounded) axis when that reaches an edge
    auto window = [&](double m, int ng, int al, int &w0, int &wn) {
        const int reach = (int)std::ceil(m + 0.5 * g.W) + 2;
        int lo = (ng / 2 - reach) & ~(al - 1);
        int hi = ((ng / 2 + reach + al - 1) / al) * al;
        if (lo <= 0 || hi >= ng) {
            lo = 0;
            hi = ((ng + al - 1) / al) * al;
        }
        w0 = lo;
        wn = hi - lo;
    };
    const double amax = umax * in.px * g.ngx, bmax = vmax * in.py * g.ngy;
    // two-level bucketing (k_t_*): one-cell keys in 64 x 64-cell bins, while
    // the bins of the window fit the first level's LDS histogram (C2: 2 first
    // planes x 59 x 61 bins); SDP_HIP_BUCKET2=0 selects the single-level
    // one-cell histogram below (A/B and tests).  Not for the fp32 predict:
    // its 32-byte records make the second move cost more than the
    // single-level count pass's atomics save (C2 prep 7.3 vs 5.3 ms); =2
    // forces it there too (tests)
    g.tiled = 0;
    g.tlx = g.tly = g.nbins = 0;
    const int b2 = env_int("SDP_HIP_BUCKET2", 1);
    // A kept bucketing (SDP_HIP_KEEP_BUCKETS, the pols of invert_ng) also
    // stays single-level: its reuse calls then run only the value pass,
    // where the two-level sort's would add the second move (C2 4 pols:
    // 57.6 vs 50 ms).
    if (b2 != 0 && (grid_mode || P.f64 || b2 == 2) &&
        (!(in.flags & SDP_HIP_KEEP_BUCKETS) || b2 == 2) &&
        env_int("SDP_HIP_BUCKET", 0) != kTileCoarse) {
        int x0, nx_, y0, ny_;
        window(amax, g.ngx, kTile, x0, nx_);
        window(bmax, g.ngy, kTile, y0, ny_);
        const int64_t nbins = (int64_t)(nx_ / kTile) * (ny_ / kTile) * g.nps;
        // the padded record total and the cell bases are 32-bit: every
        // non-empty cell may add up to 3 pad records, so the two-level sort
        // needs nvis + 3 min(nvis, cells) < 2^32 (else the single-level or
        // coarse bucketing below, whose totals are 64-bit)
        const int64_t nv = in.nrow * (int64_t)in.nchan;
        const int64_t cells = (int64_t)nx_ * ny_ * g.nps;
        const bool fits32 = !grid_mode || nv + 3 * std::min(nv, cells) < (int64_t)0xffffffffll;
        if (nbins <= kMaxBins && fits32) {
            g.tiled = 1;
            g.wx0 = x0;
            g.wnx = nx_;
            g.wy0 = y0;
            g.wny = ny_;
            g.tlx = nx_ / kTile;
            g.tly = ny_ / kTile;
            g.nbins = (int)nbins;
        }
    }
    if (!g.tiled) {
        // x (rows) only: the y stride stays ngy, since a compacted y range
        // packs the hot histogram counters of the uv core closer together and
        // measured 2x slower count-pass atomics on C2
        window(amax, g.ngx, kGridAlign, g.wx0, g.wnx);
        g.wy0 = 0;
        g.wny = g.ngy;
    }
    // bucket granularity: one-cell buckets while the dense (first plane, cell)
    // histogram stays below kMaxCellKeys (C2: 115 M keys), else 16x16-cell
    // buckets sub-sorted by cell per work item (C4's 16384^2 x 70 planes);
    // SDP_HIP_BUCKET=16 forces the latter (tests of the large-grid path)
    {
        const int64_t cell = (int64_t)g.wnx * g.wny * g.nps;
        // (the one-cell invert's 4-padded record total is 32-bit: see fits32
        // above; the coarse path checks its padded total exactly)
        const int64_t nv = in.nrow * (int64_t)in.nchan;
        const bool fits32 = !grid_mode || nv + 3 * std::min(nv, cell) < (int64_t)0xffffffffll;
        g.sub = (g.tiled || (cell <= kMaxCellKeys && fits32)) ? kTileCell : kTileCoarse;
        if (env_int("SDP_HIP_BUCKET", 0) == kTileCoarse) g.sub = kTileCoarse;
    }
    g.nty = g.wny / g.sub;
    SDP_REQUIRE(!P.f64 || g.sub == kTileCell,
                "epsilon < 1e-7 runs the fp64 NUFFT, which needs the one-cell bucket histogram "
                "(first planes x window cells <= 2^28): use a larger epsilon or SDP_HIP_FP32");
    // gridding on one-cell keys: blocks of bx x 8 cells per work item (the
    // region flushed with atomics is (bx + W - 1) x (8 + W - 1) cells)
    // (blocks of 4 x 8 and 8 x 8 cells halve the flushed atomics but measured
    // slower on C2, 4.9 and 5.5 vs 4.6 ms: the larger LDS region lowers the
    // waves per CU this latency-bound kernel runs with)
    g.bx = 2;
    g.bxs = 1;
    g.ntiles = (g.wnx / g.sub) * g.nty;
    g.grp = g.sub == kTileCell ? kGroupCell : 1;
    g.salt = 1;
    if (g.sub == kTileCoarse) {
        // salt: as many counters per bucket as 2^28 counters allow (64 at
        // most, 4 at least): a call whose visibilities crowd into few first
        // planes -- a rank of the row-by-w partition holding the dense uv
        // core -- spreads its hot buckets' serial atomics over 64 counters
        // (such a 4-way rank: count + scatter 317 -> 208 ms at salt 32); the
        // full C4 band (63 first planes) keeps 4 (salt 1 / 2 / 4 / 8 / 16
        // measured within 1 % there, profiles/r03_c4_knobs.txt)
        const int sv = env_int("SDP_HIP_SALT", 0);
        if (sv >= 1 && sv <= 64 && (sv & (sv - 1)) == 0) {
            g.salt = sv;
        } else {
            g.salt = 64;
            while (g.salt > 4 && (double)g.ntiles * g.nps * g.salt > 268435456.0) g.salt >>= 1;
        }
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
    const size_t grid_plane = (size_t)g.ngx * g.ngy * cbytes(P);
    const size_t spec_plane = 2 * (size_t)g.ny * g.ngx * cbytes(P);
    P.fft_planes = (int)std::max<size_t>(
        1, std::min<size_t>(kFftBatchMax, kFftBatchBytes / spec_plane));
    if (const char *e = std::getenv("SDP_HIP_FFT_PLANES"))  // tests: force small batches
        if (std::atoi(e) > 0) P.fft_planes = std::atoi(e);
    P.fft_planes = std::min(P.fft_planes, g.nplanes);
    const int64_t nvis = in.nrow * (int64_t)in.nchan;
    // large-grid invert: RecC records + cell bytes, then the 4-padded copy
    // (k_subsort_pad; budgeted at 1.35x -- C4's top channels pad to <= 1.5x
    // one channel at a time, less over a batch of channels)
    P.subpad = grid_mode && g.sub == kTileCoarse;
    // two-level plans: the bin-ordered records + their cell keys, then the
    // final (for the invert 4-padded, ~1.05x) copy
    const double tiled_rec = P.f64 ? sizeof(VisRec64) : grid_mode ? sizeof(RecC) : sizeof(VisRec);
    const double rec_bytes = g.tiled     ? 2.1 * tiled_rec + sizeof(uint16_t) - sizeof(unsigned)
                             : P.f64     ? sizeof(VisRec64)
                             : P.subpad  ? sizeof(RecC) + 1 + 1.35 * sizeof(RecC)
                                         : sizeof(VisRec);
    // buffers of the other kind of plan are freed, not left cached: the plane
    // budget below counts the held record buffers as reusable
    if (!P.subpad) {
        Workspace::get().drop(ws_name("recs_pad"));
        Workspace::get().drop(ws_name("rec_cls"));
    }
    for (const char *n : {"recs_a", "rec_lkey", "t_m1", "t_m2", "t_tot", "t_cbase", "t_stot"})
        if (!g.tiled) Workspace::get().drop(ws_name(n));
    for (const char *n : {"key_rank", "hist", "offs", "gsum", "gofs"})
        if (g.tiled) Workspace::get().drop(ws_name(n));
    if (grid_mode) Workspace::get().drop(ws_name("degrid_acc"));
    {
        // a record buffer held much larger than this plan needs (a predict's
        // 32-B records before a large-grid invert's 16-B ones) is freed too:
        // kept, its surplus would be counted as free but stay allocated
        const size_t want = (size_t)std::max<int64_t>(nvis, 1) *
                            (P.f64 ? sizeof(VisRec64) : P.subpad ? sizeof(RecC) : sizeof(VisRec));
        if (Workspace::get().held(ws_name("recs")) > want + want / 4 + ((size_t)256 << 20))
            Workspace::get().drop(ws_name("recs"));
    }
    const size_t hist_bytes =
        g.tiled ? ((size_t)nvis / kTChunk + 4 * (size_t)g.nbins + 512) * kBinCells * sizeof(unsigned)
                : (size_t)g.ntiles * g.nps * g.salt * 2 * sizeof(unsigned);
    const size_t need_other =
        (size_t)((double)nvis * (rec_bytes + sizeof(unsigned) + (grid_mode ? 0 : sizeof(float2)))) +
        hist_bytes + (size_t)P.fft_planes * spec_plane * (grid_mode ? 1 : 2);
    const int cp = (int)std::max<size_t>(1, grid_budget_bytes(need_other) / grid_plane);
    P.chunk_planes = std::min(cp, g.nplanes);
    P.fft_planes = std::min(P.fft_planes, P.chunk_planes);
    const size_t cf = cbytes(P) / sizeof(float2);  // float2 slots per element
    P.grid = scratch<float2>("grid", (size_t)P.chunk_planes * g.ngx * g.ngy * cf);
    P.spec = scratch<float2>("spec", (size_t)P.fft_planes * g.ny * g.ngx * cf);
    if (grid_mode) P.spec_in = band_input(P, st);
    else P.spec_adj = adj_input(P, st);

    // records per item: large enough to amortise the tile flush over dense
    // tiles, small enough that the uv core's heavy groups split into items
    // the CUs share evenly (C2, round 4: chunk 2048 / 3072 against the
    // former nvis / 16384 = 7488: gridding 3.97 / 3.94 vs 4.23 ms, the
    // degridder 5.50 / 5.53 vs 5.77, the fp64 pair 1-2 % faster)
    P.chunk = (unsigned)std::min<int64_t>(kChunkMax, std::max<int64_t>(kChunkMin, nvis / 40960));
    if (const char *e = std::getenv("SDP_HIP_CHUNK"))
        if (std::atoi(e) >= 64) P.chunk = (unsigned)std::atoi(e);
    // large grids: the 16x16-cell items are re-ordered by cell (k_subsort)
    P.subsort = g.sub == kTileCoarse;
    if (P.subsort) P.chunk = std::min<unsigned>(P.chunk, kSubChunk);
    // invert on one-cell buckets: every cell padded to a multiple of 4 records
    // (k_grid_mfma_pad); the padded record count is read back before the
    // scatter (one host sync)
    P.pad4 = grid_mode && g.sub == kTileCell && !P.f64;
    // fp64 invert on the two-level bucketing: Rec64 cells padded to 4 for the
    // MFMA gridder (a single-level plan -- windows past the LDS histogram, or
    // SDP_HIP_BUCKET2=0 -- keeps unpadded VisRec64 records and the VALU
    // gridder k_grid_f64); the fp64 predict always degrids on MFMA
    P.pad64 = grid_mode && g.tiled && P.f64;
    P.mfma64 = !grid_mode && g.sub == kTileCell && P.f64;
    // (k_degrid_f64_mfma's per-item block table holds kMaxBlk64 blocks)
    if (P.mfma64) P.chunk = std::min<unsigned>(P.chunk, (kMaxBlk64 - kGroupCell) * kBlk64);
    P.chunk &= ~63u;  // items start on 64-record batches (and 4-record K-steps)
    P.pt.nvis = nvis;
    if (g.tiled) return P;  // (records: bucket_tiled, once their padded count is known)
    P.recs = P.f64      ? scratch<VisRec>("recs", 2 * std::max<int64_t>(nvis, 1))  // VisRec64
             : P.subpad ? scratch<VisRec>("recs", (std::max<int64_t>(nvis, 1) + 1) / 2 + 1)  // RecC
                        : scratch<VisRec>("recs", std::max<int64_t>(nvis, 1));
    if (P.subpad) P.cls = scratch<uint8_t>("rec_cls", std::max<int64_t>(nvis, 1));
    return P;
}

// The weights and flags of a call as the typed bucketing passes read them
// (t_load<WT, FB>): no weights become a device 1.0f with zero strides, int32
// flags a contiguous int64 copy (a zero-stride broadcast: one element);
// dispatch() calls a kernel-launch template with the call's (WT, FB).
struct TypedIn {
    VisExtra x;
    const void *wgt;
    int64_t wrs, wcs;
    int wt, fb;
    template <class F>
    void dispatch(F launch) const {
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I4 = std::integral_constant<int, 4>;
        using I8 = std::integral_constant<int, 8>;
        if (fb == 0) {
            if (wt == 4) launch(I4{}, I0{});
            else launch(I8{}, I0{});
        } else if (fb == 1) {
            if (wt == 4) launch(I4{}, I1{});
            else launch(I8{}, I1{});
        } else {
            if (wt == 4) launch(I4{}, I8{});
            else launch(I8{}, I8{});
        }
    }
};

static TypedIn typed_inputs(const Geo &g, const Inputs &in, hipStream_t st) {
    TypedIn t;
    t.x = in.x;
    t.wgt = in.wgt;
    t.wrs = in.wrs;
    t.wcs = in.wcs;
    if (!t.wgt) {
        void *one = nullptr;
        SDP_HIP_CHECK(hipGetSymbolAddress(&one, HIP_SYMBOL(g_unit_weight)));
        t.wgt = one;
        t.wrs = t.wcs = 0;
        t.x.wgt_f64 = 0;
    }
    t.wt = t.x.wgt_f64 ? 8 : 4;
    VisExtra &x = t.x;
    if (x.fbytes == 4) {
        const bool bc = x.frs == 0 && x.fcs == 0 && x.fps == 0;
        const int np = bc ? 1 : x.npv;
        const int64_t nr = bc ? 1 : g.nrow, nc = bc ? 1 : g.nchan;
        int64_t *f64 = scratch<int64_t>("flags64", (size_t)std::max<int64_t>(nr * nc * np, 1));
        const unsigned gw = (unsigned)std::max<int64_t>(
            1, std::min<int64_t>(grid1d(nr * nc * np, 256), 65536));
        if (g.nrow > 0)
            k_widen_flags<int32_t><<<gw, 256, 0, st>>>(static_cast<const int32_t *>(x.flags), x.frs,
                                                      x.fcs, x.fps, nr, (int)nc, np, f64);
        x.flags = f64;
        x.fbytes = 8;
        x.frs = bc ? 0 : nc * np;
        x.fcs = bc ? 0 : np;
        x.fps = bc ? 0 : 1;
    }
    t.fb = x.fbytes;
    return t;
}

// Bucketing (no host sync except the 4-padded record total): histogram with
// ranks, scan, scatter of the records, work items, metadata.
static void bucket_part(Plan &P, const Inputs &in, bool grid_mode, hipStream_t st,
                        bool values_only = false,
                        const std::function<void()> &after_clear = nullptr,
                        PolsSpec *pols = nullptr) {
    const Geo &g = P.g;
    Part &pt = P.pt;
    const size_t nkeys = (size_t)g.ntiles * g.nps * g.salt;
    const int kpg = g.grp * g.salt;  // keys per work-item group
    const int64_t ngroups = (int64_t)nkeys / kpg;
    const int gpp = g.ntiles / g.grp;  // groups per first-plane value
    pt.hist = scratch<unsigned>("hist", nkeys + 1);
    pt.offs = scratch<unsigned>("offs", nkeys + 1);
    pt.nch = scratch<unsigned>("nch", ngroups + 1);
    pt.ioffs = scratch<unsigned>("ioffs", ngroups + 1);
    pt.nbad = scratch<unsigned long long>("nbad", 1);
    pt.meta = scratch<unsigned>("meta", g.nps + 5);
    // items: <= one per non-empty group plus one per chunk of (padded) records
    const bool cells = g.sub == kTileCell;
    // one-cell plans: units of ucells keys (gridding: blocks of bx x 8 cells;
    // degridding: groups of 16)
    const int ucells = kGroupCell;
    const int64_t nunits = cells ? (int64_t)nkeys / ucells : ngroups;
    const int upp = cells ? g.ntiles / ucells : gpp;
    const int64_t icap =
        std::min<int64_t>(nunits, pt.nvis) + (P.pad4 ? 4 : 1) * pt.nvis / P.chunk + 1;
    if (cells) pt.fitems = scratch<FineItem>("fitems", icap);
    else pt.items = scratch<Item>("items", icap);
    unsigned *kr = scratch<unsigned>("key_rank", std::max<int64_t>(pt.nvis, 1));
    if (!values_only) {
        SDP_HIP_CHECK(hipMemsetAsync(pt.hist, 0, (nkeys + 1) * sizeof(unsigned), st));
        SDP_HIP_CHECK(hipMemsetAsync(pt.nbad, 0, sizeof(unsigned long long), st));
        SDP_HIP_CHECK(hipMemsetAsync(pt.nch + ngroups, 0, sizeof(unsigned), st));
    }

    const unsigned nb = grid1d(std::max<int64_t>(pt.nvis, 1), 256);
    double *slots = in.x.sumwt ? scratch<double>("sumwt_slots", kSumSlots) : nullptr;
    // the typed passes' weights, flags and frequency scales (t_load)
    const TypedIn ti = typed_inputs(g, in, st);
    double *fsc = scratch<double>("t_fscale", g.nchan);
    k_fscale<<<grid1d(g.nchan, 256), 256, 0, st>>>(in.freq, g.nchan, fsc);
    // weight sums: in the count pass, or in the value pass of a reused plan
    auto launch_bucket = [&](auto scatter_tag, unsigned *counter) {
        constexpr bool S = decltype(scatter_tag)::value;
        VisRec *out = S ? P.recs : nullptr;
        double *sl = S == values_only ? slots : nullptr;
        auto go = [&](auto vt_tag, auto grid_tag, auto compact_tag, const void *visp) {
            using VT = typename decltype(vt_tag)::type;
            constexpr bool G = decltype(grid_tag)::value, C = decltype(compact_tag)::value;
            const VT *vp = static_cast<const VT *>(visp);
            ti.dispatch([&](auto wt_tag, auto fb_tag) {
                k_bucket<VT, S, G, C, decltype(wt_tag)::value, decltype(fb_tag)::value>
                    <<<nb, 256, 0, st>>>(g, pt.nvis, in.uvw, in.uvw_rs, fsc, vp, in.vrs, in.vcs,
                                         ti.wgt, ti.wrs, ti.wcs, ti.x, sl, counter, kr, out,
                                         pt.nbad, S && P.subpad ? P.cls : nullptr,
                                         S ? nullptr : P.zout);
            });
        };
        auto by_mode = [&](auto vt_tag) {
            using VT = typename decltype(vt_tag)::type;
            if (S && P.f64) {  // 64-byte VisRec64 records
                VisRec64 *o64 = reinterpret_cast<VisRec64 *>(P.recs);
                if (grid_mode)
                    k_bucket_f64<VT, true><<<nb, 256, 0, st>>>(
                        g, pt.nvis, in.uvw, in.uvw_rs, in.freq, static_cast<const VT *>(in.vis),
                        in.vrs, in.vcs, in.wgt, in.wrs, in.wcs, in.x, sl, counter, kr, o64);
                else
                    k_bucket_f64<VT, false><<<nb, 256, 0, st>>>(
                        g, pt.nvis, in.uvw, in.uvw_rs, in.freq, nullptr, 0, 0, in.wgt, in.wrs,
                        in.wcs, in.x, sl, counter, kr, o64);
                return;
            }
            // the value pass of an fp32 invert writes 16-byte RecC records
            // (one-cell and large-grid plans are both 4-padded), a predict's
            // 32-byte VisRec; the rank pass reads no visibilities (one
            // instantiation)
            if (S && grid_mode) go(vt_tag, std::true_type{}, std::true_type{}, in.vis);
            else go(TypeTag<float2>{}, std::false_type{}, std::false_type{}, nullptr);
        };
        if (S && grid_mode && in.vis_dtype == SDP_HIP_C128) by_mode(TypeTag<double2>{});
        else by_mode(TypeTag<float2>{});
    };
    if (values_only) {  // SDP_HIP_REUSE_BUCKETS: keys, ranks, offsets, items kept
        if (pt.nvis > 0) launch_bucket(std::true_type{}, pt.offs);
        SDP_HIP_CHECK(hipGetLastError());
        return;
    }
    if (after_clear) after_clear();
    if (pt.nvis > 0) launch_bucket(std::false_type{}, pt.hist);
    if (cells) {
        // offsets, pads and items from the units (k_group_sums, one 64-bit
        // scan over the units, k_group_fill)
        auto *gsum = scratch<unsigned long long>("gsum", nunits + 1);
        auto *gofs = scratch<unsigned long long>("gofs", nunits + 1);
        pt.ioffs = scratch<unsigned>("ioffs", nunits + 1);
        unsigned *pslots = nullptr;
        if (P.pad4) {
            pslots = scratch<unsigned>("pad_slots", kSumSlots);
            pt.npad = scratch<unsigned>("npad", 1);
            SDP_HIP_CHECK(hipMemsetAsync(pslots, 0, kSumSlots * sizeof(unsigned), st));
        }
        SDP_HIP_CHECK(hipMemsetAsync(gsum + nunits, 0, sizeof(unsigned long long), st));
        const unsigned gb = grid1d(nunits, 256);
        if (P.pad4)
            k_group_sums<true><<<gb, 256, 0, st>>>(nunits, ucells, pt.hist, P.chunk, gsum, pslots);
        else
            k_group_sums<false><<<gb, 256, 0, st>>>(nunits, ucells, pt.hist, P.chunk, gsum,
                                                    nullptr);
        size_t gtmp = 0;
        SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, gtmp, gsum, gofs,
                                                       (int)(nunits + 1), st));
        void *tmp = scratch<char>("scan_tmp", gtmp + 16);
        SDP_HIP_CHECK(
            hipcub::DeviceScan::ExclusiveSum(tmp, gtmp, gsum, gofs, (int)(nunits + 1), st));
        if (P.pad4) {
            // the padded record total sizes the record array (one host sync)
            unsigned long long *htot = pinned_host<unsigned long long>(48, 1);
            SDP_HIP_CHECK(hipMemcpyAsync(htot, gofs + nunits, sizeof(unsigned long long),
                                         hipMemcpyDeviceToHost, st));
            SDP_HIP_CHECK(hipStreamSynchronize(st));
            const int64_t nrc = ((int64_t)(*htot >> 32) + 1) / 2 + 1;  // RecC pairs
            P.recs = scratch<VisRec>("recs", nrc);
            if (pols) {  // the other image pols' records: same positions, same pads
                static const char *names[4] = {"recs", "recs_pol1", "recs_pol2", "recs_pol3"};
                pols->recs[0] = reinterpret_cast<RecC *>(P.recs);
                for (int q = 1; q < pols->npo; ++q)
                    pols->recs[q] = reinterpret_cast<RecC *>(scratch<VisRec>(names[q], nrc));
            }
            k_sum_pads<<<1, 256, 0, st>>>(pslots, pt.npad);
        }
        const unsigned fb = grid1d(nunits + 1, 256);
        PadMore more;
        if (pols)
            for (int q = 1; q < pols->npo; ++q) more.r[q - 1] = pols->recs[q];
        if (P.pad4)
            k_group_fill<true><<<fb, 256, 0, st>>>(nunits, upp, ucells, pt.hist, gofs, P.chunk,
                                                   pt.offs, pt.ioffs,
                                                   reinterpret_cast<RecC *>(P.recs), pt.fitems,
                                                   more);
        else
            k_group_fill<false><<<fb, 256, 0, st>>>(nunits, upp, ucells, pt.hist, gofs, P.chunk,
                                                    pt.offs, pt.ioffs, nullptr, pt.fitems);
        if (pt.nvis > 0 && pols) {
            // every image pol's value pass at once (sdp_hip_ms2dirty_vis_pols)
            SDP_REQUIRE(P.pad4 && grid_mode && !P.f64 && !P.subpad, "pols call: unsupported plan");
            auto go = [&](auto vt_tag) {
                using VT = typename decltype(vt_tag)::type;
                ti.dispatch([&](auto wt_tag, auto fb_tag) {
                    constexpr int WT = decltype(wt_tag)::value, FB = decltype(fb_tag)::value;
                    const VT *vp = static_cast<const VT *>(in.vis);
#define SDP_POLS(N)                                                                         \
    k_bucket_pols<VT, WT, FB, N><<<nb, 256, 0, st>>>(g, pt.nvis, in.uvw, in.uvw_rs, fsc, vp, \
                                                     in.vrs, in.vcs, ti.x, *pols, pt.offs, kr)
                    switch (pols->npo) {
                        case 1: SDP_POLS(1); break;
                        case 2: SDP_POLS(2); break;
                        case 3: SDP_POLS(3); break;
                        default: SDP_POLS(4); break;
                    }
#undef SDP_POLS
                });
            };
            if (in.vis_dtype == SDP_HIP_C128) go(TypeTag<double2>{});
            else go(TypeTag<float2>{});
        } else if (pt.nvis > 0) {
            launch_bucket(std::true_type{}, pt.offs);
        }
        k_part_meta<<<grid1d(g.nps + 1, 64), 64, 0, st>>>(pt.nbad, pt.offs + nkeys,
                                                          P.pad4 ? pt.npad : nullptr, pt.ioffs,
                                                          upp, g.nps, pt.meta);
        SDP_HIP_CHECK(hipGetLastError());
        return;
    }
    size_t tmp_bytes = 0;
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, pt.hist, pt.offs,
                                                   (int)(nkeys + 1), st));
    void *tmp = scratch<char>("scan_tmp", tmp_bytes + 16);
    size_t tb = tmp_bytes + 16;
    SDP_HIP_CHECK(
        hipcub::DeviceScan::ExclusiveSum(tmp, tb, pt.hist, pt.offs, (int)(nkeys + 1), st));
    if (pt.nvis > 0) launch_bucket(std::true_type{}, pt.offs);

    // work items (p0-major, so a first-plane range is a contiguous item range)
    k_items_count<<<grid1d(ngroups, 256), 256, 0, st>>>(ngroups, kpg, pt.offs, P.chunk, pt.nch);
    tb = tmp_bytes + 16;
    SDP_HIP_CHECK(
        hipcub::DeviceScan::ExclusiveSum(tmp, tb, pt.nch, pt.ioffs, (int)(ngroups + 1), st));
    k_items_fill<<<grid1d(ngroups, 256), 256, 0, st>>>(ngroups, kpg, gpp, pt.offs, pt.ioffs,
                                                       P.chunk, pt.items);
    k_part_meta<<<grid1d(g.nps + 1, 64), 64, 0, st>>>(pt.nbad, pt.offs + nkeys, nullptr, pt.ioffs,
                                                      gpp, g.nps, pt.meta);
    SDP_HIP_CHECK(hipGetLastError());
}

// Host copy of the metadata (one sync): counts, the first-plane item
// offsets (plane-chunked launches need them) and the out-of-grid check.
static void read_part_meta(Plan &P, hipStream_t st) {
    const int nps = P.g.nps;
    const size_t per = (size_t)nps + 5;
    unsigned *m = pinned_host<unsigned>(64, per);
    SDP_HIP_CHECK(hipMemcpyAsync(m, P.pt.meta, per * sizeof(unsigned), hipMemcpyDeviceToHost, st));
    SDP_HIP_CHECK(hipStreamSynchronize(st));
    const unsigned long long nbad = (unsigned long long)m[0] | ((unsigned long long)m[1] << 32);
    SDP_REQUIRE(nbad == 0,
                "visibilities outside the padded grid (or, in a batched invert, outside the "
                "sequence's bounds)");
    Part &pt = P.pt;
    pt.nrec = m[2];
    pt.nitems = m[3];
    pt.p0_items.assign(m + 4, m + 4 + nps + 1);
}

// Item range whose W-plane windows intersect planes [p_lo, p_hi).
static std::pair<unsigned, unsigned> chunk_items(const Plan &P, int p_lo, int p_hi) {
    const int a = std::max(0, p_lo - (P.g.do_w ? P.g.W : 1) + 1);
    const int b = std::min(P.g.nps - 1, p_hi - 1);
    if (a > b) return {0u, 0u};
    return {P.pt.p0_items[a], P.pt.p0_items[b + 1]};
}

template <int W, bool WS>
static void launch_grid_mfma_pad(const Plan &P, int p_lo, int p_hi, hipStream_t st) {
    // one-cell plans: one FineItem per work unit; padded sub-sorted coarse
    // plans: a coarse item's 16 FineItems per unit
    const auto r = chunk_items(P, p_lo, p_hi);
    const unsigned n = r.second - r.first;
    if (n == 0) return;
    if (P.subpad) {
        // units of 4 of a coarse item's 16 groups (2 x pairs x 2 y halves,
        // 4 x 16 cells, an 11 x 23-cell region).  C4 N = 1 gridding: 1 group
        // per unit 1001 ms, 2: 786, 4: 706, 8: 813, 16: 1078 ms -- larger
        // units flush fewer atomics (the small groups of C4's sparse cells,
        // ~120 records each, were bound by them) but hold more LDS per wave
        const unsigned nu = n * 4u;
        k_grid_mfma_pad<W, WS, 4><<<nu, 64, grid_mfma_pad_lds<4>(), st>>>(
            P.g, P.recs_pad, P.pt.fitems + 16 * (size_t)r.first, nu, (float *)P.grid, p_lo, p_hi,
            P.core);
    } else
        k_grid_mfma_pad<W, WS, 1><<<n, 64, grid_mfma_pad_lds<1>(), st>>>(
            P.g, reinterpret_cast<const RecC *>(P.recs), P.pt.fitems + r.first, n, (float *)P.grid,
            p_lo, p_hi, P.core);
}

template <int W, bool WS>
static void launch_grid_f64(const Plan &P, int p_lo, int p_hi, hipStream_t st) {
    const auto r = chunk_items(P, p_lo, p_hi);
    const unsigned n = r.second - r.first;
    if (n == 0) return;
    static const bool attr = [] {  // dynamic LDS above 64 KiB (W = 16: 106 KiB)
        SDP_HIP_CHECK(hipFuncSetAttribute((const void *)k_grid_f64<W, WS>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)grid_f64_lds<W, WS>()));
        return true;
    }();
    (void)attr;
    k_grid_f64<W, WS><<<n, 64, grid_f64_lds<W, WS>(), st>>>(
        P.g, reinterpret_cast<const VisRec64 *>(P.recs), P.pt.fitems + r.first, n,
        reinterpret_cast<double *>(P.grid), p_lo, p_hi);
}

#define SDP_W64_DISPATCH(W, CALL) \
    switch (W) {                  \
        case 9: CALL(9); break;   \
        case 10: CALL(10); break; \
        case 11: CALL(11); break; \
        case 12: CALL(12); break; \
        case 13: CALL(13); break; \
        case 14: CALL(14); break; \
        case 15: CALL(15); break; \
        default: CALL(16); break; \
    }

// The fp64 kernels' tap polynomials (es_taps_poly) for support W and shape
// beta: per tap j, the interpolant of exp(beta (sqrt(1 - x^2) - 1)), x =
// (s - W/2 + j) 2 / W, at the kPoly64 + 1 Chebyshev nodes of s in [0, 1],
// as monomial coefficients in t = 2 s - 1 ([d][j], long double sums).  One
// device table per (device, W), built on first use.
static const double *es_poly64_table(int W, double beta, hipStream_t st) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, double *> tabs;
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair(dev, W);
    auto it = tabs.find(key);
    if (it != tabs.end()) return it->second;
    constexpr int N = kPoly64 + 1;
    std::vector<double> tab((size_t)N * kPolyStride, 0.0);
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int j = 0; j < W; ++j) {
        // values at the nodes t_k = cos(pi (k + 1/2) / N)
        long double fv[N], cheb[N];
        for (int k = 0; k < N; ++k) {
            const long double t = std::cos(pi * (k + 0.5L) / N), s = 0.5L * (t + 1.0L);
            const long double x = (s - 0.5L * W + j) * 2.0L / W, y = 1.0L - x * x;
            fv[k] = y > 0 ? std::exp((long double)beta * (std::sqrt(y) - 1.0L)) : 0.0L;
        }
        for (int d = 0; d < N; ++d) {
            long double a = 0;
            for (int k = 0; k < N; ++k) a += fv[k] * std::cos(pi * d * (k + 0.5L) / N);
            cheb[d] = a * (d == 0 ? 1.0L : 2.0L) / N;
        }
        // Chebyshev -> monomial: T_0 = 1, T_1 = t, T_{n+1} = 2 t T_n - T_{n-1}
        long double mono[N] = {}, tm1[N] = {}, t0[N] = {}, t1[N] = {};
        t0[0] = 1;
        t1[1] = 1;
        for (int d = 0; d < N; ++d) {
            const long double *T = d == 0 ? t0 : t1;
            for (int e = 0; e < N; ++e) mono[e] += cheb[d] * T[e];
            if (d >= 1) {
                long double nx[N] = {};
                for (int e = 0; e + 1 < N; ++e) nx[e + 1] += 2 * t1[e];
                for (int e = 0; e < N; ++e) nx[e] -= t0[e];
                for (int e = 0; e < N; ++e) {
                    t0[e] = t1[e];
                    t1[e] = nx[e];
                }
            }
        }
        (void)tm1;
        for (int d = 0; d < N; ++d) tab[(size_t)d * kPolyStride + j] = (double)mono[d];
    }
    double *dptr = nullptr;
    SDP_HIP_CHECK(hipMalloc(&dptr, tab.size() * sizeof(double)));
    SDP_HIP_CHECK(hipMemcpyAsync(dptr, tab.data(), tab.size() * sizeof(double),
                                 hipMemcpyHostToDevice, st));
    SDP_HIP_CHECK(hipStreamSynchronize(st));
    tabs[key] = dptr;
    return dptr;
}

template <int W, bool WS>
static void launch_grid_f64_mfma(const Plan &P, int p_lo, int p_hi, hipStream_t st) {
    const auto r = chunk_items(P, p_lo, p_hi);
    const unsigned n = r.second - r.first;
    if (n == 0) return;
    static const bool attr = [] {  // dynamic LDS above 64 KiB (W >= 14)
        SDP_HIP_CHECK(hipFuncSetAttribute((const void *)k_grid_f64_mfma<W, WS>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)grid_f64m_lds<W, WS>()));
        return true;
    }();
    (void)attr;
    k_grid_f64_mfma<W, WS><<<n, 64 * f64m_waves<W, WS>(), grid_f64m_lds<W, WS>(), st>>>(
        P.g, reinterpret_cast<const Rec64 *>(P.recs), P.pt.fitems + r.first, n,
        reinterpret_cast<double *>(P.grid), p_lo, p_hi, es_poly64_table(W, P.g.beta, st));
}

template <int W, bool WS, class VT>
static void launch_degrid_f64_mfma(const Plan &P, int p_lo, int p_hi, VT *vis, int64_t vrs,
                                   int64_t vcs, int accumulate, const OutConv &oc,
                                   hipStream_t st) {
    const auto r = chunk_items(P, p_lo, p_hi);
    const unsigned n = r.second - r.first;
    if (n == 0) return;
    // records: Rec64 from the two-level bucketing, VisRec64 from the
    // single-level one (SDP_HIP_BUCKET2=0, or windows past the LDS histogram)
    auto go = [&](auto rec_tag) {
        using R = typename decltype(rec_tag)::type;
        static const bool attr = [] {  // dynamic LDS above 64 KiB
            SDP_HIP_CHECK(hipFuncSetAttribute((const void *)k_degrid_f64_mfma<W, WS, VT, R>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)degrid_f64m_lds<W, WS>()));
            return true;
        }();
        (void)attr;
        k_degrid_f64_mfma<W, WS, VT, R><<<n, 64 * kDeg64Waves, degrid_f64m_lds<W, WS>(), st>>>(
            P.g, reinterpret_cast<const R *>(P.recs), P.pt.fitems + r.first, n,
            reinterpret_cast<const double2 *>(P.grid), p_lo, p_hi, vis, vrs, vcs, accumulate, oc,
            es_poly64_table(W, P.g.beta, st));
    };
    if (P.g.tiled) go(TypeTag<Rec64>{});
    else go(TypeTag<VisRec64>{});
}

static void grid_f64(const Plan &P, int p_lo, int p_hi, hipStream_t st) {
#define SDP_G64(WW)                                                                    \
    (P.pad64 ? (P.g.do_w ? launch_grid_f64_mfma<WW, true>(P, p_lo, p_hi, st)          \
                         : launch_grid_f64_mfma<WW, false>(P, p_lo, p_hi, st))        \
             : (P.g.do_w ? launch_grid_f64<WW, true>(P, p_lo, p_hi, st)               \
                         : launch_grid_f64<WW, false>(P, p_lo, p_hi, st)))
    SDP_W64_DISPATCH(P.g.W, SDP_G64);
#undef SDP_G64
}

template <class VT>
static void degrid_f64(const Plan &P, int p_lo, int p_hi, VT *vis, int64_t vrs, int64_t vcs,
                       int accumulate, const OutConv &oc, hipStream_t st) {
    SDP_REQUIRE(P.mfma64, "the fp64 predict needs one-cell buckets");
#define SDP_D64(WW)                                                                             \
    (P.g.do_w ? launch_degrid_f64_mfma<WW, true, VT>(P, p_lo, p_hi, vis, vrs, vcs, accumulate, oc, \
                                                     st)                                        \
              : launch_degrid_f64_mfma<WW, false, VT>(P, p_lo, p_hi, vis, vrs, vcs, accumulate, \
                                                      oc, st))
    SDP_W64_DISPATCH(P.g.W, SDP_D64);
#undef SDP_D64
}

template <int W>
static void launch_grid(const Plan &P, int p_lo, int p_hi, hipStream_t st) {
    // (fp32 inverts are always 4-padded: one-cell plans by the bucketing,
    // large grids by the sub-sort)
    if (P.g.do_w) return launch_grid_mfma_pad<W, true>(P, p_lo, p_hi, st);
    return launch_grid_mfma_pad<W, false>(P, p_lo, p_hi, st);
}

// the degridder's store sink (kDegridSinkBlocks x 64 float2 per device,
// allocated once, never read)
static float2 *degrid_sink() {
    static float2 *sinks[64] = {};
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    SDP_REQUIRE(dev >= 0 && dev < 64, "device index out of range");
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (!sinks[dev])
        SDP_HIP_CHECK(hipMalloc(&sinks[dev], (size_t)kDegridSinkBlocks * 64 * sizeof(float2)));
    return sinks[dev];
}

template <int W, bool WS>
static void launch_degrid_mfma(const Plan &P, int p_lo, int p_hi, float2 *acc, hipStream_t st) {
    const size_t lds = degrid_lds_bytes<W, WS>();
    // one-cell plans: one FineItem per item; sub-sorted coarse plans: 16
    const auto r = chunk_items(P, p_lo, p_hi);
    const unsigned per = P.subsort ? 16u : 1u;
    const unsigned n = per * (r.second - r.first);
    if (n == 0) return;
    float2 *const sink = degrid_sink();
    if (P.vdirect)
        k_degrid_mfma<W, WS, true><<<n, 64, lds, st>>>(
            P.g, P.recs, n, P.pt.fitems + per * (size_t)r.first, P.grid, p_lo, p_hi, P.vdirect, sink);
    else
        k_degrid_mfma<W, WS, false><<<n, 64, lds, st>>>(
            P.g, P.recs, n, P.pt.fitems + per * (size_t)r.first, P.grid, p_lo, p_hi, acc, sink);
}

template <int W>
static void launch_degrid(const Plan &P, int p_lo, int p_hi, float2 *acc, hipStream_t st) {
    if (P.g.do_w) return launch_degrid_mfma<W, true>(P, p_lo, p_hi, acc, st);
    return launch_degrid_mfma<W, false>(P, p_lo, p_hi, acc, st);
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
    info->nvis_used = P.pt.nrec;
    info->nitems = P.pt.nitems;
    info->plane_chunk = P.chunk_planes;
    info->bucket = P.g.sub;
    info->padded = (P.pad4 || P.subpad || P.pad64) ? 1 : 0;
    info->fp64 = P.f64 ? 1 : 0;
    info->tiled = P.g.tiled;
    info->grid_launches = (P.g.nplanes + P.chunk_planes - 1) / P.chunk_planes;
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
static void exec_fft(hipfftHandle h, bool f64, void *in, void *out, int direction) {
    const hipfftResult r =
        f64 ? hipfftExecZ2Z(h, (hipfftDoubleComplex *)in, (hipfftDoubleComplex *)out, direction)
            : hipfftExecC2C(h, (hipfftComplex *)in, (hipfftComplex *)out, direction);
    if (r != HIPFFT_SUCCESS) throw Error(SDP_HIP_ERR_RUNTIME, "hipfftExec failed");
}

// element e of plane q of the resident planes (c64 or c128)
static void *plane_ptr(const Plan &P, int q, size_t e) {
    return reinterpret_cast<char *>(P.grid) +
           ((size_t)q * P.g.ngx * P.g.ngy + e) * cbytes(P);
}

static void fft_rows_y(const Plan &P, int q0, int np, int direction, hipStream_t st) {
    const Geo &g = P.g;
    const int nrow = P.row_hi - P.row_lo;
    if (nrow <= 0) return;
    hipfftHandle hr = fft_plan_1d(g.ngy, 1, g.ngy, nrow, st, P.f64);
    for (int q = q0; q < q0 + np; ++q) {
        void *p = plane_ptr(P, q, (size_t)P.row_lo * g.ngy);
        exec_fft(hr, P.f64, p, p, direction);
    }
}

// x transforms of the T rows into P.spec, in place or from `in`
static void fft_rows_x(const Plan &P, int np, int direction, hipStream_t st,
                       void *in = nullptr) {
    const Geo &g = P.g;
    hipfftHandle hc = fft_plan_1d(g.ngx, 1, g.ngx, np * g.ny, st, P.f64);
    exec_fft(hc, P.f64, in ? in : (void *)P.spec, P.spec, direction);
}

// Only the row band [row_lo, row_hi) of a plane is ever written or read.
static void zero_band(const Plan &P, int np, hipStream_t st) {
    const Geo &g = P.g;
    if (P.row_hi <= P.row_lo || np <= 0) return;
    const size_t width = (size_t)(P.row_hi - P.row_lo) * g.ngy * cbytes(P);
    for (int q = 0; q < np; ++q)
        SDP_HIP_CHECK(hipMemsetAsync(plane_ptr(P, q, (size_t)P.row_lo * g.ngy), 0, width, st));
    if (P.core.p)
        SDP_HIP_CHECK(hipMemsetAsync(P.core.p, 0,
                                     (size_t)np * P.core.nx * P.core.ny * sizeof(double2), st));
}

// The fp64 companion of the uv core (CoreAcc): a central window of
// SDP_HIP_CORE (default 128) cells square, clipped to the grid rows the
// visibilities reach, one c128 plane per resident plane (C4: 71 x 256 KiB).
// SDP_HIP_CORE=0: no companion (every flush in fp32).
static void setup_core(Plan &P) {
    P.core = CoreAcc{nullptr, 0, 0, 0, 0};
    const int cw = env_int("SDP_HIP_CORE", 128);
    if (P.f64 || cw <= 0) return;
    const Geo &g = P.g;
    const int x0 = std::max(P.row_lo, g.ngx / 2 - cw / 2), x1 = std::min(P.row_hi, g.ngx / 2 + cw / 2);
    const int y0 = std::max(0, g.ngy / 2 - cw / 2), y1 = std::min(g.ngy, g.ngy / 2 + cw / 2);
    if (x1 <= x0 || y1 <= y0) return;
    P.core = CoreAcc{scratch<double>("core64", (size_t)P.chunk_planes * (x1 - x0) * (y1 - y0) * 2),
                     x0, x1 - x0, y0, y1 - y0};
}

// planes q0 .. q0 + np - 1 of the chunk += their fp64 companion, rounded once
__global__ __launch_bounds__(256) void k_core_merge(float2 *__restrict__ grid, int ngx, int ngy,
                                                    CoreAcc c, int q0, int np) {
    const int64_t per = (int64_t)c.nx * c.ny, n = per * np;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(i / per);
        const int64_t e = i - q * per;
        const int x = (int)(e / c.ny), y = (int)(e - (int64_t)x * c.ny);
        const double2 v = reinterpret_cast<const double2 *>(c.p)[(int64_t)(q0 + q) * per + e];
        float2 &o = grid[((int64_t)(q0 + q) * ngx + c.x0 + x) * ngy + c.y0 + y];
        o = make_float2((float)((double)o.x + v.x), (float)((double)o.y + v.y));
    }
}

static void core_merge(const Plan &P, int q0, int np, hipStream_t st) {
    if (!P.core.p || np <= 0) return;
    const int64_t n = (int64_t)P.core.nx * P.core.ny * np;
    k_core_merge<<<(unsigned)std::min<int64_t>((n + 255) / 256, 8192), 256, 0, st>>>(
        P.grid, P.g.ngx, P.g.ngy, P.core, q0, np);
    SDP_HIP_CHECK(hipGetLastError());
}

static dim3 tr_grid(const Geo &g, int xrows, int np) {
    return dim3((unsigned)((xrows + kTr - 1) / kTr), (unsigned)((g.ny + kTr - 1) / kTr),
                (unsigned)np);
}

// the 16-byte c64 transposes: image rows in even pairs (ny % 4 == 0), grid
// rows and columns even (16-byte aligned pairs); tiles aligned to 64 rows
static bool tr16(const Geo &g) {
    return g.ny % 4 == 0 && g.ngy % 2 == 0 && g.ngx % 2 == 0;
}
static dim3 tr_grid16(const Geo &g, int row_lo, int row_hi, int np) {
    const int xa = row_lo & ~(kTr - 1);
    return dim3((unsigned)((row_hi - xa + kTr - 1) / kTr), (unsigned)((g.ny + kTr - 1) / kTr),
                (unsigned)np);
}

// plane-stage kernels at the plan's precision (planes q0 .. q0 + nb - 1)
static void tr_grid_to_t(const Plan &P, int q0, int nb, hipStream_t st) {
    const Geo &g = P.g;
    if (P.row_hi <= P.row_lo) return;
    const dim3 grd = tr_grid(g, P.row_hi - P.row_lo, nb), blk(kTr, kTrRows);
    if (P.f64)
        k_tr_grid_to_t<double2><<<grd, blk, 0, st>>>(
            g, static_cast<const double2 *>(plane_ptr(P, q0, 0)),
            reinterpret_cast<double2 *>(P.spec_in), P.row_lo, P.row_hi);
    else if (tr16(g))
        k_tr_grid_to_t16<<<tr_grid16(g, P.row_lo, P.row_hi, nb), blk, 0, st>>>(
            g, static_cast<const float2 *>(plane_ptr(P, q0, 0)), P.spec_in, P.row_lo, P.row_hi);
    else
        k_tr_grid_to_t<float2><<<grd, blk, 0, st>>>(
            g, static_cast<const float2 *>(plane_ptr(P, q0, 0)), P.spec_in, P.row_lo, P.row_hi);
    SDP_HIP_CHECK(hipGetLastError());
}

static void tr_t_to_grid(const Plan &P, int q0, int nb, hipStream_t st) {
    const Geo &g = P.g;
    if (P.row_hi <= P.row_lo) return;
    const dim3 grd = tr_grid(g, P.row_hi - P.row_lo, nb), blk(kTr, kTrRows);
    if (P.f64)
        k_tr_t_to_grid<double2><<<grd, blk, 0, st>>>(
            g, reinterpret_cast<const double2 *>(P.spec),
            static_cast<double2 *>(plane_ptr(P, q0, 0)), P.row_lo, P.row_hi);
    else if (tr16(g))
        k_tr_t_to_grid16<<<tr_grid16(g, P.row_lo, P.row_hi, nb), blk, 0, st>>>(
            g, P.spec, static_cast<float2 *>(plane_ptr(P, q0, 0)), P.row_lo, P.row_hi);
    else
        k_tr_t_to_grid<float2><<<grd, blk, 0, st>>>(
            g, P.spec, static_cast<float2 *>(plane_ptr(P, q0, 0)), P.row_lo, P.row_hi);
    SDP_HIP_CHECK(hipGetLastError());
}

static void screen_fwd(const Plan &P, int p_begin, int nb, double *dirty, int64_t sx, int64_t sy,
                       int accumulate, const double *tab, hipStream_t st) {
    const Geo &g = P.g;
    const dim3 grd(grid1d(g.nx, 256), g.ny);
    if (P.f64)
        k_screen_fwd_t<double2><<<grd, 256, 0, st>>>(g, reinterpret_cast<const double2 *>(P.spec),
                                                     p_begin, nb, dirty, sx, sy, accumulate, tab);
    else
        k_screen_fwd_t<float2><<<grd, 256, 0, st>>>(g, P.spec, p_begin, nb, dirty, sx, sy,
                                                    accumulate, tab);
    SDP_HIP_CHECK(hipGetLastError());
}

static void screen_adj(const Plan &P, const double *dirty, int64_t sx, int64_t sy, int p_begin,
                       int nb, const double *tab, hipStream_t st) {
    const Geo &g = P.g;
    const dim3 grd(grid1d(g.nx, 256), g.ny);
    if (P.f64)
        k_screen_adj_t<double2><<<grd, 256, 0, st>>>(g, dirty, sx, sy, p_begin, nb,
                                                     reinterpret_cast<double2 *>(P.spec_adj), tab);
    else
        k_screen_adj_t<float2><<<grd, 256, 0, st>>>(g, dirty, sx, sy, p_begin, nb, P.spec_adj, tab);
    SDP_HIP_CHECK(hipGetLastError());
}

// log2 of the x edge when the fused x-FFT + screen kernels serve the plan
// (fp32 planes, ngx a power of two in [2^7, 2^14]), else 0: hipFFT x
// transforms and the separate screens.  SDP_HIP_XFFT_FUSED=0 forces the latter.
static int xfft_log2(const Plan &P) {
    const int on = env_int("SDP_HIP_XFFT_FUSED", 1);
    const int n = P.g.ngx;
    if (P.f64 || !on || n <= 0 || (n & (n - 1)) || 2 * P.g.nx > n) return 0;
    int l = 0;
    while ((1 << l) < n) ++l;
    return (l >= 7 && l <= 14) ? l : 0;
}

// the fused FFT's twiddle bases (FxShape::tw_off), e^{+2 pi i ...} in fp64
// rounded to fp32 (the forward transforms conjugate them)
template <int LOGN>
static const float2 *fx_twiddles(hipStream_t st) {
    using S = FxShape<LOGN>;
    static const std::vector<float2> host = [] {
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
    }();
    float2 *d = scratch<float2>("fx_tw_" + std::to_string(LOGN), S::TW);
    SDP_HIP_CHECK(hipMemcpyAsync(d, host.data(), S::TW * sizeof(float2), hipMemcpyHostToDevice, st));
    return d;
}

template <int LOGN>
static void launch_xfft_screen_fwd(const Plan &P, int p_begin, int nb, double *dirty, int64_t sx,
                                   int64_t sy, int accumulate, const double *tab, hipStream_t st) {
    using S = FxShape<LOGN>;
    constexpr size_t lds = S::lds_bytes();
    static const bool attr = [] {  // dynamic LDS above 64 KiB
        SDP_HIP_CHECK(hipFuncSetAttribute((const void *)k_xfft_screen_fwd<LOGN>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        return true;
    }();
    (void)attr;
    k_xfft_screen_fwd<LOGN><<<P.g.ny, S::T, lds, st>>>(P.g, P.spec_in, P.row_lo, P.row_hi, p_begin,
                                                       nb, dirty, sx, sy, accumulate, tab,
                                                       fx_twiddles<LOGN>(st));
    SDP_HIP_CHECK(hipGetLastError());
}

// the backward x transforms of planes [p_begin, p_begin + nb) (T rows in
// spec_in) and their screens into the image: fused when xfft_log2 allows,
// else hipFFT into spec + k_screen_fwd_t.  Times the two parts into *tfft and
// *tscr (the fused kernel counts as the screen).
static void xfft_screen_fwd(const Plan &P, int p_begin, int nb, double *dirty, int64_t sx,
                            int64_t sy, int accumulate, const double *tab, hipStream_t st,
                            StageTimer &t2) {
    switch (xfft_log2(P)) {
#define SDP_FX(L) \
    case L: t2.mark(); launch_xfft_screen_fwd<L>(P, p_begin, nb, dirty, sx, sy, accumulate, tab, st); break;
    SDP_FX(7) SDP_FX(8) SDP_FX(9) SDP_FX(10) SDP_FX(11) SDP_FX(12) SDP_FX(13) SDP_FX(14)
#undef SDP_FX
    default:
        fft_rows_x(P, nb, HIPFFT_BACKWARD, st, P.spec_in);
        t2.mark();
        screen_fwd(P, p_begin, nb, dirty, sx, sy, accumulate, tab, st);
    }
    t2.mark();
}

template <int LOGN>
static void launch_screen_adj_xfft(const Plan &P, const double *dirty, int64_t sx, int64_t sy,
                                   int p_begin, int nb, const double *tab, hipStream_t st) {
    using S = FxShape<LOGN>;
    constexpr size_t lds = S::lds_bytes();
    static const bool attr = [] {  // dynamic LDS above 64 KiB
        SDP_HIP_CHECK(hipFuncSetAttribute((const void *)k_screen_adj_xfft<LOGN>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        return true;
    }();
    (void)attr;
    k_screen_adj_xfft<LOGN><<<P.g.ny, S::T, lds, st>>>(P.g, dirty, sx, sy, p_begin, nb, P.spec,
                                                       tab, fx_twiddles<LOGN>(st));
    SDP_HIP_CHECK(hipGetLastError());
}

// the predict's screens of planes [p_begin, p_begin + nb) and their forward
// x transforms into spec: fused when xfft_log2 allows, else k_screen_adj_t
// into the zero-kept input and hipFFT.  Marks t2 between the two parts (the
// fused kernel counts as the screen).
static void screen_adj_xfft(const Plan &P, const double *dirty, int64_t sx, int64_t sy,
                            int p_begin, int nb, const double *tab, hipStream_t st,
                            StageTimer &t2) {
    switch (xfft_log2(P)) {
#define SDP_FX(L) \
    case L: launch_screen_adj_xfft<L>(P, dirty, sx, sy, p_begin, nb, tab, st); t2.mark(); break;
    SDP_FX(7) SDP_FX(8) SDP_FX(9) SDP_FX(10) SDP_FX(11) SDP_FX(12) SDP_FX(13) SDP_FX(14)
#undef SDP_FX
    default:
        screen_adj(P, dirty, sx, sy, p_begin, nb, tab, st);
        t2.mark();
        fft_rows_x(P, nb, HIPFFT_FORWARD, st, P.spec_adj);
    }
}

static int cu_count() {
    static std::mutex mu;
    static std::map<int, int> cus;
    int dev = 0;
    SDP_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    auto it = cus.find(dev);
    if (it != cus.end()) return it->second;
    int n = 0;
    SDP_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    cus[dev] = std::max(n, 1);
    return cus[dev];
}

// Two-level bucketing of a tiled one-cell plan (k_t_count .. k_t_final_s):
// the count pass, bins, value pass, cell counts and bases, then (one host
// sync: the metadata, which sizes the final record array) the cell bases,
// pads, work items and the move of every record to its cell.  The weight
// sums go to `slots` (count pass; value pass when values_only).  values_only
// (SDP_HIP_REUSE_BUCKETS): the kept plan's bins, chunks and cell bases are
// valid, so only the value pass and the final move run.
static void bucket_tiled(Plan &P, const Inputs &in, bool grid_mode, hipStream_t st,
                         bool values_only, const std::function<void()> &after_clear,
                         double *slots) {
    const Geo &g = P.g;
    Part &pt = P.pt;
    const int nb = g.nbins;
    // records: 16-byte RecC (fp32 invert), 32-byte VisRec (fp32 predict,
    // SDP_HIP_BUCKET2=2 only), 48-byte Rec64 (fp64, the MFMA kernels)
    const int kind = P.f64 ? 3 : (grid_mode ? 0 : 1);
    const size_t rsz = kind == 3 ? sizeof(Rec64) : kind == 0 ? sizeof(RecC) : sizeof(VisRec);
    const int64_t nvis = pt.nvis;
    const size_t lds_bins = (size_t)nb * sizeof(unsigned);
    if (!values_only) {
        // 16 workgroups per CU (C2 prep: 4 -> 4.72, 8 -> 4.44, 16 -> 4.27 ms),
        // fewer where the per-workgroup bin offsets (t_m1: t_g1 x nb words,
        // written by the count pass, read by the value pass) would pass half
        // a word per visibility
        pt.t_g1 = env_int("SDP_HIP_TG1", 16) * cu_count();
        while (pt.t_g1 > cu_count() && (int64_t)pt.t_g1 * nb > nvis / 2) pt.t_g1 /= 2;
        pt.t_vpw = std::max<int64_t>(kT1Threads, (nvis + pt.t_g1 - 1) / pt.t_g1);
        pt.t_vpw = (pt.t_vpw + 63) / 64 * 64;
        pt.t_g1 = (int)std::max<int64_t>(1, (nvis + pt.t_vpw - 1) / pt.t_vpw);
        pt.t_maxch = (unsigned)(nvis / kTChunk + nb + 1);
        pt.t_maxseg = (unsigned)(nvis / ((int64_t)kTChunk * kTSeg) + nb + 1);
        pt.t_binc = scratch<unsigned>("t_binc", nb);
        pt.t_binbase = scratch<unsigned>("t_binbase", nb + 1);
        pt.t_segb = scratch<unsigned>("t_segb", nb);
        pt.t_nsegb = scratch<unsigned>("t_nsegb", nb);
        pt.t_segs = scratch<TSeg>("t_segs", pt.t_maxseg);
        pt.t_stot = scratch<unsigned>("t_stot", (size_t)pt.t_maxseg * kBinCells);
        pt.t_nbl = scratch<unsigned>("t_nbl", nb + 1);
        pt.t_meta_ch = scratch<unsigned>("t_meta_ch", 2);
        pt.t_chunks = scratch<TChunk>("t_chunks", pt.t_maxch);
        pt.t_binsum = scratch<unsigned long long>("t_binsum", nb);
        pt.t_bofs = scratch<unsigned long long>("t_bofs", nb + 1);
        pt.t_m1 = scratch<unsigned>("t_m1", (size_t)pt.t_g1 * nb);
        pt.t_m2 = scratch<unsigned>("t_m2", (size_t)pt.t_maxch * kBinCells);
        pt.t_tot = scratch<unsigned>("t_tot", (size_t)nb * kBinCells);
        pt.t_cbase = scratch<unsigned>("t_cbase", (size_t)nb * kBinCells);
        pt.t_lkey = scratch<uint16_t>("rec_lkey", std::max<int64_t>(nvis, 1));
        pt.t_fsc = scratch<double>("t_fscale", g.nchan);
        pt.t_a = scratch<char>("recs_a", (size_t)std::max<int64_t>(nvis, 1) * rsz);
        pt.nbad = scratch<unsigned long long>("nbad", 1);
        pt.meta = scratch<unsigned>("meta", g.nps + 6);
        SDP_HIP_CHECK(hipMemsetAsync(pt.t_binc, 0, nb * sizeof(unsigned), st));
        SDP_HIP_CHECK(hipMemsetAsync(pt.t_binsum, 0, nb * sizeof(unsigned long long), st));
        SDP_HIP_CHECK(hipMemsetAsync(pt.nbad, 0, sizeof(unsigned long long), st));
        if (after_clear) after_clear();
    }
    k_fscale<<<grid1d(g.nchan, 256), 256, 0, st>>>(in.freq, g.nchan, pt.t_fsc);
    const TypedIn ti = typed_inputs(g, in, st);
    const VisExtra &x = ti.x;
    const void *wgt = ti.wgt;
    const int64_t wrs = ti.wrs, wcs = ti.wcs;
    const int cus = cu_count();
    const unsigned gch = std::min<unsigned>(pt.t_maxch, 4u * (unsigned)cus);
    auto scatter = [&](double *sl) {
        auto go = [&](auto vt_tag, auto kind_tag, auto grid_tag) {
            using VT = typename decltype(vt_tag)::type;
            constexpr int K = decltype(kind_tag)::value;
            constexpr bool G = decltype(grid_tag)::value;
            ti.dispatch([&](auto wt_tag, auto fb_tag) {
                k_t_scatter<VT, K, G, decltype(wt_tag)::value, decltype(fb_tag)::value>
                    <<<pt.t_g1, kT1Threads, lds_bins, st>>>(
                        g, nvis, pt.t_vpw, in.uvw, in.uvw_rs, pt.t_fsc,
                        G ? static_cast<const VT *>(in.vis) : nullptr, in.vrs, in.vcs, wgt, wrs,
                        wcs, x, sl, pt.t_binbase, pt.t_m1, pt.t_a, pt.t_lkey);
            });
        };
        auto grid_kind = [&](auto vt_tag) {
            if (kind == 3) go(vt_tag, std::integral_constant<int, 3>{}, std::true_type{});
            else go(vt_tag, std::integral_constant<int, 0>{}, std::true_type{});
        };
        if (grid_mode) {
            if (in.vis_dtype == SDP_HIP_C128) grid_kind(TypeTag<double2>{});
            else grid_kind(TypeTag<float2>{});
        } else {
            // (a predict reads no visibilities: one instantiation for both dtypes)
            if (kind == 3) go(TypeTag<float2>{}, std::integral_constant<int, 3>{}, std::false_type{});
            else go(TypeTag<float2>{}, std::integral_constant<int, 1>{}, std::false_type{});
        }
    };
    auto staged = [&](auto kind_tag, auto nb_tag) {
        constexpr int K = decltype(kind_tag)::value, NB = decltype(nb_tag)::value;
        constexpr size_t lds = t_final_lds<K, NB>();
        static const bool attr = [] {  // dynamic LDS above 64 KiB
            SDP_HIP_CHECK(hipFuncSetAttribute((const void *)k_t_final_s<K, NB>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)t_final_lds<K, NB>()));
            return true;
        }();
        (void)attr;
        const int xmap = (gch % 8 == 0 && env_int("SDP_HIP_TFINAL_XCD", 1) != 0) ? 1 : 0;
        k_t_final_s<K, NB><<<gch, kTThreads, lds, st>>>(pt.t_chunks, pt.t_meta_ch, pt.t_lkey,
                                                         pt.t_m2, pt.t_stot, pt.t_cbase, pt.t_a,
                                                         P.recs, xmap);
    };
    auto final_move = [&] {
        // batches of 4096 (RecC), 2048 (VisRec, Rec64) records staged in LDS
        if (kind == 3) staged(std::integral_constant<int, 3>{}, std::integral_constant<int, 2048>{});
        else if (kind == 0) staged(std::integral_constant<int, 0>{}, std::integral_constant<int, 4096>{});
        else staged(std::integral_constant<int, 1>{}, std::integral_constant<int, 2048>{});
        SDP_HIP_CHECK(hipGetLastError());
    };
    if (values_only) {
        if (nvis > 0) {
            scatter(slots);
            final_move();
        }
        return;
    }
    if (nvis > 0)
        ti.dispatch([&](auto wt_tag, auto fb_tag) {
            k_t_count<decltype(wt_tag)::value, decltype(fb_tag)::value>
                <<<pt.t_g1, kT1Threads, lds_bins, st>>>(g, nvis, pt.t_vpw, in.uvw, in.uvw_rs,
                                                        pt.t_fsc, wgt, wrs, wcs, x, slots, pt.t_binc,
                                                        pt.t_m1, pt.nbad);
        });
    k_t_bins<<<1, kTThreads, 0, st>>>(nb, pt.t_binc, pt.t_binbase, pt.t_segb, pt.t_nsegb,
                                      pt.t_nbl, pt.t_chunks, pt.t_segs, pt.t_meta_ch);
    if (nvis > 0) scatter(nullptr);
    k_t_cellcount<<<gch, kTThreads, 0, st>>>(pt.t_chunks, pt.t_meta_ch, pt.t_lkey, pt.t_m2);
    const unsigned gseg =
        (unsigned)std::min<int64_t>((int64_t)pt.t_maxseg * (kBinCells / 256), 8192);
    k_t_segscan<<<gseg, 256, 0, st>>>(pt.t_segs, pt.t_meta_ch, pt.t_m2, pt.t_stot);
    const unsigned gcol = (unsigned)std::min<int64_t>((int64_t)nb * (kBinCells / 256), 8192);
    if (P.pad4 || P.pad64)
        k_t_cellcol<true><<<gcol, 256, 0, st>>>(pt.t_nbl, pt.t_segb, pt.t_nsegb, pt.t_stot,
                                                pt.t_tot, P.chunk, pt.t_binsum);
    else
        k_t_cellcol<false><<<gcol, 256, 0, st>>>(pt.t_nbl, pt.t_segb, pt.t_nsegb, pt.t_stot,
                                                 pt.t_tot, P.chunk, pt.t_binsum);
    k_t_binscan<<<1, kTThreads, 0, st>>>(nb, g.tlx * g.tly, g.nps, pt.t_binsum, pt.t_binbase,
                                         pt.nbad, pt.t_bofs, pt.meta);
    SDP_HIP_CHECK(hipGetLastError());
    if (slots) k_sum_slots<<<1, 64, 0, st>>>(slots, in.x.sumwt);
    // the metadata (one sync): out-of-grid check, record / item counts, the
    // first item of each first plane, the padded record total
    const int nps = g.nps;
    const size_t per = (size_t)nps + 6;
    unsigned *m = pinned_host<unsigned>(64, per);
    SDP_HIP_CHECK(hipMemcpyAsync(m, pt.meta, per * sizeof(unsigned), hipMemcpyDeviceToHost, st));
    SDP_HIP_CHECK(hipStreamSynchronize(st));
    const unsigned long long nbad = (unsigned long long)m[0] | ((unsigned long long)m[1] << 32);
    SDP_REQUIRE(nbad == 0,
                "visibilities outside the padded grid (or, in a batched invert, outside the "
                "sequence's bounds)");
    pt.nrec = m[2];
    pt.nitems = m[3];
    pt.p0_items.assign(m + 4, m + 4 + nps + 1);
    const size_t ntot = (size_t)m[5 + nps];
    P.recs = reinterpret_cast<VisRec *>(scratch<char>("recs", (ntot + 1) * rsz));
    pt.fitems = scratch<FineItem>("fitems", (size_t)pt.nitems + 1);
    const unsigned gfin = (unsigned)std::min(nb, 4096);
    if (P.pad4)
        k_t_cellfin<true, 0><<<gfin, 256, 0, st>>>(g, pt.t_nbl, pt.t_tot, pt.t_bofs, P.chunk,
                                                   pt.t_cbase, P.recs, pt.fitems);
    else if (P.pad64)
        k_t_cellfin<true, 3><<<gfin, 256, 0, st>>>(g, pt.t_nbl, pt.t_tot, pt.t_bofs, P.chunk,
                                                   pt.t_cbase, P.recs, pt.fitems);
    else
        k_t_cellfin<false, 1><<<gfin, 256, 0, st>>>(g, pt.t_nbl, pt.t_tot, pt.t_bofs, P.chunk,
                                                    pt.t_cbase, nullptr, pt.fitems);
    if (nvis > 0) final_move();
    SDP_HIP_CHECK(hipGetLastError());
}

// Bucketing with the fused weight sum (slots zeroed before the count pass,
// folded into *sumwt after it), then the metadata read back by the host.
// `after_clear` runs once the histogram clearing is queued (work put on
// another stream there does not compete with that memset).
static void bucket_all(Plan &P, const Inputs &in, bool grid_mode, hipStream_t st,
                       const std::function<void()> &after_clear = nullptr) {
    double *slots = in.x.sumwt ? scratch<double>("sumwt_slots", kSumSlots) : nullptr;
    if (slots) SDP_HIP_CHECK(hipMemsetAsync(slots, 0, kSumSlots * sizeof(double), st));
    if (P.g.tiled) {  // (reads its metadata itself)
        bucket_tiled(P, in, grid_mode, st, false, after_clear, slots);
        return;
    }
    bucket_part(P, in, grid_mode, st, false, after_clear);
    if (slots) k_sum_slots<<<1, 64, 0, st>>>(slots, in.x.sumwt);
    read_part_meta(P, st);
}

// Sub-sort of the coarse items by cell (large grids)
static void subsort_items(Plan &P, hipStream_t st) {
    Part &pt = P.pt;
    if (pt.nitems == 0) return;
    pt.fitems = scratch<FineItem>("fitems", (size_t)pt.nitems * 16);
    const unsigned ni = (unsigned)pt.nitems;
    if (!P.subpad) {
        k_subsort<true><<<ni, kSubThreads, 0, st>>>(P.g, pt.items, P.recs, pt.fitems);
        SDP_HIP_CHECK(hipGetLastError());
        return;
    }
    // padded item sizes -> item bases (scan) -> total (one host sync) -> the
    // padded, cell-ordered copy of the records
    unsigned *pcnt = scratch<unsigned>("sub_pcnt", (size_t)ni + 1);
    unsigned *pbase = scratch<unsigned>("sub_pbase", (size_t)ni + 1);
    SDP_HIP_CHECK(hipMemsetAsync(pcnt + ni, 0, sizeof(unsigned), st));
    k_sub_count<<<ni, 256, 0, st>>>(pt.items, P.cls, pcnt);
    size_t tb = 0;
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, pcnt, pbase, (int)ni + 1, st));
    void *tmp = scratch<char>("scan_tmp", tb + 16);
    SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, pcnt, pbase, (int)ni + 1, st));
    // the exact (64-bit) padded total beside the 32-bit scan: the record
    // offsets are 32-bit, so a total past 2^32 is refused, not wrapped
    unsigned long long *tot64 = scratch<unsigned long long>("sub_tot64", 1);
    k_sum_u32<<<1, 1024, 0, st>>>(pcnt, ni, tot64);
    unsigned long long *htot = pinned_host<unsigned long long>(56, 1);
    SDP_HIP_CHECK(hipMemcpyAsync(htot, tot64, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    SDP_HIP_CHECK(hipStreamSynchronize(st));
    SDP_REQUIRE(*htot < 0xffffffffull,
                "more than 2^32 padded records in one invert call: split it into batches");
    P.recs_pad = scratch<RecC>("recs_pad", (size_t)*htot + 1);
    k_subsort_pad<<<ni, kSubThreads, 0, st>>>(P.g, pt.items, reinterpret_cast<const RecC *>(P.recs),
                                              P.cls, pbase, P.recs_pad, pt.fitems);
    SDP_HIP_CHECK(hipGetLastError());
}

// Record `e` on `from` and make `to` wait for it.
static void stream_after(hipStream_t to, hipStream_t from) {
    hipEvent_t e;
    SDP_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    SDP_HIP_CHECK(hipEventRecord(e, from));
    SDP_HIP_CHECK(hipStreamWaitEvent(to, e, 0));
    SDP_HIP_CHECK(hipEventDestroy(e));
}

static int weight_is_f64(int wgt_dtype) {
    SDP_REQUIRE(wgt_dtype == SDP_HIP_F32 || wgt_dtype == SDP_HIP_F64, "weights must be f32 or f64");
    return wgt_dtype == SDP_HIP_F64 ? 1 : 0;
}

// The call's workspace slot (SDP_HIP_SLOT1), reset on every exit.
struct SlotGuard {
    explicit SlotGuard(unsigned flags) {
        const bool one = flags & SDP_HIP_SLOT1;
        SDP_REQUIRE(!one || !(flags & (SDP_HIP_KEEP_BUCKETS | SDP_HIP_REUSE_BUCKETS |
                                       SDP_HIP_BATCH_FIRST | SDP_HIP_BATCH_LAST |
                                       SDP_HIP_W_SLAB)),
                    "SDP_HIP_SLOT1 cannot be combined with kept / reused buckets, batches or "
                    "w slabs");
        ws_slot() = one ? 1 : 0;
    }
    ~SlotGuard() { ws_slot() = 0; }
};

static void ms2dirty(const Inputs &in, double *dirty, int64_t sx, int64_t sy,
                     sdp_hip_wgrid_info *info, hipStream_t st) {
    SDP_REQUIRE(in.vis == nullptr || in.vis_dtype == SDP_HIP_C64 ||
                    in.vis_dtype == SDP_HIP_C128,
                "vis must be complex64 or complex128");
    SlotGuard slot(in.flags);
    StageTimer tm(st);
    tm.mark();
    const bool keep = in.flags & SDP_HIP_KEEP_BUCKETS, reuse = in.flags & SDP_HIP_REUSE_BUCKETS;
    SDP_REQUIRE(!(keep && reuse), "SDP_HIP_KEEP_BUCKETS and SDP_HIP_REUSE_BUCKETS exclude each other");
    SDP_REQUIRE(in.bounds == nullptr || !(keep || reuse),
                "batched inverts do not keep or reuse bucketings");
    Inputs inx = in;
    // a kept bucketing holds every in-grid visibility (zero weights add exact
    // zeros); its reuse classifies them the same way (the two-level value
    // pass re-derives the bin ranks from that classification)
    inx.x.all = keep || reuse;
    Plan P = reuse ? reuse_buckets(in) : plan_geometry(inx, true, st);
    setup_core(P);
    const Geo &g = P.g;
    // batched invert: planes zeroed by the first batch, FFT + screens by the
    // last; in between they stay resident in the workspace
    const bool batched = in.bounds != nullptr;
    const bool first = !batched || (in.flags & SDP_HIP_BATCH_FIRST);
    const bool last = !batched || (in.flags & SDP_HIP_BATCH_LAST);
    if (batched) {
        SDP_REQUIRE(P.chunk_planes == g.nplanes,
                    "batched invert: the w planes do not all fit in device memory");
        check_batch_seq(P, in, first);
    }
    const double *tab = phi_table(g.W, g.beta, st);
    // the band zeroing of the first plane chunk (HBM writes) overlaps the
    // bucketing (bound by memory-side atomics): it runs on the auxiliary
    // stream after the call's earlier work on `st`; the gridding waits for it
    // (single calls only: on C4's streamed batches it measured 1-2 % slower)
    hipEvent_t zdone = nullptr;
    auto start_zero = [&] {
        if (!(first && !batched && env_int("SDP_HIP_ZERO_OVERLAP", 1) != 0)) return;
        hipStream_t aux = aux_stream();
        stream_after(aux, st);
        zero_band(P, std::min(g.nplanes, P.chunk_planes), aux);
        SDP_HIP_CHECK(hipEventCreateWithFlags(&zdone, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(zdone, aux));
    };
    if (reuse) {
        start_zero();
        // value pass only (weight sums included)
        double *slots = in.x.sumwt ? scratch<double>("sumwt_slots", kSumSlots) : nullptr;
        if (slots) SDP_HIP_CHECK(hipMemsetAsync(slots, 0, kSumSlots * sizeof(double), st));
        if (P.g.tiled) bucket_tiled(P, inx, true, st, true, nullptr, slots);
        else bucket_part(P, inx, true, st, true);
        if (slots) k_sum_slots<<<1, 64, 0, st>>>(slots, in.x.sumwt);
    } else {
        bucket_all(P, inx, true, st, start_zero);
    }
    if (P.subsort) subsort_items(P, st);
    if (keep) keep_buckets(P, in);
    const int accumulate = (in.flags & SDP_HIP_ACCUMULATE) ? 1 : 0;
    float tgrid = 0, tfft = 0, tscr = 0;
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
        {
            StageTimer tg(st);
            tg.mark();
#define SDP_LAUNCH_GRID(WW) launch_grid<WW>(P, p_lo, p_hi, st)
            if (P.f64) grid_f64(P, p_lo, p_hi, st);
            else SDP_W_DISPATCH(g.W, SDP_LAUNCH_GRID);
#undef SDP_LAUNCH_GRID
            SDP_HIP_CHECK(hipGetLastError());
            tg.mark();
            tgrid += tg.ms(0, 1);
        }
        if (last) core_merge(P, 0, np, st);
        for (int sb = 0; last && sb < np; sb += P.fft_planes) {
            const int nb = std::min(P.fft_planes, np - sb);
            StageTimer t2(st);
            t2.mark();
            fft_rows_y(P, sb, nb, HIPFFT_BACKWARD, st);
            tr_grid_to_t(P, sb, nb, st);
            xfft_screen_fwd(P, p_lo + sb, nb, dirty, sx, sy,
                            (accumulate || p_lo + sb > 0) ? 1 : 0, tab, st, t2);
            tfft += t2.ms(0, 1);
            tscr += t2.ms(1, 2);
        }
    }
    if (zdone) {  // (no plane pass ran)
        SDP_HIP_CHECK(hipStreamWaitEvent(st, zdone, 0));
        SDP_HIP_CHECK(hipEventDestroy(zdone));
    }
    if (batched && last) drop_batch_seq();
    tm.mark();
    fill_info(P, info);
    if (info) {
        // everything on the call's stream that is not gridding, FFT or screen:
        // geometry, bucketing, band zeroing not hidden behind the bucketing
        info->ms_prep = tm.on ? tm.ms(0, 1) - tgrid - tfft - tscr : 0.0f;
        info->ms_grid = tgrid;
        info->ms_fft = tfft;
        info->ms_screen = tscr;
    }
}

// All image pols of one invert_ng call in one bucketing (sdp_hip_ms2dirty_vis_pols):
// one rank pass, one value pass writing every pol's records (k_bucket_pols),
// then each pol's gridding, FFT and screens into its own image.  `in` is
// image pol 0's call (its conversion row, weights and flag pol); `ps` holds
// every pol's rows and the weights' pol stride, `dirty[q]` / `sumwt[q]` the
// outputs.  Plans the fused pass does not cover (fp64, two-level-only or
// large-grid plans) run the pols one call each, sharing a kept bucketing.
static void ms2dirty_pols(const Inputs &in, PolsSpec ps, double *const *dirty, int64_t sx,
                          int64_t sy, double *const *sumwt, sdp_hip_wgrid_info *info,
                          hipStream_t st) {
    SDP_REQUIRE(ps.npo >= 1 && ps.npo <= 4, "npol_img must be 1..4");
    SDP_REQUIRE(in.vis != nullptr && (in.vis_dtype == SDP_HIP_C64 || in.vis_dtype == SDP_HIP_C128),
                "vis must be complex64 or complex128");
    SDP_REQUIRE(ps.npo <= in.x.npv, "npol_img must not exceed npol_vis (pol q's flags mask its "
                                    "weights)");
    auto per_pol = [&] {
        for (int q = 0; q < ps.npo; ++q) {
            Inputs iq = in;
            iq.x.conv = true;
            for (int k = 0; k < 4; ++k) {
                iq.x.cre[k] = ps.cre[q][k];
                iq.x.cim[k] = ps.cim[q][k];
            }
            iq.x.fpol = q;
            iq.wgt = static_cast<const char *>(ps.wgt) +
                     q * ps.wps * (in.x.wgt_f64 ? sizeof(double) : sizeof(float));
            iq.x.sumwt = sumwt[q];
            iq.flags = (in.flags & ~(SDP_HIP_KEEP_BUCKETS | SDP_HIP_REUSE_BUCKETS)) |
                       (ps.npo > 1 ? (q == 0 ? SDP_HIP_KEEP_BUCKETS : SDP_HIP_REUSE_BUCKETS) : 0);
            ms2dirty(iq, dirty[q], sx, sy, q == ps.npo - 1 ? info : nullptr, st);
        }
    };
    if (in.eps < 1.0e-7 && !(in.flags & SDP_HIP_FP32)) {
        // (fp64: each pol its own two-level sort, as invert_ng runs them)
        for (int q = 0; q < ps.npo; ++q) {
            Inputs iq = in;
            iq.x.conv = true;
            for (int k = 0; k < 4; ++k) {
                iq.x.cre[k] = ps.cre[q][k];
                iq.x.cim[k] = ps.cim[q][k];
            }
            iq.x.fpol = q;
            iq.wgt = static_cast<const char *>(ps.wgt) +
                     q * ps.wps * (in.x.wgt_f64 ? sizeof(double) : sizeof(float));
            iq.x.sumwt = sumwt[q];
            iq.flags = in.flags & ~(SDP_HIP_KEEP_BUCKETS | SDP_HIP_REUSE_BUCKETS);
            ms2dirty(iq, dirty[q], sx, sy, q == ps.npo - 1 ? info : nullptr, st);
        }
        return;
    }
    SlotGuard slot(in.flags);
    StageTimer tm(st);
    tm.mark();
    Inputs inx = in;
    inx.x.conv = true;
    for (int k = 0; k < 4; ++k) {
        inx.x.cre[k] = ps.cre[0][k];
        inx.x.cim[k] = ps.cim[0][k];
    }
    inx.x.fpol = 0;
    inx.x.all = true;         // every in-grid visibility: the bucketing holds for every pol
    inx.x.sumwt = nullptr;    // (the value pass sums every pol's weights)
    inx.flags = (in.flags & ~SDP_HIP_REUSE_BUCKETS) | SDP_HIP_KEEP_BUCKETS;  // single-level
    Plan P = plan_geometry(inx, true, st);
    if (P.f64 || P.g.tiled || P.g.sub != kTileCell || !P.pad4 || P.subpad) {
        per_pol();
        return;
    }
    setup_core(P);
    const Geo &g = P.g;
    const double *tab = phi_table(g.W, g.beta, st);
    hipEvent_t zdone = nullptr;
    auto start_zero = [&] {
        if (env_int("SDP_HIP_ZERO_OVERLAP", 1) == 0) return;
        hipStream_t aux = aux_stream();
        stream_after(aux, st);
        zero_band(P, std::min(g.nplanes, P.chunk_planes), aux);
        SDP_HIP_CHECK(hipEventCreateWithFlags(&zdone, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(zdone, aux));
    };
    double *slots = scratch<double>("sumwt_slots_pols", 4 * kSumSlots);
    SDP_HIP_CHECK(hipMemsetAsync(slots, 0, 4 * kSumSlots * sizeof(double), st));
    for (int q = 0; q < ps.npo; ++q) ps.slots[q] = sumwt[q] ? slots + q * kSumSlots : nullptr;
    bucket_part(P, inx, true, st, false, start_zero, &ps);
    for (int q = 0; q < ps.npo; ++q)
        if (sumwt[q]) k_sum_slots<<<1, 64, 0, st>>>(ps.slots[q], sumwt[q]);
    read_part_meta(P, st);
    const int accumulate = (in.flags & SDP_HIP_ACCUMULATE) ? 1 : 0;
    float tgrid = 0, tfft = 0, tscr = 0;
    for (int q = 0; q < ps.npo; ++q) {
        P.recs = reinterpret_cast<VisRec *>(ps.recs[q]);
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
            {
                StageTimer tg(st);
                tg.mark();
#define SDP_LAUNCH_GRID(WW) launch_grid<WW>(P, p_lo, p_hi, st)
                SDP_W_DISPATCH(g.W, SDP_LAUNCH_GRID);
#undef SDP_LAUNCH_GRID
                SDP_HIP_CHECK(hipGetLastError());
                tg.mark();
                tgrid += tg.ms(0, 1);
            }
            core_merge(P, 0, np, st);
            for (int sb = 0; sb < np; sb += P.fft_planes) {
                const int nb = std::min(P.fft_planes, np - sb);
                StageTimer t2(st);
                t2.mark();
                fft_rows_y(P, sb, nb, HIPFFT_BACKWARD, st);
                tr_grid_to_t(P, sb, nb, st);
                xfft_screen_fwd(P, p_lo + sb, nb, dirty[q], sx, sy,
                                (accumulate || p_lo + sb > 0) ? 1 : 0, tab, st, t2);
                tfft += t2.ms(0, 1);
                tscr += t2.ms(1, 2);
            }
        }
    }
    if (zdone) {
        SDP_HIP_CHECK(hipStreamWaitEvent(st, zdone, 0));
        SDP_HIP_CHECK(hipEventDestroy(zdone));
    }
    P.recs = reinterpret_cast<VisRec *>(ps.recs[0]);
    tm.mark();
    fill_info(P, info);
    if (info) {
        info->ms_prep = tm.on ? tm.ms(0, 1) - tgrid - tfft - tscr : 0.0f;
        info->ms_grid = tgrid;
        info->ms_fft = tfft;
        info->ms_screen = tscr;
    }
}

static void dirty2ms(const Inputs &in, const double *dirty, int64_t sx, int64_t sy, void *vis,
                     sdp_hip_wgrid_info *info, hipStream_t st, const OutConv &oc = OutConv{},
                     int npo = 1, const double *const *dirty_q = nullptr,
                     const OutConv *oc_q = nullptr) {
    // npo > 1 (sdp_hip_dirty2ms_vis_pols): image pol q is dirty_q[q] through
    // the conversion column oc_q[q], into one output; the pols share the
    // bucketing, each has its plane stage and degridding, and one write-back
    // combines them (fp64: the degridder adds each pol itself)
    auto img = [&](int q) { return npo > 1 ? dirty_q[q] : dirty; };
    SDP_REQUIRE(in.vis_dtype == SDP_HIP_C64 || in.vis_dtype == SDP_HIP_C128,
                "vis must be complex64 or complex128");
    SlotGuard slot(in.flags);
    StageTimer tm(st);
    tm.mark();
    Plan P = plan_geometry(in, false, st);
    const Geo &g = P.g;
    const double *tab = phi_table(g.W, g.beta, st);
    const int accumulate = (in.flags & SDP_HIP_ACCUMULATE) ? 1 : 0;
    const int64_t nvis = in.nrow * (int64_t)in.nchan;
    OutConv ocz = oc;  // the visibility pols any image pol writes
    if (npo > 1) {
        ocz = oc_q[0];
        for (int k = 0; k < ocz.npv; ++k) {
            bool any = false;
            for (int q = 0; q < npo; ++q) any |= oc_q[q].cre[k] != 0.0 || oc_q[q].cim[k] != 0.0;
            ocz.cre[k] = any ? 1.0 : 0.0;
            ocz.cim[k] = 0.0;
        }
    }
    auto zero_vis = [&](hipStream_t s) {
        if (accumulate || nvis <= 0) return;
        if (in.vis_dtype == SDP_HIP_C128)
            k_zero_vis<double2><<<grid1d(nvis, 256), 256, 0, s>>>(in.nrow, in.nchan,
                                                                   (double2 *)vis, in.vrs,
                                                                   in.vcs, ocz);
        else
            k_zero_vis<float2><<<grid1d(nvis, 256), 256, 0, s>>>(in.nrow, in.nchan, (float2 *)vis,
                                                                  in.vrs, in.vcs, ocz);
        SDP_HIP_CHECK(hipGetLastError());
    };
    // all planes in one pass into plain contiguous c64 visibilities: the
    // degridder applies the record factor and writes each visibility once,
    // and on the single-level bucketing the rank pass zeroes the
    // visibilities no record reaches (no separate 1 GB zeroing pass on C2);
    // otherwise the output is zeroed first
    const bool trivial_oc = oc.npv == 1 && oc.cre[0] == 1.0 && oc.cim[0] == 0.0;
    if (npo == 1 && P.chunk_planes == g.nplanes && !accumulate && in.vis_dtype != SDP_HIP_C128 &&
        trivial_oc && in.vcs == 1 && in.vrs == in.nchan && !P.f64) {
        P.vdirect = static_cast<float2 *>(vis);
        if (!g.tiled) P.zout = P.vdirect;
    }
    auto zero_vis_unless_fused = [&](hipStream_t s) {
        if (!P.zout) zero_vis(s);
    };
    // screens + FFTs of planes [p_lo, p_lo + np) into the grid
    std::vector<std::unique_ptr<StageTimer>> stage_t;
    auto plane_stage = [&](int p_lo, int np, hipStream_t s, const double *image) {
        for (int sb = 0; sb < np; sb += P.fft_planes) {
            const int nb = std::min(P.fft_planes, np - sb);
            stage_t.emplace_back(new StageTimer(s));
            StageTimer &t2 = *stage_t.back();
            t2.mark();
            screen_adj_xfft(P, image, sx, sy, p_lo + sb, nb, tab, s, t2);
            tr_t_to_grid(P, sb, nb, s);
            fft_rows_y(P, sb, nb, HIPFFT_FORWARD, s);
            t2.mark();
        }
    };
    // the output zeroing and the first plane chunk's band zeroing (HBM
    // writes) overlap the bucketing on the auxiliary stream, once the
    // histogram clearing is queued.  With resident planes the whole plane
    // stage (screens, FFTs into the grid: it depends only on the image)
    // follows there too: C2 predict 13.01 -> 12.72 ms, at eps 1e-12 77.3 ->
    // 75.8 ms (profiles/r06_predict_planes_aux_ab.txt; round 2, with the
    // slower count pass of that time, it had measured 15.6 vs 15.4 ms)
    const bool overlap = env_int("SDP_HIP_ZERO_OVERLAP", 1) != 0;
    const bool planes_aux = overlap && P.chunk_planes == g.nplanes;
    hipEvent_t zdone = nullptr;
    auto start_aux = [&] {
        if (!overlap) return;
        hipStream_t aux = aux_stream();
        stream_after(aux, st);
        zero_vis_unless_fused(aux);
        zero_band(P, std::min(g.nplanes, P.chunk_planes), aux);
        if (planes_aux) plane_stage(0, g.nplanes, aux, img(0));
        SDP_HIP_CHECK(hipEventCreateWithFlags(&zdone, hipEventDisableTiming));
        SDP_HIP_CHECK(hipEventRecord(zdone, aux));
    };
    if (!overlap) zero_vis_unless_fused(st);
    bucket_all(P, in, false, st, start_aux);
    if (P.subsort) subsort_items(P, st);
    // (the fp64 degridder writes each visibility itself, through the pol
    // conversion, adding into the zeroed output)
    float2 *accs[4] = {};
    if (!(P.vdirect || P.f64)) {
        static const char *names[4] = {"degrid_acc", "degrid_acc1", "degrid_acc2", "degrid_acc3"};
        for (int q = 0; q < npo; ++q) {
            accs[q] = scratch<float2>(names[q], std::max<int64_t>(nvis, 1));
            SDP_HIP_CHECK(
                hipMemsetAsync(accs[q], 0, std::max<int64_t>(nvis, 1) * sizeof(float2), st));
        }
    }
    float2 *const acc = accs[0];
    float tgrid = 0, tfft = 0, tscr = 0;
    for (int q = 0; q < npo; ++q) {
      const OutConv &ocq = npo > 1 ? oc_q[q] : oc;
      float2 *const accq = accs[q];
      for (int p_lo = 0; p_lo < g.nplanes; p_lo += P.chunk_planes) {
        const int p_hi = std::min(g.nplanes, p_lo + P.chunk_planes);
        const int np = p_hi - p_lo;
        if (zdone) {
            SDP_HIP_CHECK(hipStreamWaitEvent(st, zdone, 0));
            SDP_HIP_CHECK(hipEventDestroy(zdone));
            zdone = nullptr;
            if (!planes_aux) plane_stage(p_lo, np, st, img(q));
        } else {
            zero_band(P, np, st);
            plane_stage(p_lo, np, st, img(q));
        }
        StageTimer tg(st);
        tg.mark();
#define SDP_LAUNCH_DEGRID(WW) launch_degrid<WW>(P, p_lo, p_hi, accq, st)
        if (P.f64 && in.vis_dtype == SDP_HIP_C128)
            degrid_f64<double2>(P, p_lo, p_hi, static_cast<double2 *>(vis), in.vrs, in.vcs, 1, ocq,
                                st);
        else if (P.f64)
            degrid_f64<float2>(P, p_lo, p_hi, static_cast<float2 *>(vis), in.vrs, in.vcs, 1, ocq,
                               st);
        else
            SDP_W_DISPATCH(g.W, SDP_LAUNCH_DEGRID);
#undef SDP_LAUNCH_DEGRID
        SDP_HIP_CHECK(hipGetLastError());
        tg.mark();
        tgrid += tg.ms(0, 1);
      }
    }
    if (zdone) {  // (no plane pass ran)
        SDP_HIP_CHECK(hipStreamWaitEvent(st, zdone, 0));
        SDP_HIP_CHECK(hipEventDestroy(zdone));
    }
    for (auto &t : stage_t) {
        tscr += t->ms(0, 1);
        tfft += t->ms(1, 2);
    }
    if (npo > 1 && !P.f64 && P.pt.nvis > 0) {
        const unsigned nb = std::min<unsigned>(grid1d(P.pt.nvis, 256), 16384);
        PolAccs pa;
        for (int q = 0; q < npo; ++q) {
            pa.a[q] = accs[q];
            pa.oc[q] = oc_q[q];
        }
#define SDP_FIN(VT, N)                                                                     \
    k_finalize_pols<VT, N><<<nb, 256, 0, st>>>(P.pt.nrec, in.nchan, P.recs, pa, (VT *)vis, \
                                               in.vrs, in.vcs, accumulate)
        if (in.vis_dtype == SDP_HIP_C128) {
            if (npo == 2) SDP_FIN(double2, 2);
            else if (npo == 3) SDP_FIN(double2, 3);
            else SDP_FIN(double2, 4);
        } else {
            if (npo == 2) SDP_FIN(float2, 2);
            else if (npo == 3) SDP_FIN(float2, 3);
            else SDP_FIN(float2, 4);
        }
#undef SDP_FIN
        SDP_HIP_CHECK(hipGetLastError());
    } else if (!P.vdirect && !P.f64 && P.pt.nvis > 0) {
        const unsigned nb = std::min<unsigned>(grid1d(P.pt.nvis, 256), 16384);
        if (in.vis_dtype == SDP_HIP_C128)
            k_finalize<double2><<<nb, 256, 0, st>>>(P.pt.nrec, in.nchan, P.recs, acc,
                                                    (double2 *)vis, in.vrs, in.vcs, accumulate, oc);
        else
            k_finalize<float2><<<nb, 256, 0, st>>>(P.pt.nrec, in.nchan, P.recs, acc, (float2 *)vis,
                                                   in.vrs, in.vcs, accumulate, oc);
        SDP_HIP_CHECK(hipGetLastError());
    }
    tm.mark();
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

static int ms2dirty_vis_entry(const double *uvw, int64_t uvw_row_stride, const double *freq, int nchan,
                         int64_t nrow, const void *vis, int vis_dtype, int64_t vis_row_stride,
                         int64_t vis_chan_stride, int64_t vis_pol_stride, int npol_vis,
                         const double *pol_coeff, const void *wgt, int wgt_dtype,
                         int64_t wgt_row_stride, int64_t wgt_chan_stride, const void *vis_flags,
                         int flag_bytes, int64_t flag_row_stride, int64_t flag_chan_stride,
                         int64_t flag_pol_stride, int pol, int npix_x, int npix_y,
                         double pixsize_x, double pixsize_y, double epsilon, int do_wstacking,
                         unsigned flags, const double *bounds, double *dirty, int64_t dirty_stride_x,
                         int64_t dirty_stride_y, double *sumwt, const double *shift_lmn,
                         void *stream, sdp_hip_wgrid_info *info, char *errbuf,
                         size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE((dirty != nullptr || (bounds && !(flags & SDP_HIP_BATCH_LAST))) &&
                        freq != nullptr && (uvw != nullptr || nrow == 0),
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
        in.bounds = bounds;
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
                     int64_t vis_chan_stride, const void *wgt, int wgt_dtype,
                     int64_t wgt_row_stride, int64_t wgt_chan_stride, int npix_x, int npix_y,
                     double pixsize_x,
                     double pixsize_y, double epsilon, int do_wstacking, unsigned flags,
                     double *dirty, int64_t dirty_stride_x, int64_t dirty_stride_y, void *stream,
                     sdp_hip_wgrid_info *info, char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        wstack::Inputs in{uvw,         uvw_row_stride,  freq,           nchan,
                          nrow,        vis,             vis_dtype,      vis_row_stride,
                          vis_chan_stride, wgt,         wgt_row_stride, wgt_chan_stride,
                          npix_x,      npix_y,          pixsize_x,      pixsize_y,
                          epsilon,     do_wstacking,    flags};
        in.x.wgt_f64 = wstack::weight_is_f64(wgt_dtype);
        wstack::ms2dirty(in, dirty, dirty_stride_x, dirty_stride_y, info, as_stream(stream));
    });
}

int sdp_hip_ms2dirty_batch(const double *uvw, int64_t uvw_row_stride, const double *freq,
                           int nchan, int64_t nrow, const void *vis, int vis_dtype,
                           int64_t vis_row_stride, int64_t vis_chan_stride, const void *wgt,
                           int wgt_dtype, int64_t wgt_row_stride, int64_t wgt_chan_stride,
                           int npix_x,
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
        in.x.wgt_f64 = wstack::weight_is_f64(wgt_dtype);
        in.bounds = bounds;
        wstack::ms2dirty(in, dirty, dirty_stride_x, dirty_stride_y, info, as_stream(stream));
    });
}

int sdp_hip_wstack_layout(const double *bounds, int npix_x, int npix_y, double pixsize_x,
                          double pixsize_y, double epsilon, int do_wstacking, unsigned flags,
                          sdp_hip_wgrid_info *info, char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(bounds != nullptr && info != nullptr, "null pointer argument");
        SDP_REQUIRE(npix_x > 0 && npix_y > 0 && npix_x % 2 == 0 && npix_y % 2 == 0,
                    "npix_x and npix_y must be positive and even");
        SDP_REQUIRE(pixsize_x > 0 && pixsize_y > 0, "pixel sizes must be positive");
        const double *b = bounds;
        SDP_REQUIRE(b[0] <= b[1] && b[2] >= 0 && b[3] >= 0 && b[4] > 0 && b[4] <= b[5],
                    "bounds must be {wmin <= wmax, umax >= 0, vmax >= 0, 0 < fmin <= fmax}");
        wstack::Inputs in{};
        in.nx = npix_x;
        in.ny = npix_y;
        in.px = pixsize_x;
        in.py = pixsize_y;
        in.eps = epsilon;
        in.do_w = do_wstacking;
        in.flags = flags;
        wstack::Geo g{};
        const bool f64 = epsilon < 1.0e-7 && !(flags & SDP_HIP_FP32);
        g.W = f64 ? wstack::kernel_support64(epsilon) : wstack::kernel_support(epsilon);
        const double su = (flags & SDP_HIP_FLIP_UW) ? -1.0 : 1.0;
        const double h0 = su > 0 ? b[0] : -b[1], h1 = su > 0 ? b[1] : -b[0];
        const double slo = b[4] / wstack::kCLight, shi = b[5] / wstack::kCLight;
        wstack::w_layout(in, std::min(h0 * slo, h0 * shi), std::max(h1 * slo, h1 * shi), g);
        *info = sdp_hip_wgrid_info{};
        info->support = g.W;
        info->beta = 2.30 * g.W;
        info->ngrid_x = ((2 * npix_x + wstack::kGridAlign - 1) / wstack::kGridAlign) * wstack::kGridAlign;
        info->ngrid_y = ((2 * npix_y + wstack::kGridAlign - 1) / wstack::kGridAlign) * wstack::kGridAlign;
        info->nplanes = g.nplanes;
        info->w0 = g.w0;
        info->dw = g.dw;
        info->fp64 = f64 ? 1 : 0;
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
    return ms2dirty_vis_entry(uvw, uvw_row_stride, freq, nchan, nrow, vis, vis_dtype,
                              vis_row_stride, vis_chan_stride, vis_pol_stride, npol_vis, pol_coeff,
                              wgt, wgt_dtype, wgt_row_stride, wgt_chan_stride, vis_flags,
                              flag_bytes, flag_row_stride, flag_chan_stride, flag_pol_stride, pol,
                              npix_x, npix_y, pixsize_x, pixsize_y, epsilon, do_wstacking,
                              flags & ~(SDP_HIP_BATCH_FIRST | SDP_HIP_BATCH_LAST), nullptr, dirty,
                              dirty_stride_x, dirty_stride_y, sumwt, shift_lmn, stream, info,
                              errbuf, errbuf_len);
}

int sdp_hip_ms2dirty_vis_pols(const double *uvw, int64_t uvw_row_stride, const double *freq,
                              int nchan, int64_t nrow, const void *vis, int vis_dtype,
                              int64_t vis_row_stride, int64_t vis_chan_stride,
                              int64_t vis_pol_stride, int npol_vis, const double *pol_coeff,
                              int npol_img, const void *wgt, int wgt_dtype,
                              int64_t wgt_row_stride, int64_t wgt_chan_stride,
                              int64_t wgt_pol_stride, const void *vis_flags, int flag_bytes,
                              int64_t flag_row_stride, int64_t flag_chan_stride,
                              int64_t flag_pol_stride, int npix_x, int npix_y, double pixsize_x,
                              double pixsize_y, double epsilon, int do_wstacking, unsigned flags,
                              double *dirty, int64_t dirty_stride_x, int64_t dirty_stride_y,
                              int64_t dirty_stride_pol, double *sumwt, int64_t sumwt_stride,
                              const double *shift_lmn, void *stream, sdp_hip_wgrid_info *info,
                              char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && vis != nullptr && wgt != nullptr &&
                        (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        SDP_REQUIRE(npol_vis >= 1 && npol_vis <= 4, "npol_vis must be 1..4");
        SDP_REQUIRE(npol_img >= 1 && npol_img <= npol_vis, "npol_img must be 1..npol_vis");
        SDP_REQUIRE(wgt_dtype == SDP_HIP_F32 || wgt_dtype == SDP_HIP_F64,
                    "weights must be f32 or f64");
        SDP_REQUIRE(vis_flags == nullptr || flag_bytes == 1 || flag_bytes == 4 || flag_bytes == 8,
                    "flag element size must be 1, 4 or 8 bytes");
        SDP_REQUIRE(!(flags & (SDP_HIP_KEEP_BUCKETS | SDP_HIP_REUSE_BUCKETS | SDP_HIP_BATCH_FIRST |
                               SDP_HIP_BATCH_LAST)),
                    "a pols call keeps, reuses or batches nothing");
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
        if (shift_lmn) {
            x.shift = true;
            x.sl = shift_lmn[0];
            x.sm = shift_lmn[1];
            x.sn = shift_lmn[2];
        }
        wstack::PolsSpec ps;
        ps.npo = npol_img;
        for (int q = 0; q < npol_img; ++q)
            for (int k = 0; k < npol_vis; ++k) {
                ps.cre[q][k] = pol_coeff ? pol_coeff[2 * (q * npol_vis + k)] : (q == k ? 1.0 : 0.0);
                ps.cim[q][k] = pol_coeff ? pol_coeff[2 * (q * npol_vis + k) + 1] : 0.0;
            }
        ps.wgt = wgt;
        ps.wrs = wgt_row_stride;
        ps.wcs = wgt_chan_stride;
        ps.wps = wgt_pol_stride;
        double *outs[4] = {}, *sums[4] = {};
        for (int q = 0; q < npol_img; ++q) {
            outs[q] = dirty + q * dirty_stride_pol;
            sums[q] = sumwt ? sumwt + q * sumwt_stride : nullptr;
        }
        wstack::ms2dirty_pols(in, ps, outs, dirty_stride_x, dirty_stride_y, sums, info,
                              as_stream(stream));
    });
}

int sdp_hip_ms2dirty_vis_batch(const double *uvw, int64_t uvw_row_stride, const double *freq,
                               int nchan, int64_t nrow, const void *vis, int vis_dtype,
                               int64_t vis_row_stride, int64_t vis_chan_stride,
                               int64_t vis_pol_stride, int npol_vis, const double *pol_coeff,
                               const void *wgt, int wgt_dtype, int64_t wgt_row_stride,
                               int64_t wgt_chan_stride, const void *vis_flags, int flag_bytes,
                               int64_t flag_row_stride, int64_t flag_chan_stride,
                               int64_t flag_pol_stride, int pol, int npix_x, int npix_y,
                               double pixsize_x, double pixsize_y, double epsilon,
                               int do_wstacking, unsigned flags, const double *bounds,
                               double *dirty, int64_t dirty_stride_x, int64_t dirty_stride_y,
                               double *sumwt, const double *shift_lmn, void *stream,
                               sdp_hip_wgrid_info *info, char *errbuf, size_t errbuf_len) {
    if (bounds == nullptr) {
        if (errbuf && errbuf_len) std::snprintf(errbuf, errbuf_len, "null pointer argument");
        return SDP_HIP_ERR_INVALID_ARG;
    }
    return ms2dirty_vis_entry(uvw, uvw_row_stride, freq, nchan, nrow, vis, vis_dtype,
                              vis_row_stride, vis_chan_stride, vis_pol_stride, npol_vis, pol_coeff,
                              wgt, wgt_dtype, wgt_row_stride, wgt_chan_stride, vis_flags,
                              flag_bytes, flag_row_stride, flag_chan_stride, flag_pol_stride, pol,
                              npix_x, npix_y, pixsize_x, pixsize_y, epsilon, do_wstacking, flags,
                              bounds, dirty, dirty_stride_x, dirty_stride_y, sumwt, shift_lmn,
                              stream, info, errbuf, errbuf_len);
}

int sdp_hip_dirty2ms(const double *uvw, int64_t uvw_row_stride, const double *freq, int nchan,
                     int64_t nrow, const double *dirty, int64_t dirty_stride_x,
                     int64_t dirty_stride_y, int npix_x, int npix_y, double pixsize_x,
                     double pixsize_y, const void *wgt, int wgt_dtype, int64_t wgt_row_stride,
                     int64_t wgt_chan_stride, double epsilon, int do_wstacking, unsigned flags,
                     void *vis, int vis_dtype, int64_t vis_row_stride, int64_t vis_chan_stride,
                     void *stream, sdp_hip_wgrid_info *info, char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && vis != nullptr &&
                        (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        wstack::Inputs in{uvw,         uvw_row_stride,  freq,           nchan,
                          nrow,        nullptr,         vis_dtype,      vis_row_stride,
                          vis_chan_stride, wgt,         wgt_row_stride, wgt_chan_stride,
                          npix_x,      npix_y,          pixsize_x,      pixsize_y,
                          epsilon,     do_wstacking,    flags};
        in.x.wgt_f64 = wstack::weight_is_f64(wgt_dtype);
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

int sdp_hip_dirty2ms_vis_pols(const double *uvw, int64_t uvw_row_stride, const double *freq,
                              int nchan, int64_t nrow, const double *dirty,
                              int64_t dirty_stride_x, int64_t dirty_stride_y,
                              int64_t dirty_stride_pol, int npol_img, int npix_x, int npix_y,
                              double pixsize_x, double pixsize_y, double epsilon,
                              int do_wstacking, unsigned flags, void *vis, int vis_dtype,
                              int64_t vis_row_stride, int64_t vis_chan_stride,
                              int64_t vis_pol_stride, int npol_vis, const double *pol_coeff,
                              const double *shift_lmn, void *stream, sdp_hip_wgrid_info *info,
                              char *errbuf, size_t errbuf_len) {
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(dirty != nullptr && freq != nullptr && vis != nullptr &&
                        (uvw != nullptr || nrow == 0),
                    "null pointer argument");
        SDP_REQUIRE(npol_vis >= 1 && npol_vis <= 4, "npol_vis must be 1..4");
        SDP_REQUIRE(npol_img >= 1 && npol_img <= 4, "npol_img must be 1..4");
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
        wstack::OutConv ocs[4];
        const double *imgs[4] = {};
        for (int q = 0; q < npol_img; ++q) {
            ocs[q].npv = npol_vis;
            ocs[q].vps = vis_pol_stride;
            for (int k = 0; k < npol_vis; ++k) {
                ocs[q].cre[k] = pol_coeff ? pol_coeff[2 * (q * npol_vis + k)] : (k == q ? 1.0 : 0.0);
                ocs[q].cim[k] = pol_coeff ? pol_coeff[2 * (q * npol_vis + k) + 1] : 0.0;
            }
            imgs[q] = dirty + q * dirty_stride_pol;
        }
        wstack::dirty2ms(in, dirty, dirty_stride_x, dirty_stride_y, vis, info, as_stream(stream),
                         ocs[0], npol_img, imgs, ocs);
    });
}

}  // extern "C"
