// Convolution-function (AW-projection) gridder / degridder for gfx950:
// sdp_hip_grid_cf / sdp_hip_degrid_cf, replacing the pure-Python
// chan x pol x row loops of the reference's grid_visibility_to_griddata and
// degrid_visibility_from_griddata
// (src/ska_sdp_func_python/grid_data/gridding.py:160-255, :502-590).
//
// The Python layer evaluates the reference's WCS mappings (spatial_mapping,
// gridding.py:60-157) into integer grid / sub-sample / w-plane indices per
// (channel, row).  Gridding,
//   gd[c, p, pv-dv+iv, pu-du+iu] += conj(cf[c, p, w, dv_off, du_off, iv, iu]) * V * wt,
// runs on (row, channel) entries sorted by 16x16-pixel tile of their centre
// pixel (k_cf_count: rank by atomic, hipcub scan, k_cf_scatter), split into
// work items of <= kChunk entries; one wave per (item, pol) accumulates its
// entries' footprints in an LDS tile of (16+gv-1) x (16+gu-1) fp64 complex
// cells (plain read-modify-write: one lane per tap, in-order LDS per wave)
// and flushes it once with fp64 global atomics, zero cells skipped -- one
// global add per touched cell per item instead of one per tap per entry.
// sumwt per block in LDS, then one of kSlots partial sums per pol, folded
// by k_fold_slots.  Supports too large for the LDS tile use k_grid_cf (one
// wave per entry, fp64 atomics per tap).  Degridding:
//   V = sum_{iv,iu} gd[c, p, window] * cf[c, p, w, dv_off, du_off, iv, iu]
// with the reference's edge-skip rule (gridding.py:230-237, :555-563): a row
// whose window touches pv+dv >= ny or pu+du >= nx (or < 0) is skipped.
#include <hipcub/hipcub.hpp>

#include "sdp_common.h"

namespace sdp {
namespace cfgrid {

constexpr int kThreads = 256;
constexpr int kMaxPol = 4;
constexpr int kSlots = 1024;  // partial-sum slots for sumwt / skip counts (power of two)

struct Shape {
    int64_t nrow;
    int nchan, npol, cf_nchan, nw, ndv, ndu, gv, gu, g_nchan, ny, nx;
};

__device__ __forceinline__ bool window_ok(const Shape &s, int pu, int pv) {
    const int dv = s.gv / 2, du = s.gu / 2;
    return !(pv - dv < 0 || pv + dv >= s.ny || pu - du < 0 || pu + du >= s.nx);
}

__device__ __forceinline__ size_t cf_index(const Shape &s, int c, int p, int w, int idv, int idu) {
    return ((((size_t)c * s.npol + p) * s.nw + w) * s.ndv + idv) * s.ndu + idu;
}

__global__ __launch_bounds__(kThreads) void k_grid_cf(Shape s, const int32_t *__restrict__ pu,
                                                      const int32_t *__restrict__ pv,
                                                      const int32_t *__restrict__ pwc,
                                                      const int32_t *__restrict__ pdu,
                                                      const int32_t *__restrict__ pdv,
                                                      const int32_t *__restrict__ vis_to_im,
                                                      const double2 *__restrict__ vis,
                                                      const double *__restrict__ wt,
                                                      const double2 *__restrict__ cf,
                                                      double2 *grid, double *wslots,
                                                      unsigned long long *skslots) {
    __shared__ double s_wt[kMaxPol];
    __shared__ unsigned long long s_skip;
    if (threadIdx.x < kMaxPol) s_wt[threadIdx.x] = 0.0;
    if (threadIdx.x == 0) s_skip = 0;
    __syncthreads();
    const int chan = blockIdx.y;
    const int imchan = vis_to_im[chan];
    const int lane = threadIdx.x & 63;
    const int taps = s.gv * s.gu;
    const int dv = s.gv / 2, du = s.gu / 2;
    const int64_t row = blockIdx.x * (int64_t)(kThreads / 64) + (threadIdx.x >> 6);
    if (row < s.nrow) {
        const size_t m = (size_t)chan * s.nrow + row;
        const int u0 = pu[m], v0 = pv[m];
        if (!window_ok(s, u0, v0)) {
            if (lane == 0) atomicAdd(&s_skip, (unsigned long long)s.npol);
        } else {
            const int iw = pwc[m], idu = pdu[m], idv = pdv[m];
            for (int p = 0; p < s.npol; ++p) {
                const size_t vi = ((size_t)row * s.nchan + chan) * s.npol + p;
                const double2 x = vis[vi];
                const double w = wt[vi];
                const double xr = x.x * w, xi = x.y * w;
                const double *sub =
                    reinterpret_cast<const double *>(cf + cf_index(s, imchan, p, iw, idv, idu) * taps);
                double *g = reinterpret_cast<double *>(grid + ((size_t)imchan * s.npol + p) * s.ny * s.nx);
                // one double per lane (re/im interleaved): a wave-instruction
                // covers 32 taps = whole contiguous rows of the footprint
                for (int f = lane; f < 2 * taps; f += 64) {
                    const int t = f >> 1;
                    const int iv = t / s.gu, iu = t - (t / s.gu) * s.gu;
                    const double cr = sub[2 * t], ci = sub[2 * t + 1];
                    // conj(cf) * x: re = cr xr + ci xi, im = cr xi - ci xr
                    const double val = (f & 1) ? (cr * xi - ci * xr) : (cr * xr + ci * xi);
                    double *dst = g + 2 * ((size_t)(v0 - dv + iv) * s.nx + (u0 - du + iu)) + (f & 1);
                    if (val != 0.0) atomicAdd(dst, val);
                }
                if (lane == 0) atomicAdd(&s_wt[p], w);
            }
        }
    }
    __syncthreads();
    // the block's weight / skip counts go to one of kSlots partial sums
    // (one shared address per call serialised ~1M atomics), folded by
    // k_fold_slots
    const int slot = blockIdx.x & (kSlots - 1);
    if (threadIdx.x < s.npol && s_wt[threadIdx.x] != 0.0)
        atomicAdd(&wslots[((size_t)slot * s.g_nchan + imchan) * s.npol + threadIdx.x],
                  s_wt[threadIdx.x]);
    if (threadIdx.x == 0 && s_skip) atomicAdd(&skslots[slot], s_skip);
}

// ---- sorted / LDS-tile gridding -----------------------------------------
constexpr int kTile = 16;            // tile edge (pixels) of the entry sort
constexpr unsigned kChunk = 256;     // max entries per work item
constexpr size_t kMaxTileLds = 64 * 1024;

struct CfItem {
    uint32_t b, e, key, pad;
};

// Count pass, one thread per (row, chan) entry (blockIdx.y = chan): the
// edge-skip rule, the weight sums (per block in LDS, then slots) and the
// entry's rank in its (image channel, tile) bucket
__global__ __launch_bounds__(kThreads) void k_cf_count(Shape s, int ntx, int ntiles,
                                                       const int32_t *__restrict__ pu,
                                                       const int32_t *__restrict__ pv,
                                                       const int32_t *__restrict__ vis_to_im,
                                                       const double *__restrict__ wt,
                                                       unsigned *cnt, unsigned *__restrict__ rk,
                                                       double *wslots,
                                                       unsigned long long *skslots) {
    __shared__ double s_wt[kMaxPol];
    __shared__ unsigned long long s_skip;
    if (threadIdx.x < kMaxPol) s_wt[threadIdx.x] = 0.0;
    if (threadIdx.x == 0) s_skip = 0;
    __syncthreads();
    const int chan = blockIdx.y;
    const int imchan = vis_to_im[chan];
    const int64_t row = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    bool ok = false;
    if (row < s.nrow) {
        const size_t m = (size_t)chan * s.nrow + row;
        const int u0 = pu[m], v0 = pv[m];
        ok = window_ok(s, u0, v0);
        if (!ok) {
            atomicAdd(&s_skip, (unsigned long long)s.npol);
            rk[m] = 0xffffffffu;
        } else {
            const unsigned key = (unsigned)imchan * (unsigned)ntiles +
                                 (unsigned)((v0 / kTile) * ntx + u0 / kTile);
            rk[m] = atomicAdd(&cnt[key], 1u);
        }
    }
    // weight sums: wave reduction, one LDS add per wave and pol
    for (int p = 0; p < s.npol; ++p) {
        double w = ok ? wt[((size_t)row * s.nchan + chan) * s.npol + p] : 0.0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
        if ((threadIdx.x & 63) == 0 && w != 0.0) atomicAdd(&s_wt[p], w);
    }
    __syncthreads();
    const int slot = (blockIdx.x + blockIdx.y * gridDim.x) & (kSlots - 1);
    if (threadIdx.x < s.npol && s_wt[threadIdx.x] != 0.0)
        atomicAdd(&wslots[((size_t)slot * s.g_nchan + imchan) * s.npol + threadIdx.x],
                  s_wt[threadIdx.x]);
    if (threadIdx.x == 0 && s_skip) atomicAdd(&skslots[slot], s_skip);
}

__global__ __launch_bounds__(kThreads) void k_cf_scatter(Shape s, int ntx, int ntiles,
                                                         const int32_t *__restrict__ pu,
                                                         const int32_t *__restrict__ pv,
                                                         const int32_t *__restrict__ vis_to_im,
                                                         const unsigned *__restrict__ offs,
                                                         const unsigned *__restrict__ rk,
                                                         uint32_t *__restrict__ order) {
    const int chan = blockIdx.y;
    const int64_t row = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (row >= s.nrow) return;
    const size_t m = (size_t)chan * s.nrow + row;
    const unsigned r = rk[m];
    if (r == 0xffffffffu) return;
    const int u0 = pu[m], v0 = pv[m];
    const unsigned key = (unsigned)vis_to_im[chan] * (unsigned)ntiles +
                         (unsigned)((v0 / kTile) * ntx + u0 / kTile);
    order[offs[key] + r] = (uint32_t)m;
}

__global__ void k_cf_nitems(int64_t nkeys, const unsigned *__restrict__ offs, unsigned *nit) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k >= nkeys) return;
    nit[k] = (offs[k + 1] - offs[k] + kChunk - 1) / kChunk;
}

__global__ void k_cf_items(int64_t nkeys, const unsigned *__restrict__ offs,
                           const unsigned *__restrict__ ioffs, CfItem *__restrict__ items) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k >= nkeys) return;
    const unsigned b = offs[k], e = offs[k + 1];
    unsigned o = ioffs[k];
    for (unsigned x = b; x < e; x += kChunk) items[o++] = CfItem{x, min(e, x + kChunk), (uint32_t)k, 0u};
}

__device__ __forceinline__ double lane_readd(double v, int k) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// One wave per (item, pol): the item's entries are fetched 64 at a time (one
// per lane) and broadcast; lane t owns tap t (taps > 64: t, t+64, ...).
__global__ __launch_bounds__(64) void k_cf_tile(Shape s, int ntx, int ntiles,
                                                const CfItem *__restrict__ items,
                                                const uint32_t *__restrict__ order,
                                                const int32_t *__restrict__ pu,
                                                const int32_t *__restrict__ pv,
                                                const int32_t *__restrict__ pwc,
                                                const int32_t *__restrict__ pdu,
                                                const int32_t *__restrict__ pdv,
                                                const double2 *__restrict__ vis,
                                                const double *__restrict__ wt,
                                                const double2 *__restrict__ cf, double2 *grid) {
    extern __shared__ __attribute__((aligned(16))) double2 acc[];
    const CfItem it = items[blockIdx.x];
    const int p = blockIdx.y;
    const int lane = threadIdx.x;
    const int imchan = (int)(it.key / (unsigned)ntiles);
    const int tile = (int)(it.key - (unsigned)imchan * (unsigned)ntiles);
    const int ty = tile / ntx, tx = tile - (tile / ntx) * ntx;
    const int W2 = kTile + s.gu - 1, H2 = kTile + s.gv - 1;
    const int taps = s.gv * s.gu;
    for (int i = lane; i < H2 * W2; i += 64) acc[i] = make_double2(0.0, 0.0);
    // lane's first tap: offset inside the LDS tile relative to the footprint start
    const int t0v = lane / s.gu, t0u = lane - (lane / s.gu) * s.gu;
    const int toff0 = t0v * W2 + t0u;
    for (uint32_t b0 = it.b; b0 < it.e; b0 += 64) {
        const int n = (int)min(64u, it.e - b0);
        // lane l decodes entry b0 + l
        int loff = 0;
        long long cfo = 0;
        double xr = 0.0, xi = 0.0;
        if (lane < n) {
            const uint32_t m = order[b0 + lane];
            const int chan = (int)(m / (uint32_t)s.nrow);
            const int64_t row = (int64_t)m - (int64_t)chan * s.nrow;
            loff = (pv[m] - ty * kTile) * W2 + (pu[m] - tx * kTile);
            cfo = (long long)cf_index(s, imchan, p, pwc[m], pdv[m], pdu[m]) * taps;
            const size_t vi = ((size_t)row * s.nchan + chan) * s.npol + p;
            const double2 x = vis[vi];
            const double w = wt[vi];
            xr = x.x * w;
            xi = x.y * w;
        }
        for (int k = 0; k < n; ++k) {
            const int lo = __builtin_amdgcn_readlane(loff, k);
            const long long co = ((long long)__builtin_amdgcn_readlane((int)(cfo >> 32), k) << 32) |
                                 (unsigned)__builtin_amdgcn_readlane((int)(cfo & 0xffffffffll), k);
            const double kr = lane_readd(xr, k), ki = lane_readd(xi, k);
            for (int t = lane, to = toff0; t < taps; t += 64) {
                const double2 c = cf[co + t];
                double2 a = acc[lo + to];
                // conj(cf) * x: re = cr xr + ci xi, im = cr xi - ci xr
                a.x += c.x * kr + c.y * ki;
                a.y += c.x * ki - c.y * kr;
                acc[lo + to] = a;
                if (t + 64 < taps) {
                    const int nv = (t + 64) / s.gu, nu = (t + 64) - ((t + 64) / s.gu) * s.gu;
                    to = nv * W2 + nu;
                }
            }
        }
    }
    __syncthreads();
    double *g = reinterpret_cast<double *>(grid + ((size_t)imchan * s.npol + p) * s.ny * s.nx);
    const double *fa = reinterpret_cast<const double *>(acc);
    const int v00 = ty * kTile - s.gv / 2, u00 = tx * kTile - s.gu / 2;
    for (int f = lane; f < 2 * H2 * W2; f += 64) {
        const double val = fa[f];
        if (val == 0.0) continue;
        const int c = f >> 1, lv = c / W2, lu = c - (c / W2) * W2;
        const int v = v00 + lv, u = u00 + lu;
        if (v < 0 || v >= s.ny || u < 0 || u >= s.nx) continue;
        atomicAdd(g + 2 * ((size_t)v * s.nx + u) + (f & 1), val);
    }
}

__global__ __launch_bounds__(256) void k_fold_slots(int nsum, const double *__restrict__ wslots,
                                                    const unsigned long long *__restrict__ skslots,
                                                    double *sumwt, unsigned long long *nskipped) {
    // block b < nsum: sumwt entry b; block nsum: the skip count
    const int b = blockIdx.x;
    double sw = 0.0;
    unsigned long long sk = 0;
    for (int i = threadIdx.x; i < kSlots; i += 256) {
        if (b < nsum) sw += wslots[(size_t)i * nsum + b];
        else sk += skslots[i];
    }
    __shared__ double rw[256];
    __shared__ unsigned long long rk[256];
    rw[threadIdx.x] = sw;
    rk[threadIdx.x] = sk;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            rw[threadIdx.x] += rw[threadIdx.x + o];
            rk[threadIdx.x] += rk[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (b < nsum && sumwt) sumwt[b] += rw[0];
        if (b == nsum && nskipped) *nskipped += rk[0];
    }
}

__global__ __launch_bounds__(kThreads) void k_degrid_cf(Shape s, const int32_t *__restrict__ pu,
                                                        const int32_t *__restrict__ pv,
                                                        const int32_t *__restrict__ pwc,
                                                        const int32_t *__restrict__ pdu,
                                                        const int32_t *__restrict__ pdv,
                                                        const int32_t *__restrict__ vis_to_im,
                                                        const double2 *__restrict__ grid,
                                                        const double2 *__restrict__ cf,
                                                        double2 *vis_out,
                                                        unsigned long long *skslots) {
    __shared__ unsigned long long s_skip;
    if (threadIdx.x == 0) s_skip = 0;
    __syncthreads();
    const int chan = blockIdx.y;
    const int imchan = vis_to_im[chan];
    const int lane = threadIdx.x & 63;
    const int taps = s.gv * s.gu;
    const int dv = s.gv / 2, du = s.gu / 2;
    const int64_t row = blockIdx.x * (int64_t)(kThreads / 64) + (threadIdx.x >> 6);
    if (row < s.nrow) {
        const size_t m = (size_t)chan * s.nrow + row;
        const int u0 = pu[m], v0 = pv[m];
        const bool ok = window_ok(s, u0, v0);
        if (!ok && lane == 0) atomicAdd(&s_skip, (unsigned long long)s.npol);
        const int iw = pwc[m], idu = pdu[m], idv = pdv[m];
        for (int p = 0; p < s.npol; ++p) {
            double sr = 0.0, si = 0.0;
            if (ok) {
                const double2 *sub = cf + cf_index(s, imchan, p, iw, idv, idu) * taps;
                const double2 *g = grid + ((size_t)imchan * s.npol + p) * s.ny * s.nx;
                for (int t = lane; t < taps; t += 64) {
                    const int iv = t / s.gu, iu = t - (t / s.gu) * s.gu;
                    const double2 c = sub[t];
                    const double2 a = g[(size_t)(v0 - dv + iv) * s.nx + (u0 - du + iu)];
                    sr += a.x * c.x - a.y * c.y;
                    si += a.x * c.y + a.y * c.x;
                }
                for (int o = 32; o > 0; o >>= 1) {
                    sr += __shfl_xor(sr, o);
                    si += __shfl_xor(si, o);
                }
            }
            if (lane == 0) vis_out[((size_t)row * s.nchan + chan) * s.npol + p] = make_double2(sr, si);
        }
    }
    __syncthreads();
    // skip counts go to kSlots partial sums, folded by k_fold_slots (nsum = 0)
    if (threadIdx.x == 0 && s_skip) atomicAdd(&skslots[blockIdx.x & (kSlots - 1)], s_skip);
}

static Shape make_shape(int64_t nrow, int nchan, int npol, int cf_nchan, int nw, int ndv, int ndu,
                        int gv, int gu, int g_nchan, int ny, int nx) {
    SDP_REQUIRE(nrow >= 0 && nchan > 0 && npol > 0 && npol <= kMaxPol, "bad visibility shape");
    SDP_REQUIRE(gv > 0 && gu > 0 && gv % 2 == 0 && gu % 2 == 0,
                "convolution function support must be even (gridding.py:199-201)");
    SDP_REQUIRE(cf_nchan >= g_nchan && nw > 0 && ndv > 0 && ndu > 0, "bad convolution function shape");
    SDP_REQUIRE(ny > 0 && nx > 0 && g_nchan > 0, "bad grid shape");
    return Shape{nrow, nchan, npol, cf_nchan, nw, ndv, ndu, gv, gu, g_nchan, ny, nx};
}

}  // namespace cfgrid
}  // namespace sdp

extern "C" {

int sdp_hip_grid_cf(int64_t nrowvis, int nchan_vis, int npol, const int32_t *pu,
                    const int32_t *pv, const int32_t *pwc, const int32_t *pdu,
                    const int32_t *pdv, const int32_t *vis_to_im, const void *vis,
                    const double *wt, const void *cf, int cf_nchan, int nw, int ndv, int ndu,
                    int gv, int gu, void *grid, int g_nchan, int ny, int nx, double *sumwt,
                    int64_t *nskipped, void *stream, char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    return guarded(errbuf, errbuf_len, [&] {
        const cfgrid::Shape s = cfgrid::make_shape(nrowvis, nchan_vis, npol, cf_nchan, nw, ndv,
                                                   ndu, gv, gu, g_nchan, ny, nx);
        if (nrowvis == 0) return;
        SDP_REQUIRE(pu && pv && pwc && pdu && pdv && vis_to_im && vis && wt && cf && grid,
                    "null pointer argument");
        const hipStream_t st = as_stream(stream);
        const int nsum = g_nchan * npol;
        double *wslots = scratch<double>("cf_wslots", (size_t)cfgrid::kSlots * nsum);
        auto *skslots = scratch<unsigned long long>("cf_skslots", cfgrid::kSlots);
        SDP_HIP_CHECK(hipMemsetAsync(wslots, 0, sizeof(double) * cfgrid::kSlots * nsum, st));
        SDP_HIP_CHECK(hipMemsetAsync(skslots, 0, sizeof(unsigned long long) * cfgrid::kSlots, st));
        const size_t lds = (size_t)(cfgrid::kTile + gv - 1) * (cfgrid::kTile + gu - 1) *
                           sizeof(double2);
        const int64_t nent = nrowvis * (int64_t)nchan_vis;
        if (lds <= cfgrid::kMaxTileLds && nent < (int64_t)0xffffffffll) {
            // entries sorted by (image channel, 16x16 tile), LDS-tile accumulation
            const int ntx = (nx + cfgrid::kTile - 1) / cfgrid::kTile;
            const int nty = (ny + cfgrid::kTile - 1) / cfgrid::kTile;
            const int ntiles = ntx * nty;
            const int64_t nkeys = (int64_t)ntiles * g_nchan;
            SDP_REQUIRE(nkeys < (int64_t)0x7fffffff, "grid too large for the tile sort");
            auto *cnt = scratch<unsigned>("cf_cnt", nkeys + 1);
            auto *offs = scratch<unsigned>("cf_offs", nkeys + 1);
            auto *nit = scratch<unsigned>("cf_nit", nkeys + 1);
            auto *ioffs = scratch<unsigned>("cf_ioffs", nkeys + 1);
            auto *rk = scratch<unsigned>("cf_rank", nent);
            auto *order = scratch<uint32_t>("cf_order", nent);
            SDP_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(unsigned) * (nkeys + 1), st));
            SDP_HIP_CHECK(hipMemsetAsync(nit + nkeys, 0, sizeof(unsigned), st));
            const dim3 eb((unsigned)((nrowvis + cfgrid::kThreads - 1) / cfgrid::kThreads),
                          nchan_vis);
            cfgrid::k_cf_count<<<eb, cfgrid::kThreads, 0, st>>>(s, ntx, ntiles, pu, pv, vis_to_im,
                                                                wt, cnt, rk, wslots, skslots);
            size_t tb = 0;
            SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, offs,
                                                           (int)(nkeys + 1), st));
            void *tmp = scratch<char>("cf_scan_tmp", tb + 16);
            size_t tb2 = tb + 16;
            SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, cnt, offs, (int)(nkeys + 1), st));
            cfgrid::k_cf_scatter<<<eb, cfgrid::kThreads, 0, st>>>(s, ntx, ntiles, pu, pv, vis_to_im,
                                                                  offs, rk, order);
            cfgrid::k_cf_nitems<<<grid1d(nkeys, 256), 256, 0, st>>>(nkeys, offs, nit);
            tb2 = tb + 16;
            SDP_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, nit, ioffs, (int)(nkeys + 1), st));
            unsigned nitems = 0;
            SDP_HIP_CHECK(hipMemcpyAsync(&nitems, ioffs + nkeys, sizeof(unsigned),
                                         hipMemcpyDeviceToHost, st));
            SDP_HIP_CHECK(hipStreamSynchronize(st));
            if (nitems > 0) {
                auto *items = scratch<cfgrid::CfItem>("cf_items", nitems);
                cfgrid::k_cf_items<<<grid1d(nkeys, 256), 256, 0, st>>>(nkeys, offs, ioffs, items);
                cfgrid::k_cf_tile<<<dim3(nitems, npol), 64, lds, st>>>(
                    s, ntx, ntiles, items, order, pu, pv, pwc, pdu, pdv,
                    static_cast<const double2 *>(vis), wt, static_cast<const double2 *>(cf),
                    static_cast<double2 *>(grid));
            }
        } else {
            const dim3 blocks((unsigned)((nrowvis + 3) / 4), nchan_vis);
            cfgrid::k_grid_cf<<<blocks, cfgrid::kThreads, 0, st>>>(
                s, pu, pv, pwc, pdu, pdv, vis_to_im, static_cast<const double2 *>(vis), wt,
                static_cast<const double2 *>(cf), static_cast<double2 *>(grid), wslots, skslots);
        }
        cfgrid::k_fold_slots<<<nsum + 1, 256, 0, st>>>(
            nsum, wslots, skslots, sumwt, reinterpret_cast<unsigned long long *>(nskipped));
        SDP_HIP_CHECK(hipGetLastError());
    });
}

int sdp_hip_degrid_cf(int64_t nrowvis, int nchan_vis, int npol, const int32_t *pu,
                      const int32_t *pv, const int32_t *pwc, const int32_t *pdu,
                      const int32_t *pdv, const int32_t *vis_to_im, const void *grid,
                      int g_nchan, int ny, int nx, const void *cf, int cf_nchan, int nw, int ndv,
                      int ndu, int gv, int gu, void *vis_out, int64_t *nskipped, void *stream,
                      char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    return guarded(errbuf, errbuf_len, [&] {
        const cfgrid::Shape s = cfgrid::make_shape(nrowvis, nchan_vis, npol, cf_nchan, nw, ndv,
                                                   ndu, gv, gu, g_nchan, ny, nx);
        if (nrowvis == 0) return;
        SDP_REQUIRE(pu && pv && pwc && pdu && pdv && vis_to_im && grid && cf && vis_out,
                    "null pointer argument");
        const hipStream_t st = as_stream(stream);
        auto *skslots = scratch<unsigned long long>("cfd_skslots", cfgrid::kSlots);
        SDP_HIP_CHECK(hipMemsetAsync(skslots, 0, sizeof(unsigned long long) * cfgrid::kSlots, st));
        const dim3 blocks((unsigned)((nrowvis + 3) / 4), nchan_vis);
        cfgrid::k_degrid_cf<<<blocks, cfgrid::kThreads, 0, st>>>(
            s, pu, pv, pwc, pdu, pdv, vis_to_im, static_cast<const double2 *>(grid),
            static_cast<const double2 *>(cf), static_cast<double2 *>(vis_out), skslots);
        if (nskipped)
            cfgrid::k_fold_slots<<<1, 256, 0, st>>>(0, nullptr, skslots, nullptr,
                                                   reinterpret_cast<unsigned long long *>(nskipped));
        SDP_HIP_CHECK(hipGetLastError());
    });
}

}  // extern "C"
