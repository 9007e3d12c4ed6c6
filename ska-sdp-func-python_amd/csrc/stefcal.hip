// Batched antenna-gain solve by iterative substitution ("StefCal") for
// gfx950: sdp_hip_solve_gains, replacing the numpy loops of the reference's
// solve_gaintable inner solvers (src/ska_sdp_func_python/calibration/
// solvers.py:148-539).
//
// A "solve" is one gain-table row; it holds nchan x ncomp independent
// sub-problems (ncomp = 1 scalar, 4 for the 2x2 element-wise matrix forms)
// that share one convergence test, exactly as the reference's
// change = max|g - g_last| over antennas AND channels (solvers.py:268, :427).
//
// Device layout (fp32 storage, fp64 arithmetic):
//   x, w   [solve][chan][comp][dense]  normalised point-source vis/weight in
//          the dense column-block baseline layout (dense_off below)
//   g, gw  [solve][chan][comp][antenna]   current gains / gain weights
// Per iteration two launches: k_iter (one 256-thread workgroup per active
// sub-problem: baselines streamed once with lane = station a2, register sums
// for a2 and lane-reduced sums for a1 added to LDS with ds_add_f64, then the
// substitution, phase normalisation, refant rotation, damping and the
// per-row max change) and k_commit (row-level convergence).  The host polls
// the converged-row count every few iterations.
#include <cmath>
#include <vector>

#include <type_traits>

#include "sdp_common.h"

namespace sdp {
namespace stefcal {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxAnts = 1024;

enum Mode { kScalar = 0, kMatrix = 1, kNoCross = 2 };

struct Dims {
    int nsolve, nants, nbl, nchan, npol, ncomp, nrec, mode;
    size_t nd;  // dense entries per sub-solve (dense_size)
    int phase_only, refant;
    double tol, damping;
};

__device__ __forceinline__ size_t sub_index(const Dims &d, int s, int chan, int comp) {
    return ((size_t)s * d.nchan + chan) * d.ncomp + comp;
}

// input pol feeding component `comp`, or -1 (component has no data)
__device__ __forceinline__ int comp_pol(const Dims &d, int comp) {
    if (d.mode == kScalar) return 0;
    if (d.mode == kMatrix) return comp;
    if (comp == 1 || comp == 2) return -1;  // no cross-hand data
    return d.npol == 2 ? (comp == 0 ? 0 : 1) : comp;
}

__device__ __forceinline__ unsigned long long dbits(double v) {
    return (unsigned long long)__double_as_longlong(v);
}

// max over the row of wb (solvers.py:167: xwt / max(xwt))
__global__ void k_rowmax(Dims d, const double *__restrict__ wb, unsigned long long *rowmax) {
    const size_t per = (size_t)d.nbl * d.nchan * d.npol;
    const int s = blockIdx.y;
    double m = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < per;
         i += (size_t)gridDim.x * blockDim.x)
        m = fmax(m, fabs(wb[(size_t)s * per + i]));
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0 && m > 0.0) atomicMax(&rowmax[s], dbits(m));
}

// x = xb / wb, w = wb / max  (masked where wb <= 0), into [s][chan][comp][dense]:
// an LDS-tiled transpose of each solve's [bl][chan*pol] block (coalesced
// reads along chan*pol, coalesced writes along bl).  Tile kTr x kTr with
// kTr x 8 threads: 64 when a solve has >= 64 (chan, comp) columns (C5's 256
// channels: 6.03 -> 4.83 ms per 4096-solve batch against 32,
// profiles/r02_fill_tile_ab.txt), else 32 so that narrow solves (one channel,
// 1-4 comps) leave fewer load lanes idle.
template <int kTr>
__global__ __launch_bounds__(kTr * 8) void k_fill(Dims d, const double2 *__restrict__ xb,
                                              const double *__restrict__ wb,
                                              const unsigned long long *__restrict__ rowmax,
                                              const int32_t *__restrict__ dpos, float2 *x,
                                              float *w) {
    __shared__ float2 sx[kTr][kTr + 1];
    __shared__ float sw[kTr][kTr + 1];
    const int s = blockIdx.z;
    const int b0 = blockIdx.x * kTr, c0 = blockIdx.y * kTr;  // c = chan * ncomp + comp
    const int ncc = d.nchan * d.ncomp;
    const double mx = __longlong_as_double((long long)rowmax[s]);
    for (int r = threadIdx.y; r < kTr; r += 8) {
        const int b = b0 + r, c = c0 + threadIdx.x;
        float2 xv = make_float2(0.0f, 0.0f);
        float wv = 0.0f;
        if (b < d.nbl && c < ncc) {
            const int chan = c / d.ncomp, comp = c - chan * d.ncomp;
            const int p = comp_pol(d, comp);
            if (p >= 0) {
                const size_t src = (((size_t)s * d.nbl + b) * d.nchan + chan) * d.npol + p;
                const double ww = wb[src];
                if (ww > 0.0 && mx > 0.0) {
                    const double2 xx = xb[src];
                    xv = make_float2((float)(xx.x / ww), (float)(xx.y / ww));
                    wv = (float)(ww / mx);
                }
            }
        }
        sx[r][threadIdx.x] = xv;
        sw[r][threadIdx.x] = wv;
    }
    __syncthreads();
    for (int r = threadIdx.y; r < kTr; r += 8) {
        const int c = c0 + r, b = b0 + threadIdx.x;
        const int dp = b < d.nbl ? dpos[b] : -1;
        if (dp >= 0 && c < ncc) {
            const size_t dst = ((size_t)s * ncc + c) * d.nd + dp;
            x[dst] = sx[threadIdx.x][r];
            w[dst] = sw[threadIdx.x][r];
        }
    }
}

// gains [s][ant][chan][r1][r2] (c128) -> working [s][chan][comp][ant]
__global__ void k_load_gains(Dims d, const double2 *__restrict__ gin,
                             const double *__restrict__ gwin, double2 *g, double *gw) {
    const size_t total = (size_t)d.nsolve * d.nchan * d.ncomp * d.nants;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int a = (int)(i % d.nants);
        const size_t sub = i / d.nants;
        const int comp = (int)(sub % d.ncomp);
        const int chan = (int)((sub / d.ncomp) % d.nchan);
        const int s = (int)(sub / ((size_t)d.ncomp * d.nchan));
        const size_t src = (((size_t)s * d.nants + a) * d.nchan + chan) * d.ncomp + comp;
        double2 v = gin[src];
        if (d.mode != kScalar && (comp == 1 || comp == 2)) v = make_double2(0.0, 0.0);  // :418-419
        g[i] = v;
        gw[i] = gwin[src];  // returned unchanged when no iteration runs
    }
}

#ifndef SDP_STEFCAL_PERMLANE
#define SDP_STEFCAL_PERMLANE 1
#endif
// a + b after exchanging the upper half of `a` with the lower half of `b`
// (H = 32: wave halves, v_permlane32_swap; H = 16: odd / even 16-lane rows,
// v_permlane16_swap): lanes with bit H clear get a[l] + a[l ^ H], lanes with
// it set b[l] + b[l ^ H]
template <int H>
__device__ __forceinline__ double swap_sum(double a, double b) {
    const unsigned alo = (unsigned)__double_as_longlong(a),
                   ahi = (unsigned)((unsigned long long)__double_as_longlong(a) >> 32);
    const unsigned blo = (unsigned)__double_as_longlong(b),
                   bhi = (unsigned)((unsigned long long)__double_as_longlong(b) >> 32);
    unsigned r0a, r0b, r1a, r1b;
    if constexpr (H == 32) {
        const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
        r0a = lo[0]; r0b = lo[1]; r1a = hi[0]; r1b = hi[1];
    } else {
        const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
        r0a = lo[0]; r0b = lo[1]; r1a = hi[0]; r1b = hi[1];
    }
    const double na = __longlong_as_double((long long)(((unsigned long long)r1a << 32) | r0a));
    const double nb = __longlong_as_double((long long)(((unsigned long long)r1b << 32) | r0b));
    return na + nb;
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// Dense column-block layout of a sub-solve's canonical baselines (a1 < a2):
// block c holds antennas a2 in [64c, 64c + 64) against rows a1 in
// [0, rows(c)), rows(c) = min(64c + 63, na - 1), row-major with 64 entries
// per row (entry = a2 - 64c).  Entries with no baseline (a1 >= a2 inside the
// diagonal block, flagged or absent baselines) carry weight 0.  About 12 %
// padding at 512 stations buys a layout in which lane = a2 for a whole block:
// the a2-side sums stay in registers and every row is one coalesced 768-B
// read.
__host__ __device__ __forceinline__ int dense_rows(int c, int na) {
    return min(64 * c + 63, na - 1);
}
__host__ __device__ __forceinline__ size_t dense_off(int c, int na) {
    size_t o = 0;
    for (int k = 0; k < c; ++k) o += (size_t)dense_rows(k, na) * 64;
    return o;
}
__host__ __device__ __forceinline__ size_t dense_size(int na) {
    return dense_off((na + 63) / 64, na);
}

// canonical baseline b -> its dense entry
__global__ void k_dense_pos(int na, int nbl, const int32_t *__restrict__ row_start,
                            const int32_t *__restrict__ ant2, int32_t *dpos) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbl) return;
    int lo = 0, hi = na;  // largest a1 with row_start[a1] <= b
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (row_start[mid] <= b) lo = mid;
        else hi = mid;
    }
    const int a1 = lo, a2 = ant2[b], c = a2 >> 6;
    // not canonical (a2 <= a1) or out of range: dropped
    dpos[b] = (a2 > a1 && a2 < na) ? (int32_t)(dense_off(c, na) + (size_t)a1 * 64 + (a2 & 63)) : -1;
}

// One 256-thread workgroup per sub-solve.  Wave w takes column blocks in
// snake order (w, 2W-1-w, 2W+w, ...) so the triangle's block sizes balance.
// Lane = a2: per row a1 of the block the lane adds g1 conj(x) w and |g1|^2 w
// to its register sums (antenna a2's side) and forms g2 x w, |g2|^2 w for
// antenna a1's side; those are summed over the 64 lanes for 8 rows at a time
// by one reduce-scatter butterfly and added to the shared LDS sums with
// ds_add_f64 (one per row and block; the register sums once per block).
// Rows are loaded 8 ahead of use.
constexpr int kRowsInFlight = 8;
__global__ __launch_bounds__(kThreads) void k_iter(Dims d, const float2 *__restrict__ x,
                                                   const float *__restrict__ w,
                                                   const double2 *__restrict__ g, double2 *gnext,
                                                   double *gwnext, const int32_t *__restrict__ done,
                                                   unsigned long long *change) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int sub = blockIdx.x;
    const int s = sub / (d.ncomp * d.nchan);
    if (done[s]) return;
    const int na = d.nants;
    double2 *gl = reinterpret_cast<double2 *>(lds);      // [na]
    double2 *top = gl + na;                              // [na]
    double *gp = reinterpret_cast<double *>(top + na) + na;  // [na] |g|^2 (after bot)
    double *bot = reinterpret_cast<double *>(top + na);  // [na]
    const size_t gbase = (size_t)sub * na;
    const size_t xbase = (size_t)sub * d.nd;
    for (int a = threadIdx.x; a < na; a += kThreads) {
        const double2 ga = g[gbase + a];
        gl[a] = ga;
        gp[a] = ga.x * ga.x + ga.y * ga.y;
        top[a] = make_double2(0.0, 0.0);
        bot[a] = 0.0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR block math
    constexpr int K = kRowsInFlight;
    static_assert(K == 8, "the reduce-scatter below sums 8 rows");
    const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
    const int nblk = (na + 63) / 64;
    for (int k = 0; k * kWaves < nblk; ++k) {
        const int c = (k & 1) ? (k + 1) * kWaves - 1 - wave : k * kWaves + wave;
        if (c >= nblk) continue;
        const int a2 = 64 * c + lane;
        const double2 g2 = a2 < na ? gl[a2] : make_double2(0.0, 0.0);
        const double p2 = g2.x * g2.x + g2.y * g2.y;
        double ax = 0.0, ay = 0.0, ab = 0.0;
        const int rows = dense_rows(c, na);
        // buffer loads: the block base in the descriptor, the row offset in
        // an SGPR, the lane offset a constant VGPR (no per-load 64-bit
        // address arithmetic); rows past the block end read the last row and
        // are masked to weight 0
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(x + xbase + dense_off(c, na)), 0, rows * 64 * (int)sizeof(float2), 0x00020000);
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(w + xbase + dense_off(c, na)), 0, rows * 64 * (int)sizeof(float), 0x00020000);
        auto load = [&](int r0, float2 (&bx)[K], float (&bw)[K]) {
#pragma unroll
            for (int u = 0; u < K; ++u) {
                const int r = min(r0 + u, rows - 1);
                const auto xv = __builtin_amdgcn_raw_buffer_load_b64(
                    rx, lane * (int)sizeof(float2), r * 64 * (int)sizeof(float2), 0);
                const float wl = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    rw, lane * (int)sizeof(float), r * 64 * (int)sizeof(float), 0));
                bx[u] = make_float2(__uint_as_float(xv[0]), __uint_as_float(xv[1]));
                bw[u] = r0 + u < rows ? wl : 0.0f;
            }
        };
        auto process = [&](int r0, const float2 (&bx)[K], const float (&bw)[K]) {
            double pr[K], pi[K], pb[K];
#pragma unroll
            for (int u = 0; u < K; ++u) {
                const double2 g1 = gl[min(r0 + u, na - 1)];
                const double p1 = gp[min(r0 + u, na - 1)];
                const double wv = bw[u];
                const float2 xv = wv != 0.0 ? bx[u] : make_float2(0.0f, 0.0f);
                const double xr = xv.x * wv, xi = xv.y * wv;
                // antenna a2 (i = a1): x[a1,a2] = conj(x_b)
                ax += g1.x * xr + g1.y * xi;
                ay += g1.y * xr - g1.x * xi;
                ab += p1 * wv;
                // antenna a1 (i = a2): x[a2,a1] = x_b
                pr[u] = g2.x * xr - g2.y * xi;
                pi[u] = g2.x * xi + g2.y * xr;
                pb[u] = p2 * wv;
            }
            // reduce-scatter over the 64 lanes: after the xor-32/16/8 halvings
            // lane l holds row (l >> 3) & 7 summed over 8 lanes; xor 4/2/1
            // finish it
            double q4r[4], q4i[4], q4b[4];
            double q2r[2], q2i[2], q2b[2];
#if SDP_STEFCAL_PERMLANE
            // the two first halvings as VALU lane swaps (gfx950
            // v_permlane32_swap / v_permlane16_swap): after swapping the upper
            // half of A = row i with the lower half of B = row i + 4, A + B is
            // row i on lanes 0-31 and row i + 4 on lanes 32-63
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                q4r[i] = swap_sum<32>(pr[i], pr[i + 4]);
                q4i[i] = swap_sum<32>(pi[i], pi[i + 4]);
                q4b[i] = swap_sum<32>(pb[i], pb[i + 4]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                q2r[i] = swap_sum<16>(q4r[i], q4r[i + 2]);
                q2i[i] = swap_sum<16>(q4i[i], q4i[i + 2]);
                q2b[i] = swap_sum<16>(q4b[i], q4b[i + 2]);
            }
#else
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                q4r[i] = (b5 ? pr[i + 4] : pr[i]) + __shfl_xor(b5 ? pr[i] : pr[i + 4], 32);
                q4i[i] = (b5 ? pi[i + 4] : pi[i]) + __shfl_xor(b5 ? pi[i] : pi[i + 4], 32);
                q4b[i] = (b5 ? pb[i + 4] : pb[i]) + __shfl_xor(b5 ? pb[i] : pb[i + 4], 32);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                q2r[i] = (b4 ? q4r[i + 2] : q4r[i]) + __shfl_xor(b4 ? q4r[i] : q4r[i + 2], 16);
                q2i[i] = (b4 ? q4i[i + 2] : q4i[i]) + __shfl_xor(b4 ? q4i[i] : q4i[i + 2], 16);
                q2b[i] = (b4 ? q4b[i + 2] : q4b[i]) + __shfl_xor(b4 ? q4b[i] : q4b[i + 2], 16);
            }
#endif
            double tr = (b3 ? q2r[1] : q2r[0]) + __shfl_xor(b3 ? q2r[0] : q2r[1], 8);
            double ti = (b3 ? q2i[1] : q2i[0]) + __shfl_xor(b3 ? q2i[0] : q2i[1], 8);
            double tb = (b3 ? q2b[1] : q2b[0]) + __shfl_xor(b3 ? q2b[0] : q2b[1], 8);
#pragma unroll
            for (int m = 4; m > 0; m >>= 1) {
                tr += __shfl_xor(tr, m);
                ti += __shfl_xor(ti, m);
                tb += __shfl_xor(tb, m);
            }
            // row of lane l: bit 5 -> +4, bit 4 -> +2, bit 3 -> +1
            const int a1 = r0 + ((lane >> 3) & 7);
            if ((lane & 7) == 0 && a1 < rows && tb != 0.0) {
                atomicAdd(&top[a1].x, tr);
                atomicAdd(&top[a1].y, ti);
                atomicAdd(&bot[a1], tb);
            }
        };
        // two register buffers in ping-pong (a copy between them would wait
        // for the prefetch it is meant to overlap)
        float2 xa[K], xb_[K];
        float wa[K], wb_[K];
        // (sched_barrier: keep each prefetch issued ahead of the other
        // buffer's arithmetic instead of sunk below it)
        load(0, xa, wa);
        for (int r0 = 0; r0 < rows; r0 += 2 * K) {
            load(r0 + K, xb_, wb_);
            __builtin_amdgcn_sched_barrier(0);
            process(r0, xa, wa);
            load(r0 + 2 * K, xa, wa);
            __builtin_amdgcn_sched_barrier(0);
            if (r0 + K < rows) process(r0 + K, xb_, wb_);
        }
        if (a2 < na && ab != 0.0) {
            atomicAdd(&top[a2].x, ax);
            atomicAdd(&top[a2].y, ay);
            atomicAdd(&bot[a2], ab);
        }
    }
    __syncthreads();
    // substitution (solvers.py:308-319 / :466-477), new gains into top[0]
    for (int a = threadIdx.x; a < na; a += kThreads) {
        double tx = 0.0, ty = 0.0, bb = 0.0;
        tx = top[a].x;
        ty = top[a].y;
        bb = bot[a];
        double2 ng = bb > 0.0 ? make_double2(tx / bb, ty / bb) : make_double2(0.0, 0.0);
        if (d.phase_only) {
            const double m = sqrt(ng.x * ng.x + ng.y * ng.y);
            if (m > 0.0) ng = make_double2(ng.x / m, ng.y / m);
        }
        top[a] = ng;
        bot[a] = (d.mode == kScalar) ? (bb > 0.0 ? bb : 0.0) : bb;
    }
    __syncthreads();
    // refant rotation (scalar only, :265-266): multiply by exp(-i angle(g_ref))
    double2 rot = make_double2(1.0, 0.0);
    if (d.mode == kScalar) {
        const double2 gr = top[d.refant];
        const double m = sqrt(gr.x * gr.x + gr.y * gr.y);
        if (m > 0.0) rot = make_double2(gr.x / m, -gr.y / m);
    }
    double cmax = 0.0;
    for (int a = threadIdx.x; a < na; a += kThreads) {
        const double2 gold = gl[a];
        double2 ng = cmul(top[a], rot);
        double2 out;
        double ch;
        if (d.mode == kScalar) {  // damp, then change (:267-268)
            out = make_double2((1.0 - d.damping) * ng.x + d.damping * gold.x,
                               (1.0 - d.damping) * ng.y + d.damping * gold.y);
            ch = hypot(out.x - gold.x, out.y - gold.y);
        } else {  // change, then average (:427-428)
            ch = hypot(ng.x - gold.x, ng.y - gold.y);
            out = make_double2(0.5 * (ng.x + gold.x), 0.5 * (ng.y + gold.y));
        }
        cmax = fmax(cmax, ch);
        gnext[gbase + a] = out;
        gwnext[gbase + a] = bot[a];
    }
    for (int o = 32; o > 0; o >>= 1) cmax = fmax(cmax, __shfl_xor(cmax, o));
    if (lane == 0) atomicMax(&change[s], dbits(cmax));
}

__global__ void k_commit(Dims d, int it, double2 *g, double *gw, const double2 *__restrict__ gnext,
                         const double *__restrict__ gwnext, int32_t *done,
                         const unsigned long long *__restrict__ change_cur,
                         unsigned long long *change_next, int *ndone) {
    const size_t per = (size_t)d.nchan * d.ncomp * d.nants;
    const size_t total = (size_t)d.nsolve * per;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(i / per);
        if (done[s]) continue;
        const double ch = __longlong_as_double((long long)change_cur[s]);
        double2 v = gnext[i];
        const bool conv = ch < d.tol;
        if (conv && d.mode == kScalar && d.phase_only) {  // :270-272
            const double m = sqrt(v.x * v.x + v.y * v.y);
            if (m > 0.0) v = make_double2(v.x / m, v.y / m);
        }
        g[i] = v;
        gw[i] = gwnext[i];
    }
    // row bookkeeping: one thread per solve
    for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < (size_t)d.nsolve;
         s += (size_t)gridDim.x * blockDim.x) {
        change_next[s] = 0ull;
    }
}

__global__ void k_mark_done(Dims d, int it, int32_t *done, const unsigned long long *change_cur,
                            int *ndone) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= d.nsolve || done[s]) return;
    const double ch = __longlong_as_double((long long)change_cur[s]);
    if (ch < d.tol) {
        done[s] = it + 1;
        atomicAdd(ndone, 1);
    }
}

// rows that did not converge: phase-only normalisation (:280-282), niter+1
__global__ void k_finish(Dims d, int niter, double2 *g, const int32_t *__restrict__ done,
                         int32_t *niter_out) {
    const size_t per = (size_t)d.nchan * d.ncomp * d.nants;
    const size_t total = (size_t)d.nsolve * per;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(i / per);
        if (done[s]) continue;
        if (d.mode == kScalar && d.phase_only) {
            double2 v = g[i];
            const double m = sqrt(v.x * v.x + v.y * v.y);
            if (m > 0.0) g[i] = make_double2(v.x / m, v.y / m);
        }
    }
    for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < (size_t)d.nsolve;
         s += (size_t)gridDim.x * blockDim.x)
        niter_out[s] = done[s] ? done[s] : niter + 1;
}

// residual (solvers.py:481-539): sqrt(sum w |x - g_a1 conj(g_a2)|^2 / sum w)
__global__ __launch_bounds__(kThreads) void k_residual(Dims d, const float2 *__restrict__ x,
                                                       const float *__restrict__ w,
                                                       const double2 *__restrict__ g,
                                                       double *residual) {
    __shared__ double red[2][kWaves];
    const int sub = blockIdx.x;
    const int na = d.nants;
    const size_t gbase = (size_t)sub * na;
    const size_t xbase = (size_t)sub * d.nd;
    double r = 0.0, sw = 0.0;
    const int nblk = (na + 63) / 64;
    for (int c = 0; c < nblk; ++c) {
        const int a2 = 64 * c + (threadIdx.x & 63);
        if (a2 >= na) continue;
        const double2 g2 = g[gbase + a2];
        const size_t off = xbase + dense_off(c, na) + (threadIdx.x & 63);
        for (int a1 = threadIdx.x >> 6; a1 < dense_rows(c, na); a1 += kWaves) {
            const double wv = w[off + (size_t)a1 * 64];
            if (wv == 0.0) continue;
            const double2 g1 = g[gbase + a1];
            const double mr = g1.x * g2.x + g1.y * g2.y;  // g1 conj(g2)
            const double mi = g1.y * g2.x - g1.x * g2.y;
            const float2 xv = x[off + (size_t)a1 * 64];
            const double er = xv.x - mr, ei = xv.y - mi;
            r += wv * (er * er + ei * ei);
            sw += wv;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        r += __shfl_xor(r, o);
        sw += __shfl_xor(sw, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = r;
        red[1][threadIdx.x >> 6] = sw;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double rr = 0.0, ss = 0.0;
        for (int k = 0; k < kWaves; ++k) {
            rr += red[0][k];
            ss += red[1][k];
        }
        residual[sub] = ss > 0.0 ? sqrt(rr / ss) : 0.0;
    }
}

// working [s][chan][comp][ant] -> outputs [s][ant][chan][comp]
__global__ void k_store(Dims d, const double2 *__restrict__ g, const double *__restrict__ gw,
                        double2 *gout, double *gwout) {
    const size_t total = (size_t)d.nsolve * d.nchan * d.ncomp * d.nants;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int a = (int)(i % d.nants);
        const size_t sub = i / d.nants;
        const int comp = (int)(sub % d.ncomp);
        const int chan = (int)((sub / d.ncomp) % d.nchan);
        const int s = (int)(sub / ((size_t)d.ncomp * d.nchan));
        const size_t o = (((size_t)s * d.nants + a) * d.nchan + chan) * d.ncomp + comp;
        gout[o] = g[i];
        gwout[o] = gw[i];
    }
}

static unsigned blocks_for(size_t n) {
    size_t b = (n + 255) / 256;
    return (unsigned)std::max<size_t>(1, std::min<size_t>(b, 65535));
}

static void solve(const Dims &d, const int32_t *row_start, const int32_t *ant2, const void *xb,
                  const double *wb, void *gain, double *gwt, double *residual,
                  int32_t *niter_out, int niter, hipStream_t st) {
    const size_t nsub = (size_t)d.nsolve * d.nchan * d.ncomp;
    const size_t nx = nsub * d.nd;
    const size_t ng = nsub * d.nants;
    float2 *x = scratch<float2>("sc_x", std::max<size_t>(nx, 1));
    float *w = scratch<float>("sc_w", std::max<size_t>(nx, 1));
    double2 *g = scratch<double2>("sc_g", ng);
    double2 *gn = scratch<double2>("sc_gn", ng);
    double *gw = scratch<double>("sc_gw", ng);
    double *gwn = scratch<double>("sc_gwn", ng);
    auto *rowmax = scratch<unsigned long long>("sc_rowmax", d.nsolve);
    auto *change = scratch<unsigned long long>("sc_change", 2 * (size_t)d.nsolve);
    int32_t *done = scratch<int32_t>("sc_done", d.nsolve);
    int *ndone = scratch<int>("sc_ndone", 1);
    int32_t *dpos = scratch<int32_t>("sc_dpos", std::max(d.nbl, 1));
    SDP_HIP_CHECK(hipMemsetAsync(w, 0, nx * sizeof(float), st));  // padding entries: weight 0
    if (d.nbl > 0)
        k_dense_pos<<<(d.nbl + 255) / 256, 256, 0, st>>>(d.nants, d.nbl, row_start, ant2, dpos);
    SDP_HIP_CHECK(hipMemsetAsync(rowmax, 0, d.nsolve * sizeof(unsigned long long), st));
    SDP_HIP_CHECK(hipMemsetAsync(change, 0, 2 * (size_t)d.nsolve * sizeof(unsigned long long), st));
    SDP_HIP_CHECK(hipMemsetAsync(done, 0, d.nsolve * sizeof(int32_t), st));
    SDP_HIP_CHECK(hipMemsetAsync(ndone, 0, sizeof(int), st));

    const size_t per = (size_t)d.nbl * d.nchan * d.npol;
    k_rowmax<<<dim3(std::max<unsigned>(1, std::min<unsigned>(64, (unsigned)((per + 255) / 256))),
                    d.nsolve),
               256, 0, st>>>(d, wb, rowmax);
    auto fill = [&](auto tile) {
        constexpr int kTr = decltype(tile)::value;
        const dim3 grd((unsigned)((d.nbl + kTr - 1) / kTr),
                       (unsigned)((d.nchan * d.ncomp + kTr - 1) / kTr), (unsigned)d.nsolve);
        k_fill<kTr><<<grd, dim3(kTr, 8), 0, st>>>(d, static_cast<const double2 *>(xb), wb,
                                                  rowmax, dpos, x, w);
    };
    if (d.nchan * d.ncomp >= 64)
        fill(std::integral_constant<int, 64>{});
    else
        fill(std::integral_constant<int, 32>{});
    k_load_gains<<<blocks_for(ng), 256, 0, st>>>(d, static_cast<const double2 *>(gain), gwt, g,
                                                  gw);
    SDP_HIP_CHECK(hipGetLastError());

    const size_t lds = (size_t)d.nants * (2 * sizeof(double2) + 2 * sizeof(double));
    if (lds > 65536)
        SDP_HIP_CHECK(hipFuncSetAttribute((const void *)k_iter,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int it = 0;
    for (; it < niter; ++it) {
        unsigned long long *cur = change + (size_t)(it & 1) * d.nsolve;
        unsigned long long *nxt = change + (size_t)((it + 1) & 1) * d.nsolve;
        k_iter<<<(unsigned)nsub, kThreads, lds, st>>>(d, x, w, g, gn, gwn, done, cur);
        k_commit<<<blocks_for(ng), 256, 0, st>>>(d, it, g, gw, gn, gwn, done, cur, nxt, ndone);
        k_mark_done<<<(d.nsolve + 255) / 256, 256, 0, st>>>(d, it, done, cur, ndone);
        SDP_HIP_CHECK(hipGetLastError());
        if ((it & 3) == 3 || it == niter - 1) {
            int h = 0;
            SDP_HIP_CHECK(hipMemcpyAsync(&h, ndone, sizeof(int), hipMemcpyDeviceToHost, st));
            SDP_HIP_CHECK(hipStreamSynchronize(st));
            if (h >= d.nsolve) break;
        }
    }
    k_finish<<<blocks_for(ng), 256, 0, st>>>(d, niter, g, done, niter_out);
    k_residual<<<(unsigned)nsub, kThreads, 0, st>>>(d, x, w, g, residual);
    k_store<<<blocks_for(ng), 256, 0, st>>>(d, g, gw, static_cast<double2 *>(gain), gwt);
    SDP_HIP_CHECK(hipGetLastError());
}

}  // namespace stefcal
}  // namespace sdp

extern "C" int sdp_hip_solve_gains(int nsolve, int nants, int nbl, const int32_t *row_start,
                                   const int32_t *ant2, int nchan, int npol, int mode,
                                   const void *xb, const double *wb, void *gain, double *gwt,
                                   double *residual, int32_t *niter_out, int niter, double tol,
                                   int phase_only, int refant, double damping, void *stream,
                                   char *errbuf, size_t errbuf_len) {
    using namespace sdp;
    return guarded(errbuf, errbuf_len, [&] {
        SDP_REQUIRE(nsolve >= 0 && nants > 0 && nbl >= 0 && nchan > 0, "bad sizes");
        SDP_REQUIRE(nants <= stefcal::kMaxAnts, "at most 1024 antennas per solve");
        SDP_REQUIRE(mode >= 0 && mode <= 2, "mode must be 0 (scalar), 1 (matrix) or 2 (nocross)");
        SDP_REQUIRE(mode != 0 || npol == 1, "scalar mode needs npol == 1");
        SDP_REQUIRE(mode != 1 || npol == 4, "matrix mode needs npol == 4");
        SDP_REQUIRE(mode != 2 || npol == 2 || npol == 4, "nocross mode needs npol 2 or 4");
        SDP_REQUIRE(refant >= 0 && refant < nants, "refant out of range");
        SDP_REQUIRE(niter >= 0, "niter must be >= 0");
        if (nsolve == 0) return;
        SDP_REQUIRE(row_start && ant2 && xb && wb && gain && gwt && residual && niter_out,
                    "null pointer argument");
        stefcal::Dims d;
        d.nsolve = nsolve;
        d.nants = nants;
        d.nbl = nbl;
        d.nd = stefcal::dense_size(nants);
        d.nchan = nchan;
        d.npol = npol;
        d.mode = mode;
        d.ncomp = mode == 0 ? 1 : 4;
        d.nrec = mode == 0 ? 1 : 2;
        d.phase_only = phase_only;
        d.refant = refant;
        d.tol = tol;
        d.damping = damping;
        stefcal::solve(d, row_start, ant2, xb, wb, gain, gwt, residual, niter_out, niter,
                       as_stream(stream));
    });
}
