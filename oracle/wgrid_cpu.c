/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- never linked by the product path.
 *
 * Plain-C + OpenMP restatement of the w-stacking adjoint NUFFT (ms2dirty)
 * and of its adjoint, the forward NUFFT (dirty2ms), that the reference binds
 * through ducc0.wgridder (ducc0 0.27.0, poetry.lock:305-306; call sites
 * src/ska_sdp_func_python/imaging/ng.py:240-256 (invert, epsilon=1e-12,
 * double_precision_accumulation=True) and ng.py:99-129 (predict)).
 * ducc0 is not vendored under /root/reference and cannot be built or
 * installed here.  This file is (1) the full-size checker of the HIP path in
 * tests/ and (2) the CPU baseline of bench.py ("kind": "port").  The
 * algorithm is the one stated in oracle/nufft_oracle.py (wgrid_ms2dirty) and
 * SURVEY.md Appendix A:
 *
 *   ES kernel phi(t) = exp(beta (sqrt(1 - (2t/W)^2) - 1)), sigma = 2,
 *   W = ceil(-log10(eps/10)), beta = 2.30 W;
 *   w planes w_p = w0 + p dw with dw = 1/(2 tmax), vis pre-phased by
 *   exp(2 pi i w s0); per plane: grid, 2-D inverse FFT pruned to the npix
 *   window, multiply by exp(2 pi i w_p (n - 1 - s0)) and accumulate; finally
 *   divide by the kernel's Fourier transform in x, y and w and by n.
 *
 * Two precisions (argument `prec`):
 *   0  "single": fp32 taps and fp32 grid, W in [2, 8], epsilon floored at
 *      1e-7 -- the arithmetic the HIP path performs (matched-precision CPU
 *      baseline);
 *   1  "double": fp64 taps, fp64 grid and fp64 visibilities, W in [2, 16]
 *      (epsilon = 1e-12 gives W = 13, ~1e-12 kernel error) -- the reference's
 *      ducc0 call with double_precision_accumulation=True.
 *
 * Output is ducc0's convention: dirty[x * npix_y + y], l_x = (x - nx/2) px.
 *
 * Parallelism (load-balanced for concentrated uv coverage such as the
 * SKA-MID core, where a handful of cells take millions of samples): the
 * visibilities are counting-sorted by 32 x 32-cell tile; every tile's list is
 * cut into tasks of <= TASK visibilities; a task accumulates into a private
 * tile buffer (all its planes) and adds it into the resident planes under the
 * locks of the <= 4 tiles its halo reaches.  FFT rows/columns and the image
 * accumulation are OpenMP loops.
 *
 * Also here: exact direct sums at sampled pixels / rows (the definition ducc0
 * approximates to epsilon), used as the absolute anchor of the full-size
 * tests.
 */
#include <complex.h>
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#define C_LIGHT 299792458.0
#define TILE 32
#define TASK 16384
#define MAXW 16

typedef double complex cf64;

typedef struct {
    int W, nchan, ngx, ngy, ntr, ntc, do_w, nplanes;
    double beta, px, py, s0, dw, w0;
} Geo;

typedef struct {
    int ic, jc, p0;
    double fu, fv, fw, w;
} Coord;

static int kernel_support(double eps, int prec) {
    const double floor_eps = prec ? 1e-15 : 1e-7;
    const int wmax = prec ? MAXW : 8;
    if (eps < floor_eps) eps = floor_eps;
    int w = (int)ceil(-log10(eps / 10.0));
    return w < 2 ? 2 : (w > wmax ? wmax : w);
}

static double es(double t, int W, double beta) {
    double x = 2.0 * t / W, y = 1.0 - x * x;
    return y > 0.0 ? exp(beta * (sqrt(y) - 1.0)) : 0.0;
}

/* Phi(xi) = int_{-W/2}^{W/2} phi(t) cos(2 pi t xi) dt, 128-point Gauss-Legendre. */
static double gl_x[128], gl_w[128];
static int gl_ready = 0;
static void gauss_legendre(void) {
    if (gl_ready) return;
    const int n = 128;
    for (int i = 0; i < n; ++i) {
        double z = cos(M_PI * (i + 0.75) / (n + 0.5)), pp = 0.0;
        for (int it = 0; it < 100; ++it) {
            double p1 = 1.0, p2 = 0.0;
            for (int j = 0; j < n; ++j) {
                double p3 = p2;
                p2 = p1;
                p1 = ((2.0 * j + 1.0) * z * p2 - j * p3) / (j + 1);
            }
            pp = n * (z * p1 - p2) / (z * z - 1.0);
            double z1 = z;
            z = z1 - p1 / pp;
            if (fabs(z - z1) < 1e-15) break;
        }
        gl_x[i] = z;
        gl_w[i] = 2.0 / ((1.0 - z * z) * pp * pp);
    }
    gl_ready = 1;
}
static double es_fourier_quad(double xi, int W, double beta) {
    double s = 0.0;
    for (int i = 0; i < 128; ++i) {
        double t = 0.25 * W * (gl_x[i] + 1.0);
        s += 0.25 * W * gl_w[i] * es(t, W, beta) * cos(2.0 * M_PI * t * xi);
    }
    return 2.0 * s;
}

/* tabulated Phi on [0, 0.5] with 4-point Lagrange interpolation */
#define NTAB 8193
static double phi_tab[NTAB + 3];
static void phi_table(int W, double beta) {
    for (int i = 0; i < NTAB + 3; ++i) phi_tab[i] = es_fourier_quad((i - 1) * (0.5 / (NTAB - 1)), W, beta);
}
static double es_fourier(double xi) {
    const double h = 0.5 / (NTAB - 1), t = xi / h;
    int i = (int)t;
    if (i > NTAB - 2) i = NTAB - 2;
    const double f = t - i;
    const double *y = phi_tab + i; /* y[0..3] at nodes i-1, i, i+1, i+2 */
    return -f * (f - 1) * (f - 2) / 6 * y[0] + (f + 1) * (f - 1) * (f - 2) / 2 * y[1] -
           (f + 1) * f * (f - 2) / 2 * y[2] + (f + 1) * f * (f - 1) / 6 * y[3];
}

/* ---------------- FFT: iterative radix-2 (power-of-two) or direct DFT ---- */
typedef struct {
    int n, pow2;
    cf64 *tw; /* exp(+2 pi i k / n), k < n */
    int *rev;
} fft_plan;

static void plan_init(fft_plan *p, int n) {
    p->n = n;
    p->pow2 = (n & (n - 1)) == 0;
    p->tw = malloc(sizeof(cf64) * n);
    for (int k = 0; k < n; ++k) p->tw[k] = cexp(2.0 * M_PI * I * (double)k / n);
    p->rev = malloc(sizeof(int) * n);
    int lg = 0;
    while ((1 << lg) < n) ++lg;
    for (int i = 0; i < n; ++i) {
        int r = 0;
        for (int b = 0; b < lg; ++b) r |= ((i >> b) & 1) << (lg - 1 - b);
        p->rev[i] = p->pow2 ? r : i;
    }
}
static void plan_free(fft_plan *p) {
    free(p->tw);
    free(p->rev);
}

/* in-place backward (exp(+i)) unnormalised transform of x[0..n) */
static void fft_bwd(const fft_plan *p, cf64 *x, cf64 *tmp) {
    const int n = p->n;
    if (!p->pow2) {
        for (int k = 0; k < n; ++k) {
            cf64 s = 0;
            for (int j = 0; j < n; ++j) s += x[j] * p->tw[(int)(((int64_t)j * k) % n)];
            tmp[k] = s;
        }
        memcpy(x, tmp, sizeof(cf64) * n);
        return;
    }
    for (int i = 0; i < n; ++i)
        if (p->rev[i] > i) {
            cf64 t = x[i];
            x[i] = x[p->rev[i]];
            x[p->rev[i]] = t;
        }
    for (int len = 2; len <= n; len <<= 1) {
        const int half = len >> 1, step = n / len;
        for (int i = 0; i < n; i += len)
            for (int j = 0; j < half; ++j) {
                cf64 a = x[i + j], b = x[i + j + half] * p->tw[j * step];
                x[i + j] = a + b;
                x[i + j + half] = a - b;
            }
    }
}
static void fft_fwd(const fft_plan *p, cf64 *x, cf64 *tmp) {
    for (int i = 0; i < p->n; ++i) x[i] = conj(x[i]);
    fft_bwd(p, x, tmp);
    for (int i = 0; i < p->n; ++i) x[i] = conj(x[i]);
}

/* ---------------- geometry (shared by both directions) ------------------ */
static void geometry(Geo *g, const double *uvw, const double *freq, int nchan, int64_t nrow,
                     int npix_x, int npix_y, double pixsize_x, double pixsize_y, double epsilon,
                     int prec, int do_wstacking) {
    g->W = kernel_support(epsilon, prec);
    g->beta = 2.30 * g->W;
    g->nchan = nchan;
    g->ngx = 2 * npix_x;
    g->ngy = 2 * npix_y;
    g->ntr = (g->ngx + TILE - 1) / TILE;
    g->ntc = (g->ngy + TILE - 1) / TILE;
    g->px = pixsize_x;
    g->py = pixsize_y;
    g->do_w = do_wstacking;
    g->s0 = 0.0;
    g->dw = 1.0;
    g->w0 = 0.0;
    g->nplanes = 1;
    if (!do_wstacking) return;
    double wmin = 1e300, wmax = -1e300;
#pragma omp parallel for reduction(min : wmin) reduction(max : wmax) schedule(static)
    for (int64_t r = 0; r < nrow; ++r)
        for (int c = 0; c < nchan; ++c) {
            double w = uvw[3 * r + 2] * freq[c] / C_LIGHT;
            if (w < wmin) wmin = w;
            if (w > wmax) wmax = w;
        }
    double lmax = (npix_x / 2) * pixsize_x, mmax = (npix_y / 2) * pixsize_y;
    double r2 = lmax * lmax + mmax * mmax;
    if (r2 > 1.0) r2 = 1.0;
    double tmax = 1.0 - sqrt(1.0 - r2);
    const int W = g->W;
    g->s0 = 0.5 * tmax;
    g->dw = tmax > 0 ? 1.0 / (2.0 * tmax) : 1.0;
    g->w0 = wmin - (0.5 * W - 0.5) * g->dw;
    g->nplanes = (int)floor((wmax - g->w0) / g->dw - 0.5 * W) + 1 + W;
}

static void vis_coord(const Geo *g, const double *uvw, int64_t r, double f, Coord *c) {
    const double s = f / C_LIGHT;
    const double a = uvw[3 * r] * s * g->px * g->ngx;
    const double b = uvw[3 * r + 1] * s * g->py * g->ngy;
    c->w = uvw[3 * r + 2] * s;
    const double fa = floor(a - 0.5 * g->W), fb = floor(b - 0.5 * g->W);
    c->ic = (((int)fa + 1 + g->ngx / 2) % g->ngx + g->ngx) % g->ngx;
    c->jc = (((int)fb + 1 + g->ngy / 2) % g->ngy + g->ngy) % g->ngy;
    c->fu = fa + 1.0 - a;
    c->fv = fb + 1.0 - b;
    c->p0 = 0;
    c->fw = 0.0;
    if (g->do_w) {
        const double pw = (c->w - g->w0) / g->dw, fp = floor(pw - 0.5 * g->W);
        c->p0 = (int)fp + 1;
        if (c->p0 < 0) c->p0 = 0;
        if (c->p0 > g->nplanes - g->W) c->p0 = g->nplanes - g->W;
        c->fw = fp + 1.0 - pw;
    }
}

#define REAL float
#define SFX _f
#define EXP expf
#define SQRT sqrtf
#include "wgrid_cpu_kern.h"
#undef REAL
#undef SFX
#undef EXP
#undef SQRT
#define REAL double
#define SFX _d
#define EXP exp
#define SQRT sqrt
#include "wgrid_cpu_kern.h"
#undef REAL
#undef SFX
#undef EXP
#undef SQRT


/* large zeroed buffers: 2 MiB-aligned, transparent huge pages requested,
   zeroed by all threads (first touch in parallel, outside any lock) */
static void *big_zeroed(size_t bytes) {
    const size_t al = (size_t)2 << 20;
    const size_t n = (bytes + al - 1) / al * al;
    void *p = aligned_alloc(al, n);
    if (!p) return NULL;
    madvise(p, n, MADV_HUGEPAGE);
#pragma omp parallel for schedule(static)
    for (size_t o = 0; o < n; o += al) memset((char *)p + o, 0, al);
    return p;
}

static inline cf64 grid_load(const void *grid, size_t i, int prec) {
    if (prec) return ((const double *)grid)[2 * i] + I * ((const double *)grid)[2 * i + 1];
    return (double)((const float *)grid)[2 * i] + I * (double)((const float *)grid)[2 * i + 1];
}
static inline void grid_store(void *grid, size_t i, cf64 v, int prec) {
    if (prec) {
        ((double *)grid)[2 * i] = creal(v);
        ((double *)grid)[2 * i + 1] = cimag(v);
    } else {
        ((float *)grid)[2 * i] = (float)creal(v);
        ((float *)grid)[2 * i + 1] = (float)cimag(v);
    }
}

/* ---------------- ms2dirty ---------------------------------------------- */
int wgrid_cpu_ms2dirty(const double *uvw, const double *freq, int nchan, int64_t nrow,
                       const void *vis /* complex [nrow][nchan] or NULL */, int vis_f64,
                       const void *wgt /* [nrow][nchan] or NULL */, int wgt_f64, int npix_x,
                       int npix_y, double pixsize_x, double pixsize_y, double epsilon,
                       int do_wstacking, int prec, double *dirty, int nthreads, double *t_grid,
                       double *t_fft, int *support_out, int *nplanes_out) {
    if (npix_x % 2 || npix_y % 2) return 1;
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const int64_t nvis = nrow * nchan;
    if (nvis >= (int64_t)UINT32_MAX) return 2;
    gauss_legendre();
    Geo g;
    geometry(&g, uvw, freq, nchan, nrow, npix_x, npix_y, pixsize_x, pixsize_y, epsilon, prec,
             do_wstacking);
    const int W = g.W;
    phi_table(W, g.beta);
    if (support_out) *support_out = W;
    if (nplanes_out) *nplanes_out = g.nplanes;
    const int ngx = g.ngx, ngy = g.ngy;
    const double tg0 = omp_get_wtime();

    /* counting sort of the gridded visibilities by tile (per-thread
       histograms over contiguous visibility ranges) */
    const int nkey = g.ntr * g.ntc;
    const int nth = omp_get_max_threads();
    uint32_t *key = malloc(sizeof(uint32_t) * nvis);
    int64_t *hist = calloc((size_t)nth * (nkey + 1), sizeof(int64_t));
    int64_t *cnt = calloc((size_t)nkey + 1, sizeof(int64_t));
    const size_t rsz = prec ? sizeof(rec_t_d) : sizeof(rec_t_f);
    void *recs = NULL;
#pragma omp parallel
    {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        const int64_t lo = nvis * t / nt, hi = nvis * (t + 1) / nt;
        int64_t *h = hist + (size_t)t * (nkey + 1);
        for (int64_t v = lo; v < hi; ++v) {
            const int64_t r = v / nchan;
            const int c = (int)(v - r * nchan);
            double wt = 1.0;
            if (wgt) wt = wgt_f64 ? ((const double *)wgt)[v] : (double)((const float *)wgt)[v];
            int zero = wt == 0.0;
            if (vis && !zero) {
                zero = vis_f64 ? (((const double *)vis)[2 * v] == 0.0 &&
                                  ((const double *)vis)[2 * v + 1] == 0.0)
                               : (((const float *)vis)[2 * v] == 0.0f &&
                                  ((const float *)vis)[2 * v + 1] == 0.0f);
            }
            key[v] = UINT32_MAX;
            if (zero) continue;
            Coord cd;
            vis_coord(&g, uvw, r, freq[c], &cd);
            key[v] = (uint32_t)((cd.ic / TILE) * g.ntc + cd.jc / TILE);
            h[key[v]]++;
        }
#pragma omp barrier
#pragma omp single
        {
            int64_t run = 0;
            for (int k = 0; k < nkey; ++k) {
                cnt[k] = run;
                for (int tt = 0; tt < nt; ++tt) {
                    int64_t *hh = hist + (size_t)tt * (nkey + 1);
                    const int64_t c = hh[k];
                    hh[k] = run;
                    run += c;
                }
            }
            cnt[nkey] = run;
            recs = malloc(rsz * (size_t)(run + 1));
        }
        /* scatter pass: decoded records at their sorted positions (sequential
           reads of the inputs; the gridding tasks then read contiguously) */
        for (int64_t v = lo; v < hi; ++v) {
            if (key[v] == UINT32_MAX) continue;
            const int64_t pos = h[key[v]]++;
            if (prec)
                decode_d(&g, uvw, freq, vis, vis_f64, wgt, wgt_f64, v, (rec_t_d *)recs + pos);
            else
                decode_f(&g, uvw, freq, vis, vis_f64, wgt, wgt_f64, v, (rec_t_f *)recs + pos);
        }
    }
    free(key);
    free(hist);

    /* tasks: (tile, [b, e)) with e - b <= TASK */
    int64_t ntask = 0;
    for (int k = 0; k < nkey; ++k) ntask += (cnt[k + 1] - cnt[k] + TASK - 1) / TASK;
    int64_t *tb = malloc(sizeof(int64_t) * (ntask + 1)), *te = malloc(sizeof(int64_t) * (ntask + 1));
    int *tt_tile = malloc(sizeof(int) * (ntask + 1));
    {
        int64_t i = 0;
        for (int k = 0; k < nkey; ++k)
            for (int64_t b = cnt[k]; b < cnt[k + 1]; b += TASK) {
                tb[i] = b;
                te[i] = b + TASK < cnt[k + 1] ? b + TASK : cnt[k + 1];
                tt_tile[i++] = k;
            }
    }
    const size_t plane = (size_t)ngx * ngy;
    const size_t esz = prec ? sizeof(double) : sizeof(float);
    void *grid = big_zeroed(plane * 2 * (size_t)g.nplanes * esz); /* [plane][x][y] complex */
    omp_lock_t *locks = malloc(sizeof(omp_lock_t) * nkey);
    for (int k = 0; k < nkey; ++k) omp_init_lock(&locks[k]);
    const size_t bufsz = (size_t)(TILE + W - 1) * (TILE + W - 1) * 2 * g.nplanes;
#pragma omp parallel
    {
        void *buf = malloc(bufsz * esz);
#pragma omp for schedule(dynamic, 1)
        for (int64_t i = 0; i < ntask; ++i) {
            if (prec)
                grid_task_d(&g, (const rec_t_d *)recs + tb[i], te[i] - tb[i], tt_tile[i], buf,
                            grid, locks);
            else
                grid_task_f(&g, (const rec_t_f *)recs + tb[i], te[i] - tb[i], tt_tile[i], buf,
                            grid, locks);
        }
        free(buf);
    }
    for (int k = 0; k < nkey; ++k) omp_destroy_lock(&locks[k]);
    free(locks);
    free(tb);
    free(te);
    free(tt_tile);
    free(recs);
    free(cnt);
    const double tg = omp_get_wtime() - tg0;

    cf64 *rowbuf = malloc(sizeof(cf64) * (size_t)ngx * npix_y); /* [ngx][npix_y] after row FFT */
    double *acc = calloc((size_t)npix_x * npix_y, sizeof(double));
    /* per-pixel w-screen phasor exp(2 pi i w_p (n - 1 - s0)), advanced plane
       by plane by the pixel's step exp(2 pi i dw (n - 1 - s0)) */
    cf64 *scr = NULL, *stp = NULL;
    if (do_wstacking) {
        scr = malloc(sizeof(cf64) * (size_t)npix_x * npix_y);
        stp = malloc(sizeof(cf64) * (size_t)npix_x * npix_y);
#pragma omp parallel for schedule(static)
        for (int x = 0; x < npix_x; ++x)
            for (int y = 0; y < npix_y; ++y) {
                const double l = (x - npix_x / 2) * pixsize_x, m = (y - npix_y / 2) * pixsize_y;
                const double r2 = l * l + m * m;
                const double nt = r2 < 1.0 ? r2 / (sqrt(1.0 - r2) + 1.0) - g.s0 : 0.0;
                const double t0 = g.w0 * nt, t1 = g.dw * nt;
                scr[(size_t)x * npix_y + y] = cexp(2.0 * M_PI * I * (t0 - rint(t0)));
                stp[(size_t)x * npix_y + y] = cexp(2.0 * M_PI * I * (t1 - rint(t1)));
            }
    }
    fft_plan px, py;
    plan_init(&px, ngx);
    plan_init(&py, ngy);
    double tf = 0.0;
    enum { CB = 8 }; /* columns per block of the column pass */
    for (int p = 0; p < g.nplanes; ++p) {
        const char *gp = (const char *)grid + 2 * plane * esz * (size_t)p;
        const double t1 = omp_get_wtime();
        /* pruned 2-D backward FFT: rows (length ngy) keep npix_y outputs
           (all-zero rows skipped), then columns (length ngx) keep npix_x
           outputs, CB columns gathered per pass over rowbuf */
#pragma omp parallel
        {
            const int nl = ngx > ngy ? ngx : ngy;
            cf64 *line = malloc(sizeof(cf64) * nl * CB);
            cf64 *tmp = malloc(sizeof(cf64) * nl);
#pragma omp for schedule(static)
            for (int i = 0; i < ngx; ++i) {
                int nz = 0;
                for (int j = 0; j < ngy; ++j) {
                    line[j] = grid_load(gp, (size_t)i * ngy + j, prec);
                    nz |= line[j] != 0;
                }
                cf64 *dst = rowbuf + (size_t)i * npix_y;
                if (!nz) {
                    memset(dst, 0, sizeof(cf64) * npix_y);
                    continue;
                }
                fft_bwd(&py, line, tmp);
                for (int y = 0; y < npix_y; ++y) {
                    const int Y = y - npix_y / 2;
                    dst[y] = line[(Y % ngy + ngy) % ngy];
                }
            }
#pragma omp for schedule(static)
            for (int y0 = 0; y0 < npix_y; y0 += CB) {
                const int nb = npix_y - y0 < CB ? npix_y - y0 : CB;
                for (int i = 0; i < ngx; ++i)
                    for (int b = 0; b < nb; ++b) line[(size_t)b * nl + i] = rowbuf[(size_t)i * npix_y + y0 + b];
                for (int b = 0; b < nb; ++b) {
                    cf64 *ln = line + (size_t)b * nl;
                    const int y = y0 + b;
                    fft_bwd(&px, ln, tmp);
                    const int Y = y - npix_y / 2;
                    for (int x = 0; x < npix_x; ++x) {
                        const int X = x - npix_x / 2;
                        const size_t k = (size_t)x * npix_y + y;
                        cf64 h = ln[(X % ngx + ngx) % ngx];
                        if ((X + Y) & 1) h = -h; /* centred-grid storage */
                        double val;
                        if (do_wstacking) {
                            const double l = X * pixsize_x, m = Y * pixsize_y;
                            if (l * l + m * m >= 1.0) continue;
                            val = creal(h * scr[k]);
                            scr[k] *= stp[k];
                        } else {
                            val = creal(h);
                        }
                        acc[k] += val;
                    }
                }
            }
            free(line);
            free(tmp);
        }
        tf += omp_get_wtime() - t1;
    }
    free(scr);
    free(stp);

    /* grid correction */
    double *cx = malloc(sizeof(double) * npix_x), *cy = malloc(sizeof(double) * npix_y);
    for (int x = 0; x < npix_x; ++x) cx[x] = 1.0 / es_fourier(fabs((double)(x - npix_x / 2)) / ngx);
    for (int y = 0; y < npix_y; ++y) cy[y] = 1.0 / es_fourier(fabs((double)(y - npix_y / 2)) / ngy);
#pragma omp parallel for schedule(static)
    for (int x = 0; x < npix_x; ++x)
        for (int y = 0; y < npix_y; ++y) {
            double v = acc[(size_t)x * npix_y + y] * cx[x] * cy[y];
            if (do_wstacking) {
                const double l = (x - npix_x / 2) * pixsize_x, m = (y - npix_y / 2) * pixsize_y;
                const double r2 = l * l + m * m;
                if (r2 >= 1.0) {
                    v = 0.0;
                } else {
                    const double nm1 = -r2 / (sqrt(1.0 - r2) + 1.0);
                    v /= es_fourier(fabs(g.dw * (-nm1 - g.s0))) * (nm1 + 1.0);
                }
            }
            dirty[(size_t)x * npix_y + y] = v;
        }
    free(cx);
    free(cy);
    free(acc);
    free(rowbuf);
    free(grid);
    plan_free(&px);
    plan_free(&py);
    if (t_grid) *t_grid = tg;
    if (t_fft) *t_fft = tf;
    return 0;
}

/* ---------------- dirty2ms (the adjoint of ms2dirty) -------------------- */
/* ducc0-convention dirty2ms (predict_ng's call, ng.py:99): every step of
 * ms2dirty transposed.  The corrected image (1 / Phi in x and y; for
 * w-stacking also 1 / (Phi_w(dw (n - 1 - s0)) n)) is, per w plane, multiplied
 * by exp(-2 pi i w_p (n - 1 - s0)), placed on the centred grid and
 * forward-FFT'd (columns then rows, pruned on input); all planes stay
 * resident and each visibility interpolates its W^3 taps, times
 * exp(-2 pi i w s0) and its weight.  vis_out: complex double [nrow][nchan];
 * zero-weight visibilities are 0. */
int wgrid_cpu_dirty2ms(const double *uvw, const double *freq, int nchan, int64_t nrow,
                       const double *dirty /* [npix_x][npix_y] */, const void *wgt, int wgt_f64,
                       int npix_x, int npix_y, double pixsize_x, double pixsize_y,
                       double epsilon, int do_wstacking, int prec, double *vis_out, int nthreads,
                       double *t_degrid, double *t_fft, int *support_out, int *nplanes_out) {
    if (npix_x % 2 || npix_y % 2) return 1;
    if (nthreads > 0) omp_set_num_threads(nthreads);
    gauss_legendre();
    Geo g;
    geometry(&g, uvw, freq, nchan, nrow, npix_x, npix_y, pixsize_x, pixsize_y, epsilon, prec,
             do_wstacking);
    const int W = g.W;
    phi_table(W, g.beta);
    if (support_out) *support_out = W;
    if (nplanes_out) *nplanes_out = g.nplanes;
    const int ngx = g.ngx, ngy = g.ngy;
    const size_t npix = (size_t)npix_x * npix_y;

    /* corrected image and each pixel's n - 1 - s0 */
    double *img = malloc(sizeof(double) * npix), *nt = malloc(sizeof(double) * npix);
    double *cx = malloc(sizeof(double) * npix_x), *cy = malloc(sizeof(double) * npix_y);
    for (int x = 0; x < npix_x; ++x) cx[x] = 1.0 / es_fourier(fabs((double)(x - npix_x / 2)) / ngx);
    for (int y = 0; y < npix_y; ++y) cy[y] = 1.0 / es_fourier(fabs((double)(y - npix_y / 2)) / ngy);
#pragma omp parallel for schedule(static)
    for (int x = 0; x < npix_x; ++x)
        for (int y = 0; y < npix_y; ++y) {
            const size_t k = (size_t)x * npix_y + y;
            double v = dirty[k] * cx[x] * cy[y];
            nt[k] = 0.0;
            if (do_wstacking) {
                const double l = (x - npix_x / 2) * pixsize_x, m = (y - npix_y / 2) * pixsize_y;
                const double r2 = l * l + m * m;
                if (r2 >= 1.0) {
                    v = 0.0;
                } else {
                    const double nm1 = -r2 / (sqrt(1.0 - r2) + 1.0);
                    nt[k] = -nm1 - g.s0;
                    v /= es_fourier(fabs(g.dw * nt[k])) * (nm1 + 1.0);
                }
            }
            img[k] = v;
        }
    free(cx);
    free(cy);

    const size_t plane = (size_t)ngx * ngy;
    const size_t esz = prec ? sizeof(double) : sizeof(float);
    void *grid = big_zeroed(esz * 2 * plane * g.nplanes); /* [plane][x][y] complex */
    cf64 *colbuf = malloc(sizeof(cf64) * (size_t)ngx * npix_y); /* [ngx][npix_y] */
    fft_plan px, py;
    plan_init(&px, ngx);
    plan_init(&py, ngy);
    double tf = 0.0;
    for (int p = 0; p < g.nplanes; ++p) {
        const double wp = g.w0 + p * g.dw;
        char *gp = (char *)grid + 2 * plane * esz * (size_t)p;
        const double t1 = omp_get_wtime();
#pragma omp parallel
        {
            const int nl = ngx > ngy ? ngx : ngy;
            cf64 *line = malloc(sizeof(cf64) * nl), *tmp = malloc(sizeof(cf64) * nl);
#pragma omp for schedule(static)
            for (int y = 0; y < npix_y; ++y) {
                const int Y = y - npix_y / 2;
                memset(line, 0, sizeof(cf64) * ngx);
                for (int x = 0; x < npix_x; ++x) {
                    const int X = x - npix_x / 2;
                    const size_t k = (size_t)x * npix_y + y;
                    cf64 h = img[k];
                    if (do_wstacking) h *= cexp(-2.0 * M_PI * I * wp * nt[k]);
                    if ((X + Y) & 1) h = -h; /* centred-grid storage */
                    line[(X % ngx + ngx) % ngx] = h;
                }
                fft_fwd(&px, line, tmp);
                for (int i = 0; i < ngx; ++i) colbuf[(size_t)i * npix_y + y] = line[i];
            }
#pragma omp for schedule(static)
            for (int i = 0; i < ngx; ++i) {
                memset(line, 0, sizeof(cf64) * ngy);
                for (int y = 0; y < npix_y; ++y) {
                    const int Y = y - npix_y / 2;
                    line[(Y % ngy + ngy) % ngy] = colbuf[(size_t)i * npix_y + y];
                }
                fft_fwd(&py, line, tmp);
                for (int j = 0; j < ngy; ++j) grid_store(gp, (size_t)i * ngy + j, line[j], prec);
            }
            free(line);
            free(tmp);
        }
        tf += omp_get_wtime() - t1;
    }
    free(colbuf);
    free(img);
    free(nt);

    /* degrid: rows in parallel, a row's channels in order (neighbouring uv) */
    const double tg0 = omp_get_wtime();
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t r = 0; r < nrow; ++r)
        for (int c = 0; c < nchan; ++c) {
            const int64_t k = r * nchan + c;
            double wt = 1.0;
            if (wgt) wt = wgt_f64 ? ((const double *)wgt)[k] : (double)((const float *)wgt)[k];
            vis_out[2 * k] = vis_out[2 * k + 1] = 0.0;
            if (wt == 0.0) continue;
            Coord cd;
            vis_coord(&g, uvw, r, freq[c], &cd);
            cf64 v = prec ? degrid_one_d(&g, grid, &cd) : degrid_one_f(&g, grid, &cd);
            v *= wt;
            if (do_wstacking) v *= cexp(-2.0 * M_PI * I * (cd.w * g.s0 - rint(cd.w * g.s0)));
            vis_out[2 * k] = creal(v);
            vis_out[2 * k + 1] = cimag(v);
        }
    const double tg = omp_get_wtime() - tg0;
    free(grid);
    plan_free(&px);
    plan_free(&py);
    if (t_degrid) *t_degrid = tg;
    if (t_fft) *t_fft = tf;
    return 0;
}

/* ---------------- exact direct sums (ducc0's definition) ---------------- */
/* phase of visibility (row, chan) at pixel (l, m, n - 1), in turns:
 * (u l + v m - w (n - 1)) f / c (oracle/nufft_oracle.py).  A row's channels
 * are handled by a complex recurrence when the frequencies are uniformly
 * spaced (re-anchored every 16 channels), else by one sincos each. */
static int uniform_freq(const double *freq, int nchan) {
    if (nchan < 3) return 0;
    const double df = (freq[nchan - 1] - freq[0]) / (nchan - 1);
    for (int c = 0; c < nchan; ++c)
        if (fabs(freq[c] - (freq[0] + c * df)) > 1e-9 * fabs(freq[c])) return 0;
    return 1;
}

static void row_phasors(double turns_per_hz, const double *freq, int nchan, int uni, cf64 *ph) {
    if (!uni) {
        for (int c = 0; c < nchan; ++c) ph[c] = cexp(2.0 * M_PI * I * turns_per_hz * freq[c]);
        return;
    }
    const double df = (freq[nchan - 1] - freq[0]) / (nchan - 1);
    const cf64 step = cexp(2.0 * M_PI * I * turns_per_hz * df);
    for (int c = 0; c < nchan; ++c) {
        if ((c & 15) == 0) {
            const double t = turns_per_hz * freq[c];
            ph[c] = cexp(2.0 * M_PI * I * (t - rint(t)));
        } else {
            ph[c] = ph[c - 1] * step;
        }
    }
}

/* dirty at npts pixels (px[i], py[i]) (0-based, ducc0 layout) */
int wgrid_cpu_exact_pixels(const double *uvw, const double *freq, int nchan, int64_t nrow,
                           const void *vis, int vis_f64, const void *wgt, int wgt_f64, int npix_x,
                           int npix_y, double pixsize_x, double pixsize_y, int do_wstacking,
                           int npts, const int *pxs, const int *pys, double *out, int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const int uni = uniform_freq(freq, nchan);
    double *l = malloc(sizeof(double) * npts), *m = malloc(sizeof(double) * npts),
           *nm1 = malloc(sizeof(double) * npts);
    for (int i = 0; i < npts; ++i) {
        l[i] = (pxs[i] - npix_x / 2) * pixsize_x;
        m[i] = (pys[i] - npix_y / 2) * pixsize_y;
        const double r2 = l[i] * l[i] + m[i] * m[i];
        nm1[i] = r2 < 1.0 ? -r2 / (sqrt(1.0 - r2) + 1.0) : 0.0;
        out[i] = 0.0;
    }
#pragma omp parallel
    {
        double *part = calloc(npts, sizeof(double));
        cf64 *ph = malloc(sizeof(cf64) * nchan);
#pragma omp for schedule(dynamic, 256)
        for (int64_t r = 0; r < nrow; ++r) {
            const double u = uvw[3 * r], v = uvw[3 * r + 1], w = uvw[3 * r + 2];
            for (int i = 0; i < npts; ++i) {
                const double t = (u * l[i] + v * m[i] - (do_wstacking ? w * nm1[i] : 0.0)) / C_LIGHT;
                row_phasors(t, freq, nchan, uni, ph);
                double s = 0.0;
                for (int c = 0; c < nchan; ++c) {
                    const int64_t k = r * nchan + c;
                    double wt = 1.0;
                    if (wgt) wt = wgt_f64 ? ((const double *)wgt)[k] : (double)((const float *)wgt)[k];
                    double vr = 1.0, vi = 0.0;
                    if (vis) {
                        if (vis_f64) {
                            vr = ((const double *)vis)[2 * k];
                            vi = ((const double *)vis)[2 * k + 1];
                        } else {
                            vr = ((const float *)vis)[2 * k];
                            vi = ((const float *)vis)[2 * k + 1];
                        }
                    }
                    s += wt * (vr * creal(ph[c]) - vi * cimag(ph[c]));
                }
                part[i] += s;
            }
        }
#pragma omp critical
        for (int i = 0; i < npts; ++i) out[i] += part[i];
        free(part);
        free(ph);
    }
    for (int i = 0; i < npts; ++i) {
        const double r2 = l[i] * l[i] + m[i] * m[i];
        if (do_wstacking) out[i] = r2 < 1.0 ? out[i] / (nm1[i] + 1.0) : 0.0;
    }
    free(l);
    free(m);
    free(nm1);
    return 0;
}

/* visibilities of nsel rows (all channels) predicted exactly from the dense
 * image dirty[npix_x][npix_y]: vis = wgt sum_pix dirty / n exp(-2 pi i phase);
 * out: complex double [nsel][nchan] */
int wgrid_cpu_exact_rows(const double *uvw, const double *freq, int nchan, int nsel,
                         const int64_t *rows, const double *dirty, int npix_x, int npix_y,
                         double pixsize_x, double pixsize_y, int do_wstacking, double *out,
                         int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const int uni = uniform_freq(freq, nchan);
    const size_t nout = (size_t)nsel * nchan;
    memset(out, 0, sizeof(double) * 2 * nout);
#pragma omp parallel
    {
        cf64 *part = calloc(nout, sizeof(cf64));
        cf64 *ph = malloc(sizeof(cf64) * nchan);
#pragma omp for schedule(dynamic, 4)
        for (int x = 0; x < npix_x; ++x) {
            const double l = (x - npix_x / 2) * pixsize_x;
            for (int y = 0; y < npix_y; ++y) {
                const double val = dirty[(size_t)x * npix_y + y];
                if (val == 0.0) continue;
                const double m = (y - npix_y / 2) * pixsize_y, r2 = l * l + m * m;
                if (do_wstacking && r2 >= 1.0) continue;
                const double nm1 = r2 < 1.0 ? -r2 / (sqrt(1.0 - r2) + 1.0) : 0.0;
                const double a = do_wstacking ? val / (nm1 + 1.0) : val;
                for (int s = 0; s < nsel; ++s) {
                    const double *q = uvw + 3 * rows[s];
                    const double t = -(q[0] * l + q[1] * m - (do_wstacking ? q[2] * nm1 : 0.0)) / C_LIGHT;
                    row_phasors(t, freq, nchan, uni, ph);
                    cf64 *o = part + (size_t)s * nchan;
                    for (int c = 0; c < nchan; ++c) o[c] += a * ph[c];
                }
            }
        }
#pragma omp critical
        for (size_t i = 0; i < nout; ++i) {
            out[2 * i] += creal(part[i]);
            out[2 * i + 1] += cimag(part[i]);
        }
        free(part);
        free(ph);
    }
    return 0;
}
