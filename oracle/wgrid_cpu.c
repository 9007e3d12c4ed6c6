/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- never linked by the product path.
 *
 * Plain-C + OpenMP restatement of the w-stacking adjoint NUFFT (ms2dirty)
 * and of its adjoint, the forward NUFFT (dirty2ms, at the end of this file),
 * that the reference binds through ducc0.wgridder (ducc0 0.27.0,
 * poetry.lock:305-306; call sites src/ska_sdp_func_python/imaging/ng.py:240
 * and ng.py:99).
 * ducc0 is not vendored under /root/reference and cannot be built or
 * installed here, so this is the CPU baseline of bench.py ("kind": "port")
 * and a second checker for the HIP path.  The algorithm is the one stated in
 * oracle/nufft_oracle.py (wgrid_ms2dirty) and SURVEY.md Appendix A:
 *
 *   ES kernel phi(t) = exp(beta (sqrt(1 - (2t/W)^2) - 1)), sigma = 2,
 *   W = ceil(-log10(eps/10)) in [2, 8], beta = 2.30 W;
 *   w planes w_p = w0 + p dw with dw = 1/(2 tmax), vis pre-phased by
 *   exp(2 pi i w s0); per plane: grid (complex float, like ducc0 for fp32
 *   input), 2-D inverse FFT pruned to the npix window, multiply by
 *   exp(2 pi i w_p (n - 1 - s0)) and accumulate; finally divide by the
 *   kernel's Fourier transform in x, y and w and by n.
 *
 * Output is ducc0's convention: dirty[x * npix_y + y], l_x = (x - nx/2) px.
 * Parallelism: all w planes stay resident (as on the GPU), visibilities are
 * bucketed by 32 x 32-cell tiles and gridded strip by strip (32-row strips,
 * even strips then odd strips, so no two threads touch the same grid row);
 * each visibility's u/v/w taps are evaluated once.  FFT rows/columns and the
 * image accumulation are OpenMP loops.
 */
#include <complex.h>
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define C_LIGHT 299792458.0
#define STRIP 32

typedef float complex cf32;
typedef double complex cf64;

static int kernel_support(double eps) {
    if (eps < 1e-7) eps = 1e-7;
    int w = (int)ceil(-log10(eps / 10.0));
    return w < 2 ? 2 : (w > 8 ? 8 : w);
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
static double es_fourier(double xi, int W, double beta) {
    (void)W;
    (void)beta;
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

/* ---------------- w-plane geometry (shared by both directions) ---------- */
static void w_geometry(const double *uvw, const double *freq, int nchan, int64_t nrow, int npix_x,
                       int npix_y, double pixsize_x, double pixsize_y, int W, int do_wstacking,
                       double *s0, double *dw, double *w0, int *nplanes) {
    double wmin = 1e300, wmax = -1e300;
    for (int64_t r = 0; r < nrow; ++r)
        for (int c = 0; c < nchan; ++c) {
            double w = uvw[3 * r + 2] * freq[c] / C_LIGHT;
            if (w < wmin) wmin = w;
            if (w > wmax) wmax = w;
        }
    *s0 = 0.0;
    *dw = 1.0;
    *w0 = 0.0;
    *nplanes = 1;
    if (do_wstacking) {
        double lmax = (npix_x / 2) * pixsize_x, mmax = (npix_y / 2) * pixsize_y;
        double r2 = lmax * lmax + mmax * mmax;
        if (r2 > 1.0) r2 = 1.0;
        double tmax = 1.0 - sqrt(1.0 - r2);
        *s0 = 0.5 * tmax;
        *dw = tmax > 0 ? 1.0 / (2.0 * tmax) : 1.0;
        *w0 = wmin - (0.5 * W - 0.5) * *dw;
        *nplanes = (int)floor((wmax - *w0) / *dw - 0.5 * W) + 1 + W;
    }
}

/* ---------------- ms2dirty ---------------------------------------------- */
int wgrid_cpu_ms2dirty(const double *uvw, const double *freq, int nchan, int64_t nrow,
                       const float *vis /* c64 interleaved [nrow][nchan] or NULL */,
                       const float *wgt /* [nrow][nchan] or NULL */, int npix_x, int npix_y,
                       double pixsize_x, double pixsize_y, double epsilon, int do_wstacking,
                       double *dirty, int nthreads, double *t_grid, double *t_fft) {
    if (npix_x % 2 || npix_y % 2) return 1;
    if (nthreads > 0) omp_set_num_threads(nthreads);
    gauss_legendre();
    const int W = kernel_support(epsilon);
    const double beta = 2.30 * W;
    phi_table(W, beta);
    const int ngx = 2 * npix_x, ngy = 2 * npix_y;
    const int64_t nvis = nrow * nchan;

    double s0, dw, w0;
    int nplanes;
    w_geometry(uvw, freq, nchan, nrow, npix_x, npix_y, pixsize_x, pixsize_y, W, do_wstacking, &s0,
               &dw, &w0, &nplanes);

    /* per-vis records bucketed by (strip, tile column) of 32 x 32 cells;
       all w planes stay resident (like the GPU path), so each visibility's
       u/v/w taps are evaluated once and it is gridded in one pass */
    const int ntc = (ngy + STRIP - 1) / STRIP;
    const int nstrip = (ngx + STRIP - 1) / STRIP;
    const int64_t nkey = (int64_t)nstrip * ntc;
    int64_t *cnt = calloc((size_t)nkey + 1, sizeof(int64_t));
    int32_t *key = malloc(sizeof(int32_t) * nvis);
    typedef struct {
        float re, im, fu, fv, fw;
        int32_t ic, jc, p0;
    } rec_t;
    rec_t *rec = malloc(sizeof(rec_t) * (nvis + 1));
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nrow; ++r)
        for (int c = 0; c < nchan; ++c) {
            const int64_t k = r * nchan + c;
            float wt = wgt ? wgt[k] : 1.0f;
            float re = vis ? vis[2 * k] : 1.0f, im = vis ? vis[2 * k + 1] : 0.0f;
            key[k] = -1;
            if (wt == 0.0f || (re == 0.0f && im == 0.0f)) continue;
            const double s = freq[c] / C_LIGHT;
            const double a = uvw[3 * r] * s * pixsize_x * ngx;
            const double b = uvw[3 * r + 1] * s * pixsize_y * ngy;
            const double w = uvw[3 * r + 2] * s;
            const double fa = floor(a - 0.5 * W), fb = floor(b - 0.5 * W);
            rec_t q;
            q.ic = (((int)fa + 1 + ngx / 2) % ngx + ngx) % ngx;
            q.jc = (((int)fb + 1 + ngy / 2) % ngy + ngy) % ngy;
            q.fu = (float)(fa + 1.0 - a);
            q.fv = (float)(fb + 1.0 - b);
            q.p0 = 0;
            q.fw = 0.0f;
            cf64 v = (re + I * im) * (double)wt;
            if (do_wstacking) {
                const double pw = (w - w0) / dw, fp = floor(pw - 0.5 * W);
                q.p0 = (int)fp + 1;
                q.fw = (float)(fp + 1.0 - pw);
                v *= cexp(2.0 * M_PI * I * w * s0);
            }
            q.re = (float)creal(v);
            q.im = (float)cimag(v);
            rec[k] = q;
            key[k] = (q.ic / STRIP) * ntc + q.jc / STRIP;
        }
    for (int64_t k = 0; k < nvis; ++k)
        if (key[k] >= 0) cnt[key[k] + 1]++;
    for (int64_t i = 0; i < nkey; ++i) cnt[i + 1] += cnt[i];
    int64_t *order = malloc(sizeof(int64_t) * (cnt[nkey] + 1));
    {
        int64_t *fill = malloc(sizeof(int64_t) * nkey);
        memcpy(fill, cnt, sizeof(int64_t) * nkey);
        for (int64_t k = 0; k < nvis; ++k)
            if (key[k] >= 0) order[fill[key[k]]++] = k;
        free(fill);
    }
    free(key);

    const size_t plane = (size_t)ngx * ngy;
    float *grid = calloc(plane * 2 * nplanes, sizeof(float)); /* [plane][x][y] complex */
    cf64 *rowbuf = malloc(sizeof(cf64) * (size_t)ngx * npix_y); /* [ngx][npix_y] after row FFT */
    double *acc = calloc((size_t)npix_x * npix_y, sizeof(double));
    fft_plan px, py;
    plan_init(&px, ngx);
    plan_init(&py, ngy);
    double tg = 0.0, tf = 0.0;
    const float fbeta = (float)beta, fihw = 2.0f / W;

    double tg0 = omp_get_wtime();
    /* strips of one parity never share grid rows (W <= 8 < STRIP); with an
       odd strip count the last strip wraps onto strip 0, so it runs alone */
    const int nst_even = nstrip & ~1;
    for (int parity = 0; parity < 3; ++parity) {
        const int lo = parity < 2 ? parity : nst_even, hi = parity < 2 ? nst_even : nstrip;
#pragma omp parallel for schedule(dynamic, 1)
        for (int st = lo; st < hi; st += 2) {
            for (int64_t k = cnt[(int64_t)st * ntc]; k < cnt[(int64_t)(st + 1) * ntc]; ++k) {
                const rec_t *q = &rec[order[k]];
                float ku[8], kw[8], kv2[16];
                for (int t = 0; t < W; ++t) {
                    float x = (q->fu + t) * fihw, y = 1.0f - x * x;
                    ku[t] = y > 0.0f ? expf(fbeta * (sqrtf(y) - 1.0f)) : 0.0f;
                    x = (q->fv + t) * fihw;
                    y = 1.0f - x * x;
                    kv2[2 * t] = kv2[2 * t + 1] = y > 0.0f ? expf(fbeta * (sqrtf(y) - 1.0f)) : 0.0f;
                    x = (q->fw + t) * fihw;
                    y = 1.0f - x * x;
                    kw[t] = do_wstacking ? (y > 0.0f ? expf(fbeta * (sqrtf(y) - 1.0f)) : 0.0f)
                                         : (t == 0 ? 1.0f : 0.0f);
                }
                const int nq = do_wstacking ? W : 1;
                const int fast = q->jc + W <= ngy;
                for (int qq = 0; qq < nq; ++qq) {
                    float *pl = grid + 2 * plane * (size_t)(q->p0 + qq);
                    for (int t = 0; t < W; ++t) {
                        int gi = q->ic + t;
                        if (gi >= ngx) gi -= ngx;
                        const float f = ku[t] * kw[qq];
                        float cv[16];
                        for (int e = 0; e < 8; ++e) {
                            cv[2 * e] = q->re * f;
                            cv[2 * e + 1] = q->im * f;
                        }
                        float *row = pl + 2 * (size_t)gi * ngy;
                        if (fast && W == 8) {
                            float *dst = row + 2 * q->jc;
                            for (int e = 0; e < 16; ++e) dst[e] += cv[e] * kv2[e];
                        } else {
                            for (int tt = 0; tt < W; ++tt) {
                                int gj = q->jc + tt;
                                if (gj >= ngy) gj -= ngy;
                                row[2 * gj] += cv[2 * tt] * kv2[2 * tt];
                                row[2 * gj + 1] += cv[2 * tt + 1] * kv2[2 * tt + 1];
                            }
                        }
                    }
                }
            }
        }
    }
    tg = omp_get_wtime() - tg0;

    for (int p = 0; p < nplanes; ++p) {
        const float *gp = grid + 2 * plane * (size_t)p;
        double t1 = omp_get_wtime();
        /* pruned 2-D backward FFT: rows (length ngy) keep npix_y outputs,
           then columns (length ngx) keep npix_x outputs */
#pragma omp parallel
        {
            cf64 *line = malloc(sizeof(cf64) * (ngx > ngy ? ngx : ngy));
            cf64 *tmp = malloc(sizeof(cf64) * (ngx > ngy ? ngx : ngy));
#pragma omp for schedule(static)
            for (int i = 0; i < ngx; ++i) {
                for (int j = 0; j < ngy; ++j)
                    line[j] = gp[2 * ((size_t)i * ngy + j)] + I * gp[2 * ((size_t)i * ngy + j) + 1];
                fft_bwd(&py, line, tmp);
                for (int y = 0; y < npix_y; ++y) {
                    const int Y = y - npix_y / 2;
                    rowbuf[(size_t)i * npix_y + y] = line[(Y % ngy + ngy) % ngy];
                }
            }
#pragma omp for schedule(static)
            for (int y = 0; y < npix_y; ++y) {
                for (int i = 0; i < ngx; ++i) line[i] = rowbuf[(size_t)i * npix_y + y];
                fft_bwd(&px, line, tmp);
                const int Y = y - npix_y / 2;
                for (int x = 0; x < npix_x; ++x) {
                    const int X = x - npix_x / 2;
                    cf64 h = line[(X % ngx + ngx) % ngx];
                    if ((X + Y) & 1) h = -h; /* centred-grid storage */
                    double val;
                    if (do_wstacking) {
                        const double l = X * pixsize_x, m = Y * pixsize_y, r2 = l * l + m * m;
                        if (r2 >= 1.0) continue;
                        const double nm1 = -r2 / (sqrt(1.0 - r2) + 1.0);
                        const double ph = 2.0 * M_PI * (w0 + p * dw) * (-nm1 - s0);
                        val = creal(h) * cos(ph) - cimag(h) * sin(ph);
                    } else {
                        val = creal(h);
                    }
                    acc[(size_t)x * npix_y + y] += val;
                }
            }
            free(line);
            free(tmp);
        }
        tf += omp_get_wtime() - t1;
    }

    /* grid correction */
    double *cx = malloc(sizeof(double) * npix_x), *cy = malloc(sizeof(double) * npix_y);
    for (int x = 0; x < npix_x; ++x) cx[x] = 1.0 / es_fourier(fabs((double)(x - npix_x / 2)) / ngx, W, beta);
    for (int y = 0; y < npix_y; ++y) cy[y] = 1.0 / es_fourier(fabs((double)(y - npix_y / 2)) / ngy, W, beta);
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
                    v /= es_fourier(fabs(dw * (-nm1 - s0)), W, beta) * (nm1 + 1.0);
                }
            }
            dirty[(size_t)x * npix_y + y] = v;
        }
    free(cx);
    free(cy);
    free(acc);
    free(rowbuf);
    free(grid);
    free(rec);
    free(order);
    free(cnt);
    plan_free(&px);
    plan_free(&py);
    if (t_grid) *t_grid = tg;
    if (t_fft) *t_fft = tf;
    return 0;
}

/* ---------------- dirty2ms (the adjoint of ms2dirty) -------------------- */
static void fft_fwd(const fft_plan *p, cf64 *x, cf64 *tmp) {
    for (int i = 0; i < p->n; ++i) x[i] = conj(x[i]);
    fft_bwd(p, x, tmp);
    for (int i = 0; i < p->n; ++i) x[i] = conj(x[i]);
}

/* ducc0-convention dirty2ms (predict_ng's call, ng.py:99): every step of
 * ms2dirty transposed.  The corrected image (1 / Phi in x and y; for
 * w-stacking also 1 / (Phi_w(dw (n - 1 - s0)) n)) is, per w plane, multiplied
 * by exp(-2 pi i w_p (n - 1 - s0)), placed on the centred grid and
 * forward-FFT'd (columns then rows, pruned on input); all planes stay
 * resident and each visibility interpolates its W^3 taps, times
 * exp(-2 pi i w s0) and its weight.  vis_out: complex double [nrow][nchan];
 * zero-weight visibilities are 0. */
int wgrid_cpu_dirty2ms(const double *uvw, const double *freq, int nchan, int64_t nrow,
                       const double *dirty /* [npix_x][npix_y] */, const float *wgt,
                       int npix_x, int npix_y, double pixsize_x, double pixsize_y,
                       double epsilon, int do_wstacking, double *vis_out, int nthreads,
                       double *t_degrid, double *t_fft) {
    if (npix_x % 2 || npix_y % 2) return 1;
    if (nthreads > 0) omp_set_num_threads(nthreads);
    gauss_legendre();
    const int W = kernel_support(epsilon);
    const double beta = 2.30 * W;
    phi_table(W, beta);
    const int ngx = 2 * npix_x, ngy = 2 * npix_y;
    double s0, dw, w0;
    int nplanes;
    w_geometry(uvw, freq, nchan, nrow, npix_x, npix_y, pixsize_x, pixsize_y, W, do_wstacking, &s0,
               &dw, &w0, &nplanes);
    const size_t npix = (size_t)npix_x * npix_y;

    /* corrected image and each pixel's n - 1 - s0 */
    double *img = malloc(sizeof(double) * npix), *nt = malloc(sizeof(double) * npix);
    double *cx = malloc(sizeof(double) * npix_x), *cy = malloc(sizeof(double) * npix_y);
    for (int x = 0; x < npix_x; ++x) cx[x] = 1.0 / es_fourier(fabs((double)(x - npix_x / 2)) / ngx, W, beta);
    for (int y = 0; y < npix_y; ++y) cy[y] = 1.0 / es_fourier(fabs((double)(y - npix_y / 2)) / ngy, W, beta);
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
                    nt[k] = -nm1 - s0;
                    v /= es_fourier(fabs(dw * nt[k]), W, beta) * (nm1 + 1.0);
                }
            }
            img[k] = v;
        }
    free(cx);
    free(cy);

    const size_t plane = (size_t)ngx * ngy;
    float *grid = malloc(sizeof(float) * 2 * plane * nplanes); /* [plane][x][y] complex */
    cf64 *colbuf = malloc(sizeof(cf64) * (size_t)ngx * npix_y); /* [ngx][npix_y] */
    fft_plan px, py;
    plan_init(&px, ngx);
    plan_init(&py, ngy);
    double tf = 0.0;
    for (int p = 0; p < nplanes; ++p) {
        const double wp = w0 + p * dw;
        float *gp = grid + 2 * plane * (size_t)p;
        double t1 = omp_get_wtime();
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
                float *row = gp + 2 * (size_t)i * ngy;
                for (int j = 0; j < ngy; ++j) {
                    row[2 * j] = (float)creal(line[j]);
                    row[2 * j + 1] = (float)cimag(line[j]);
                }
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
    const float fbeta = (float)beta, fihw = 2.0f / W;
    const double tg0 = omp_get_wtime();
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t r = 0; r < nrow; ++r)
        for (int c = 0; c < nchan; ++c) {
            const int64_t k = r * nchan + c;
            const float wt = wgt ? wgt[k] : 1.0f;
            vis_out[2 * k] = vis_out[2 * k + 1] = 0.0;
            if (wt == 0.0f) continue;
            const double s = freq[c] / C_LIGHT;
            const double a = uvw[3 * r] * s * pixsize_x * ngx;
            const double b = uvw[3 * r + 1] * s * pixsize_y * ngy;
            const double w = uvw[3 * r + 2] * s;
            const double fa = floor(a - 0.5 * W), fb = floor(b - 0.5 * W);
            const int ic = (((int)fa + 1 + ngx / 2) % ngx + ngx) % ngx;
            const int jc = (((int)fb + 1 + ngy / 2) % ngy + ngy) % ngy;
            const float fu = (float)(fa + 1.0 - a), fv = (float)(fb + 1.0 - b);
            int p0 = 0;
            float fw = 0.0f;
            if (do_wstacking) {
                const double pw = (w - w0) / dw, fp = floor(pw - 0.5 * W);
                p0 = (int)fp + 1;
                fw = (float)(fp + 1.0 - pw);
            }
            float ku[8], kv[8], kw[8];
            for (int t = 0; t < W; ++t) {
                float x = (fu + t) * fihw, y = 1.0f - x * x;
                ku[t] = y > 0.0f ? expf(fbeta * (sqrtf(y) - 1.0f)) : 0.0f;
                x = (fv + t) * fihw;
                y = 1.0f - x * x;
                kv[t] = y > 0.0f ? expf(fbeta * (sqrtf(y) - 1.0f)) : 0.0f;
                x = (fw + t) * fihw;
                y = 1.0f - x * x;
                kw[t] = do_wstacking ? (y > 0.0f ? expf(fbeta * (sqrtf(y) - 1.0f)) : 0.0f)
                                     : (t == 0 ? 1.0f : 0.0f);
            }
            const int nq = do_wstacking ? W : 1;
            const int fast = jc + W <= ngy;
            double sr = 0.0, si = 0.0;
            for (int q = 0; q < nq; ++q) {
                const float *pl = grid + 2 * plane * (size_t)(p0 + q);
                float qr = 0.0f, qi = 0.0f;
                for (int t = 0; t < W; ++t) {
                    int gi = ic + t;
                    if (gi >= ngx) gi -= ngx;
                    const float *row = pl + 2 * (size_t)gi * ngy;
                    float rr = 0.0f, ri = 0.0f;
                    if (fast) {
                        const float *src = row + 2 * jc;
                        for (int tt = 0; tt < W; ++tt) {
                            rr += kv[tt] * src[2 * tt];
                            ri += kv[tt] * src[2 * tt + 1];
                        }
                    } else {
                        for (int tt = 0; tt < W; ++tt) {
                            int gj = jc + tt;
                            if (gj >= ngy) gj -= ngy;
                            rr += kv[tt] * row[2 * gj];
                            ri += kv[tt] * row[2 * gj + 1];
                        }
                    }
                    qr += ku[t] * rr;
                    qi += ku[t] * ri;
                }
                sr += kw[q] * qr;
                si += kw[q] * qi;
            }
            cf64 v = (sr + I * si) * (double)wt;
            if (do_wstacking) v *= cexp(-2.0 * M_PI * I * w * s0);
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
