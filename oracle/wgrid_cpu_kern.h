/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- included twice by wgrid_cpu.c, once
 * with REAL = float (SFX _f: fp32 taps and grid, the precision the HIP path
 * computes in) and once with REAL = double (SFX _d: fp64 taps and grid, the
 * reference's double_precision_accumulation=True call of ducc0,
 * src/ska_sdp_func_python/imaging/ng.py:240-256).
 */
#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SFX)

static inline REAL FN(es_tap)(REAL t, REAL ihw, REAL beta) {
    const REAL x = t * ihw, y = (REAL)1 - x * x;
    return y > (REAL)0 ? EXP(beta * (SQRT(y) - (REAL)1)) : (REAL)0;
}

/* ms2dirty gridding of one task: visibilities order[b..e) of one TILE x
 * TILE-cell tile, accumulated into the thread's private tile buffer (all
 * touched planes) and then added into the resident planes under the locks
 * of the (up to) four tiles the footprint halo reaches.  scratch holds the
 * decoded records of the task. */
typedef struct {
    REAL re, im, fu, fv, fw;
    int ic, jc, p0;
} FN(rec_t);

/* the records of one task into the private tile buffer; W is a literal at
   every call site, so the tap loops unroll and vectorise */
static inline __attribute__((always_inline)) void FN(grid_recs)(
    const FN(rec_t) *recs, int64_t n, REAL *buf, size_t pl, int pmin, const int W,
    const int RY, int ibase, int jbase, const Geo *g, REAL ihw, REAL beta) {
    const int do_w = g->do_w, nq = do_w ? W : 1;
    for (int64_t k = 0; k < n; ++k) {
        const FN(rec_t) *q = &recs[k];
        int ic = q->ic - ibase, jc = q->jc - jbase;
        if (ic < 0) ic += g->ngx;
        if (jc < 0) jc += g->ngy;
        REAL ku[MAXW], kv2[2 * MAXW], kw[MAXW];
        for (int t = 0; t < W; ++t) {
            ku[t] = FN(es_tap)(q->fu + (REAL)t, ihw, beta);
            kv2[2 * t] = kv2[2 * t + 1] = FN(es_tap)(q->fv + (REAL)t, ihw, beta);
            kw[t] = do_w ? FN(es_tap)(q->fw + (REAL)t, ihw, beta) : (REAL)(t == 0);
        }
        for (int qq = 0; qq < nq; ++qq) {
            REAL *p = buf + pl * (size_t)(q->p0 - pmin + qq);
            const REAL cr = q->re * kw[qq], ci = q->im * kw[qq];
            for (int t = 0; t < W; ++t) {
                REAL cv[2 * MAXW];
                for (int x = 0; x < 2 * W; x += 2) {
                    cv[x] = cr * ku[t];
                    cv[x + 1] = ci * ku[t];
                }
                REAL *row = p + 2 * ((size_t)(ic + t) * RY + jc);
                for (int x = 0; x < 2 * W; ++x) row[x] += cv[x] * kv2[x];
            }
        }
    }
}

/* one visibility -> record (global footprint origin), written by the
   scatter pass of the counting sort */
static inline void FN(decode)(const Geo *g, const double *uvw, const double *freq,
                              const void *vis, int vis_f64, const void *wgt, int wgt_f64,
                              int64_t v, FN(rec_t) *q) {
    const int64_t r = v / g->nchan;
    const int c = (int)(v - r * g->nchan);
    Coord cd;
    vis_coord(g, uvw, r, freq[c], &cd);
    double wt = 1.0;
    if (wgt) wt = wgt_f64 ? ((const double *)wgt)[v] : (double)((const float *)wgt)[v];
    double re = 1.0, im = 0.0;
    if (vis) {
        if (vis_f64) {
            re = ((const double *)vis)[2 * v];
            im = ((const double *)vis)[2 * v + 1];
        } else {
            re = ((const float *)vis)[2 * v];
            im = ((const float *)vis)[2 * v + 1];
        }
    }
    cf64 val = (re + I * im) * wt;
    if (g->do_w) val *= cexp(2.0 * M_PI * I * (cd.w * g->s0 - rint(cd.w * g->s0)));
    q->re = (REAL)creal(val);
    q->im = (REAL)cimag(val);
    q->fu = (REAL)cd.fu;
    q->fv = (REAL)cd.fv;
    q->fw = (REAL)cd.fw;
    q->ic = cd.ic;
    q->jc = cd.jc;
    q->p0 = cd.p0;
}

static void FN(grid_task)(const Geo *g, const FN(rec_t) *recs, int64_t n, int tile, REAL *buf,
                          REAL *grid, omp_lock_t *locks) {
    const int W = g->W, RX = TILE + W - 1, RY = TILE + W - 1;
    const int ntc = g->ntc, tx = tile / ntc, ty = tile - tx * ntc;
    const int ibase = tx * TILE, jbase = ty * TILE;
    const REAL ihw = (REAL)2 / (REAL)W, beta = (REAL)g->beta;
    int pmin = 1 << 30, pmax = -1;
    for (int64_t k = 0; k < n; ++k) {
        if (recs[k].p0 < pmin) pmin = recs[k].p0;
        if (recs[k].p0 > pmax) pmax = recs[k].p0;
    }
    if (pmax < 0) return;
    const int np = pmax - pmin + (g->do_w ? W : 1);
    const size_t pl = (size_t)RX * RY * 2;
    memset(buf, 0, sizeof(REAL) * pl * np);
    switch (W) {
#define CASE_W(w)                                                                        \
    case w:                                                                              \
        FN(grid_recs)(recs, n, buf, pl, pmin, w, RY, ibase, jbase, g, ihw, beta);                 \
        break;
        CASE_W(2) CASE_W(3) CASE_W(4) CASE_W(5) CASE_W(6) CASE_W(7) CASE_W(8) CASE_W(9)
        CASE_W(10) CASE_W(11) CASE_W(12) CASE_W(13) CASE_W(14) CASE_W(15) CASE_W(16)
#undef CASE_W
    }
    /* merge: the buffer spans this tile and the halo in the tiles at +1 in x
       and/or y (W - 1 < TILE); their locks are taken in ascending order */
    int lk[4], nl = 0;
    const int ntr = g->ntr;
    const int txs[2] = {tx, (tx + 1) % ntr}, tys[2] = {ty, (ty + 1) % ntc};
    for (int a = 0; a < 2; ++a)
        for (int c = 0; c < 2; ++c) {
            const int id = txs[a] * ntc + tys[c];
            int dup = 0;
            for (int m = 0; m < nl; ++m) dup |= lk[m] == id;
            if (!dup) lk[nl++] = id;
        }
    for (int i = 1; i < nl; ++i)
        for (int j = i; j > 0 && lk[j - 1] > lk[j]; --j) {
            const int t = lk[j];
            lk[j] = lk[j - 1];
            lk[j - 1] = t;
        }
    for (int i = 0; i < nl; ++i) omp_set_lock(&locks[lk[i]]);
    const size_t plane = (size_t)g->ngx * g->ngy;
    for (int p = 0; p < np; ++p) {
        const REAL *s = buf + pl * (size_t)p;
        REAL *gp = grid + 2 * plane * (size_t)(pmin + p);
        for (int x = 0; x < RX; ++x) {
            int gx = ibase + x;
            if (gx >= g->ngx) gx -= g->ngx;
            REAL *dst = gp + 2 * (size_t)gx * g->ngy;
            const REAL *src = s + 2 * (size_t)x * RY;
            if (jbase + RY <= g->ngy) {
                REAL *d = dst + 2 * jbase;
                for (int y = 0; y < 2 * RY; ++y) d[y] += src[y];
            } else {
                for (int y = 0; y < RY; ++y) {
                    int gy = jbase + y;
                    if (gy >= g->ngy) gy -= g->ngy;
                    dst[2 * gy] += src[2 * y];
                    dst[2 * gy + 1] += src[2 * y + 1];
                }
            }
        }
    }
    for (int i = nl - 1; i >= 0; --i) omp_unset_lock(&locks[lk[i]]);
}

/* dirty2ms degridding of one visibility (reads the resident planes) */
static cf64 FN(degrid_one)(const Geo *g, const REAL *grid, const Coord *cd) {
    const int W = g->W;
    const REAL ihw = (REAL)2 / (REAL)W, beta = (REAL)g->beta;
    REAL ku[MAXW], kv[MAXW], kw[MAXW];
    for (int t = 0; t < W; ++t) {
        ku[t] = FN(es_tap)((REAL)cd->fu + (REAL)t, ihw, beta);
        kv[t] = FN(es_tap)((REAL)cd->fv + (REAL)t, ihw, beta);
        kw[t] = g->do_w ? FN(es_tap)((REAL)cd->fw + (REAL)t, ihw, beta) : (REAL)(t == 0);
    }
    const int nq = g->do_w ? W : 1;
    const size_t plane = (size_t)g->ngx * g->ngy;
    const int fast = cd->jc + W <= g->ngy;
    REAL sr = 0, si = 0;
    for (int q = 0; q < nq; ++q) {
        const REAL *pl = grid + 2 * plane * (size_t)(cd->p0 + q);
        REAL qr = 0, qi = 0;
        for (int t = 0; t < W; ++t) {
            int gi = cd->ic + t;
            if (gi >= g->ngx) gi -= g->ngx;
            const REAL *row = pl + 2 * (size_t)gi * g->ngy;
            REAL rr = 0, ri = 0;
            if (fast) {
                const REAL *src = row + 2 * cd->jc;
                for (int tt = 0; tt < W; ++tt) {
                    rr += kv[tt] * src[2 * tt];
                    ri += kv[tt] * src[2 * tt + 1];
                }
            } else {
                for (int tt = 0; tt < W; ++tt) {
                    int gj = cd->jc + tt;
                    if (gj >= g->ngy) gj -= g->ngy;
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
    return (double)sr + I * (double)si;
}

#undef FN
#undef CAT
#undef CAT_
