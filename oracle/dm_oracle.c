/*
 * dm_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (deepmatching_stereo_matching_amd/) never links or calls it.
 *
 * It follows the reference step by step, deliberately WITHOUT the algebraic shortcuts
 * the HIP kernels take (pooling before normalisation / rectification, on-demand level-0
 * recomputation), so that it checks them:
 *
 *   dmo_corr_l0    Correlation_map._create_atomic_patch + _create_simple_initial_co_map
 *                  (misc/Correlation_map.py:51-87) with Feature_value.__call__ / min_max
 *                  (misc/Feature_value.py:32-43) and the pinned matchTemplate arithmetic
 *                  of oracle/cv2_shim/cv2.py (OpenCV's own arithmetic is unpinnable).
 *   dmo_rectify    Correlation_map._rectification  (misc/Correlation_map.py:158-159)
 *   dmo_aggregate  Correlation_map._aggregation    (misc/Correlation_map.py:89-130),
 *                  Maxpool = nn.MaxPool2d(3, 2, padding=1) (:176-184), NaN-propagating.
 *   dmo_match      Matching.__call__ (misc/Matching.py:211-222): _initial_move_map
 *                  (:80-96), _B / _calc_match (:98-149), _calc_near_match (:58-78),
 *                  _sub_pix_cal / _sub_pix_compute (:165-209).  (_filter: oracle.py.)
 *   dmo_cal_map    Calc_difference.cal_map (misc/Calc_difference.py:26-49).
 *
 * pow() is the C library's, as numpy's float64 power is in the reference (which itself
 * may differ by 1 ulp between machines: SVML vs libm, see DESIGN.md "Numerics").
 *
 * Parity pinned by the tests/golden npz fixtures, generated from the reference itself.
 * Build: oracle/Makefile  (gcc -O2 -fopenmp -ffp-contract=off; no fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../deepmatching_stereo_matching_amd/csrc/dm_pow.h"

#define DMO_NORMED 5 /* cv2.TM_CCOEFF_NORMED */
#define DMO_CCOEFF 4 /* cv2.TM_CCOEFF */

/* ---- level 0 -------------------------------------------------------------------- */
/* Per-window sums of the template image: sI[q] = sum(I), bq[q] = f32(1/sqrt(f64 dI)). */
typedef struct {
    const uint8_t *img, *tmpl;
    int W, ws, h0, w0, method, formula;
    int64_t *sI, *dI;
    float *bq;
} l0_src;

/* ZNCC formula: 0 = the pinned one the kernels evaluate,
 *   y = f32(num) * f32(1/sqrt(f64 dI)), r = clamp(y * f32(1/sqrt(f64 dT)));
 * 1 = SURVEY.md 8(c)'s, r = f32(clamp(num / sqrt(f64 dT * f64 dI))) (OpenCV's double-
 * precision division, one rounding).  1 exists only to MEASURE the difference
 * (tools/zncc_pin.py); the goldens and every parity test use 0. */
static int g_zncc = 0;
void dmo_set_zncc_formula(int f) { g_zncc = f; }

static int l0_init(l0_src *s, const uint8_t *img, const uint8_t *tmpl, int H, int W, int ws,
                   int method)
{
    if (ws < 1 || (ws & 1) == 0 || H < ws || W < ws || ws > 21) return -1;
    if (method != DMO_NORMED && method != DMO_CCOEFF) return -2;
    s->img = img; s->tmpl = tmpl; s->W = W; s->ws = ws; s->method = method;
    s->formula = g_zncc;
    s->h0 = H - ws + 1; s->w0 = W - ws + 1;
    const int n = ws * ws;
    const long P = (long)s->h0 * s->w0;
    s->sI = malloc(sizeof(int64_t) * P);
    s->dI = malloc(sizeof(int64_t) * P);
    s->bq = malloc(sizeof(float) * P);
    for (int q0 = 0; q0 < s->h0; ++q0)
        for (int q1 = 0; q1 < s->w0; ++q1) {
            int64_t a = 0, a2 = 0;
            for (int u = 0; u < ws; ++u)
                for (int v = 0; v < ws; ++v) {
                    int64_t x = tmpl[(long)(q0 + u) * W + q1 + v];
                    a += x; a2 += x * x;
                }
            long q = (long)q0 * s->w0 + q1;
            int64_t dI = (int64_t)n * a2 - a * a;
            s->sI[q] = a;
            s->dI[q] = dI;
            s->bq[q] = dI == 0 ? 0.0f : (float)(1.0 / sqrt((double)dI));
        }
    return 0;
}

static void l0_free(l0_src *s) { free(s->sI); free(s->dI); free(s->bq); }

/* Row p of the level-0 volume: Feature_value(patch p, template) = matchTemplate with the
 * pinned formula (oracle/cv2_shim/cv2.py), then min_max (misc/Feature_value.py:32-43), in
 * float32.  acc: w0 int32 scratch.  sum(T*I) <= 21*21*255*255 fits int32 exactly. */
static void l0_row(const l0_src *s, long p, float *row, int32_t *acc)
{
    const int ws = s->ws, W = s->W, h0 = s->h0, w0 = s->w0, n = ws * ws;
    const long P = (long)h0 * w0;
    const int p0 = (int)(p / w0), p1 = (int)(p % w0);
    int T[21 * 21];
    int64_t sT = 0, sT2 = 0;
    for (int u = 0; u < ws; ++u)
        for (int v = 0; v < ws; ++v) {
            int x = s->img[(long)(p0 + u) * W + p1 + v];
            T[u * ws + v] = x; sT += x; sT2 += (int64_t)x * x;
        }
    const int64_t dT = (int64_t)n * sT2 - sT * sT;
    const float a = dT == 0 ? 0.0f : (float)(1.0 / sqrt((double)dT));
    const float inv_n = (float)(1.0 / n);
    for (int q0 = 0; q0 < h0; ++q0) {
        for (int q1 = 0; q1 < w0; ++q1) acc[q1] = 0;
        for (int u = 0; u < ws; ++u)
            for (int v = 0; v < ws; ++v) {
                const int32_t t = T[u * ws + v];
                const uint8_t *ir = s->tmpl + (long)(q0 + u) * W + v;
                for (int q1 = 0; q1 < w0; ++q1) acc[q1] += t * (int32_t)ir[q1];
            }
        float *o = row + (long)q0 * w0;
        for (int q1 = 0; q1 < w0; ++q1) {
            const long q = (long)q0 * w0 + q1;
            const int64_t num = (int64_t)n * acc[q1] - sT * s->sI[q];
            float r;
            if (s->method == DMO_CCOEFF) {
                r = (float)num * inv_n;
            } else if (dT == 0) {
                r = 1.0f;
            } else if (s->formula == 1) {
                if (s->dI[q] == 0) {
                    r = 0.0f;
                } else {
                    double d = (double)num / sqrt((double)dT * (double)s->dI[q]);
                    r = (float)(d < -1.0 ? -1.0 : (d > 1.0 ? 1.0 : d));
                }
            } else {
                const float y = (float)num * s->bq[q];
                r = y * a;
                r = r < -1.0f ? -1.0f : (r > 1.0f ? 1.0f : r);
            }
            o[q1] = r;
        }
    }
    /* Feature_value.min_max: (x - min) / (max - min) in float32 */
    float mn = row[0], mx = row[0];
    for (long q = 1; q < P; ++q) {
        if (row[q] < mn) mn = row[q];
        if (row[q] > mx) mx = row[q];
    }
    const float den = mx - mn;
    for (long q = 0; q < P; ++q) row[q] = (row[q] - mn) / den;
}

/* img/tmpl: uint8 H x W row-major.  l0: [h0*w0][h0*w0] float32, h0 = H-ws+1.
 * Correlation_map._create_atomic_patch + _create_simple_initial_co_map (:51-87). */
int dmo_corr_l0(const uint8_t *img, const uint8_t *tmpl, int H, int W, int ws,
                int method, float *l0)
{
    l0_src s;
    int rc = l0_init(&s, img, tmpl, H, W, ws, method);
    if (rc) return rc;
    const long P = (long)s.h0 * s.w0;
    #pragma omp parallel
    {
        int32_t *acc = malloc(sizeof(int32_t) * s.w0);
        #pragma omp for schedule(dynamic, 1)
        for (long p = 0; p < P; ++p) l0_row(&s, p, l0 + p * P, acc);
        free(acc);
    }
    l0_free(&s);
    return 0;
}

/* Rows of selected patches only (out: [n][P] float32): the level-0 values the C5 tests
 * sample from an S = 256 tile without materialising its 17 GB volume. */
int dmo_corr_l0_rows(const uint8_t *img, const uint8_t *tmpl, int H, int W, int ws, int method,
                     const int64_t *patches, long n, float *out)
{
    l0_src s;
    int rc = l0_init(&s, img, tmpl, H, W, ws, method);
    if (rc) return rc;
    const long P = (long)s.h0 * s.w0;
    for (long k = 0; k < n; ++k)
        if (patches[k] < 0 || patches[k] >= P) { l0_free(&s); return -3; }
    #pragma omp parallel
    {
        int32_t *acc = malloc(sizeof(int32_t) * s.w0);
        #pragma omp for schedule(dynamic, 1)
        for (long k = 0; k < n; ++k) l0_row(&s, patches[k], out + k * P, acc);
        free(acc);
    }
    l0_free(&s);
    return 0;
}

/* Distance between the two ZNCC formulas on one pair's level 0 (tools/zncc_pin.py):
 * st[0] = values that differ, st[1] = max float32 ulp distance (finite values),
 * st[2] = NaN positions that differ, st[3] = rows (patches) with any difference;
 * max_abs = max |a - b| over finite values. */
static long ulp_dist(float a, float b)
{
    int32_t ia, ib;
    memcpy(&ia, &a, 4); memcpy(&ib, &b, 4);
    if (ia < 0) ia = (int32_t)0x80000000 - ia;
    if (ib < 0) ib = (int32_t)0x80000000 - ib;
    long d = (long)ia - (long)ib;
    return d < 0 ? -d : d;
}

int dmo_zncc_formula_diff(const uint8_t *img, const uint8_t *tmpl, int H, int W, int ws, int method,
                          long *st, double *max_abs)
{
    l0_src s0, s1;
    const int keep = g_zncc;
    g_zncc = 0;
    int rc = l0_init(&s0, img, tmpl, H, W, ws, method);
    g_zncc = 1;
    if (!rc) rc = l0_init(&s1, img, tmpl, H, W, ws, method);
    g_zncc = keep;
    if (rc) return rc;
    const long P = (long)s0.h0 * s0.w0;
    long nd = 0, mu = 0, nn = 0, rows = 0;
    double ma = 0.0;
    #pragma omp parallel reduction(+:nd, nn, rows) reduction(max:mu, ma)
    {
        int32_t *acc = malloc(sizeof(int32_t) * s0.w0);
        float *a = malloc(sizeof(float) * P), *b = malloc(sizeof(float) * P);
        #pragma omp for schedule(dynamic, 1)
        for (long p = 0; p < P; ++p) {
            l0_row(&s0, p, a, acc);
            l0_row(&s1, p, b, acc);
            long d_row = 0;
            for (long q = 0; q < P; ++q) {
                const int na = isnan(a[q]), nb = isnan(b[q]);
                if (na || nb) { if (na != nb) { ++nn; ++d_row; } continue; }
                if (a[q] != b[q]) {
                    ++d_row;
                    const long u = ulp_dist(a[q], b[q]);
                    if (u > mu) mu = u;
                    const double ad = fabs((double)a[q] - (double)b[q]);
                    if (ad > ma) ma = ad;
                }
            }
            nd += d_row;
            rows += d_row > 0;
        }
        free(acc); free(a); free(b);
    }
    st[0] = nd; st[1] = mu; st[2] = nn; st[3] = rows;
    *max_abs = ma;
    l0_free(&s0); l0_free(&s1);
    return 0;
}

/* ---- rectification: out = (double)in ** lam ------------------------------------- */
/* pow mode 0: the C library's pow (as numpy on this host); mode 1: the build's pinned
 * dm_pow14 (dm_pow.h), which the GPU kernels use -- GPU parity tests select it so that
 * every float64 output can be compared bit for bit. */
static int g_pow_mode = 0;
static const double POW_TAB[] = DM_POW_TAB_INIT;
static const double POW_G[] = DM_POW_G_INIT;
static const double POWF_C[] = DM_POWF_C_INIT;
static const double POWF_P[] = DM_POWF_P_INIT;
static const double POWF_G[] = DM_POWF_G_INIT;
static const dm_pow_tabs POW_TABS = {POWF_C, POWF_P, POWF_G, POW_TAB, POW_G};

void dmo_set_pow_mode(int mode) { g_pow_mode = mode; }

double dmo_pow14(double x) { return dm_pow14(x, &POW_TABS); }

static inline double rect(double x, double lam)
{
    return g_pow_mode == 1 ? dm_pow14(x, &POW_TABS) : pow(x, lam);
}

void dmo_rectify_f32(const float *in, long n, double lam, double *out)
{
    #pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) out[i] = rect((double)in[i], lam);
}

void dmo_rectify_f64(double *inout, long n, double lam)
{
    #pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) inout[i] = rect(inout[i], lam);
}

/* torch max_pool2d semantics: -inf padding, NaN propagates */
static inline double nanmax(double acc, double v)
{
    return (v > acc || isnan(v)) ? v : acc;
}

/* ---- aggregation: in (h,w,h,w) f64 -> out (h/2,w/2,h/2,w/2) f64, NOT rectified ----- */
int dmo_aggregate(const double *in, int h, int w, double *out)
{
    if ((h & 1) || (w & 1)) return -1;
    const int h2 = h / 2, w2 = w / 2;
    const long P = (long)h * w, P2 = (long)h2 * w2;
    double *R = malloc(sizeof(double) * P * P2);
    /* res[i, j] = Maxpool(map[i, j]) for every p */
    #pragma omp parallel for schedule(static)
    for (long p = 0; p < P; ++p) {
        const double *m = in + p * P;
        double *r = R + p * P2;
        for (int u = 0; u < h2; ++u)
            for (int v = 0; v < w2; ++v) {
                double acc = -INFINITY;
                for (int a = 2 * u - 1; a <= 2 * u + 1; ++a) {
                    if (a < 0 || a >= h) continue;
                    for (int b = 2 * v - 1; b <= 2 * v + 1; ++b) {
                        if (b < 0 || b >= w) continue;
                        acc = nanmax(acc, m[(long)a * w + b]);
                    }
                }
                r[(long)u * w2 + v] = acc;
            }
    }
    /* output[i, j] = (ul + ur + ll + lr) / 4, left to right */
    #pragma omp parallel for schedule(static)
    for (long c = 0; c < P2; ++c) {
        const int i = (int)(c / w2), j = (int)(c % w2);
        const double *ul = R + ((long)(2 * i) * w + 2 * j) * P2;
        const double *ur = R + ((long)(2 * i) * w + 2 * j + 1) * P2;
        const double *ll = R + ((long)(2 * i + 1) * w + 2 * j) * P2;
        const double *lr = R + ((long)(2 * i + 1) * w + 2 * j + 1) * P2;
        double *o = out + c * P2;
        for (long k = 0; k < P2; ++k) o[k] = (ul[k] + ur[k] + ll[k] + lr[k]) / 4;
    }
    free(R);
    return 0;
}

/* ---- matching ------------------------------------------------------------------- */
/* _calc_near_match on map M (h x w) = co_map[p]; returns row, col, score */
static void near_match(const double *M, int h, int w, int pd0, int pd1, double *o)
{
    double win[9];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            const int r = pd0 - 1 + a, c = pd1 - 1 + b;
            win[a * 3 + b] = (r < 0 || r >= h || c < 0 || c >= w) ? 0.0 : M[(long)r * w + c];
        }
    /* np.argmax: first maximum, a NaN wins at its first occurrence; np.max -> NaN */
    int m = 0, has_nan = isnan(win[0]);
    double best = win[0];
    if (!has_nan)
        for (int k = 1; k < 9; ++k) {
            if (isnan(win[k])) { m = k; has_nan = 1; break; }
            if (win[k] > best) { best = win[k]; m = k; }
        }
    if (!has_nan && best < 0.0001) m = 4;
    o[0] = (double)(pd0 + m / 3 - 1);
    o[1] = (double)(pd1 + m % 3 - 1);
    o[2] = win[m] + M[(long)pd0 * w + pd1];
}

static double sub_pix_compute(double r0, double r1, double r_)
{
    if (r0 > r1 && r0 > r_) return -(r1 - r_) / (2 * (r1 + r_ - 2 * r0));
    return 0;
}

/* Matching._sub_pix_cal for one pixel (misc/Matching.py:177-209) on its rectified level-0
 * map M (h0 x w0): rows, then columns.  c = int(entry) indexes co_map_list[0][i, j] the numpy
 * way: an index in [-N, N) is valid and a negative one wraps, any other raises IndexError ->
 * bare except -> i - d_x (j - d_y).  The row step reads (c0 - 1 | c0 | c0 + 1, c1), the
 * column step (c0, c1 - 1 | c1 | c1 + 1).  (NaN / huge entries: the reference's int() raises
 * outside the try; taken as the except branch here.) */
static int py_index(double v) { return (v == v && fabs(v) < 1073741824.0) ? (int)v : -0x40000000; }
static int py_in(int k, int n) { return k >= -n && k < n; }
static int py_wrap(int k, int n) { return k < 0 ? k + n : k; }

static void sub_pix_one(const double *M, int h0, int w0, int i, int j, double *m0, double *m1)
{
    const int c0 = py_index(*m0), c1 = py_index(*m1);
    const double d_x = i - *m0;
    double v = i - d_x;                                  /* IndexError branch */
    if (py_in(c0 - 1, h0) && py_in(c0 + 1, h0) && py_in(c1, w0)) {
        const long b = py_wrap(c1, w0);
        const double r0 = M[(long)py_wrap(c0, h0) * w0 + b], r1 = M[(long)py_wrap(c0 + 1, h0) * w0 + b],
                     r_ = M[(long)py_wrap(c0 - 1, h0) * w0 + b];
        v = v + sub_pix_compute(r0, r1, r_);
    }
    *m0 = v;
    const double d_y = j - *m1;
    v = j - d_y;
    if (py_in(c1 - 1, w0) && py_in(c1 + 1, w0) && py_in(c0, h0)) {
        const long a = (long)py_wrap(c0, h0) * w0;
        const double r0 = M[a + py_wrap(c1, w0)], r1 = M[a + py_wrap(c1 + 1, w0)],
                     r_ = M[a + py_wrap(c1 - 1, w0)];
        v = v + sub_pix_compute(r0, r1, r_);
    }
    *m1 = v;
}

static const int OFF[4][2] = {{1, 1}, {0, 1}, {1, 0}, {0, 0}};   /* _B's o order (:111) */

/* _initial_move_map + _B down to level `stop` (misc/Matching.py:80-149); cur holds the
 * (3, h, w) map of level `stop` on return.  levels[l] for l >= stop must be present. */
static void descend(const double *const *levels, int nlev, int h0, int w0, int stop,
                    double **pcur, double **pnxt)
{
    double *cur = *pcur, *nxt = *pnxt;
    int h = h0 >> (nlev - 1), w = w0 >> (nlev - 1);
    const double *L = levels[nlev - 1];
    long P = (long)h * w;
    for (int i = 0; i < h; ++i)
        for (int j = 0; j < w; ++j) {
            double o[3];
            near_match(L + ((long)i * w + j) * P, h, w, i, j, o);
            for (int k = 0; k < 3; ++k) cur[k * P + (long)i * w + j] = o[k];
        }
    for (int l = nlev - 2; l >= stop; --l) {
        const int hn = h * 2, wn = w * 2;
        const long Pn = (long)hn * wn;
        L = levels[l];
        for (int i = 0; i < h; ++i)
            for (int j = 0; j < w; ++j) {
                const long pc = (long)i * w + j;
                const int64_t b0 = (int64_t)(cur[pc] * 2), b1 = (int64_t)(cur[P + pc] * 2);
                for (int k = 0; k < 4; ++k) {
                    const int p0 = 2 * i + OFF[k][0], p1 = 2 * j + OFF[k][1];
                    double o[3];
                    near_match(L + ((long)p0 * wn + p1) * Pn, hn, wn,
                               (int)(b0 + OFF[k][0]), (int)(b1 + OFF[k][1]), o);
                    for (int c = 0; c < 3; ++c) nxt[c * Pn + (long)p0 * wn + p1] = o[c];
                }
            }
        double *t = cur; cur = nxt; nxt = t;
        h = hn; w = wn; P = Pn;
    }
    *pcur = cur; *pnxt = nxt;
}

/* levels[l]: (h0>>l, w0>>l, h0>>l, w0>>l) f64 rectified.  out: (3, h0, w0) f64. */
int dmo_match(const double *const *levels, int nlev, int h0, int w0, int sub_pix,
              double *out)
{
    if (nlev < 2) return -1; /* Matching._B indexes co_map_list[-2] unconditionally */
    double *cur = malloc(sizeof(double) * 3 * (size_t)h0 * w0);
    double *nxt = malloc(sizeof(double) * 3 * (size_t)h0 * w0);
    descend(levels, nlev, h0, w0, 0, &cur, &nxt);
    const long P = (long)h0 * w0;
    if (sub_pix)
        for (int i = 0; i < h0; ++i)
            for (int j = 0; j < w0; ++j) {
                const long pc = (long)i * w0 + j;
                sub_pix_one(levels[0] + pc * P, h0, w0, i, j, &cur[pc], &cur[P + pc]);
            }
    memcpy(out, cur, sizeof(double) * 3 * P);
    free(cur); free(nxt);
    return 0;
}

/* ---- streaming mode: tiles whose level 0 does not fit in host memory (C5, S = 256) ---- *
 * The same arithmetic in the same order as dmo_corr_l0 -> pyramid -> dmo_match, but level 0
 * is never stored: each level-1 cell recomputes its four children's level-0 rows, rectifies
 * them (_rectification, :158-159), max-pools them (:101-103) and averages the four pooled
 * maps (:109-122) before the cell's own rectification (:148); the last descent step of
 * Matching (level 0) and the sub-pixel fit recompute each pixel's level-0 row. */

/* rectified level-0 row of patch p: x[q] = rect(min-max ZNCC) as float64 */
static void l0_row_rect(const l0_src *s, long p, double lam, float *row, double *x, int32_t *acc)
{
    const long P = (long)s->h0 * s->w0;
    l0_row(s, p, row, acc);
    for (long q = 0; q < P; ++q) x[q] = rect((double)row[q], lam);
}

/* level 1 (rectified): l1 [(h0/2)(w0/2)][(h0/2)(w0/2)] float64 */
int dmo_corr_level1_stream(const uint8_t *img, const uint8_t *tmpl, int H, int W, int ws,
                           int method, double lam, double *l1)
{
    l0_src s;
    int rc = l0_init(&s, img, tmpl, H, W, ws, method);
    if (rc) return rc;
    const int h0 = s.h0, w0 = s.w0, h1 = h0 / 2, w1 = w0 / 2;
    if ((h0 & 1) || (w0 & 1)) { l0_free(&s); return -4; }
    const long P = (long)h0 * w0, P1 = (long)h1 * w1;
    #pragma omp parallel
    {
        int32_t *acc = malloc(sizeof(int32_t) * w0);
        float *row = malloc(sizeof(float) * P);
        double *x = malloc(sizeof(double) * P);
        double *R = malloc(sizeof(double) * 4 * P1);
        #pragma omp for schedule(dynamic, 1)
        for (long c = 0; c < P1; ++c) {
            const int i = (int)(c / w1), j = (int)(c % w1);
            /* children in the reference's summation order: ul, ur, ll, lr */
            const long child[4] = {(long)(2 * i) * w0 + 2 * j, (long)(2 * i) * w0 + 2 * j + 1,
                                   (long)(2 * i + 1) * w0 + 2 * j, (long)(2 * i + 1) * w0 + 2 * j + 1};
            for (int k = 0; k < 4; ++k) {
                l0_row_rect(&s, child[k], lam, row, x, acc);
                double *r = R + k * P1;
                for (int u = 0; u < h1; ++u)
                    for (int v = 0; v < w1; ++v) {
                        double m = -INFINITY;
                        for (int a = 2 * u - 1; a <= 2 * u + 1; ++a) {
                            if (a < 0 || a >= h0) continue;
                            for (int b = 2 * v - 1; b <= 2 * v + 1; ++b) {
                                if (b < 0 || b >= w0) continue;
                                m = nanmax(m, x[(long)a * w0 + b]);
                            }
                        }
                        r[(long)u * w1 + v] = m;
                    }
            }
            double *o = l1 + c * P1;
            for (long k = 0; k < P1; ++k)
                o[k] = rect((R[k] + R[P1 + k] + R[2 * P1 + k] + R[3 * P1 + k]) / 4, lam);
        }
        free(acc); free(row); free(x); free(R);
    }
    l0_free(&s);
    return 0;
}

/* Matching()() with level 0 recomputed: levels[0] is ignored (may be NULL), levels[1..] as
 * dmo_match.  out: (3, h0, w0) f64. */
int dmo_match_stream(const uint8_t *img, const uint8_t *tmpl, int H, int W, int ws, int method,
                     double lam, const double *const *levels, int nlev, int sub_pix, double *out)
{
    if (nlev < 2) return -1;
    l0_src s;
    int rc = l0_init(&s, img, tmpl, H, W, ws, method);
    if (rc) return rc;
    const int h0 = s.h0, w0 = s.w0, h1 = h0 / 2, w1 = w0 / 2;
    const long P = (long)h0 * w0, P1 = (long)h1 * w1;
    double *cur = malloc(sizeof(double) * 3 * (size_t)P);
    double *nxt = malloc(sizeof(double) * 3 * (size_t)P);
    descend(levels, nlev, h0, w0, 1, &cur, &nxt);           /* level-1 map in cur */
    #pragma omp parallel
    {
        int32_t *acc = malloc(sizeof(int32_t) * w0);
        float *row = malloc(sizeof(float) * P);
        double *x = malloc(sizeof(double) * P);
        #pragma omp for schedule(dynamic, 1)
        for (long pc = 0; pc < P1; ++pc) {
            const int i = (int)(pc / w1), j = (int)(pc % w1);
            const int64_t b0 = (int64_t)(cur[pc] * 2), b1 = (int64_t)(cur[P1 + pc] * 2);
            for (int k = 0; k < 4; ++k) {
                const int p0 = 2 * i + OFF[k][0], p1 = 2 * j + OFF[k][1];
                const long p = (long)p0 * w0 + p1;
                l0_row_rect(&s, p, lam, row, x, acc);
                double o[3];
                near_match(x, h0, w0, (int)(b0 + OFF[k][0]), (int)(b1 + OFF[k][1]), o);
                if (sub_pix) sub_pix_one(x, h0, w0, p0, p1, &o[0], &o[1]);
                for (int c = 0; c < 3; ++c) nxt[c * P + p] = o[c];
            }
        }
        free(acc); free(row); free(x);
    }
    memcpy(out, nxt, sizeof(double) * 3 * P);
    free(cur); free(nxt);
    l0_free(&s);
    return 0;
}

/* mode: 0 elevation (j - map[1]), 1 elevation2 (i - map[0]), 2 distance */
int dmo_cal_map(const double *map, int h, int w, int mode, double *out)
{
    const long P = (long)h * w;
    if (mode < 0 || mode > 2) return -1;
    for (int i = 0; i < h; ++i)
        for (int j = 0; j < w; ++j) {
            const long k = (long)i * w + j;
            if (mode == 0) out[k] = (double)j - map[P + k];
            else if (mode == 1) out[k] = (double)i - map[k];
            else {
                const double a = (double)i - map[k], b = (double)j - map[P + k];
                out[k] = sqrt(a * a + b * b);
            }
        }
    return 0;
}

/* ---- Gauss-Seidel post-processing ---------------------------- *
 * Plain sequential loops in the reference's own order, no scheduling: they check the
 * dependency-level execution of dm_postproc.hip.  exp() is the pinned dm_exp shared with
 * the kernels (numpy's own exp is 1 ulp apart on some inputs; the goldens hold it). */
#include "../deepmatching_stereo_matching_amd/csrc/dm_exp.h"

static inline long pyix(long i, long n) { return i < 0 ? i + n : i; } /* python's a[-1] */

/* misc/optimize_loop.py:15-37 on an already thresholded map (image_threshold, :40-44, is
 * the caller's np.where); returns error, the backward sweep's sum of |x - d|. */
double dmo_optimize_loop(double *img, const double *coef, int wc, int h, int w, int s0, int s1,
                         int e, double alpha)
{
    (void)h;
    /* forward (:18-25) */
    for (int i = e; i < s0 - e - 1; ++i)
        for (int j = e; j < s1 - e - 1; ++j) {
            double *m = img;
            const double sum_d = ((m[(long)i * w + pyix(j - 1, w)] + m[(long)i * w + j + 1]) +
                                  m[pyix(i - 1, h) * w + j]) + m[(long)(i + 1) * w + j];
            const double a = coef[(long)i * wc + j];
            const double d_new = (-a * m[(long)i * w + j] + alpha * sum_d) / (-a + 4.0 * alpha);
            m[(long)i * w + j] = d_new;
        }
    /* backward (:27-36): `i = size[0] - i - 1` rebinds the outer variable every inner step */
    double error = 0.0;
    for (int i0 = e; i0 < s0 - e - 1; ++i0) {
        int i = i0;
        for (int j0 = e; j0 < s1 - e - 1; ++j0) {
            i = s0 - i - 1;
            const int j = s1 - j0 - 1;
            double *m = img;
            const double sum_d = ((m[(long)i * w + pyix(j - 1, w)] + m[(long)i * w + j + 1]) +
                                  m[pyix(i - 1, h) * w + j]) + m[(long)(i + 1) * w + j];
            const double a = coef[(long)i * wc + j];
            const double d_new = (-a * m[(long)i * w + j] + alpha * sum_d) / (-a + 4.0 * alpha);
            error += fabs(m[(long)i * w + j] - d_new);
            m[(long)i * w + j] = d_new;
        }
    }
    return error;
}

/* misc/opt_loop.py make_weight (:60-85); color: [s0-e][s1-e][W][W] zero-filled by the caller */
void dmo_make_weight(const double *guide, int w, int s0, int s1, int e, double den_c, double den_s,
                     double *gauss, double *color)
{
    const int W = 2 * e + 1;
    for (int i = 0; i < W; ++i)
        for (int j = 0; j < W; ++j)
            gauss[i * W + j] = dm_exp(-((double)((i - e) * (i - e) + (j - e) * (j - e))) / den_s);
    const long cw = s1 - e;
    for (int i = e; i < s0 - e - 1; ++i)
        for (int j = e; j < s1 - e - 1; ++j) {
            double *out = color + ((long)(i - e) * cw + (j - e)) * W * W;
            for (int a = 0; a < W; ++a)
                for (int b = 0; b < W; ++b) {
                    double c = guide[(long)i * w + j] - guide[(long)(i - e + a) * w + (j - e + b)];
                    c = -1.0 * c * c / den_c;
                    out[a * W + b] = dm_exp(c);
                }
        }
}

/* numpy pairwise summation (contiguous, n elements): < 8 sequential, <= 128 eight
 * accumulators, else split at n/2 rounded down to a multiple of 8 (recursive) */
static double np_sum(const double *a, long n)
{
    if (n < 8) {
        double res = -0.0;
        for (long i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return np_sum(a, n2) + np_sum(a + n2, n - n2);
}

/* misc/opt_loop.py optimize_loop_bilateral_horizon (:16-35) / _vertical (:39-58); returns error */
double dmo_opt_loop_bilateral(double *img, const double *color, const double *gauss, const double *coef,
                              int hc, int wc, int w, int s0, int s1, int e, int vertical)
{
    const int W = 2 * e + 1, n = W * W;
    const long cw = s1 - e;
    double *p1 = malloc(sizeof(double) * n), *p2 = malloc(sizeof(double) * n);
    const double c0 = coef[pyix(e, hc) * wc + pyix(e, wc)];
    const double cp = vertical ? coef[pyix(e + 1, hc) * wc + e] : coef[pyix(e, hc) * wc + e + 1];
    const double cm = vertical ? coef[pyix(e - 1, hc) * wc + e] : coef[pyix(e, hc) * wc + pyix(e - 1, wc)];
    double error = 0.0;
    for (int i = e; i < s0 - e - 1; ++i)
        for (int j = e; j < s1 - e - 1; ++j) {
            const double *cwt = color + ((long)(i - e) * cw + (j - e)) * n;
            const double a = -(c0 - (cp + cm) / 2.0);
            const double x = img[(long)i * w + j];
            const double b = x - (cp - cm) / 2.0 / (-2.0 * c0 + cp + cm);
            for (int k = 0; k < n; ++k) {
                p2[k] = gauss[k] * cwt[k];
                p1[k] = p2[k] * img[(long)(i - e + k / W) * w + (j - e + k % W)];
            }
            const double d_new = (-a * b + np_sum(p1, n)) / (-a + np_sum(p2, n));
            error += fabs(img[(long)i * w + j] - d_new);
            img[(long)i * w + j] = d_new;
        }
    free(p1);
    free(p2);
    (void)hc;
    return error;
}

double dmo_exp(double x) { return dm_exp(x); }
