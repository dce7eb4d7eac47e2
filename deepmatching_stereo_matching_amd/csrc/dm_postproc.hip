// dm_postproc.hip -- gfx950 kernels + C ABI of the Gauss-Seidel post-processing loops
// (SURVEY.md 8(f) row 4): misc/optimize_loop.py optimize_loop (:15-37) / image_threshold
// (:40-44) and misc/opt_loop.py optimize_loop_bilateral_horizon (:16-35),
// optimize_loop_bilateral_vertical (:39-58), make_weight (:60-85).
//
// The reference updates one pixel at a time, in place, in a fixed order (row-major; the
// backward sweep of optimize_loop in its own order, see gs_cell).  Every update reads the
// current values of its neighbourhood, so the result depends on that order.  Here a sweep
// runs as a dependency-level schedule (dm_gs_schedule, host): update u gets level
//   1 + max(level of the last writer of every cell u reads,
//           level of every reader of u's own cell since its last write)
// so all updates of one level are independent and every read sees exactly the value the
// sequential order gives it.  One workgroup walks the levels with a barrier between them;
// the arithmetic per update is the reference's, operation for operation (float64,
// -ffp-contract=off), so the maps are bit-identical to the sequential loops.  The error
// sums (`error += abs(...)`) are taken in sequence order by one dependent chain (k_seq_sum).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/dmstereo.h"
#include "dm_exp.h"

// error reporting lives in dm_kernels.hip (one thread-local message per thread)
__attribute__((visibility("hidden"))) int dm_vfail(int code, const char *fmt, va_list ap);

static int pfail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    const int r = dm_vfail(code, fmt, ap);
    va_end(ap);
    return r;
}

#define PHIP_TRY(x)                                                                          \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return pfail(DM_ERR_HIP, "HIP error: %s (%d)", hipGetErrorString(e_), (int)e_); \
    } while (0)

// python index semantics for the only negative index the loops can form (-1)
__host__ __device__ __forceinline__ int pyix(int i, int n) { return i < 0 ? i + n : i; }

struct GsGeo {
    int kind, h, w, s0, s1, e, nj;
};

// cell (r, c) of update s (sequence position) of a sweep.
//  FWD4 / BILAT: i = e + s / nj, j = e + s % nj  (optimize_loop.py:18-19, opt_loop.py:23-24)
//  BWD4 (optimize_loop.py:27-31): `i = size[0] - i - 1` rebinds the OUTER loop variable at
//  every inner step, so i alternates: inner step k even -> row s0-1-(e+o), k odd -> e+o;
//  the column is s1-1-(e+k).
__host__ __device__ __forceinline__ void gs_cell(const GsGeo &g, int s, int &r, int &c)
{
    const int o = s / g.nj, k = s - o * g.nj;
    if (g.kind == DM_GS_BWD4) {
        r = (k & 1) ? g.e + o : g.s0 - 1 - (g.e + o);
        c = g.s1 - 1 - (g.e + k);
    } else {
        r = g.e + o;
        c = g.e + k;
    }
}

static GsGeo gs_geo(int kind, int h, int w, int s0, int s1, int e)
{
    GsGeo g;
    g.kind = kind; g.h = h; g.w = w; g.s0 = s0; g.s1 = s1; g.e = e;
    g.nj = s1 - 2 * e - 1 > 0 ? s1 - 2 * e - 1 : 0;
    return g;
}

static long long gs_count(const GsGeo &g)
{
    const long long ni = g.s0 - 2 * g.e - 1;
    return (ni > 0 && g.nj > 0) ? ni * g.nj : 0;
}

// ---------------------------------------------------------------------------------------
// numpy's pairwise float64 sum (the order np.sum gives a contiguous array of n elements:
// 8 accumulators up to 128 elements, halving above), elements produced on the fly by f(m)
// ---------------------------------------------------------------------------------------
template <int D, typename F>
__device__ double np_pairwise(const F &f, int m0, int n)
{
    if (n < 8) {
        double res = -0.0;
        for (int i = 0; i < n; ++i) res += f(m0 + i);
        return res;
    }
    if (D == 0 || n <= 128) {
        double r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = f(m0 + k);
        int i = 8;
        for (; i < n - (n % 8); i += 8) {
#pragma unroll
            for (int k = 0; k < 8; ++k) r[k] += f(m0 + i + k);
        }
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += f(m0 + i);
        return res;
    }
    if constexpr (D > 0) {
        int n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise<D - 1>(f, m0, n2) + np_pairwise<D - 1>(f, m0 + n2, n - n2);
    }
    return 0.0;
}

// ---------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------
// image_threshold (optimize_loop.py:40-44): np.where(a > hi, hi, a), then np.where(a < lo, lo, a)
__global__ void k_threshold(const double *in, size_t n, double lo, double hi, double *out)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = in[i];
    v = v > hi ? hi : v;
    out[i] = v < lo ? lo : v;
}

// optimize_loop (optimize_loop.py:15-37): forward then backward sweep of
//   d = (-a * x + alpha * (L + R + U + D)) / (-a + 4 alpha),  a = coefficient[i, j]
// one workgroup, levels of each sweep separated by barriers; diff[s] = |x - d| (backward)
__global__ __launch_bounds__(1024) void k_optimize_loop(double *img, const double *coef, int wc, double alpha,
                                                        GsGeo gf, const int32_t *__restrict__ ford,
                                                        const int32_t *__restrict__ foff, int fnl, GsGeo gb,
                                                        const int32_t *__restrict__ bord,
                                                        const int32_t *__restrict__ boff, int bnl, double *diff)
{
    const int h = gf.h, w = gf.w;
    for (int pass = 0; pass < 2; ++pass) {
        const GsGeo &g = pass ? gb : gf;
        const int32_t *ord = pass ? bord : ford;
        const int32_t *off = pass ? boff : foff;
        const int nl = pass ? bnl : fnl;
        for (int l = 0; l < nl; ++l) {
            const int b = off[l], e = off[l + 1];
            for (int idx = b + (int)threadIdx.x; idx < e; idx += (int)blockDim.x) {
                const int s = ord[idx];
                int r, c;
                gs_cell(g, s, r, c);
                double *row = img + (size_t)r * w;
                const double x = row[c];
                const double sum = ((row[pyix(c - 1, w)] + row[c + 1]) + img[(size_t)pyix(r - 1, h) * w + c]) +
                                   img[(size_t)(r + 1) * w + c];
                const double a = coef[(size_t)r * wc + c];
                const double d = ((-a) * x + alpha * sum) / ((-a) + 4.0 * alpha);
                if (pass) diff[s] = fabs(x - d);
                row[c] = d;
            }
            __syncthreads();
        }
    }
}

// make_weight (opt_loop.py:60-85): gauss[a][b] = exp(-(float((a-e)^2 + (b-e)^2)) / den_s);
// color[ci][cj][a][b] = exp(((-c) * c) / den_c), c = guide[i][j] - guide[i-e+a][j-e+b],
// (i, j) = (ci + e, cj + e) for ci <= s0-2e-2, cj <= s1-2e-2, zero elsewhere (np.zeros)
__global__ void k_make_weight(const double *guide, int w, int s0, int s1, int e, double den_c, double den_s,
                              double *gauss, double *color)
{
    const int W = 2 * e + 1, n = W * W;
    const int cw = s1 - e;
    const size_t total = (size_t)(s0 - e) * cw * n;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx < (size_t)n) {
        const int a = (int)idx / W - e, b = (int)idx % W - e;
        gauss[idx] = dm_exp(-((double)(a * a + b * b)) / den_s);
    }
    if (idx >= total) return;
    const int m = (int)(idx % n);
    const size_t cell = idx / n;
    const int ci = (int)(cell / cw), cj = (int)(cell % cw);
    double v = 0.0;
    if (ci <= s0 - 2 * e - 2 && cj <= s1 - 2 * e - 2) {
        const int i = ci + e, j = cj + e;
        const double c = guide[(size_t)i * w + j] - guide[(size_t)(ci + m / W) * w + (cj + m % W)];
        v = dm_exp(((-c) * c) / den_c);
    }
    color[idx] = v;
}

// optimize_loop_bilateral_horizon / _vertical (opt_loop.py:16-35 / :39-58):
//   a = -(c0 - (c+ + c-) / 2.0);  b = x - (c+ - c-) / 2.0 / (-2.0 c0 + c+ + c-)
//   d = (-a * b + sum(g * cw * sub)) / (-a + sum(g * cw))        (numpy pairwise sums)
// c0 = coefficient[e, e]; c+/c- = coefficient[e, e+-1] (horizontal) or [e+-1, e] (vertical)
__global__ __launch_bounds__(1024) void k_bilateral(double *img, const double *color, const double *gauss,
                                                    const double *coef, int hc, int wc, int vertical, GsGeo g,
                                                    const int32_t *__restrict__ ord, const int32_t *__restrict__ off,
                                                    int nl, double *diff)
{
    __shared__ double gs[31 * 31];
    const int e = g.e, W = 2 * e + 1, n = W * W, w = g.w, cwc = g.s1 - e;
    for (int m = threadIdx.x; m < n; m += blockDim.x) gs[m] = gauss[m];
    const int er = pyix(e, hc), ec = pyix(e, wc);
    const double c0 = coef[(size_t)er * wc + ec];
    const double cp = vertical ? coef[(size_t)pyix(e + 1, hc) * wc + ec] : coef[(size_t)er * wc + pyix(e + 1, wc)];
    const double cm = vertical ? coef[(size_t)pyix(e - 1, hc) * wc + ec] : coef[(size_t)er * wc + pyix(e - 1, wc)];
    const double a = -(c0 - (cp + cm) / 2.0);
    const double K = (cp - cm) / 2.0 / (((-2.0) * c0 + cp) + cm);
    __syncthreads();
    for (int l = 0; l < nl; ++l) {
        const int b0 = off[l], b1 = off[l + 1];
        for (int idx = b0 + (int)threadIdx.x; idx < b1; idx += (int)blockDim.x) {
            const int s = ord[idx];
            int i, j;
            gs_cell(g, s, i, j);
            const double *cw = color + ((size_t)(i - e) * cwc + (j - e)) * n;
            const double *sub = img + (size_t)(i - e) * w + (j - e);
            const double x = img[(size_t)i * w + j];
            const double bb = x - K;
            auto f1 = [&](int m) { return (gs[m] * cw[m]) * sub[(size_t)(m / W) * w + (m % W)]; };
            auto f2 = [&](int m) { return gs[m] * cw[m]; };
            const double S1 = np_pairwise<3>(f1, 0, n);
            const double S2 = np_pairwise<3>(f2, 0, n);
            const double d = ((-a) * bb + S1) / ((-a) + S2);
            diff[s] = fabs(x - d);
            img[(size_t)i * w + j] = d;
        }
        __syncthreads();
    }
}

#include "dm_gs_pf.h"

// sum of diff[0..n) in sequence order (the reference's `error += ...`): one dependent chain
// of float64 adds that no reordering may shorten.  One wave: chunks of 64 consecutive values
// are loaded coalesced (one per lane, SEQ_D chunks in flight) and fed to the chain through
// v_readlane into SGPRs, so the chain runs at the add latency instead of one memory round
// trip per few elements (the one-lane loop took 36.7 ms per 1M values).
__device__ __forceinline__ double readlane_d(double v, int k)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, k);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), k);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

constexpr int SEQ_D = 4;

__global__ __launch_bounds__(64) void k_seq_sum(const double *__restrict__ v, long long n, double *out)
{
    const int lane = (int)threadIdx.x;
    const long long nc = (n + 63) / 64;
    double x[SEQ_D];
#pragma unroll
    for (int d = 0; d < SEQ_D; ++d) {
        const long long i = (long long)d * 64 + lane;
        x[d] = i < n ? v[i] : 0.0;
    }
    double acc = 0.0; // every lane carries the same chain
    for (long long c = 0; c < nc; c += SEQ_D) {
#pragma unroll
        for (int d = 0; d < SEQ_D; ++d) {
            const long long cc = c + d;
            if (cc >= nc) break; // uniform
            const double cur = x[d];
            const long long i = (cc + SEQ_D) * 64 + lane;
            x[d] = i < n ? v[i] : 0.0;
            const long long m = n - cc * 64;
            if (m >= 64) {
#pragma unroll
                for (int k = 0; k < 64; ++k) acc += readlane_d(cur, k);
            } else {
                for (int k = 0; k < (int)m; ++k) acc += readlane_d(cur, k);
            }
        }
    }
    if (lane == 0) *out = acc;
}

// (SGPR-fed from wave-uniform s_load blocks instead of readlane measured slower on MI355X:
// 22 vs 13.8 ms per 1M values -- the chain waits on the scalar loads)
static void seq_sum(const double *d, long long n, double *out, hipStream_t st)
{
    k_seq_sum<<<1, 64, 0, st>>>(d, n, out);
}

// ---------------------------------------------------------------------------------------
// host: dependency levels of a sweep
// ---------------------------------------------------------------------------------------
static int check_sweep(int kind, int h, int w, int s0, int s1, int e)
{
    if (kind != DM_GS_FWD4 && kind != DM_GS_BWD4 && kind != DM_GS_BILAT)
        return pfail(DM_ERR_ARG, "unknown sweep kind %d", kind);
    if (h < 1 || w < 1 || e < 0) return pfail(DM_ERR_ARG, "bad map %dx%d / exclusion %d", h, w, e);
    if (s0 > h || s1 > w || s0 < 0 || s1 < 0)
        return pfail(DM_ERR_SHAPE, "size (%d, %d) exceeds the map (%d, %d)", s0, s1, h, w);
    if (kind == DM_GS_BILAT && e > 15) return pfail(DM_ERR_UNSUPPORTED, "exclusion %d > 15 not supported", e);
    const GsGeo g = gs_geo(kind, h, w, s0, s1, e);
    if (gs_count(g) == 0) return DM_OK;
    if (kind != DM_GS_BILAT) {
        // highest row / column any update touches (r + 1, c + 1): python raises IndexError
        const int rmax = kind == DM_GS_FWD4 ? s0 - e - 1 : s0 - e, cmax = kind == DM_GS_FWD4 ? s1 - e - 1 : s1 - e;
        if (rmax >= h || cmax >= w) return pfail(DM_ERR_SHAPE, "list index out of range (index %d, %d of a %dx%d map)",
                                                 rmax, cmax, h, w);
    }
    return DM_OK;
}

extern "C" {

int dm_gs_schedule(int32_t kind, int32_t h, int32_t w, int32_t s0, int32_t s1, int32_t excl, int32_t *order,
                   int32_t *level_off, int32_t *n_levels)
{
    int rc = check_sweep(kind, h, w, s0, s1, excl);
    if (rc) return rc;
    if (!n_levels) return pfail(DM_ERR_ARG, "null n_levels");
    const GsGeo g = gs_geo(kind, h, w, s0, s1, excl);
    const long long n = gs_count(g);
    *n_levels = 0;
    if (n == 0) {
        if (level_off) level_off[0] = 0;
        return DM_OK;
    }
    if (!order || !level_off) return pfail(DM_ERR_ARG, "null order / level_off");
    if (n > 0x7fffffffLL) return pfail(DM_ERR_UNSUPPORTED, "sweep of %lld updates", n);
    std::vector<int32_t> lastw((size_t)h * w, -1), maxr((size_t)h * w, -1), lev((size_t)n);
    const int e = excl;
    int cells[4 * 31 * 31 + 8];
    int top = -1;
    for (long long s = 0; s < n; ++s) {
        int r, c;
        gs_cell(g, (int)s, r, c);
        int nc = 0;
        if (kind == DM_GS_BILAT) {
            for (int a = -e; a <= e; ++a)
                for (int b = -e; b <= e; ++b) cells[nc++] = (r + a) * w + (c + b);
        } else {
            cells[nc++] = r * w + pyix(c - 1, w);
            cells[nc++] = r * w + c + 1;
            cells[nc++] = pyix(r - 1, h) * w + c;
            cells[nc++] = (r + 1) * w + c;
            cells[nc++] = r * w + c;
        }
        const int own = r * w + c;
        int L = lastw[own] > maxr[own] ? lastw[own] : maxr[own];
        for (int k = 0; k < nc; ++k) L = lastw[cells[k]] > L ? lastw[cells[k]] : L;
        ++L;
        for (int k = 0; k < nc; ++k)
            if (maxr[cells[k]] < L) maxr[cells[k]] = L;
        lastw[own] = L;
        maxr[own] = -1;
        lev[(size_t)s] = L;
        if (L > top) top = L;
    }
    const int nl = top + 1;
    std::vector<int32_t> cnt((size_t)nl + 1, 0);
    for (long long s = 0; s < n; ++s) ++cnt[(size_t)lev[(size_t)s] + 1];
    for (int l = 0; l < nl; ++l) cnt[(size_t)l + 1] += cnt[(size_t)l];
    for (int l = 0; l <= nl; ++l) level_off[l] = cnt[(size_t)l];
    for (long long s = 0; s < n; ++s) order[cnt[(size_t)lev[(size_t)s]]++] = (int32_t)s;
    *n_levels = nl;
    return DM_OK;
}

int dm_image_threshold(const double *d_in, size_t n, double lo, double hi, double *d_out, void *stream)
{
    if (n == 0) return DM_OK;
    if (!d_in || !d_out) return pfail(DM_ERR_ARG, "null pointer");
    k_threshold<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(d_in, n, lo, hi, d_out);
    PHIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_optimize_loop(double *d_img, const double *d_coef, int32_t hc, int32_t wc, int32_t h, int32_t w, int32_t s0,
                     int32_t s1, int32_t excl, double alpha, const int32_t *d_fwd_order, const int32_t *d_fwd_off,
                     int32_t fwd_levels, const int32_t *d_bwd_order, const int32_t *d_bwd_off, int32_t bwd_levels,
                     double *d_diff, double *d_error, void *stream)
{
    int rc = check_sweep(DM_GS_FWD4, h, w, s0, s1, excl);
    if (rc) return rc;
    rc = check_sweep(DM_GS_BWD4, h, w, s0, s1, excl);
    if (rc) return rc;
    if (!d_img || !d_error) return pfail(DM_ERR_ARG, "null image / error pointer");
    const GsGeo gf = gs_geo(DM_GS_FWD4, h, w, s0, s1, excl), gb = gs_geo(DM_GS_BWD4, h, w, s0, s1, excl);
    const long long n = gs_count(gf);
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        PHIP_TRY(hipMemsetAsync(d_error, 0, sizeof(double), st));
        return DM_OK;
    }
    // coefficient[i, j] for every updated cell (rows <= s0-1-e, cols <= s1-1-e)
    if (!d_coef || hc < s0 - excl || wc < s1 - excl)
        return pfail(DM_ERR_SHAPE, "coefficient %dx%d does not cover the sweep (size %d, %d, exclusion %d)", hc, wc,
                     s0, s1, excl);
    if (!d_fwd_order || !d_fwd_off || !d_bwd_order || !d_bwd_off || !d_diff || fwd_levels < 1 || bwd_levels < 1)
        return pfail(DM_ERR_ARG, "missing schedule / diff buffer");
    if (gs_pf())
        k_optimize_loop_pf<<<1, 1024, 0, st>>>(d_img, d_coef, wc, alpha, gf, d_fwd_order, d_fwd_off, fwd_levels, gb,
                                               d_bwd_order, d_bwd_off, bwd_levels, d_diff);
    else
        k_optimize_loop<<<1, 1024, 0, st>>>(d_img, d_coef, wc, alpha, gf, d_fwd_order, d_fwd_off, fwd_levels, gb,
                                            d_bwd_order, d_bwd_off, bwd_levels, d_diff);
    PHIP_TRY(hipGetLastError());
    seq_sum(d_diff, n, d_error, st);
    PHIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_make_weight(const double *d_guide, int32_t h, int32_t w, int32_t s0, int32_t s1, int32_t excl,
                   double den_color, double den_space, double *d_gauss, double *d_color, void *stream)
{
    if (!d_gauss || !d_color || (!d_guide && s0 > 0)) return pfail(DM_ERR_ARG, "null pointer");
    if (excl < 0 || excl > 15) return pfail(DM_ERR_UNSUPPORTED, "exclusion %d outside 0..15", excl);
    if (s0 > h || s1 > w) return pfail(DM_ERR_SHAPE, "size (%d, %d) exceeds the guide (%d, %d)", s0, s1, h, w);
    if (s0 - excl < 0 || s1 - excl < 0)
        return pfail(DM_ERR_SHAPE, "negative dimensions are not allowed (size %d, %d, exclusion %d)", s0, s1, excl);
    const int W = 2 * excl + 1;
    const size_t total = (size_t)(s0 - excl) * (s1 - excl) * W * W;
    const size_t work = total > (size_t)W * W ? total : (size_t)W * W;
    k_make_weight<<<(unsigned)((work + 255) / 256), 256, 0, (hipStream_t)stream>>>(d_guide, w, s0, s1, excl, den_color,
                                                                                  den_space, d_gauss, d_color);
    PHIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_opt_loop_bilateral(double *d_img, const double *d_color, const double *d_gauss, const double *d_coef,
                          int32_t hc, int32_t wc, int32_t h, int32_t w, int32_t s0, int32_t s1, int32_t excl,
                          int32_t vertical, const int32_t *d_order, const int32_t *d_off, int32_t n_levels,
                          double *d_diff, double *d_error, void *stream)
{
    int rc = check_sweep(DM_GS_BILAT, h, w, s0, s1, excl);
    if (rc) return rc;
    if (!d_img || !d_error) return pfail(DM_ERR_ARG, "null image / error pointer");
    const GsGeo g = gs_geo(DM_GS_BILAT, h, w, s0, s1, excl);
    const long long n = gs_count(g);
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        PHIP_TRY(hipMemsetAsync(d_error, 0, sizeof(double), st));
        return DM_OK;
    }
    // coefficient[e, e], [e, e +- 1] / [e +- 1, e] with python's -1 wrap
    if (!d_coef || hc < 1 || wc < 1 || excl >= hc || excl >= wc || (vertical ? excl + 1 >= hc : excl + 1 >= wc))
        return pfail(DM_ERR_SHAPE, "index %d is out of bounds for the %dx%d coefficient", excl + 1, hc, wc);
    if (!d_color || !d_gauss || !d_order || !d_off || !d_diff || n_levels < 1)
        return pfail(DM_ERR_ARG, "missing weights / schedule / diff buffer");
    const int vt = vertical ? 1 : 0;
#define DM_BILAT_PF(E_, LPU_, R_, NT_)                                                                            \
    k_bilateral_pf<E_, LPU_, R_, NT_><<<1, NT_, 0, st>>>(d_img, d_color, d_gauss, d_coef, hc, wc, vt, g, d_order, d_off,  \
                                                 n_levels, d_diff)
    const bool pf = gs_pf();
    // lanes per update, prefetched rounds, workgroup size: ~n/(e+1) updates per level of an
    // n = 1024 map prefetched without spilling (128 VGPRs per lane at 1024 lanes, 256 at 512)
    if (pf && excl == 1) DM_BILAT_PF(1, 4, 1, 1024);
    else if (pf && excl == 2) DM_BILAT_PF(2, 4, 1, 1024);
    else if (pf && excl == 3) DM_BILAT_PF(3, 4, 2, 512);
    else if (pf && excl == 4) DM_BILAT_PF(4, 8, 2, 512);
    else if (pf && excl == 5) DM_BILAT_PF(5, 8, 1, 512);
    else
        k_bilateral<<<1, 1024, 0, st>>>(d_img, d_color, d_gauss, d_coef, hc, wc, vt, g, d_order, d_off, n_levels,
                                        d_diff);
#undef DM_BILAT_PF
    PHIP_TRY(hipGetLastError());
    seq_sum(d_diff, n, d_error, st);
    PHIP_TRY(hipGetLastError());
    return DM_OK;
}

} // extern "C"
