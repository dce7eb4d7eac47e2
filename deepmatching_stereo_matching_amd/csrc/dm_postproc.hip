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
// sums (`error += abs(...)`) are the sequence-order float64 sums, bit for bit, computed as
// integer prefix sums between binade crossings (k_seq_sum_seg).
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

// The same sum without the dependent chain: binade segments.  Every term is >= 0 (an
// absolute difference), so the running sum s only grows.  While s stays in one binade
// [2^e, 2^(e+1)) -- ulp u = 2^(e-52); below 2^-1022, u = 2^-1074 -- every partial sum is a
// multiple of u and a step rounds as RN(s + d) = s + u * inc with inc an integer:
//   inc = RN(d / u)                       when d / u is not a tie,
//   inc = floor(d / u) + (p ^ (q & 1))    for a tie (fraction exactly 1/2; q = floor(d / u)),
// where p = (s / u) mod 2: round-half-even picks the even multiple, and s / u is even after
// every tie.  (Ties are common: differences of nearby doubles carry few significant bits.)
// So a run of steps is an integer prefix sum whose increments depend on one parity bit, and
// that is a scan over the monoid of segments {f: parity in -> parity out, T: parity in ->
// increment sum}: (A then B).f(p) = B.f(A.f(p)), (A then B).T(p) = A.T(p) + B.T(A.f(p)).
// One workgroup scans a chunk of 8192 terms in parallel, exactly.  A step is taken by itself,
// as the reference's one float64 add, where the binade changes: s + inc u reaches 2^(e+1), or
// d is not finite or not below 2^(e+1) -- once per binade the sum climbs (a few dozen over a
// sweep).  NaN / inf in s: the rest is added one by one (NaN + x, inf + x as the chain does).
// A negative term (dm_seq_sum is a public entry; the reference's callers only pass abs())
// is also a step of its own, and once s is negative the rest is added one by one.
// Bit-identical to k_seq_sum (tests/test_seq_sum_gpu.py).
constexpr int SEG_T = 1024, SEG_E = 8, SEG_CH = SEG_T * SEG_E;

struct SegSum {   // a run of steps: parity out and increment sum, for parity in 0 / 1
    unsigned f0, f1;
    unsigned long long T0, T1;
};

__device__ __forceinline__ SegSum seg_then(const SegSum &A, const SegSum &B)
{
    SegSum r;
    r.f0 = A.f0 ? B.f1 : B.f0;
    r.f1 = A.f1 ? B.f1 : B.f0;
    r.T0 = A.T0 + (A.f0 ? B.T1 : B.T0);
    r.T1 = A.T1 + (A.f1 ? B.T1 : B.T0);
    return r;
}

__device__ __forceinline__ SegSum seg_shfl_up(const SegSum &x, int o)
{
    SegSum r;
    r.f0 = __shfl_up(x.f0, o);
    r.f1 = __shfl_up(x.f1, o);
    r.T0 = __shfl_up(x.T0, o);
    r.T1 = __shfl_up(x.T1, o);
    return r;
}

__global__ __launch_bounds__(SEG_T) void k_seq_sum_seg(const double *__restrict__ v, long long n, double *out)
{
    typedef unsigned long long u64;
    constexpr int NWV = SEG_T / 64;
    __shared__ SegSum wagg[2][NWV];             // per-wave aggregates (double-buffered)
    __shared__ long long wmin[2][NWV];          // per-wave first binade change
    __shared__ double snext[2];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const SegSum ident = {0u, 1u, 0ull, 0ull};
    double s = 0.0;
    long long k0 = 0;
    for (int it = 0; k0 < n; it ^= 1) {
        if (!(s >= 0.0 && s < INFINITY)) { // NaN, inf or a negative sum (uniform): the chain
            if (t == 0) {
                for (long long k = k0; k < n; ++k) s += v[k];
                *out = s;
            }
            return;
        }
        // binade of s: u = 2^-sh; its top B = 2^(e+1) = top * u
        int sh;
        u64 top;
        if (s < 0x1p-1022) { sh = 1074; top = 1ull << 52; }
        else { sh = 52 - ilogb(s); top = 1ull << 53; }
        const u64 base = (u64)ldexp(s, sh);
        const double B = ldexp((double)top, -sh);
        const long long kt = k0 + (long long)t * SEG_E;
        u64 q[SEG_E];
        unsigned tie = 0;      // bit i: term i is a tie
        int lbad = SEG_E;      // the thread's first term that changes the binade by itself
        SegSum th = ident;
#pragma unroll
        for (int i = 0; i < SEG_E; ++i) {
            const double d = kt + i < n ? v[kt + i] : 0.0;
            const double f = ldexp(d, sh);    // exact (d < B: f < 2^53)
            const double fl = floor(f);
            const bool bad = !(d >= 0.0 && d < B);   // negative terms: a step of their own
            const bool ti = !bad && f - fl == 0.5;
            q[i] = bad ? 0ull : (u64)(ti ? fl : rint(f));
            if (bad && lbad == SEG_E) lbad = i;
            tie |= (unsigned)ti << i;
            const unsigned qo = (unsigned)(q[i] & 1ull);
            SegSum e;
            if (ti) { e.f0 = 0u; e.f1 = 0u; e.T0 = q[i] + qo; e.T1 = q[i] + (qo ^ 1u); }
            else { e.f0 = qo; e.f1 = qo ^ 1u; e.T0 = q[i]; e.T1 = q[i]; }
            th = seg_then(th, e);
        }
        // inclusive scan of the thread segments over the wave
        SegSum inc = th;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const SegSum y = seg_shfl_up(inc, o);
            if (lane >= o) inc = seg_then(y, inc);
        }
        SegSum ex = seg_shfl_up(inc, 1);           // exclusive within the wave
        if (lane == 0) ex = ident;
        if (lane == 63) wagg[it][wave] = inc;
        __syncthreads();
        SegSum pre = ident, all = ident;
#pragma unroll
        for (int w2 = 0; w2 < NWV; ++w2) {
            const SegSum a = wagg[it][w2];
            if (w2 < wave) pre = seg_then(pre, a);
            all = seg_then(all, a);
        }
        pre = seg_then(pre, ex);
        // the thread's first step that changes the binade (P then holds the prefix before it)
        const unsigned p0 = (unsigned)(base & 1ull);
        unsigned p = p0 ? pre.f1 : pre.f0;
        u64 P = p0 ? pre.T1 : pre.T0;
        long long fb = LLONG_MAX;
#pragma unroll
        for (int i = 0; i < SEG_E; ++i) {
            if (fb != LLONG_MAX) continue;
            const unsigned qo = (unsigned)(q[i] & 1ull);
            const bool ti = (tie >> i) & 1u;
            const u64 d_inc = ti ? q[i] + (p ^ qo) : q[i];
            if (i == lbad || base + P + d_inc >= top) {
                fb = (long long)t * SEG_E + i;
            } else {
                P += d_inc;
                p = ti ? 0u : (p ^ qo);
            }
        }
        long long m = fb;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const long long y = __shfl_xor(m, o);
            m = y < m ? y : m;
        }
        if (lane == 0) wmin[it][wave] = m;
        __syncthreads();
        long long j = LLONG_MAX;
#pragma unroll
        for (int w2 = 0; w2 < NWV; ++w2) j = wmin[it][w2] < j ? wmin[it][w2] : j;
        if (j == LLONG_MAX) {    // the whole chunk in one binade
            s = ldexp((double)(base + (p0 ? all.T1 : all.T0)), -sh);
            k0 += SEG_CH;
        } else {                 // s at step j exactly, then step j as the reference adds it
            if (fb == j) snext[it] = ldexp((double)(base + P), -sh) + v[k0 + j];
            __syncthreads();
            s = snext[it];
            k0 += j + 1;
        }
    }
    if (t == 0) *out = s;
}

// DM_SEQ_SUM=chain: the dependent-chain kernel (A/B)
static void seq_sum(const double *d, long long n, double *out, hipStream_t st)
{
    const char *e = getenv("DM_SEQ_SUM");
    if (e && !strcmp(e, "chain")) k_seq_sum<<<1, 64, 0, st>>>(d, n, out);
    else k_seq_sum_seg<<<1, SEG_T, 0, st>>>(d, n, out);
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

int dm_seq_sum(const double *d_v, int64_t n, double *d_out, void *stream)
{
    if (n < 0 || (n > 0 && !d_v) || !d_out) return pfail(DM_ERR_ARG, "bad sequence sum arguments");
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        PHIP_TRY(hipMemsetAsync(d_out, 0, sizeof(double), st));
        return DM_OK;
    }
    seq_sum(d_v, (long long)n, d_out, st);
    PHIP_TRY(hipGetLastError());
    return DM_OK;
}

} // extern "C"
