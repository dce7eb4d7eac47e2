/*
 * dm_pow.h -- the pinned float64 rectification pow(x, 1.4).
 *
 * Replaces numpy's ``map ** self.lam`` (misc/Correlation_map.py:41,158-159) on every
 * path of the build.  numpy's float64 power is itself platform-dependent (libm vs SVML:
 * 1 ulp apart on ~5 % of inputs), so the build pins this evaluation: IEEE double
 * + - * and fma only, no division, no libm, hence bit-identical on x86-64 hosts (gcc,
 * -ffp-contract=off) and on gfx950 (hipcc, -ffp-contract=off).  Accuracy: error terms
 * ~2^-60 relative before one final rounding: <= 1 ulp, nearly always correctly rounded
 * (tests/test_pow.py measures it against a 60-digit decimal evaluation).
 *
 * Algorithm and constants: gen_pow_tables.py.  Tables are passed by pointer (dm_pow_tabs)
 * so GPU kernels can serve the fast-path tables from LDS.
 *
 * Plain C99 (also compiled by the C oracle); DM_HD adds __host__ __device__ under hipcc.
 */
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "dm_pow_tables.h"

#if defined(__HIPCC__)
#define DM_HD __host__ __device__
#else
#define DM_HD
#endif

typedef struct dm_pow_tabs {
    const double *fc;  /* fast: [DM_POWF_NT] c_i                                 */
    const double *fp;  /* fast: [DM_POWF_NT][2] (1/c_i)^y  hi, lo                 */
    const double *fg;  /* fast: [1 - DM_POWF_EMIN][2] 2^(yE) = G (1 + g): G, g   */
    const double *tab; /* slow: [DM_POW_NT][3] c_i, (1/c_i)^y hi, lo             */
    const double *g;   /* slow: [5][2] 2^(j/5) hi, lo                            */
} dm_pow_tabs;

DM_HD static inline uint64_t dm_bits_f64(double x)
{
    uint64_t b;
    memcpy(&b, &x, 8);
    return b;
}

DM_HD static inline double dm_f64_bits(uint64_t b)
{
    double x;
    memcpy(&x, &b, 8);
    return x;
}

/* fast path, x in [2^DM_POWF_EMIN, 1]: one table row, degree-5 series, one 2^(yE) row
 * {G, g} with 2^(yE) = G (1 + g); g enters the series' last step, and
 * x^y ~ G (Phi + Phi q + Plo) = fma(Phi, G, fma(Phi, q, Plo) * G) (gen_pow_tables.py) */
DM_HD static inline double dm_pow14_fast(double x, const double *fc, const double *fp, const double *fg)
{
    const uint64_t b = dm_bits_f64(x);
    const int E = (int)(b >> 52) - 1023;
    const double M = dm_f64_bits((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const int i = (int)((b >> 43) & (DM_POWF_NT - 1));
    const double r = fma(M, fc[i], -1.0);                  /* |r| <= 2^-10 */
    const int e = E - DM_POWF_EMIN;
    const double G = fg[2 * e], g = fg[2 * e + 1];         /* 2^(yE) = G (1 + g) */
    double q = DM_POWF_B5;
    q = fma(q, r, DM_POWF_B4);
    q = fma(q, r, DM_POWF_B3);
    q = fma(q, r, DM_POWF_B2);
    q = fma(q, r, DM_POWF_B1);
    q = fma(q, r, g);                                      /* (1+r)^y - 1 + g */
    const double Phi = fp[2 * i], Plo = fp[2 * i + 1];     /* (1/c_i)^y */
    const double s = fma(Phi, q, Plo) * G;
    return fma(Phi, G, s);
}

/* slow path: every other input (0, NaN, inf, negatives, x > 1, x < 2^EMIN) */
/* noinline: kept out of the kernels' hot loops (reached only for 0, NaN, x > 1, tiny x) */
DM_HD static __attribute__((noinline)) double dm_pow14_slow(double x, const double *tab, const double *g)
{
    if (!(x > 0.0) || x == INFINITY) {
        if (x == 0.0) return 0.0;          /* pow(+-0, 1.4) = +0 */
        if (x == INFINITY) return x;
        return (x - x) / (x - x) + x;      /* NaN in -> NaN out; x < 0 -> NaN */
    }
    int sh = 0;
    if (x < 0x1p-1022) { x *= 0x1p54; sh = 54; }
    const uint64_t b = dm_bits_f64(x);
    const int E = (int)(b >> 52) - 1023 - sh;
    const double M = dm_f64_bits((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const double *T = tab + 3 * (int)((b >> 44) & 0xFF);
    const double r = fma(M, T[0], -1.0);                   /* |r| <= 2^-9 */
    double q = DM_POW_B7;
    q = fma(q, r, DM_POW_B6);
    q = fma(q, r, DM_POW_B5);
    q = fma(q, r, DM_POW_B4);
    q = fma(q, r, DM_POW_B3);
    q = fma(q, r, DM_POW_B2);
    q = fma(q, r, DM_POW_B1);
    q = q * r;
    const double Bhi = T[1];
    const double Blo = fma(T[1], q, T[2]);
    const int t7 = 7 * E;
    const int k = t7 >= 0 ? t7 / 5 : -((-t7 + 4) / 5);   /* floor(7E/5) */
    const int j = t7 - 5 * k;
    const double Ghi = g[2 * j], Glo = g[2 * j + 1];       /* 2^(j/5) */
    const double c = (double)E * DM_POW_KDELTA;            /* 2^(yE - 7E/5) - 1 */
    const double Zhi = Bhi * Ghi;
    double s = fma(Bhi, Ghi, -Zhi);
    s = fma(Bhi, Glo, s);
    s = fma(Blo, Ghi, s);
    s = fma(s, c, s);
    s = fma(Zhi, c, s);
    double res = Zhi + s;
    int kk = k;
    if (kk < -1000) { res *= 0x1p-600; kk += 600; }
    if (kk > 1000) { res *= 0x1p600; kk -= 600; }
    return res * dm_f64_bits((uint64_t)(1023 + kk) << 52);
}

/* x ** 1.4 for the double y = 1.4 (0x3FF6666666666666) */
DM_HD static inline double dm_pow14(double x, const dm_pow_tabs *t)
{
    if (x >= DM_POWF_XMIN && x <= 1.0) return dm_pow14_fast(x, t->fc, t->fp, t->fg);
    return dm_pow14_slow(x, t->tab, t->g);
}
