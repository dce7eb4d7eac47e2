/*
 * dm_pow.h -- the pinned float64 rectification pow(x, 1.4).
 *
 * Replaces numpy's ``map ** self.lam`` (misc/Correlation_map.py:41,158-159) on every
 * path of the build.  numpy's float64 power is itself platform-dependent (libm vs SVML:
 * 1 ulp apart on ~5 % of inputs), so the build pins this evaluation: IEEE double
 * + - * and fma only, no division, no libm, hence bit-identical on x86-64 hosts (gcc,
 * -ffp-contract=off) and on gfx950 (hipcc, -ffp-contract=off).  Accuracy: all error
 * terms are ~2^-60 relative before one final rounding, i.e. near-correctly rounded
 * (tests/test_pow.py measures it against a 60-digit decimal reference).
 *
 * Algorithm and constants: gen_pow_tables.py.  The tables are passed by pointer so the
 * GPU kernels can read them from LDS or constant memory.
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

/* x ** 1.4 for the double y = 1.4 (0x3FF6666666666666).  tab: DM_POW_TAB_INIT (flat,
 * [256][3] = {c_i, (1/c_i)^y hi, lo}); g: DM_POW_G_INIT ([5][2] = 2^(j/5) hi, lo). */
DM_HD static inline double dm_pow14(double x, const double *tab, const double *g)
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
    q = q * r;                                             /* (1+r)^y - 1 */
    const double Bhi = T[1];
    const double Blo = fma(T[1], q, T[2]);                 /* M^y = Bhi + Blo */
    const int t7 = 7 * E;
    const int k = t7 >= 0 ? t7 / 5 : -((-t7 + 4) / 5);   /* floor(7E/5) */
    const int j = t7 - 5 * k;
    const double Ghi = g[2 * j], Glo = g[2 * j + 1];       /* 2^(j/5) */
    const double c = (double)E * DM_POW_KDELTA;            /* 2^(yE - 7E/5) - 1 */
    const double Zhi = Bhi * Ghi;
    double s = fma(Bhi, Ghi, -Zhi);
    s = fma(Bhi, Glo, s);
    s = fma(Blo, Ghi, s);                                  /* M^y 2^(j/5) = Zhi + s */
    s = fma(s, c, s);                                      /* ... * (1 + c)        */
    s = fma(Zhi, c, s);
    double res = Zhi + s;
    int kk = k;
    if (kk < -1000) { res *= 0x1p-600; kk += 600; }
    if (kk > 1000) { res *= 0x1p600; kk -= 600; }
    return res * dm_f64_bits((uint64_t)(1023 + kk) << 52);
}
