/*
 * dm_exp.h -- the pinned float64 exp() of the Gauss-Seidel post-processing weights.
 *
 * Replaces numpy's ``np.exp`` in misc/opt_loop.py:69 (spatial weights) and :80 (colour
 * weights) on every path of the build.  numpy's float64 exp is platform-dependent (SIMD
 * vs libm kernels, <= 1 ulp apart), so the build pins one evaluation shared by the HIP
 * kernels (dm_postproc.hip) and the C oracle (oracle/dm_oracle.c): IEEE double + - * and
 * fma only, no table, no libm -- bit-identical on x86-64 (gcc, -ffp-contract=off) and on
 * gfx950 (hipcc, -ffp-contract=off).
 *
 * Algorithm: k = rint(x / ln2) (fma + 1.5*2^52 shifter), r = x - k ln2 in two fma steps
 * (ln2 split hi/lo), |r| <= ln2/2; exp(r) = (1 + r) + r^2 q(r) with q the Taylor series
 * to r^13 (truncation < 2^-57 relative) and 1 + r carried as a Fast2Sum pair, so only
 * the final addition and the small r^2 q term round; exp = exp(r) * 2^k with the scaling
 * split in two for the overflow and subnormal edges.  Error < 0.6 ulp;
 * tests/test_postproc.py measures it against a 50-digit evaluation.
 *
 * Plain C99 (also compiled by the C oracle); DM_HD adds __host__ __device__ under hipcc.
 */
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if !defined(DM_HD)
#if defined(__HIPCC__)
#define DM_HD __host__ __device__
#else
#define DM_HD
#endif
#endif

DM_HD static inline double dm_exp_scale(double y, int k)
{
    /* y * 2^k for y in [0.7, 1.5], k in [-1080, 1025]: two exact power-of-two factors */
    int k1 = k / 2, k2 = k - k1;
    uint64_t b1 = (uint64_t)(1023 + k1) << 52, b2 = (uint64_t)(1023 + k2) << 52;
    double f1, f2;
    memcpy(&f1, &b1, 8);
    memcpy(&f2, &b2, 8);
    return (y * f1) * f2;
}

DM_HD static inline double dm_exp(double x)
{
    if (x != x) return x + x;                                   /* NaN */
    if (x > 0x1.62e42fefa39efp+9) return x * 0x1p1023;          /* > log(DBL_MAX): +inf */
    if (x < -0x1.74910d52d3052p+9) return 0.0;                  /* < log(2^-1075): +0 */
    const double SH = 0x1.8p52;
    const double kd = fma(x, 0x1.71547652b82fep+0, SH) - SH;   /* rint(x / ln2) */
    double r = fma(-kd, 0x1.62e42fefa3800p-1, x);               /* ln2 hi (trailing zeros) */
    r = fma(-kd, 0x1.ef35793c76730p-45, r);                     /* ln2 lo */
    double p = 0x1.6124613a86d09p-33;                           /* 1/13! */
    p = fma(p, r, 0x1.1eed8eff8d898p-29);                       /* 1/12! */
    p = fma(p, r, 0x1.ae64567f544e4p-26);                       /* 1/11! */
    p = fma(p, r, 0x1.27e4fb7789f5cp-22);                       /* 1/10! */
    p = fma(p, r, 0x1.71de3a556c734p-19);                       /* 1/9!  */
    p = fma(p, r, 0x1.a01a01a01a01ap-16);                       /* 1/8!  */
    p = fma(p, r, 0x1.a01a01a01a01ap-13);                       /* 1/7!  */
    p = fma(p, r, 0x1.6c16c16c16c17p-10);                       /* 1/6!  */
    p = fma(p, r, 0x1.1111111111111p-7);                        /* 1/5!  */
    p = fma(p, r, 0x1.5555555555555p-5);                        /* 1/4!  */
    p = fma(p, r, 0x1.5555555555555p-3);                        /* 1/3!  */
    p = fma(p, r, 0.5);                                         /* 1/2!  */
    const double t = (r * r) * p;                               /* expm1(r) - r */
    const double hi = 1.0 + r;                                  /* Fast2Sum: |1| >= |r| */
    const double lo = (1.0 - hi) + r;
    return dm_exp_scale(hi + (lo + t), (int)kd);
}
