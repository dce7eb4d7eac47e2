// dm_kernels.hip -- gfx950 kernels + C ABI (include/dmstereo.h) of the DeepMatching stereo
// correlation engine.  Reference: Yuki-Kumon/deepmatching_stereo_matching, misc/*.py.
//
// Numerics (DESIGN.md "Numerics"): the level-0 value of patch p against window q is
//   num = n*sum(T'I') - sum(T')*sum(I')      exact int32 (T' = T-128, I' = I-128; shift-free)
//   y   = f32(num) * b_q                      b_q = f32(1/sqrt(dI)) (0 if dI == 0) | 1 (CCOEFF)
//   r   = clamp(y * a_p, -1, 1)               a_p = f32(1/sqrt(dT)) | f32(1/n) (CCOEFF, no clamp)
//   x   = (r - rmin_p) / (rmax_p - rmin_p)    float32, Feature_value.min_max
//   L0  = pow14(x)                            float64, Correlation_map._rectification
// y -> r -> x -> pow14 is monotone non-decreasing for a fixed p, so MaxPool and min/max are
// taken on y and only pooled values are normalised and rectified.  All float ops are
// explicit-rounding (__fmul_rn etc.); the file is compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "../../include/dmstereo.h"
#include "dm_pow.h"

__constant__ double c_pow_tab[DM_POW_NT * 3] = DM_POW_TAB_INIT;
__constant__ double c_pow_g[10] = DM_POW_G_INIT;
__constant__ double c_powf_c[DM_POWF_NT] = DM_POWF_C_INIT;
__constant__ double c_powf_p[DM_POWF_NT * 2] = DM_POWF_P_INIT;
__constant__ double c_powf_g[(1 - DM_POWF_EMIN) * 2] = DM_POWF_G_INIT;

// Kernels of a pair's tail (stats, levels >= 3, matching, sub-pixel, stitch) run beside the next
// pair's level kernel, whose waves are older and win the SIMD's age-ordered issue arbitration on
// nearly every cycle; a tail wave then waits for the few idle issue slots between its loads
// and holds its wave slot ~20x longer than alone (profiles/r03y_gaps.txt).  With
// DM_TAIL_PRIO, tail waves raise their priority (s_setprio) so their short, latency-bound
// instruction streams issue as soon as they are ready.
#ifdef DM_TAIL_PRIO
#define DM_TAIL_ENTRY() __builtin_amdgcn_s_setprio(3)
#else
#define DM_TAIL_ENTRY() ((void)0)
#endif

__device__ __forceinline__ double pow14(double x)
{
    if (x >= DM_POWF_XMIN && x <= 1.0) return dm_pow14_fast(x, c_powf_c, c_powf_p, c_powf_g);
    return dm_pow14_slow(x, c_pow_tab, c_pow_g);
}

// Fast-path tables staged in LDS by the level-1 kernels (gathers with random rows: strides
// of 8 and 16 B spread over the banks; one 32-B row per index conflicted 4x more, measured):
//   fp[i]   = (1/c_i)^y hi, lo                              per mantissa index
//   fc32[i] = c_i as float32 (exact: 10 significant bits); float64 callers widen it (exact)
//   gz[k]   = 2^(yE) as {G, g} for E = k - 1 + EMIN (1 <= k < DM_GZ_ROWS);  gz[0] = 0 (x == 0
//             -> +0);  gz[DM_GZ_ROWS] = NaN (pow14_q4's row for a NaN input)
//   g32[b]  = 2^(yE) for the f32 biased exponent b = E + 127 (1 <= b <= 127); g32[255] = NaN
//             (x = NaN -> NaN); g32[0] = 0.  Rows 128..254 (x > 1) are never read by the
//             level kernels, whose float32 inputs are in [0, 1] or NaN: with fill(hole = true)
//             they are left unwritten and the level kernel keeps its own exchange arrays there
//             (G32_HOLE bytes from &g32[128]), which keeps its LDS within 20 KB.
// Same constants and the same operation sequence as dm_pow14_fast, so every variant below
// returns dm_pow14's value on its domain.
#define DM_GZ_ROWS (2 - DM_POWF_EMIN)
typedef double dm_d2 __attribute__((ext_vector_type(2)));
// 16-B rows as one vector: ds_read_b128 (4 LDS cycles, 64 banks) instead of ds_read2_b64
// (8 cycles, 32 banks) -- MI355X_MICROARCH.md section LDS
// (measured: c_i on a 16-B stride, so that the c_i and (1/c_i)^y reads share one i*16
// address, saves one VALU per pow but ran 2 % slower -- the b64 reads then use half the
// banks -- as did splitting (1/c_i)^y into hi / lo arrays on c_i's 8-B stride)
struct PowLds {
    dm_d2 fp[DM_POWF_NT];
    dm_d2 gz[DM_GZ_ROWS + 1];
    dm_d2 g32[256];
    float fc32[DM_POWF_NT]; // c_i has 10 significant bits (gen_pow_tables.py): exact in float32
};
constexpr int G32_HOLE = 127 * 16;  // g32 rows 128..254

__device__ __forceinline__ void pow_lds_fill(PowLds &t, int tid, int nthreads, bool hole = false)
{
    for (int i = tid; i < DM_POWF_NT; i += nthreads) {
        t.fc32[i] = (float)c_powf_c[i];
        t.fp[i] = dm_d2{c_powf_p[2 * i], c_powf_p[2 * i + 1]};
    }
    for (int k = tid; k <= DM_GZ_ROWS; k += nthreads) {
        t.gz[k] = k == DM_GZ_ROWS ? dm_d2{(double)NAN, (double)NAN}
                  : k ? dm_d2{c_powf_g[2 * (k - 1)], c_powf_g[2 * (k - 1) + 1]} : dm_d2{0.0, 0.0};
    }
    for (int b = tid; b < 256; b += nthreads) {
        if (hole && b >= 128 && b < 255) continue;
        const int e = b - 127 - DM_POWF_EMIN; // row of c_powf_g
        const bool in = b >= 1 && b <= 127 && e >= 0;
        t.g32[b] = in ? dm_d2{c_powf_g[2 * e], c_powf_g[2 * e + 1]}
                   : b == 255 ? dm_d2{(double)NAN, (double)NAN} : dm_d2{0.0, 0.0};
    }
}

// fma(a, b, c) with the constant c read from an SGPR pair by the VOP3 form: left to itself the
// compiler keeps the polynomial's constants in VGPR pairs (for v_fmac_f64's tied addend) hoisted
// out of the level kernels' loops -- 8 VGPRs held for a pow that runs once per row pair
__device__ __forceinline__ double fma_sc(double a, double b, double c)
{
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

// dm_pow14_fast's arithmetic from r = fma(M, c_i, -1), table index i and 2^(yE) row G = {G, g}
template <typename T>
__device__ __forceinline__ double pow14_core_r(double r, int i, dm_d2 G, const T &t)
{
    double q = fma_sc(r, DM_POWF_B5, DM_POWF_B4);
    q = fma_sc(q, r, DM_POWF_B3);
    q = fma_sc(q, r, DM_POWF_B2);
    q = fma_sc(q, r, DM_POWF_B1);
    q = fma(q, r, G.y);
    const dm_d2 Pr = t.fp[i];
    const double s = fma(Pr.x, q, Pr.y) * G.x;
    return fma(Pr.x, G.x, s);
}

template <typename T>
__device__ __forceinline__ double pow14_core(double M, int i, dm_d2 G, const T &t)
{
    return pow14_core_r(fma(M, (double)t.fc32[i], -1.0), i, G, t);
}

// float64 input.  Exact dm_pow14 on [2^EMIN, 1] and 0; other inputs read in-bounds rows and
// return garbage (NaN: callers add a NaN term).
__device__ __forceinline__ double pow14_zd(double x, const PowLds &t)
{
    const uint64_t b = dm_bits_f64(x);
    const unsigned hi = (unsigned)(b >> 32);
    const double M = dm_f64_bits((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const int i = (int)((hi >> 11) & (DM_POWF_NT - 1));
    const int be = (int)((hi >> 20) & 0x7FF);
    const int k = min(max(be - (1022 + DM_POWF_EMIN), 0), DM_GZ_ROWS - 1);
    return pow14_core(M, i, t.gz[k], t);
}

// pow14(s / 4) for s == 0, NaN, or s / 4 in [2^EMIN, 1]: /4 of a normal double only lowers
// its biased exponent by 2 (same mantissa, same table index), so the scaling is folded into
// the row index -- no multiply.  NaN reads the NaN row and returns NaN.
__device__ __forceinline__ double pow14_q4(double s, const PowLds &t)
{
    const uint64_t b = dm_bits_f64(s);
    const unsigned hi = (unsigned)(b >> 32);
    const double M = dm_f64_bits((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const int i = (int)((hi >> 11) & (DM_POWF_NT - 1));
    const int be = (int)((hi >> 20) & 0x7FF);
    const int k = min(max(be - (1024 + DM_POWF_EMIN), 0), DM_GZ_ROWS);
    return pow14_core(M, i, t.gz[k], t);
}

// float32 input (widened exactly): exact dm_pow14((double)x) for x == 0 and for normal
// x in [2^EMIN, 1] (f32 subnormals would need renormalising: callers never produce them);
// NaN -> NaN (the g32 NaN row).  Fewer integer ops than pow14_zd: exponent, index and
// mantissa come straight from the f32 bits, and r = M c_i - 1 is exact in float32 (24-bit M,
// 10-bit c_i, |r| < 2^-9), so one float32 FMA forms the float64 FMA's value.
// The LDS byte offsets come straight from the f32 bits, two VOP2 ops each (2.2 issue cycles
// apiece, tools/valu_probe.hip) instead of a bfe, a shift and a mad_u32_u24 (4 + 2.2 + 4):
// fp row i (16 B) at (u >> 10) & 0x1FF0, fc32[i] at a quarter of that, g32 row be at
// (u >> 19) & 0xFF0.
// M = (u & 0x7FFFFF) | 1.0f as v_bitop3_b32 (2.1 issue cycles) instead of v_and_or_b32 (4);
// `mant` is 0x7FFFFF in a VGPR (an SGPR operand costs the VOP3 forms 4 cycles).
static_assert(DM_POWF_NT == 512, "pow14_zf's offsets assume 9 mantissa index bits");
__device__ __forceinline__ unsigned mant_mask_vgpr()
{
    unsigned m;
    asm volatile("v_mov_b32 %0, 0x7fffff" : "=v"(m));
    return m;
}
template <typename T>
__device__ __forceinline__ double pow14_zf(float x, const T &t, unsigned mant = 0x7FFFFFu)
{
    const unsigned u = __float_as_uint(x);
    // bitop3 truth table 0xEA = (src0 & src1) | src2
    const float M = __uint_as_float(__builtin_amdgcn_bitop3_b32(u, mant, 0x3F800000u, 0xEA));
    const unsigned ofp = (u >> 10) & 0x1FF0u, og = (u >> 19) & 0xFF0u;
    const float ci = *(const float *)((const char *)t.fc32 + (ofp >> 2));
    const dm_d2 G = *(const dm_d2 *)((const char *)t.g32 + og);
    const dm_d2 Pr = *(const dm_d2 *)((const char *)t.fp + ofp);
    const double r = (double)__builtin_fmaf(M, ci, -1.0f);
    double q = DM_POWF_B5;
    q = fma(q, r, DM_POWF_B4);
    q = fma(q, r, DM_POWF_B3);
    q = fma(q, r, DM_POWF_B2);
    q = fma(q, r, DM_POWF_B1);
    q = fma(q, r, G.y);
    const double s = fma(Pr.x, q, Pr.y) * G.x;
    return fma(Pr.x, G.x, s);
}

__device__ __forceinline__ double pow14_lds(double x, const PowLds &t)
{
    if (x >= DM_POWF_XMIN && x <= 1.0) return pow14_zd(x, t);
    return dm_pow14_slow(x, c_pow_tab, c_pow_g);
}

// pow14 for the fused level-1/level-2 kernels, branch-free.  Their inputs are 0, NaN or in
// [2^-297, 1]: x = f32 in [0, 1] gives x^1.4 >= 2^-208.6 (f32's least subnormal is 2^-149),
// the /4 child sums of those are >= 2^-210.6, their powers >= 2^-294.9 and the level-2 sums
// >= 2^-297 -- all inside the fast path's [2^DM_POWF_EMIN, 1], so this equals pow14 there.
static_assert(DM_POWF_EMIN <= -297, "fast-path table must cover every level-1/level-2 input");
__device__ __forceinline__ double pow14_k(double x, const PowLds &t)
{
    return pow14_zd(x, t) + (x - x); // 0 -> +0 (zero row), NaN -> NaN
}

// The float64 pows of the pruned level kernel (round 6, k_level12_prune in dm_prune.h) without
// the gz rows: that kernel's level-1 x buffers need the LDS the 5 KB of gz took.  The 2^(yE) row
// of a double whose exponent E is in [-126, 0] is g32[E + 127] -- the same {G, g} constants as
// gz[E - EMIN + 1] -- so pow14_core gives the same bits; zero reads g32[0] = {0, 0} as gz[0]; NaN
// (and the out-of-domain s / 4 > 1 of pow14_q4) the NaN row g32[255] as gz[DM_GZ_ROWS]; the rare
// E < -126 takes dm_pow14_fast with the constant-memory tables (the same constants and
// operations as pow14_core: fma(M, c_i, -1), the series, fma(Phi, G, fma(Phi, q, Plo) G)), or 0
// below 2^EMIN where gz's clamp gives 0.  So pow14_q4g == pow14_q4 and pow14_kg == pow14_k bit
// for bit on EVERY double (tests/test_pow_gpu.py through dm_pow14_variant).  T: any table
// struct with fp, g32, fc32 (PowLds, PowLdsG).
template <typename T>
__device__ __forceinline__ double pow14_q4g(double s, const T &t)
{
    const uint64_t b = dm_bits_f64(s);
    const unsigned hi = (unsigned)(b >> 32);
    const double M = dm_f64_bits((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const int i = (int)((hi >> 11) & (DM_POWF_NT - 1));
    const int be = (int)((hi >> 20) & 0x7FF);
    int row = be - 898;                       // E(s / 4) + 127 = be - 1025 + 127
    if (be != 0 && row < 1) [[unlikely]] {    // s / 4 < 2^-126 (and not 0)
        if (be - 1025 < DM_POWF_EMIN) return 0.0;
        return dm_pow14_fast(ldexp(s, -2), c_powf_c, c_powf_p, c_powf_g);
    }
    row = be == 0 ? 0 : (row > 127 ? 255 : row);
    return pow14_core_r(fma(M, (double)t.fc32[i], -1.0), i, t.g32[row], t);
}

template <typename T>
__device__ __forceinline__ double pow14_kg(double x, const T &t)
{
    const uint64_t b = dm_bits_f64(x);
    const unsigned hi = (unsigned)(b >> 32);
    const double M = dm_f64_bits((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const int i = (int)((hi >> 11) & (DM_POWF_NT - 1));
    const int be = (int)((hi >> 20) & 0x7FF);
    int row = be - 896;                       // E + 127
    if (be != 0 && row < 1) [[unlikely]] {    // x < 2^-126 (and not 0)
        if (be - 1023 < DM_POWF_EMIN) return 0.0 + (x - x);
        return dm_pow14_fast(x, c_powf_c, c_powf_p, c_powf_g) + (x - x);
    }
    row = be == 0 ? 0 : (row > 127 ? 127 : row);   // (pow14_zd's clamp: x > 1 reads the E = 0 row)
    return pow14_core_r(fma(M, (double)t.fc32[i], -1.0), i, t.g32[row], t) + (x - x);
}

// the pow tables without gz (k_level12_prune): fp, g32 (rows 128..254 a hole the kernel uses for
// its exchange arrays), fc32
struct PowLdsG {
    dm_d2 fp[DM_POWF_NT];
    dm_d2 g32[256];
    float fc32[DM_POWF_NT];
};

__device__ __forceinline__ void pow_lds_fill_g(PowLdsG &t, int tid, int nthreads)
{
    for (int i = tid; i < DM_POWF_NT; i += nthreads) {
        t.fc32[i] = (float)c_powf_c[i];
        t.fp[i] = dm_d2{c_powf_p[2 * i], c_powf_p[2 * i + 1]};
    }
    for (int b = tid; b < 256; b += nthreads) {
        if (b >= 128 && b < 255) continue;
        const int e = b - 127 - DM_POWF_EMIN;
        const bool in = b >= 1 && b <= 127 && e >= 0;
        t.g32[b] = in ? dm_d2{c_powf_g[2 * e], c_powf_g[2 * e + 1]}
                   : b == 255 ? dm_d2{(double)NAN, (double)NAN} : dm_d2{0.0, 0.0};
    }
}

// ------------------------------------------------------------------------------------
// geometry + workspace views
// ------------------------------------------------------------------------------------
struct Geo {
    const uint8_t *img1, *img2;
    int pitch1, pitch2;
    const int *org;
    int T, h0, w0, ws, method;
};

struct Stats {
    int *sT;    // sum(T') per patch         [T][P]
    float *aP;  // a_p                        [T][P]
    int *sI;    // sum(I') per window         [T][P]
    float *bQ;  // b_q                        [T][P]
    float *rmn; // min_q r(p, q)              [T][P]
    float *rmx; // max_q r(p, q)              [T][P]
};

static Stats stats_view(void *base, int T, int P)
{
    Stats s;
    char *c = (char *)base;
    const size_t n = (size_t)T * P;
    s.sT = (int *)c;
    s.aP = (float *)(c + 4 * n);
    s.sI = (int *)(c + 8 * n);
    s.bQ = (float *)(c + 12 * n);
    s.rmn = (float *)(c + 16 * n);
    s.rmx = (float *)(c + 20 * n);
    return s;
}

__device__ __forceinline__ float r_of_y(float y, float a, int method)
{
    if (method == DM_TM_CCOEFF) return __fmul_rn(y, a);
    if (a == 0.0f) return 1.0f; // constant patch: OpenCV returns 1 everywhere
    const float r = __fmul_rn(y, a);
    return r < -1.0f ? -1.0f : (r > 1.0f ? 1.0f : r);
}

__device__ __forceinline__ float y_of_num(int num, float b) { return __fmul_rn((float)num, b); }

__device__ __forceinline__ float norm_x(float r, float mn, float mx)
{
    return __fdiv_rn(__fsub_rn(r, mn), __fsub_rn(mx, mn));
}

// Same value as norm_x, for a fixed patch: Markstein's correction of q = a * RN(1/den) is the
// correctly rounded a/den for normal operands (Handbook of FP arithmetic, Markstein's
// theorem; 5.4e8 random pairs checked).  Reachable operands are never subnormal: |r| is
// 0 or >= ~1e-9 (f32(num) is an integer, a_p, b_q >= ~3e-5), so a = r - mn is 0 or
// >= ~1e-16 and den is 0 or >= ~1e-16; den == 0 (constant map) gives NaN like 0/0.
// rinv = __frcp_rn(den) is computed once per patch.
__device__ __forceinline__ float norm_mk(float r, float mn, float den, float rinv)
{
    const float a = __fsub_rn(r, mn);
    const float q = __fmul_rn(a, rinv);
    const float e = __fmaf_rn(-q, den, a);
    return __fmaf_rn(e, rinv, q);
}

// r_of_y with the clamp as one v_med3_f32 (r is never NaN)
__device__ __forceinline__ float r_of_y_fast(float y, float a, int method)
{
    const float r = __fmul_rn(y, a);
    if (method == DM_TM_CCOEFF) return r;
    return a == 0.0f ? 1.0f : __builtin_amdgcn_fmed3f(r, -1.0f, 1.0f);
}

// ------------------------------------------------------------------------------------
// K1: per-patch / per-window moments
// ------------------------------------------------------------------------------------
__global__ void k_stats(Geo g, Stats s)
{
    DM_TAIL_ENTRY();
    const int P = g.h0 * g.w0;
    const int t = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int p0 = p / g.w0, p1 = p % g.w0;
    const int r0 = g.org[2 * t] + p0, c0 = g.org[2 * t + 1] + p1;
    const int n = g.ws * g.ws;
    int sa = 0, sa2 = 0, sb = 0, sb2 = 0;
    for (int u = 0; u < g.ws; ++u)
        for (int v = 0; v < g.ws; ++v) {
            const int a = (int)g.img1[(size_t)(r0 + u) * g.pitch1 + c0 + v] - 128;
            const int b = (int)g.img2[(size_t)(r0 + u) * g.pitch2 + c0 + v] - 128;
            sa += a; sa2 += a * a; sb += b; sb2 += b * b;
        }
    const long long dT = (long long)n * sa2 - (long long)sa * sa;
    const long long dI = (long long)n * sb2 - (long long)sb * sb;
    float ap, bq;
    if (g.method == DM_TM_CCOEFF) {
        ap = (float)(1.0 / (double)n);
        bq = 1.0f;
    } else {
        ap = dT == 0 ? 0.0f : (float)(1.0 / sqrt((double)dT));
        bq = dI == 0 ? 0.0f : (float)(1.0 / sqrt((double)dI));
    }
    const size_t o = (size_t)t * P + p;
    s.sT[o] = sa; s.aP[o] = ap; s.sI[o] = sb; s.bQ[o] = bq;
}

// num = n * acc - sT * sI with full-rate v_mul_i32_i24 (v_mul_lo_u32 is quarter rate): every
// operand fits 24 signed bits (n <= 225, |acc| <= 225 * 128^2 < 2^23, |sT|, |sI| <= 225 * 128)
// and |num| <= n^2 * 128^2 < 2^31 (Cauchy-Schwarz), so the low 32 bits are the exact value
__device__ __forceinline__ int num_of(int n, int acc, int sT, int sI) { return __mul24(n, acc) - __mul24(sT, sI); }

// exact numerator for (patch p0,p1 ; window q0,q1) of tile t, read from global images
__device__ int num_global(const Geo &g, int t, int p0, int p1, int q0, int q1, int sT, int sI)
{
    const int ro = g.org[2 * t], co = g.org[2 * t + 1];
    int acc = 0;
    for (int u = 0; u < g.ws; ++u) {
        const uint8_t *a = g.img1 + (size_t)(ro + p0 + u) * g.pitch1 + co + p1;
        const uint8_t *b = g.img2 + (size_t)(ro + q0 + u) * g.pitch2 + co + q1;
        for (int v = 0; v < g.ws; ++v) acc += ((int)a[v] - 128) * ((int)b[v] - 128);
    }
    return num_of(g.ws * g.ws, acc, sT, sI);
}

// rectified level-0 value L0[p][q] (co_map_list[0]), evaluated on demand
__device__ double l0_value(const Geo &g, const Stats &s, int t, int p0, int p1, int q0, int q1)
{
    const int P = g.h0 * g.w0;
    const size_t op = (size_t)t * P + p0 * g.w0 + p1, oq = (size_t)t * P + q0 * g.w0 + q1;
    const int num = num_global(g, t, p0, p1, q0, q1, s.sT[op], s.sI[oq]);
    const float r = r_of_y(y_of_num(num, s.bQ[oq]), s.aP[op], g.method);
    return pow14((double)norm_x(r, s.rmn[op], s.rmx[op]));
}

// Level-1 value of cell (I, J) at (u, v), on demand: MaxPool(3,2,1) of the four children's
// rectified level-0 maps, (ul+ur+ll+lr)/4, rectify -- the same expression as k_aggregate
// (Correlation_map.py:89-130) evaluated on l0_value, for matching when the fused
// level-1/level-2 kernel kept level 1 on chip.
__device__ double l1_value(const Geo &g, const Stats &s, int t, int I, int J, int u, int v)
{
    double acc = 0.0;
    for (int ch = 0; ch < 4; ++ch) {
        const int p0 = 2 * I + (ch >> 1), p1 = 2 * J + (ch & 1);
        double mx = -INFINITY;
        for (int a = 2 * u - 1; a <= 2 * u + 1; ++a) {
            if (a < 0 || a >= g.h0) continue;
            for (int b = 2 * v - 1; b <= 2 * v + 1; ++b) {
                if (b < 0 || b >= g.w0) continue;
                const double x = l0_value(g, s, t, p0, p1, a, b);
                mx = (x > mx || isnan(x)) ? x : mx;
            }
        }
        acc = ch == 0 ? mx : acc + mx;
    }
    return pow14(acc / 4.0);
}

#include "dm_mfma.h"
#include "dm_strip.h"
#include "dm_prune.h"

// ------------------------------------------------------------------------------------
// K2 (generic): one workgroup per level-1 cell (= 2x2 block of patches p).  For each
// child p in reference order ul, ur, ll, lr: y over all windows q -> LDS, block min/max,
// MaxPool(3,2,1) on y, normalise + rectify the pooled values, accumulate the children
// in order; finally /4 and rectify -> level 1.  Requires P <= DM_GENERIC_MAX_P.
// ------------------------------------------------------------------------------------
#define DM_GENERIC_MAX_P 16384
#define K2_THREADS 256

template <int WS>
__global__ __launch_bounds__(K2_THREADS) void k_level1_generic(Geo g, Stats s, double *L1)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int h0 = g.h0, w0 = g.w0, P = h0 * w0;
    const int h1 = h0 / 2, w1 = w0 / 2, P1 = h1 * w1;
    const int t = blockIdx.y, cell = blockIdx.x;
    const int I = cell / w1, J = cell % w1;
    const int Wc = w0 + WS - 1, Hc = h0 + WS - 1;
    const int tid = threadIdx.x;
    float *ymap = (float *)smem;                                   // [P]
    double *acc = (double *)(smem + (size_t)P * 4);                // [P1]
    float *red = (float *)(smem + (size_t)P * 4 + (size_t)P1 * 8); // [2*K2_THREADS/64]
    signed char *crop = (signed char *)(red + 2 * (K2_THREADS / 64));
    signed char *patch = crop + Hc * Wc;                           // [WS*WS]

    const int ro = g.org[2 * t], co = g.org[2 * t + 1];
    for (int i = tid; i < Hc * Wc; i += K2_THREADS) {
        const int r = i / Wc, c = i % Wc;
        crop[i] = (signed char)((int)g.img2[(size_t)(ro + r) * g.pitch2 + co + c] - 128);
    }
    const size_t tb = (size_t)t * P;
    const int n = WS * WS;
    for (int ch = 0; ch < 4; ++ch) {
        const int p0 = 2 * I + (ch >> 1), p1 = 2 * J + (ch & 1);
        const int p = p0 * w0 + p1;
        __syncthreads(); // previous child done with patch / ymap / red
        if (tid < n) {
            const int u = tid / WS, v = tid % WS;
            patch[tid] = (signed char)((int)g.img1[(size_t)(ro + p0 + u) * g.pitch1 + co + p1 + v] - 128);
        }
        __syncthreads();
        int Tr[WS * WS];
#pragma unroll
        for (int k = 0; k < WS * WS; ++k) Tr[k] = patch[k];
        const int sT = s.sT[tb + p];
        const float ap = s.aP[tb + p];
        float ymn = INFINITY, ymx = -INFINITY;
        for (int q = tid; q < P; q += K2_THREADS) {
            const int q0 = q / w0, q1 = q % w0;
            int a = 0;
#pragma unroll
            for (int u = 0; u < WS; ++u)
#pragma unroll
                for (int v = 0; v < WS; ++v) a += Tr[u * WS + v] * (int)crop[(q0 + u) * Wc + q1 + v];
            const float y = y_of_num(num_of(n, a, sT, s.sI[tb + q]), s.bQ[tb + q]);
            ymap[q] = y;
            ymn = fminf(ymn, y);
            ymx = fmaxf(ymx, y);
        }
        // block min / max
        for (int off = 32; off > 0; off >>= 1) {
            ymn = fminf(ymn, __shfl_xor(ymn, off));
            ymx = fmaxf(ymx, __shfl_xor(ymx, off));
        }
        if ((tid & 63) == 0) { red[tid >> 6] = ymn; red[K2_THREADS / 64 + (tid >> 6)] = ymx; }
        __syncthreads();
        ymn = red[0]; ymx = red[K2_THREADS / 64];
        for (int k = 1; k < K2_THREADS / 64; ++k) {
            ymn = fminf(ymn, red[k]);
            ymx = fmaxf(ymx, red[K2_THREADS / 64 + k]);
        }
        const float rmn = r_of_y(ymn, ap, g.method), rmx = r_of_y(ymx, ap, g.method);
        if (tid == 0) { s.rmn[tb + p] = rmn; s.rmx[tb + p] = rmx; }
        // pooled, normalised, rectified child accumulated in reference order
        for (int k = tid; k < P1; k += K2_THREADS) {
            const int u = k / w1, v = k % w1;
            float m = -INFINITY;
            for (int a = 2 * u - 1; a <= 2 * u + 1; ++a) {
                if (a < 0 || a >= h0) continue;
                for (int b = 2 * v - 1; b <= 2 * v + 1; ++b) {
                    if (b < 0 || b >= w0) continue;
                    m = fmaxf(m, ymap[a * w0 + b]);
                }
            }
            const double val = pow14((double)norm_x(r_of_y(m, ap, g.method), rmn, rmx));
            acc[k] = ch == 0 ? val : acc[k] + val;
        }
    }
    __syncthreads();
    double *out = L1 + ((size_t)t * P1 + cell) * P1;
    for (int k = tid; k < P1; k += K2_THREADS) out[k] = pow14(acc[k] / 4.0);
}

static size_t k2_lds_bytes(int h0, int w0, int ws)
{
    const size_t P = (size_t)h0 * w0, P1 = P / 4;
    return P * 4 + P1 * 8 + 2 * (K2_THREADS / 64) * 4 + (size_t)(h0 + ws - 1) * (w0 + ws - 1) + ws * ws;
}

// ------------------------------------------------------------------------------------
// level-0 volume (co_map) materialisation: pass 1 min/max, pass 2 coalesced f32 stores
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_minmax(Geo g, Stats s)
{
    const int P = g.h0 * g.w0, t = blockIdx.y, p = blockIdx.x;
    const int p0 = p / g.w0, p1 = p % g.w0;
    const size_t tb = (size_t)t * P;
    const int sT = s.sT[tb + p];
    const float ap = s.aP[tb + p];
    float ymn = INFINITY, ymx = -INFINITY;
    for (int q = threadIdx.x; q < P; q += 256) {
        const float y = y_of_num(num_global(g, t, p0, p1, q / g.w0, q % g.w0, sT, s.sI[tb + q]), s.bQ[tb + q]);
        ymn = fminf(ymn, y);
        ymx = fmaxf(ymx, y);
    }
    __shared__ float red[8];
    for (int off = 32; off > 0; off >>= 1) {
        ymn = fminf(ymn, __shfl_xor(ymn, off));
        ymx = fmaxf(ymx, __shfl_xor(ymx, off));
    }
    if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = ymn; red[4 + (threadIdx.x >> 6)] = ymx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        ymn = fminf(fminf(red[0], red[1]), fminf(red[2], red[3]));
        ymx = fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7]));
        s.rmn[tb + p] = r_of_y(ymn, ap, g.method);
        s.rmx[tb + p] = r_of_y(ymx, ap, g.method);
    }
}

template <typename OT>
__global__ __launch_bounds__(256) void k_volume(Geo g, Stats s, OT *l0)
{
    const int P = g.h0 * g.w0, t = blockIdx.y, p = blockIdx.x;
    const int p0 = p / g.w0, p1 = p % g.w0;
    const size_t tb = (size_t)t * P;
    const int sT = s.sT[tb + p];
    const float ap = s.aP[tb + p], mn = s.rmn[tb + p], mx = s.rmx[tb + p];
    OT *row = l0 + (tb + p) * P;
    for (int q = threadIdx.x; q < P; q += 256) {
        const float y = y_of_num(num_global(g, t, p0, p1, q / g.w0, q % g.w0, sT, s.sI[tb + q]), s.bQ[tb + q]);
        row[q] = (OT)norm_x(r_of_y(y, ap, g.method), mn, mx);
    }
}

template <typename F>
__global__ void k_rectify(const F *in, size_t n, double *out)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = pow14((double)in[i]);
}

// the in-kernel pow14 forms on arbitrary inputs (dm_pow14_variant): tables in LDS exactly as
// the level kernel holds them
template <int V>
__global__ __launch_bounds__(256) void k_pow_variant(const double *in, size_t n, double *out)
{
    __shared__ PowLds plds;
    pow_lds_fill(plds, threadIdx.x, 256);
    __syncthreads();
    const unsigned mant = mant_mask_vgpr();
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double x = in[i];
        double r;
        if constexpr (V == DM_POW_F32) r = pow14_zf((float)x, plds, mant);
        else if constexpr (V == DM_POW_Q4) r = pow14_q4(x, plds);
        else if constexpr (V == DM_POW_K) r = pow14_k(x, plds);
        else if constexpr (V == DM_POW_Q4G) r = pow14_q4g(x, plds);
        else if constexpr (V == DM_POW_KG) r = pow14_kg(x, plds);
        else r = pow14_lds(x, plds);
        out[i] = r;
    }
}

// ------------------------------------------------------------------------------------
// pyramid step for levels >= 1 (float64 in, float64 out)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ double nanmax(double acc, double v) { return (v > acc || isnan(v)) ? v : acc; }

// one output value of the aggregation step: tile t, rem = cell * P2 + position
__device__ __forceinline__ void aggregate_at(const double *in, int h, int w, int rectify, size_t t, size_t rem,
                                             double *out)
{
    const int h2 = h / 2, w2 = w / 2;
    const size_t P = (size_t)h * w, P2 = (size_t)h2 * w2;
    const int cell = (int)(rem / P2), k = (int)(rem % P2);
    const int I = cell / w2, J = cell % w2, u = k / w2, v = k % w2;
    double acc = 0.0;
    for (int ch = 0; ch < 4; ++ch) {
        const int c = (2 * I + (ch >> 1)) * w + 2 * J + (ch & 1);
        const double *m = in + (t * P + c) * P;
        double mx = -INFINITY;
        for (int a = 2 * u - 1; a <= 2 * u + 1; ++a) {
            if (a < 0 || a >= h) continue;
            for (int b = 2 * v - 1; b <= 2 * v + 1; ++b) {
                if (b < 0 || b >= w) continue;
                mx = nanmax(mx, m[(size_t)a * w + b]);
            }
        }
        acc = ch == 0 ? mx : acc + mx;
    }
    out[t * P2 * P2 + rem] = rectify ? pow14(acc / 4.0) : acc / 4.0;
}

__global__ void k_aggregate(const double *in, int T, int h, int w, int rectify, double *out)
{
    DM_TAIL_ENTRY();
    const size_t P2 = (size_t)(h / 2) * (w / 2);
    const size_t total = (size_t)T * P2 * P2;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x)
        aggregate_at(in, h, w, rectify, idx / (P2 * P2), idx % (P2 * P2), out);
}

// Same result as k_aggregate, streaming: one workgroup per (tile, output cell, band of
// output rows), thread (child, v) owns output column v of one child map and walks the
// band's input rows once (MaxPool columns 2v-1..2v+1, rows streamed), so every input byte
// is read once from HBM, coalesced.  Children are summed in ul, ur, ll, lr order through
// LDS.  W2 = w/2 columns per child, 4*W2 threads, BR output rows per band.
// VEC (16-B aligned input, W2 in {16, 32, 64}: a child's lanes never straddle a wave): one
// 16-B load of columns 2v, 2v+1 per lane and row; column 2v-1 is lane v-1's second value.
#define AGG_LDS_DOUBLES 4096
template <bool VEC>
__global__ __launch_bounds__(256) void k_aggregate_rows(const double *in, int T, int h, int w, int BR, int rectify,
                                                        double *out)
{
    DM_TAIL_ENTRY();
    extern __shared__ double pooled[]; // [child][band row][v]: 4 * BR * W2 doubles (dynamic, so
                                       // small bands do not cap the workgroups per CU)
    const int h2 = h / 2, W2 = w / 2;
    const size_t P = (size_t)h * w, P2 = (size_t)h2 * W2;
    const int nb = (h2 + BR - 1) / BR;
    const int band = blockIdx.x % nb, cell = (int)((blockIdx.x / nb) % P2), t = (int)(blockIdx.x / nb / P2);
    const int I = cell / W2, J = cell % W2;
    const int tid = threadIdx.x, ch = tid / W2, v = tid % W2;
    const int u0 = band * BR, u1 = min(u0 + BR, h2);
    if (ch < 4) {
        const int cc = (2 * I + (ch >> 1)) * w + 2 * J + (ch & 1);
        const double *m = in + ((size_t)t * P + cc) * P;
        double cprev = -INFINITY, R = -INFINITY;
        const int a0 = max(2 * u0 - 1, 0), a1 = 2 * u1 - 1;
        constexpr int CH = 8; // rows per batch of loads in flight
        for (int ab = a0; ab <= a1; ab += CH) {
            double cmv[CH];
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const int a = min(ab + k, a1);
                const double *row = m + (size_t)a * w;
                if constexpr (VEC) {
                    const dm_d2 x = *(const dm_d2 *)(row + 2 * v);
                    const double l = __shfl(x.y, (int)(threadIdx.x & 63) - 1);
                    cmv[k] = nanmax(nanmax(v > 0 ? l : -INFINITY, x.x), x.y);
                } else {
                    const double x1 = row[2 * v], x2 = row[2 * v + 1], x0 = v > 0 ? row[2 * v - 1] : -INFINITY;
                    cmv[k] = nanmax(nanmax(x0, x1), x2);
                }
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) {
            const int a = ab + k;
            if (a > a1) break;
            const double cm = cmv[k];
            if ((a & 1) == 0) {
                R = a == 0 ? cm : nanmax(cprev, cm);
            } else {
                if (a >= 2 * u0) {
                    R = nanmax(R, cm);
                    pooled[(ch * BR + (a >> 1) - u0) * W2 + v] = R;
                }
                cprev = cm;
            }
            }
        }
    }
    __syncthreads();
    const int nout = (u1 - u0) * W2;
    for (int i = tid; i < nout; i += blockDim.x) {
        const int ur = i / W2, vv = i % W2;
        double acc = pooled[(0 * BR + ur) * W2 + vv];
        acc = acc + pooled[(1 * BR + ur) * W2 + vv];
        acc = acc + pooled[(2 * BR + ur) * W2 + vv];
        acc = acc + pooled[(3 * BR + ur) * W2 + vv];
        out[((size_t)t * P2 + cell) * P2 + (size_t)(u0 + ur) * W2 + vv] = rectify ? pow14(acc / 4.0) : acc / 4.0;
    }
}

// ------------------------------------------------------------------------------------
// matching (Matching.py)
// ------------------------------------------------------------------------------------
struct Levels {
    const double *lv[32];
};

// Matching._calc_near_match (:58-78) on a 3x3 zero-padded window of values win[9]
__device__ __forceinline__ void near_pick(const double *win, int pd0, int pd1, double *o)
{
    int m = 0;
    bool nan_seen = isnan(win[0]);
    double best = win[0];
    if (!nan_seen) {
        for (int k = 1; k < 9; ++k) {
            if (isnan(win[k])) { m = k; nan_seen = true; break; }
            if (win[k] > best) { best = win[k]; m = k; }
        }
    }
    if (!nan_seen && best < 0.0001) m = 4;
    o[0] = (double)(pd0 + m / 3 - 1);
    o[1] = (double)(pd1 + m % 3 - 1);
    o[2] = win[m] + win[4];
}

__device__ __forceinline__ void window_lvl(const double *M, int h, int w, int pd0, int pd1, double *win)
{
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            const int r = pd0 - 1 + a, c = pd1 - 1 + b;
            win[a * 3 + b] = (r < 0 || r >= h || c < 0 || c >= w) ? 0.0 : M[(size_t)r * w + c];
        }
}

// top of the pyramid (_initial_move_map, :80-96): p_dot = p, for entry p of tile t
// Map buffers of the matching phases hold one (3, h, w) map per tile: tile t's at map + t * ms
// (ms = 3 h w: the maps of a level packed).
__device__ __forceinline__ void match_top_at(const double *LK, int h, int w, size_t t, size_t p, double *map, size_t ms)
{
    const size_t P = (size_t)h * w;
    const int i = (int)(p / w), j = (int)(p % w);
    double win[9], o[3];
    window_lvl(LK + (t * P + p) * P, h, w, i, j, win);
    near_pick(win, i, j, o);
    double *mt = map + t * ms;
    mt[p] = o[0]; mt[P + p] = o[1]; mt[2 * P + p] = o[2];
}

__global__ void k_match_top(const double *LK, int T, int h, int w, double *map)
{
    DM_TAIL_ENTRY();
    const size_t P = (size_t)h * w;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)T * P) return;
    match_top_at(LK, h, w, idx / P, idx % P, map, 3 * P);
}

__device__ __forceinline__ double sub_pix_compute(double r0, double r1, double r_)
{
    if (r0 > r1 && r0 > r_) return -(r1 - r_) / (2.0 * (r1 + r_ - 2.0 * r0));
    return 0.0;
}

// one _B step (:98-139): parent map (h x w) -> child map (2h x 2w) on level L (materialised
// when L != nullptr, else level lev = 0 or 1 on demand); at level 0 optionally _sub_pix_cal (:177-209)
__device__ __forceinline__ void match_step_at(const Geo &g, const Stats &s, const double *L, int lev, int h, int w,
                                              int t, int pc, const double *pmap, size_t pms, double *cmap, size_t cms)
{
    const int hn = 2 * h, wn = 2 * w;
    const size_t P = (size_t)h * w, Pn = (size_t)hn * wn;
    const int p0 = pc / wn, p1 = pc % wn;
    const int o0 = p0 & 1, o1 = p1 & 1;
    const size_t par = (size_t)(p0 >> 1) * w + (p1 >> 1);
    const double *pm = pmap + (size_t)t * pms;
    const int pd0 = (int)(long long)(pm[par] * 2) + o0;
    const int pd1 = (int)(long long)(pm[P + par] * 2) + o1;
    double win[9], o[3];
    if (L) {
        window_lvl(L + ((size_t)t * Pn + pc) * Pn, hn, wn, pd0, pd1, win);
    } else {
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                const int r = pd0 - 1 + a, c = pd1 - 1 + b;
                win[a * 3 + b] = (r < 0 || r >= hn || c < 0 || c >= wn) ? 0.0
                                 : lev == 0 ? l0_value(g, s, t, p0, p1, r, c) : l1_value(g, s, t, p0, p1, r, c);
            }
    }
    near_pick(win, pd0, pd1, o);
    double *cm_ = cmap + (size_t)t * cms;
    cm_[pc] = o[0]; cm_[Pn + pc] = o[1]; cm_[2 * Pn + pc] = o[2];
}

__global__ void k_match_step(Geo g, Stats s, const double *L, int lev, int T, int h, int w,
                             const double *pmap, double *cmap)
{
    DM_TAIL_ENTRY();
    const size_t Pn = (size_t)(2 * h) * (2 * w);
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)T * Pn) return;
    match_step_at(g, s, L, lev, h, w, (int)(idx / Pn), (int)(idx % Pn), pmap, 3 * (size_t)h * w, cmap, 3 * Pn);
}

// Level-0 values of one patch on demand with its taps in registers (WS known at compile
// time): the same expression as l0_value.
template <int WS>
struct PatchL0 {
    // row u's taps as packed signed bytes (v_dot4_i32_i8 operands): NW4 full words of taps
    // 4m..4m+3, then (WS % 4 != 0) one tail word with the WS % 4 remaining taps in its low
    // bytes and zeros above -- the tail is one more dot4, not WS % 4 extract + multiply-adds
    static constexpr int NW4 = WS / 4, NT = WS % 4 ? 1 : 0, NWD = NW4 + NT;
    int Tw[WS][NWD];
    int sT;
    float ap, rmn, rmx;
    // tap k = T'[k / WS][k % WS] (k known at compile time after unrolling)
    __device__ int tap(int k) const
    {
        const int u = k / WS, v = k % WS;
        return ((int)((unsigned)Tw[u][v >> 2] << (24 - 8 * (v & 3)))) >> 24;
    }
    __device__ void load(const Geo &g, const Stats &s, int t, int p0, int p1)
    {
        const int ro = g.org[2 * t], co = g.org[2 * t + 1];
        const uint8_t *a = g.img1 + (size_t)(ro + p0) * g.pitch1 + co + p1;
        int T8[WS * WS];
#pragma unroll
        for (int k = 0; k < WS * WS; ++k) T8[k] = (int)a[(size_t)(k / WS) * g.pitch1 + (k % WS)] - 128;
#pragma unroll
        for (int u = 0; u < WS; ++u) {
#pragma unroll
            for (int m = 0; m < NWD; ++m) {
                unsigned w = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (4 * m + k < WS) w |= (unsigned)(T8[u * WS + 4 * m + k] & 0xFF) << (8 * k);
                Tw[u][m] = (int)w;
            }
        }
        const size_t op = (size_t)t * g.h0 * g.w0 + (size_t)p0 * g.w0 + p1;
        sT = s.sT[op]; ap = s.aP[op]; rmn = s.rmn[op]; rmx = s.rmx[op];
    }
    // Integer dot products sum_k T'_k I'_k of this patch against the NI x NJ windows whose
    // top-left window is (qa0, qb0).  The (NI+WS-1) x (NJ+WS-1) image region must lie inside
    // the tile.  Per region row: its aligned dwords (each holds a needed byte, so no load
    // leaves the page of a valid byte), re-aligned by the row's byte offset (v_alignbyte),
    // bytes made signed (^ 0x80 = b - 128 as int8), then v_dot4_i32_i8 over four taps at a
    // time: (NB+3)/4 loads per row instead of one byte load per tap and window.  Exact
    // integers, so the sums equal the byte-wise ones.
    // emit(i, acc_row) is called for window row i as soon as its last image row is in, so a
    // caller that consumes rows at once keeps only WS rows of sums live.
    template <int NI, int NJ, typename F>
    __device__ void grid_rows(const Geo &g, int t, int qa0, int qb0, F &&emit) const
    {
        int acc[NI][NJ];
        constexpr int NB = NJ + WS - 1, NE = (NB + 3) / 4, ND = (NB + 6) / 4;
        const int ro = g.org[2 * t], co = g.org[2 * t + 1];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = 0;
        const uint8_t *rp0 = g.img2 + (size_t)(ro + qa0) * g.pitch2 + co + qb0;
#pragma unroll
        for (int r = 0; r < NI + WS - 1; ++r) {
            const uint8_t *rp = rp0 + (size_t)r * (unsigned)g.pitch2;
            const unsigned off = (unsigned)((uintptr_t)rp & 3u);
            const unsigned *A = (const unsigned *)(rp - off);
            unsigned D[ND + 1], E[NE + 1];
#pragma unroll
            for (int d = 0; d < ND; ++d) D[d] = (4 * d <= NB - 1 || 4 * d < (int)off + NB) ? A[d] : 0u;
            D[ND] = 0u;
#pragma unroll
            for (int e = 0; e < NE; ++e) E[e] = __builtin_amdgcn_alignbyte(D[e + 1], D[e], off) ^ 0x80808080u;
            E[NE] = 0u;
#pragma unroll
            for (int u = 0; u < WS; ++u) {
                const int i = r - u;
                if (i < 0 || i >= NI) continue;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    int a = acc[i][j];
                    // the tail word's zero taps meet bytes past the window (or E's zero pad)
#pragma unroll
                    for (int m = 0; m < NWD; ++m) {
                        const int b0 = j + 4 * m;
                        const unsigned w = (b0 & 3) ? __builtin_amdgcn_alignbyte(E[(b0 >> 2) + 1], E[b0 >> 2], b0 & 3)
                                                    : E[b0 >> 2];
                        a = __builtin_amdgcn_sdot4(Tw[u][m], (int)w, a, false);
                    }
                    acc[i][j] = a;
                }
            }
            if (r - (WS - 1) >= 0 && r - (WS - 1) < NI) emit(r - (WS - 1), acc[r - (WS - 1)]);
        }
    }
    template <int NI, int NJ>
    __device__ void grid_acc(const Geo &g, int t, int qa0, int qb0, int (&out)[NI][NJ]) const
    {
        grid_rows<NI, NJ>(g, t, qa0, qb0, [&](int i, const int (&row)[NJ]) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) out[i][j] = row[j];
        });
    }
    // rectified level 0 from an integer dot sum (the expression of value() below)
    __device__ double rect(const Geo &g, const Stats &s, int t, int q0, int q1, int acc) const
    {
        const size_t oq = (size_t)t * g.h0 * g.w0 + (size_t)q0 * g.w0 + q1;
        const float r = r_of_y(y_of_num(num_of(WS * WS, acc, sT, s.sI[oq]), s.bQ[oq]), ap, g.method);
        return pow14((double)norm_x(r, rmn, rmx));
    }
    __device__ double value(const Geo &g, const Stats &s, int t, int q0, int q1) const
    {
        const int ro = g.org[2 * t], co = g.org[2 * t + 1];
        const uint8_t *b = g.img2 + (size_t)(ro + q0) * g.pitch2 + co + q1;
        int acc = 0;
#pragma unroll
        for (int k = 0; k < WS * WS; ++k) acc += tap(k) * ((int)b[(size_t)(k / WS) * g.pitch2 + (k % WS)] - 128);
        const size_t oq = (size_t)t * g.h0 * g.w0 + (size_t)q0 * g.w0 + q1;
        const float r = r_of_y(y_of_num(num_of(WS * WS, acc, sT, s.sI[oq]), s.bQ[oq]), ap, g.method);
        return pow14((double)norm_x(r, rmn, rmx));
    }
};

// lane 4q + L of every quad (DPP quad_perm [L, L, L, L]), for a float64 value: two v_mov_dpp
template <int L>
__device__ __forceinline__ double quad_bcast(double v)
{
    constexpr int qp = L | (L << 2) | (L << 4) | (L << 6);
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, qp, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), qp, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// The _B step onto level 1 when level 1 was never stored (dm_corr_level12 without level 1):
// four lanes per entry, one per child patch of the level-1 cell.  A lane computes y on the
// 7x7 level-0 neighbourhood its entry's 3x3 level-1 window pools from, takes the MaxPool on
// y (monotone: same as pooling the rectified values), normalises and rectifies the 9 pooled
// values; the 4 lanes sum them in ul, ur, ll, lr order, /4, rectify -- the arithmetic of
// k_level1_mfq / k_aggregate, so the window equals the stored level 1 bit for bit.
// Entry pc of tile t, child ch = lane & 3: the four lanes of a quad must run together (DPP);
// a dead quad (live false) computes an entry of its tile and stores nothing.
template <int WS>
__device__ __forceinline__ void match_step_l1_at(const Geo &g, const Stats &s, int t, int pc, int ch, bool live,
                                                 const double *pmap, size_t pms, double *cmap, size_t cms)
{
    constexpr int ws = WS, n = WS * WS;
    const int h0 = g.h0, w0 = g.w0;
    const int h1 = h0 / 2, w1 = w0 / 2, h = h1 / 2, w = w1 / 2;
    const size_t P = (size_t)h0 * w0, P1 = (size_t)h1 * w1, Pp = (size_t)h * w;
    const int p0 = pc / w1, p1 = pc % w1;
    const double *pm = pmap + (size_t)t * pms;
    const size_t par = (size_t)(p0 >> 1) * w + (p1 >> 1);
    const int pd0 = (int)(long long)(pm[par] * 2) + (p0 & 1);
    const int pd1 = (int)(long long)(pm[Pp + par] * 2) + (p1 & 1);
    // child patch (level-0 patch coordinates) and its statistics
    const int pp0 = 2 * p0 + (ch >> 1), pp1 = 2 * p1 + (ch & 1);
    const int ro = g.org[2 * t], co = g.org[2 * t + 1];
    PatchL0<WS> pt;
    pt.load(g, s, t, pp0, pp1);
    const int sT = pt.sT;
    const float ap = pt.ap, rmn = pt.rmn, rmx = pt.rmx;
    // MaxPool(3,2,1) on y over level-0 rows/cols 2*pd - 3 .. 2*pd + 3 (-inf outside the map):
    // R[a][b] = max of y[2a..2a+2][2b..2b+2]
    float R[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) R[a][b] = -INFINITY;
    const int qa0 = 2 * pd0 - 3, qb0 = 2 * pd1 - 3;
    auto pool_row = [&](int i, const float (&yr)[7]) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (i < 2 * a || i > 2 * a + 2) continue;
#pragma unroll
            for (int b = 0; b < 3; ++b) R[a][b] = fmaxf(R[a][b], fmaxf(fmaxf(yr[2 * b], yr[2 * b + 1]), yr[2 * b + 2]));
        }
    };
    bool fast = false;
    if constexpr (WS <= 7) fast = qa0 >= 0 && qa0 + 6 < h0 && qb0 >= 0 && qb0 + 6 < w0;
    if constexpr (WS <= 7) {
        if (fast) { // all 49 windows inside: one pass over their (WS+6)^2 image bytes
            int acc[7][7];
            pt.template grid_acc<7, 7>(g, t, qa0, qb0, acc);
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                float yr[7];
#pragma unroll
                for (int j = 0; j < 7; ++j) {
                    const size_t oq = (size_t)t * P + (size_t)(qa0 + i) * w0 + qb0 + j;
                    yr[j] = y_of_num(num_of(n, acc[i][j], sT, s.sI[oq]), s.bQ[oq]);
                }
                pool_row(i, yr);
            }
        }
    }
    if (!fast) { // map border (rare): byte loads, one window row at a time
#pragma unroll 1
        for (int i = 0; i < 7; ++i) {
            float yr[7];
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                const int qa = qa0 + i, qb = qb0 + j;
                if (qa < 0 || qa >= h0 || qb < 0 || qb >= w0) { yr[j] = -INFINITY; continue; }
                const uint8_t *b = g.img2 + (size_t)(ro + qa) * g.pitch2 + co + qb;
                int acc = 0;
#pragma unroll
                for (int k = 0; k < n; ++k) acc += pt.tap(k) * ((int)b[(size_t)(k / ws) * g.pitch2 + (k % ws)] - 128);
                const size_t oq = (size_t)t * P + (size_t)qa * w0 + qb;
                yr[j] = y_of_num(num_of(n, acc, sT, s.sI[oq]), s.bQ[oq]);
            }
            pool_row(i, yr);
        }
    }
    // the 9 window sums: every lane of the entry's quad gets all four children (DPP quad
    // broadcasts, in ul, ur, ll, lr order) and forms every sum; lane ch then rectifies the sums
    // of positions k = ch, ch + 4 (selected per lane, so the wave issues 2 sum-pows, not 8) and
    // every lane that of k = 8; lane 0 collects the window (out-of-range positions: 0,
    // Matching's zero padding)
    double sk[9];
    bool ink[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int a = k / 3, b = k % 3;
        const int u = pd0 - 1 + a, v = pd1 - 1 + b;
        double pv = 0.0;
        ink[k] = u >= 0 && u < h1 && v >= 0 && v < w1;
        if (ink[k]) pv = pow14((double)norm_x(r_of_y(R[a][b], ap, g.method), rmn, rmx));
        const double v0 = quad_bcast<0>(pv), v1 = quad_bcast<1>(pv), v2 = quad_bcast<2>(pv), v3 = quad_bcast<3>(pv);
        sk[k] = (((v0 + v1) + v2) + v3) / 4.0;
    }
    double mine[3];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const double x = ch == 0 ? sk[4 * m] : ch == 1 ? sk[4 * m + 1] : ch == 2 ? sk[4 * m + 2] : sk[4 * m + 3];
        const bool in = ch == 0 ? ink[4 * m] : ch == 1 ? ink[4 * m + 1] : ch == 2 ? ink[4 * m + 2] : ink[4 * m + 3];
        mine[m] = in ? pow14(x) : 0.0;
    }
    mine[2] = ink[8] ? pow14(sk[8]) : 0.0;
    double win[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const double m = mine[k >> 2];
        win[k] = (k & 3) == 0 ? quad_bcast<0>(m) : (k & 3) == 1 ? quad_bcast<1>(m)
                 : (k & 3) == 2 ? quad_bcast<2>(m) : quad_bcast<3>(m);
    }
    if (!live || ch != 0) return;
    double o[3];
    near_pick(win, pd0, pd1, o);
    double *cm_ = cmap + (size_t)t * cms;
    cm_[pc] = o[0]; cm_[P1 + pc] = o[1]; cm_[2 * P1 + pc] = o[2];
}

template <int WS, int MW = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MW))) void k_match_step_l1(Geo g, Stats s, int T, const double *pmap, double *cmap)
{
    DM_TAIL_ENTRY();
    const size_t P1 = (size_t)(g.h0 / 2) * (g.w0 / 2);
    const size_t gid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t e = gid >> 2;
    const bool live = e < (size_t)T * P1;
    const size_t ee = live ? e : 0;
    match_step_l1_at<WS>(g, s, (int)(ee / P1), (int)(ee % P1), (int)(gid & 3), live, pmap, 3 * (P1 / 4), cmap, 3 * P1);
}

// Matching._sub_pix_cal (:177-209) on the final map, in place.  L0: materialised rectified
// level 0 ([T][P0][P0], P0 = h0 w0) or nullptr (on demand from images + stats).  The map is
// hm x wm: h0 x w0 after a descent to level 0, a coarser level's when the descent stops
// above it -- the reference still reads co_map_list[0] at (i, j, row, col) of that map
// (:182-186), so the level-0 patch is (i, j) and the bounds are level 0's window sides.
// An entry is any float (dm_subpix_map accepts arbitrary maps), indexed the way numpy indexes
// co_map_list[0][i, j, c0 +- 1, c1] with c = int(value): an index in [-N, N) is valid and a
// negative one wraps (value + N); any other index raises IndexError, caught by the bare
// except (:193-194, :205-206), which writes i - d_x (j - d_y).  The row refinement reads
// (c0 - 1, c1), (c0, c1), (c0 + 1, c1), so it needs c0 in [-h0 + 1, h0 - 2] and c1 in
// [-w0, w0); the column one c1 in [-w0 + 1, w0 - 2] and c0 in [-h0, h0).  (A NaN or an
// entry beyond int range makes the reference's int() raise outside the try; here it takes
// the except branch.)
__device__ __forceinline__ int py_index(double v)
{
    return (v == v && fabs(v) < 1073741824.0) ? (int)v : -0x40000000; // int(): truncation
}

__device__ __forceinline__ bool py_in(int k, int n) { return k >= -n && k < n; }
__device__ __forceinline__ int py_wrap(int k, int n) { return k < 0 ? k + n : k; }

__global__ void k_subpix(Geo g, Stats s, const double *L0, int T, int h0, int w0, int hm, int wm, double *map)
{
    DM_TAIL_ENTRY();
    const size_t P = (size_t)h0 * w0, Pm = (size_t)hm * wm;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)T * Pm) return;
    const int t = (int)(idx / Pm), pc = (int)(idx % Pm);
    const int p0 = pc / wm, p1 = pc % wm;
    double *mt = map + (size_t)t * 3 * Pm;
    const double *M = L0 ? L0 + ((size_t)t * P + (size_t)p0 * w0 + p1) * P : nullptr;
    // (r_, c_) already wrapped into [0, h0) x [0, w0)
#define L0V(r_, c_) (M ? M[(size_t)(r_) * w0 + (c_)] : l0_value(g, s, t, p0, p1, (r_), (c_)))
    const double row = mt[pc], col = mt[Pm + pc];
    const int c0 = py_index(row), c1 = py_index(col);
    const double dx = (double)p0 - row;
    double nrow = (double)p0 - dx; // the except branch
    if (py_in(c0 - 1, h0) && py_in(c0 + 1, h0) && py_in(c1, w0)) {
        const int a = py_wrap(c0, h0), b = py_wrap(c1, w0);
        nrow = nrow + sub_pix_compute(L0V(a, b), L0V(py_wrap(c0 + 1, h0), b), L0V(py_wrap(c0 - 1, h0), b));
    }
    const double dy = (double)p1 - col;
    double ncol = (double)p1 - dy;
    if (py_in(c1 - 1, w0) && py_in(c1 + 1, w0) && py_in(c0, h0)) {
        const int a = py_wrap(c0, h0), b = py_wrap(c1, w0);
        ncol = ncol + sub_pix_compute(L0V(a, b), L0V(a, py_wrap(c1 + 1, w0)), L0V(a, py_wrap(c1 - 1, w0)));
    }
#undef L0V
    mt[pc] = nrow;
    mt[Pm + pc] = ncol;
}

// Matching._filter (:224-255), square maps: per interior pixel the rounded (half-even)
// mean / median of the neighbouring integer displacements.  in -> out (score copied).
__global__ void k_filter(const double *in, double *out, int T, int h, int w, int fw, int median)
{
    DM_TAIL_ENTRY();
    const size_t P = (size_t)h * w;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)T * P) return;
    const int t = (int)(idx / P), k = (int)(idx % P);
    const int i = k / w, j = k % w;
    const double *mi = in + (size_t)t * 3 * P;
    double *mo = out + (size_t)t * 3 * P;
    const int ex = (fw - 1) / 2;
    double r0 = mi[k], r1 = mi[P + k];
    if (i >= ex && i < h - ex && j >= ex && j < w - ex) {
        long long d1[49], d2[49];
        int n = 0;
        for (int a = i - ex; a <= i + ex; ++a)
            for (int b = j - ex; b <= j + ex; ++b) {
                d1[n] = (long long)mi[P + (size_t)a * w + b] - b; // d_map  = map[1] - j
                d2[n] = (long long)mi[(size_t)a * w + b] - a;     // d_map2 = map[0] - i
                ++n;
            }
        double v1, v2;
        if (median) {
            for (int x = 1; x < n; ++x) // insertion sort, n <= 49
                for (int y = x; y > 0 && d1[y - 1] > d1[y]; --y) { long long q = d1[y]; d1[y] = d1[y - 1]; d1[y - 1] = q; }
            for (int x = 1; x < n; ++x)
                for (int y = x; y > 0 && d2[y - 1] > d2[y]; --y) { long long q = d2[y]; d2[y] = d2[y - 1]; d2[y - 1] = q; }
            v1 = (double)d1[n / 2];
            v2 = (double)d2[n / 2];
        } else {
            long long s1 = 0, s2 = 0;
            for (int x = 0; x < n; ++x) { s1 += d1[x]; s2 += d2[x]; }
            v1 = (double)s1 / (double)n;
            v2 = (double)s2 / (double)n;
        }
        r1 = rint(v1) + (double)j; // python round(): half to even
        r0 = rint(v2) + (double)i;
    }
    mo[k] = r0;
    mo[P + k] = r1;
    mo[2 * P + k] = mi[2 * P + k];
}

__global__ void k_cal_map(const double *map, int T, int h, int w, int mode, double *out)
{
    DM_TAIL_ENTRY();
    const size_t P = (size_t)h * w;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)T * P) return;
    const size_t t = idx / P, k = idx % P;
    const int i = (int)(k / w), j = (int)(k % w);
    const double *m = map + t * 3 * P;
    double v;
    if (mode == DM_CAL_ELEVATION) v = (double)j - m[P + k];
    else if (mode == DM_CAL_ELEVATION2) v = (double)i - m[k];
    else {
        const double a = (double)i - m[k], b = (double)j - m[P + k];
        v = sqrt(a * a + b * b);
    }
    out[idx] = v;
}

// misc/sub_pix_cal.py:22-53 (image_threshold: misc/optimize_loop.py:40-44)
__device__ __forceinline__ double thr3(double v) { v = v > 3.0 ? 3.0 : v; return v < -3.0 ? -3.0 : v; }

__global__ void k_sub_pix_cal(const double *arr, const double *co, int h, int w, int dir, double ratio,
                              double *out)
{
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)h * w) return;
    const int i = (int)(idx / w), j = (int)(idx % w);
    const double d = thr3(arr[idx]);
    double dis = d;
    if (i >= 1 && i < h - 1 && j >= 1 && j < w - 1) {
        const size_t pl = dir == 0 ? idx + w : idx + 1, mi = dir == 0 ? idx - w : idx - 1;
        const double r0 = co[idx] * ratio, r1 = co[pl] * ratio, r_ = co[mi] * ratio;
        dis = d - (r1 - r_) / (2.0 * (r1 + r_ - 2.0 * r0));
        if (fabs(d - dis) > 1.0) dis = d;
    }
    out[idx] = thr3(dis);
}

struct Modes {
    int m[8];
};

__global__ void k_stitch(const double *match, int n0, int n1, int h0, int w0, int s0, int s1,
                         Modes modes, int nmodes, double *dmap, double *score, int Hout, int Wout)
{
    DM_TAIL_ENTRY();
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)Hout * Wout) return;
    const int y = (int)(idx / Wout), x = (int)(idx % Wout);
    const int i = min(y / s0, n0 - 1), j = min(x / s1, n1 - 1);
    const int ly = y - i * s0, lx = x - j * s1;
    const size_t HW = (size_t)Hout * Wout;
    if (ly >= h0 || lx >= w0) {
        for (int k = 0; k < nmodes; ++k) dmap[k * HW + idx] = NAN;
        score[idx] = NAN;
        return;
    }
    const size_t P = (size_t)h0 * w0, l = (size_t)ly * w0 + lx;
    const double *m = match + (size_t)(j * n0 + i) * 3 * P;
    for (int k = 0; k < nmodes; ++k) {
        double v;
        if (modes.m[k] == DM_CAL_ELEVATION) v = (double)lx - m[P + l];
        else if (modes.m[k] == DM_CAL_ELEVATION2) v = (double)ly - m[l];
        else {
            const double a = (double)ly - m[l], b = (double)lx - m[P + l];
            v = sqrt(a * a + b * b);
        }
        dmap[k * HW + idx] = v;
    }
    score[idx] = m[2 * P + l];
}

// ------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------
static thread_local char g_err[512];

// shared with dm_postproc.hip (not exported)
__attribute__((visibility("hidden"))) int dm_vfail(int code, const char *fmt, va_list ap)
{
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    return code;
}

static int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    dm_vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_TRY(x)                                                                          \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) return fail(DM_ERR_HIP, "HIP error: %s (%d)", hipGetErrorString(e_), (int)e_); \
    } while (0)

static int check_tiles(const dm_tiles *b)
{
    if (!b || !b->d_img1 || !b->d_img2 || !b->d_origins) return fail(DM_ERR_ARG, "null tile batch / pointer");
    if (b->T < 1 || b->h0 < 1 || b->w0 < 1) return fail(DM_ERR_ARG, "empty batch (T=%d, h0=%d, w0=%d)", b->T, b->h0, b->w0);
    if (b->ws < 1 || (b->ws & 1) == 0)
        return fail(DM_ERR_SHAPE, "window_size must be odd (got %d): Correlation_map.py:63-64 broadcast error", b->ws);
    if (b->ws > 15) return fail(DM_ERR_UNSUPPORTED, "window_size %d > 15 not supported", b->ws);
    if (b->method != DM_TM_CCOEFF && b->method != DM_TM_CCOEFF_NORMED)
        return fail(DM_ERR_ARG, "invalid feature method %d", b->method);
    return DM_OK;
}

static Geo make_geo(const dm_tiles *b)
{
    Geo g;
    g.img1 = b->d_img1; g.img2 = b->d_img2;
    g.pitch1 = b->pitch1; g.pitch2 = b->pitch2;
    g.org = b->d_origins;
    g.T = b->T; g.h0 = b->h0; g.w0 = b->w0; g.ws = b->ws; g.method = b->method;
    return g;
}

static inline size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

static size_t base_stats_bytes(const dm_tiles *b) { return (size_t)6 * 4 * (size_t)b->T * b->h0 * b->w0; }

// level-1 kernel variant, a function of the tile shape only (no environment, no state): 3 =
// the column-split MFMA kernel k_level1_mfq where the shape allows it, 0 = the generic kernel.
// dm_corr_stats lays the window operands out for the variant, and every later call on the same
// batch re-derives the same decision from the same dm_tiles.
static int level1_variant(const dm_tiles *b)
{
    return mf16_eligible(b) ? 3 : 0;
}

// waves per workgroup of k_level1_mfq (and the window layout dm_corr_stats writes for it):
// column group width GW = G/NW tiles of 16 windows per wave.  GW = 4 (two pooled columns per
// lane: the left neighbour of the second is in the lane, level 2 pools in the lane) where the
// width gives 1, 2 or 4 such waves and the packed-y path applies (one wave: two cell blocks per
// workgroup, launch_mfq_t); GW = 2 otherwise.  Same box,
// bit-identical (tools/kbench.py, profiles/r03k_*): C3 (S=128) 7.96 -> 7.72 ms with 2 waves of
// GW = 4 instead of 4 waves of GW = 2 (137 VGPRs: 3 waves/SIMD instead of 5), C5 (S=256)
// 549 -> 487 ms with 4 waves instead of 8.
static int mfq_nw(const dm_tiles *b)
{
    const int G = b->w0 / 16;
    const bool g4 = b->ws * b->ws <= 25 && G % 4 == 0 && (G / 4 == 1 || G / 4 == 2 || G / 4 == 4);
    if (g4) return G / 4;
    return G / 2 < 8 ? G / 2 : 8;
}

// second window region: the column-group layout of k_volume_ls (GW = 16 B of output per
// lane), prepped by dm_corr_volume(_f16) itself
static bool volume_ls_shape(const dm_tiles *b)   // sizes the workspace: no environment knobs
{
    return mf16_eligible(b) && b->ws <= 5 && (b->h0 % 4) == 0 && ((size_t)(b->h0 / 4) * (b->w0 / 4)) % 8 == 0;
}


// the row-pair strips of sweep 1 (k_prep_strips): the three GW = 4 instances of the level kernel
// (packed y, ws <= 5; every wave sweeps 64 windows = 2 strip tiles per row pair)
#ifndef DM_S1
#define DM_S1 1   // 0: sweep 1 on the 16 x 16 tiles (A/B build switch)
#endif
static bool strip_shape(const dm_tiles *b)   // sizes the workspace: no environment knobs
{
    if (!DM_S1 || !mf16_eligible(b) || b->ws > 5) return false;
    const int G = b->w0 / 16;
    return G % 4 == 0 && (G / 4 == 1 || G / 4 == 2 || G / 4 == 4);
}

// both sweeps on the strips (k_level12_strip, dm_strip.h) for the strip shapes whose bit is set
// in DM_S2 (1: w0 = 64, C2; 2: w0 = 128, C3; 4: w0 = 256, C5); dm_corr_stats then skips the
// 16 x 16 window operands (k_prep_windows16), which nothing else reads there.  Same box, bit-
// identical (profiles/r05_strip_ab.txt): C5 27.06 / 27.04 ms against 27.44 / 27.30, C2 0.498
// against 0.504 ms (mean of 4), C3 7.30 / 7.32 against 7.19 / 7.18 -- there k_level1_mfq stays
// (the strip kernel issues 3.6 % more VALU instructions and 29 % more LDS ones per launch: its
// lane holds two cells' normalisation constants and carries two windows' odd rows; fewer MFMA
// cycles do not make up for it at 4 waves per SIMD, and at 3 the lost occupancy costs more)
#ifndef DM_S2
#define DM_S2 5
#endif
static bool strip2_shape(const dm_tiles *b)
{
    return strip_shape(b) && ((DM_S2 >> (b->w0 == 64 ? 0 : b->w0 == 128 ? 1 : 2)) & 1);
}

static size_t strip_bytes(const dm_tiles *b)
{
    const size_t rows = (size_t)b->T * (b->h0 / 2);
    return rows * (b->w0 / 32) * 1024 + rows * b->w0 * 16;
}

static void strip_views(const dm_tiles *b, void *d_stats, dm_v4i **Bs, dm_v4i **Ss)
{
    const size_t extra = mf16_extra_bytes(b);
    char *base = (char *)d_stats + align256(base_stats_bytes(b)) + align256(extra) +
                 (volume_ls_shape(b) ? align256(extra) : 0);
    *Bs = (dm_v4i *)base;
    *Ss = (dm_v4i *)(base + (size_t)b->T * (b->h0 / 2) * (b->w0 / 32) * 1024);
}

static void mfma_views2(const dm_tiles *b, void *d_stats, dm_v4i **Bw, int2 **QS)
{
    const int G = b->w0 / 16;
    char *base = (char *)d_stats + align256(base_stats_bytes(b)) + align256(mf16_extra_bytes(b));
    *Bw = (dm_v4i *)base;
    *QS = (int2 *)(base + (size_t)b->T * b->h0 * G * 1024);
}

static void mfma_views(const dm_tiles *b, void *d_stats, dm_v4i **Bw, int2 **QS)
{
    const int G = b->w0 / 16, KS = (b->ws * b->ws + 63) / 64;
    char *base = (char *)d_stats + align256(base_stats_bytes(b));
    *Bw = (dm_v4i *)base;
    *QS = (int2 *)(base + (size_t)b->T * b->h0 * G * KS * 1024);
}

static inline unsigned nblk(size_t n, unsigned bs)
{
    size_t b = (n + bs - 1) / bs;
    return (unsigned)(b > 0x7fffffff ? 0x7fffffff : b);
}

// The ws = 5 on-demand matching kernels run in one-wave workgroups, which fit in the wave slot
// a retiring level-kernel wave leaves (a 4-wave workgroup needs a free slot on every SIMD of a
// CU at once): the pipelined C3 bench -0.35 % per pair, same box (profiles/r03z2_tail.txt).
static constexpr unsigned TAIL_WG = 64u;


// the last _B step (onto level 0) with level 0 on demand, patch taps in registers
template <int WS>
__device__ __forceinline__ void match_step_l0_at(const Geo &g, const Stats &s, int t, int pc, const double *pmap,
                                                 size_t pms, double *cmap, size_t cms)
{
    const int hn = g.h0, wn = g.w0, h = hn / 2, w = wn / 2;
    const size_t Pp = (size_t)h * w, Pn = (size_t)hn * wn;
    const int p0 = pc / wn, p1 = pc % wn;
    const double *pm = pmap + (size_t)t * pms;
    const size_t par = (size_t)(p0 >> 1) * w + (p1 >> 1);
    const int pd0 = (int)(long long)(pm[par] * 2) + (p0 & 1);
    const int pd1 = (int)(long long)(pm[Pp + par] * 2) + (p1 & 1);
    PatchL0<WS> pt;
    pt.load(g, s, t, p0, p1);
    double win[9], o[3];
    bool fast = false;
    if constexpr (WS <= 7) fast = pd0 >= 1 && pd0 + 1 < hn && pd1 >= 1 && pd1 + 1 < wn;
    if constexpr (WS <= 7) {
        if (fast) { // the 3x3 windows in one pass over their (WS+2)^2 image bytes
            int acc[3][3];
            pt.template grid_acc<3, 3>(g, t, pd0 - 1, pd1 - 1, acc);
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) win[a * 3 + b] = pt.rect(g, s, t, pd0 - 1 + a, pd1 - 1 + b, acc[a][b]);
        }
    }
    if (!fast) {
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                const int r = pd0 - 1 + a, c = pd1 - 1 + b;
                win[a * 3 + b] = (r < 0 || r >= hn || c < 0 || c >= wn) ? 0.0 : pt.value(g, s, t, r, c);
            }
    }
    near_pick(win, pd0, pd1, o);
    double *cm_ = cmap + (size_t)t * cms;
    cm_[pc] = o[0]; cm_[Pn + pc] = o[1]; cm_[2 * Pn + pc] = o[2];
}

template <int WS, int MW = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MW))) void k_match_step_l0(Geo g, Stats s, int T, const double *pmap, double *cmap)
{
    DM_TAIL_ENTRY();
    const size_t Pn = (size_t)g.h0 * g.w0;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)T * Pn) return;
    match_step_l0_at<WS>(g, s, (int)(idx / Pn), (int)(idx % Pn), pmap, 3 * (Pn / 4), cmap, 3 * Pn);
}

// _sub_pix_cal with level 0 on demand, patch taps in registers (see k_subpix)
template <int WS>
__device__ __forceinline__ void subpix_at(const Geo &g, const Stats &s, int t, int pc, double *map, size_t ms)
{
    const int h0 = g.h0, w0 = g.w0;
    const size_t P = (size_t)h0 * w0;
    const int p0 = pc / w0, p1 = pc % w0;
    double *mt = map + (size_t)t * ms;
    PatchL0<WS> pt;
    pt.load(g, s, t, p0, p1);
    const double row = mt[pc], col = mt[P + pc];
    const int c0 = (int)row, c1 = (int)col;
    if constexpr (WS <= 7) {
        if (c0 >= 1 && c0 + 1 < h0 && c1 >= 1 && c1 + 1 < w0) {
            // interior: the five values (centre, up/down, left/right) from one 3x3 pass, and
            // neither the IndexError nor the -1 wrap branch applies
            int acc[3][3];
            pt.template grid_acc<3, 3>(g, t, c0 - 1, c1 - 1, acc);
            const double r0 = pt.rect(g, s, t, c0, c1, acc[1][1]);
            mt[pc] = ((double)p0 - ((double)p0 - row)) +
                     sub_pix_compute(r0, pt.rect(g, s, t, c0 + 1, c1, acc[2][1]), pt.rect(g, s, t, c0 - 1, c1, acc[0][1]));
            mt[P + pc] = ((double)p1 - ((double)p1 - col)) +
                         sub_pix_compute(r0, pt.rect(g, s, t, c0, c1 + 1, acc[1][2]), pt.rect(g, s, t, c0, c1 - 1, acc[1][0]));
            return;
        }
    }
    const double r0 = pt.value(g, s, t, c0, c1);
    const double dx = (double)p0 - row;
    double nrow, ncol;
    if (c0 + 1 >= h0) {
        nrow = (double)p0 - dx;
    } else {
        const int cm = c0 - 1 < 0 ? h0 - 1 : c0 - 1;
        nrow = ((double)p0 - dx) + sub_pix_compute(r0, pt.value(g, s, t, c0 + 1, c1), pt.value(g, s, t, cm, c1));
    }
    const double dy = (double)p1 - col;
    if (c1 + 1 >= w0) {
        ncol = (double)p1 - dy;
    } else {
        const int cm = c1 - 1 < 0 ? w0 - 1 : c1 - 1;
        ncol = ((double)p1 - dy) + sub_pix_compute(r0, pt.value(g, s, t, c0, c1 + 1), pt.value(g, s, t, c0, cm));
    }
    mt[pc] = nrow;
    mt[P + pc] = ncol;
}

template <int WS, int MW = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MW))) void k_subpix_t(Geo g, Stats s, int T, double *map)
{
    DM_TAIL_ENTRY();
    const size_t P = (size_t)g.h0 * g.w0;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (idx >= (size_t)T * P) return;
    subpix_at<WS>(g, s, (int)(idx / P), (int)(idx % P), map, 3 * P);
}

template <int WS>
static int launch_level1(const dm_tiles *b, Stats s, double *L1, hipStream_t st)
{
    const size_t lds = k2_lds_bytes(b->h0, b->w0, WS);
    static bool attr_set = false; // idempotent attribute, benign race
    if (!attr_set) {
        HIP_TRY(hipFuncSetAttribute((const void *)k_level1_generic<WS>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    dim3 grid((b->h0 / 2) * (b->w0 / 2), b->T);
    k_level1_generic<WS><<<grid, K2_THREADS, lds, st>>>(make_geo(b), s, L1);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

#ifndef DM_C5_NB
#define DM_C5_NB 1   // four-wave cell blocks per workgroup of the S = 256 level kernel
#endif
#ifndef DM_C3_MINW
#define DM_C3_MINW 4   // waves per SIMD k_level1_mfq's S = 128 instance is compiled for
#endif
#ifndef DM_C3_MW
#define DM_C3_MW 4   // waves per SIMD the S = 128 strip kernel is compiled for
#endif
#ifndef DM_C3_NB
#define DM_C3_NB 2   // two-wave cell blocks per workgroup of the S = 128 level kernel
#endif
#ifndef DM_C2_NB
#define DM_C2_NB 4   // one-wave cell blocks per workgroup of the S = 64 level kernel
#endif
// the C3 level kernel with pruned child pows when DM_PRUNE is set (dm_prune.h) -> launched?
template <bool OK>
static bool prune_c3(const Geo &gg, const Stats &s, double *L1, double *L2, const dm_v4i *Bw, const int2 *QS,
                     const dm_v4i *Bs, const dm_v4i *Ss, unsigned grid, hipStream_t st)
{
    if constexpr (DM_PRUNE && OK) {
        if (Bs && L1 == nullptr && L2 != nullptr) {
            k_level12_prune<2, DM_C3_NB, DM_C3_MINW><<<grid, 64 * 2 * DM_C3_NB, 0, st>>>(gg, s, L2, Bw, QS, Bs, Ss);
            return true;
        }
    }
    (void)gg; (void)s; (void)L1; (void)L2; (void)Bw; (void)QS; (void)Bs; (void)Ss; (void)grid; (void)st;
    return false;
}

template <bool L2F, bool YF>
static int launch_mfq_t(const dm_tiles *b, Stats s, const dm_v4i *Bw, const int2 *QS, double *L1, double *L2,
                        hipStream_t st, const dm_v4i *Bs, const dm_v4i *Ss)
{
    const int KS = (b->ws * b->ws + 63) / 64, NW = mfq_nw(b), GW = b->w0 / 16 / NW;
    const unsigned grid = (unsigned)(b->T * (b->h0 / 4) * (b->w0 / 4));
    const Geo gg = make_geo(b);
    // the fused path (L2F) normalises with the clamp bit of the Markstein step (norm_clamp in
    // dm_mfma.h); the level-1-only path keeps the v_med3_f32 form
    constexpr bool CL = L2F;
    // GW = 4 with 4 waves (S = 256, C5): 4 waves/SIMD register budget
    if (KS == 1 && GW == 4 && NW == 4) {
        constexpr int NBc = DM_C5_NB;
        const size_t bpt = (size_t)(b->h0 / 4) * (b->w0 / 4);
        if (bpt % NBc) return fail(DM_ERR_UNSUPPORTED, "cell blocks per tile not a multiple of %d (fill_ptab: a workgroup in one tile)", NBc);
        if (Bs && (DM_S2 & 4)) k_level12_strip<4, NBc, L2F, CL, 4><<<grid / NBc, 64 * 4 * NBc, 0, st>>>(gg, s, L1, L2, Bs, Ss);
        else if (Bs) k_level1_mfq<1, 4, 4 * NBc, 4, L2F, YF, NBc, CL, YF><<<grid / NBc, 64 * 4 * NBc, 0, st>>>(gg, s, Bw, QS, L1, L2, Bs, Ss);
        else k_level1_mfq<1, 4, 4 * NBc, 4, L2F, YF, NBc, CL><<<grid / NBc, 64 * 4 * NBc, 0, st>>>(gg, s, Bw, QS, L1, L2);
        HIP_TRY(hipGetLastError());
        return DM_OK;
    }
    // GW = 4 with one wave per cell block (S = 64, C2): C2_NB cell blocks per workgroup share
    // the pow tables (one-wave workgroups would hold 20 KB of LDS per wave: 2 waves/SIMD).
    // 4 blocks: C2 level kernel 0.540 -> 0.503-0.509 ms against 2 (same box,
    // profiles/r04g_c2nb4.txt): half the table fills and workgroup starts per wave
    if (KS == 1 && GW == 4 && NW == 1) {
        constexpr int NBc = DM_C2_NB;
        const size_t bpt = (size_t)(b->h0 / 4) * (b->w0 / 4);
        if (bpt % NBc) return fail(DM_ERR_UNSUPPORTED, "cell blocks per tile not a multiple of %d (fill_ptab: a workgroup in one tile)", NBc);
        if (Bs && (DM_S2 & 1)) k_level12_strip<1, NBc, L2F, CL, 4><<<grid / NBc, 64 * NBc, 0, st>>>(gg, s, L1, L2, Bs, Ss);
        else if (Bs) k_level1_mfq<1, 4, NBc, 4, L2F, YF, NBc, CL, YF><<<grid / NBc, 64 * NBc, 0, st>>>(gg, s, Bw, QS, L1, L2, Bs, Ss);
        else k_level1_mfq<1, 4, NBc, 4, L2F, YF, NBc, CL><<<grid / NBc, 64 * NBc, 0, st>>>(gg, s, Bw, QS, L1, L2);
        HIP_TRY(hipGetLastError());
        return DM_OK;
    }
    // GW = 4 with 2 waves (C3): 20 KB of LDS (the exchange arrays in the pow tables' hole)
    // allow 8 workgroups per CU, so a 4 waves/SIMD register budget (<= 128 VGPRs)
    if (KS == 1 && GW == 4 && NW == 2) {
        constexpr int NBc = DM_C3_NB;
        const size_t bpt = (size_t)(b->h0 / 4) * (b->w0 / 4);
        if (bpt % NBc) return fail(DM_ERR_UNSUPPORTED, "cell blocks per tile not a multiple of %d (fill_ptab: a workgroup in one tile)", NBc);
        if (Bs && (DM_S2 & 2)) k_level12_strip<2, NBc, L2F, CL, DM_C3_MW><<<grid / NBc, 64 * 2 * NBc, 0, st>>>(gg, s, L1, L2, Bs, Ss);
        // level 1 not stored: the child pows pruned to the level-2 window maxima (dm_prune.h;
        // DM_PRUNE, off: measured slower)
        else if (prune_c3<L2F && YF>(gg, s, L1, L2, Bw, QS, Bs, Ss, grid / NBc, st)) {}
        else if (Bs) k_level1_mfq<1, 4, 2 * NBc, DM_C3_MINW, L2F, YF, NBc, CL, YF><<<grid / NBc, 64 * 2 * NBc, 0, st>>>(gg, s, Bw, QS, L1, L2, Bs, Ss);
        else k_level1_mfq<1, 4, 2 * NBc, 4, L2F, YF, NBc, CL><<<grid / NBc, 64 * 2 * NBc, 0, st>>>(gg, s, Bw, QS, L1, L2);
        HIP_TRY(hipGetLastError());
        return DM_OK;
    }
    // GW = 2 (ws > 5, or widths without a 4-tile split): register budget 5 waves/SIMD
#define DM_MQ(KS_, GW_, NW_) if (KS == KS_ && GW == GW_ && NW == NW_) { k_level1_mfq<KS_, GW_, NW_, 5, L2F, YF><<<grid, 64 * NW_, 0, st>>>(gg, s, Bw, QS, L1, L2); HIP_TRY(hipGetLastError()); return DM_OK; }
    DM_MQ(1, 2, 1) DM_MQ(1, 2, 2) DM_MQ(1, 2, 4) DM_MQ(1, 2, 8)
    if constexpr (!YF) {
        DM_MQ(2, 2, 1) DM_MQ(2, 2, 2) DM_MQ(2, 2, 4) DM_MQ(2, 2, 8)
        DM_MQ(3, 2, 1) DM_MQ(3, 2, 2) DM_MQ(3, 2, 4) DM_MQ(3, 2, 8)
        DM_MQ(4, 2, 1) DM_MQ(4, 2, 2) DM_MQ(4, 2, 4) DM_MQ(4, 2, 8)
    }
#undef DM_MQ
    return fail(DM_ERR_UNSUPPORTED, "no column-split instance for KS=%d GW=%d NW=%d", KS, GW, NW);
}

// the packed-f32 y (YF) needs n <= 25 (see y_of_acc)
template <bool L2F>
static int launch_mfq(const dm_tiles *b, void *d_stats, double *L1, double *L2, hipStream_t st)
{
    dm_v4i *Bw;
    int2 *QS;
    mfma_views(b, d_stats, &Bw, &QS);
    const Stats s = stats_view(d_stats, b->T, b->h0 * b->w0);
    dm_v4i *Bs = nullptr, *Ss = nullptr;
    if (strip_shape(b)) strip_views(b, d_stats, &Bs, &Ss);
    if (b->ws <= 5) return launch_mfq_t<L2F, true>(b, s, Bw, QS, L1, L2, st, Bs, Ss);
    return launch_mfq_t<L2F, false>(b, s, Bw, QS, L1, L2, st, nullptr, nullptr);
}

// LDS-shared-window volume kernel (k_volume_ls): ws <= 5 on the MFMA shapes, 8 waves (patch
// blocks) per workgroup, nontemporal stores
// The w0 = 128 (C3) instances: store runs (TR), register budget (waves per SIMD, MW) and
// nontemporal stores (NT) per output type, chosen by same-box A/B with bit-identical output
// (profiles/r04h_vol.txt, volume checksums; r04g_vtr.txt).  binary16 with the min/max known
// (no min/max sweep): 2 x 512-B runs per store, 144 VGPRs, 6.78 -> 6.61-6.69 ms on 64 tiles
// (6.75 -> 6.42-6.46 on a second box); 1-KB runs (194 VGPRs) 6.94-6.99, plain stores 9.1-9.3
// (the window loads then compete with write-allocate traffic).  The standalone binary16
// volume keeps 256-B runs: its min/max sweep needs the occupancy (runs of 2 / 4: 8.8-9.1 ms
// against 7.85-7.94).
#ifndef DM_VL_H_TR
#define DM_VL_H_TR 2
#endif
#ifndef DM_VL_H_NT
#define DM_VL_H_NT 1
#endif
#ifndef DM_VL_H_NW
#define DM_VL_H_NW 4   // waves (16-patch blocks) per workgroup: 144 VGPRs allow 3 four-wave
#endif          // workgroups per CU against 1 of 8 waves: 6.81 -> 6.52-6.54 ms (r04q_vol_nw.txt); 2 waves 6.66
// float32: 1-KB runs compiled for 4 waves per SIMD (128 VGPRs, 4 spilled) 14.27 -> 13.60-13.71 ms
// standalone, 13.69 -> 13.07-13.11 ms with the min/max known; 1-KB runs at 186 VGPRs 14.0 /
// 16.5 (plain), 2 x 512 B 14.1-14.3.
// w0 = 256 (C5): binary16 with the min/max known, float32 (A/B switches, 256-B runs by default)
#ifndef DM_VL_H2_TR
#define DM_VL_H2_TR 0
#endif
#ifndef DM_VL_H2_NW
#define DM_VL_H2_NW 8
#endif
#ifndef DM_VL_F2_TR
#define DM_VL_F2_TR 0
#endif
#ifndef DM_VL_F2_MW
#define DM_VL_F2_MW 1
#endif
#ifndef DM_VL_HS_NW
#define DM_VL_HS_NW 8   // binary16 standalone (w0 = 128): waves per workgroup
#endif
#ifndef DM_VL_HS_TR
#define DM_VL_HS_TR 0   // binary16 standalone (w0 = 128): 256-B chunks per store run (2 with 4 or 8
#endif                  // waves: 8.24-8.29 against 8.04-8.10 ms, profiles/r05w_volume_ws_ab.txt)
#ifndef DM_VL_F_NW
#define DM_VL_F_NW 8    // float32 (w0 = 128): waves per workgroup
#endif
#ifndef DM_VL_F_TR
#define DM_VL_F_TR 4
#endif
#ifndef DM_VL_F_MW
#define DM_VL_F_MW 4
#endif
#ifndef DM_VL_F_NT
#define DM_VL_F_NT 1
#endif
// the min/max sweep of the volume kernels without a known min/max on the row-pair strips
// dm_corr_stats leaves for the strip shapes (32 x 32 x 32 i8 MFMA, as the level kernel's sweep 1)
#ifndef DM_VS1
#define DM_VS1 1
#endif
template <typename OT>
static int launch_volume_ls(const dm_tiles *b, void *d_stats, const Stats &s, OT *out, hipStream_t st,
                            int have_mm = 0)
{
    if (!volume_ls_shape(b)) return DM_ERR_UNSUPPORTED;
    dm_v4i *Bs = nullptr, *Ss = nullptr;
    if (DM_VS1 && !have_mm && strip_shape(b)) strip_views(b, d_stats, &Bs, &Ss);
    const int G = b->w0 / 16, nw = 8;
    const size_t bpt = (size_t)(b->h0 / 4) * (b->w0 / 4);
    if (bpt % nw) return DM_ERR_UNSUPPORTED;
    // the window operands in k_volume_ls's layout, in the second window region
    dm_v4i *Bw;
    int2 *QS;
    mfma_views2(b, d_stats, &Bw, &QS);
    const size_t n = (size_t)b->T * b->h0 * G * 16;
    const int GW = (int)(16 / sizeof(OT)) < G ? (int)(16 / sizeof(OT)) : G;   // = k_volume_ls's GW
    if (b->ws == 5) k_prep_windows16<5><<<nblk(n, 256), 256, 0, st>>>(make_geo(b), G, GW, 1, Bw, QS);
    else k_prep_windows16<0><<<nblk(n, 256), 256, 0, st>>>(make_geo(b), G, GW, 1, Bw, QS);
    HIP_TRY(hipGetLastError());
    const unsigned grid = (unsigned)(b->T * bpt / nw);
    const Geo gg = make_geo(b);
    if (G == 8) {
        if constexpr (sizeof(OT) == 2) {
            if (have_mm) {
                constexpr int NWh = DM_VL_H_NW;
                if (bpt % NWh) return DM_ERR_UNSUPPORTED;
                k_volume_ls<8, NWh, DM_VL_H_NT, OT, DM_VL_H_TR><<<(unsigned)(b->T * bpt / NWh), 64 * NWh, 0, st>>>(
                    gg, s, Bw, QS, out, have_mm, Bs, Ss);
                HIP_TRY(hipGetLastError());
                return DM_OK;
            }
            if constexpr (DM_VL_HS_NW != 8 || DM_VL_HS_TR != 0) {
                constexpr int NWs = DM_VL_HS_NW;
                if (bpt % NWs) return DM_ERR_UNSUPPORTED;
                k_volume_ls<8, NWs, true, OT, DM_VL_HS_TR><<<(unsigned)(b->T * bpt / NWs), 64 * NWs, 0, st>>>(gg, s, Bw, QS, out, have_mm, Bs, Ss);
                HIP_TRY(hipGetLastError());
                return DM_OK;
            }
        } else {
            constexpr int NWf = DM_VL_F_NW;
            if (bpt % NWf) return DM_ERR_UNSUPPORTED;
            k_volume_ls<8, NWf, DM_VL_F_NT, OT, DM_VL_F_TR, DM_VL_F_MW><<<(unsigned)(b->T * bpt / NWf), 64 * NWf, 0, st>>>(
                gg, s, Bw, QS, out, have_mm, Bs, Ss);
            HIP_TRY(hipGetLastError());
            return DM_OK;
        }
    }
    if (G == 16) {   // w0 = 256 (C5)
        if constexpr (sizeof(OT) == 2) {
            if (have_mm) {
                constexpr int NWh = DM_VL_H2_NW;
                if (bpt % NWh) return DM_ERR_UNSUPPORTED;
                k_volume_ls<16, NWh, true, OT, DM_VL_H2_TR><<<(unsigned)(b->T * bpt / NWh), 64 * NWh, 0, st>>>(
                    gg, s, Bw, QS, out, have_mm, Bs, Ss);
                HIP_TRY(hipGetLastError());
                return DM_OK;
            }
        } else {
            k_volume_ls<16, 8, true, OT, DM_VL_F2_TR, DM_VL_F2_MW><<<grid, 64 * 8, 0, st>>>(gg, s, Bw, QS, out, have_mm, Bs, Ss);
            HIP_TRY(hipGetLastError());
            return DM_OK;
        }
    }
#define DM_VL(G_) if (G == G_) { k_volume_ls<G_, 8, true, OT><<<grid, 64 * 8, 0, st>>>(gg, s, Bw, QS, out, have_mm, Bs, Ss); HIP_TRY(hipGetLastError()); return DM_OK; }
    DM_VL(2) DM_VL(4) DM_VL(8) DM_VL(16)
#undef DM_VL
    return DM_ERR_UNSUPPORTED;
}

// the MFMA volume for the shapes k_volume_ls does not take (ws > 5; GW = 2 there): integer y,
// nontemporal stores, a row staged in LDS where 16 x w0 floats fit
template <typename OT>
static int launch_volume_mfq(const dm_tiles *b, void *d_stats, const Stats &s, OT *out, hipStream_t st)
{
    dm_v4i *Bw;
    int2 *QS;
    mfma_views(b, d_stats, &Bw, &QS);
    const int KS = (b->ws * b->ws + 63) / 64, GW = b->w0 / 16 / mfq_nw(b);
    const size_t waves = (size_t)b->T * (b->h0 / 4) * (b->w0 / 4);
    const unsigned vgrid = (unsigned)((waves + 3) / 4);
    const bool lds = b->w0 <= 128;
    const Geo gg = make_geo(b);
#define DM_VQ(KS_, LS_) if (KS == KS_ && GW == 2 && lds == LS_) { k_volume_mfq<KS_, 2, false, true, LS_, OT><<<vgrid, 256, 0, st>>>(gg, s, Bw, QS, out); HIP_TRY(hipGetLastError()); return DM_OK; }
    DM_VQ(1, true) DM_VQ(1, false) DM_VQ(2, true) DM_VQ(2, false)
    DM_VQ(3, true) DM_VQ(3, false) DM_VQ(4, true) DM_VQ(4, false)
#undef DM_VQ
    return DM_ERR_UNSUPPORTED;
}

extern "C" {

int dm_abi_version(void) { return 110; }

#define DM_STR2(x) #x
#define DM_STR(x) DM_STR2(x)
const char *dm_build_config(void)
{
    return "S1=" DM_STR(DM_S1) " S2=" DM_STR(DM_S2) " PRUNE=" DM_STR(DM_PRUNE) " STRIP_WAVESYNC=" DM_STR(DM_STRIP_WAVESYNC) " VS1=" DM_STR(DM_VS1) " VS1_LDS=" DM_STR(DM_VS1_LDS) " XCD_MAP=" DM_STR(DM_XCD_MAP) " C2_NB=" DM_STR(DM_C2_NB) " C3_NB=" DM_STR(DM_C3_NB) " C3_MW=" DM_STR(DM_C3_MW) " C3_MINW=" DM_STR(DM_C3_MINW) " C5_NB=" DM_STR(DM_C5_NB)
           " VL_H_TR=" DM_STR(DM_VL_H_TR) " VL_H_NT=" DM_STR(DM_VL_H_NT) " VL_H_NW=" DM_STR(DM_VL_H_NW)
           " VL_H2_TR=" DM_STR(DM_VL_H2_TR) " VL_H2_NW=" DM_STR(DM_VL_H2_NW) " VL_F2_TR=" DM_STR(DM_VL_F2_TR)
           " VL_F2_MW=" DM_STR(DM_VL_F2_MW) " VL_HS_NW=" DM_STR(DM_VL_HS_NW) " VL_HS_TR=" DM_STR(DM_VL_HS_TR) " VL_F_NW=" DM_STR(DM_VL_F_NW)
           " VL_F_TR=" DM_STR(DM_VL_F_TR) " VL_F_MW=" DM_STR(DM_VL_F_MW) " VL_F_NT=" DM_STR(DM_VL_F_NT);
}

#if DM_CLOCK_STAMP
// diagnostic builds only (DM_CLOCK_STAMP, dm_mfma.h): the level kernels' per-workgroup clock
// stamps of the last launch, {shader start, shader end, real start, real end} per workgroup
int dm_diag_clock_stamps(unsigned long long *host, int nwg)
{
    if (nwg < 0 || nwg > 65536) return fail(DM_ERR_ARG, "nwg %d outside 0 .. 65536", nwg);
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(dm_clock_stamps), (size_t)nwg * 4 * sizeof(unsigned long long)));
    return DM_OK;
}
#endif

const char *dm_last_error(void) { return g_err; }

size_t dm_stats_bytes(const dm_tiles *b)
{
    if (!b) return 0;
    size_t n = base_stats_bytes(b), extra = 0;
    if (b->ws >= 1 && b->ws <= 15 && b->T > 0 && b->h0 > 0 && b->w0 > 0 && mf16_eligible(b))
        extra = mf16_extra_bytes(b);
    if (!extra) return n;
    size_t tot = align256(n) + align256(extra);
    if (volume_ls_shape(b)) tot += align256(extra);   // + the GW = G region (k_volume_ls)
    if (strip_shape(b)) tot += strip_bytes(b);        // + the row-pair strips (sweep 1)
    return tot;
}

int dm_corr_stats(const dm_tiles *b, void *d_stats, void *stream)
{
    int rc = check_tiles(b);
    if (rc) return rc;
    if (!d_stats) return fail(DM_ERR_ARG, "null stats workspace");
    const int P = b->h0 * b->w0;
    dim3 grid(nblk(P, 256), b->T);
    k_stats<<<grid, 256, 0, (hipStream_t)stream>>>(make_geo(b), stats_view(d_stats, b->T, P));
    HIP_TRY(hipGetLastError());
    const int var = level1_variant(b);
    if (var) { // MFMA-B-ordered windows + packed per-window stats for dm_corr_level1
        dm_v4i *Bw;
        int2 *QS;
        mfma_views(b, d_stats, &Bw, &QS);
        const int G = b->w0 / 16, KS = (b->ws * b->ws + 63) / 64;
        const size_t n = (size_t)b->T * b->h0 * G * 16;
        const int GW = G / mfq_nw(b);
        if (!strip2_shape(b)) {
            if (b->ws == 5) k_prep_windows16<5><<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(make_geo(b), G, GW, KS, Bw, QS);
            else k_prep_windows16<0><<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(make_geo(b), G, GW, KS, Bw, QS);
            HIP_TRY(hipGetLastError());
        }
        if (strip_shape(b)) {
            dm_v4i *Bs, *Ss;
            strip_views(b, d_stats, &Bs, &Ss);
            const size_t ns = (size_t)b->T * (b->h0 / 2) * b->w0;
            if (b->ws == 5) k_prep_strips<5><<<nblk(ns, 256), 256, 0, (hipStream_t)stream>>>(make_geo(b), Bs, Ss);
            else k_prep_strips<0><<<nblk(ns, 256), 256, 0, (hipStream_t)stream>>>(make_geo(b), Bs, Ss);
            HIP_TRY(hipGetLastError());
        }
    }
    return DM_OK;
}

int dm_corr_level1(const dm_tiles *b, void *d_stats, double *d_level1, void *stream)
{
    int rc = check_tiles(b);
    if (rc) return rc;
    if (!d_stats || !d_level1) return fail(DM_ERR_ARG, "null workspace / output");
    if ((b->h0 & 1) || (b->w0 & 1))
        return fail(DM_ERR_SHAPE, "could not broadcast: map sides %dx%d must be even (Correlation_map.py:96-103)", b->h0, b->w0);
    const int P = b->h0 * b->w0;
    Stats s = stats_view(d_stats, b->T, P);
    hipStream_t st = (hipStream_t)stream;
    const int var = level1_variant(b);
    if (var == 3) return launch_mfq<false>(b, d_stats, d_level1, nullptr, st);
    if (P > DM_GENERIC_MAX_P || k2_lds_bytes(b->h0, b->w0, b->ws) > 160 * 1024)
        return fail(DM_ERR_UNSUPPORTED, "tile too large for the generic level-1 kernel (P=%d)", P);
    switch (b->ws) {
    case 1: return launch_level1<1>(b, s, d_level1, st);
    case 3: return launch_level1<3>(b, s, d_level1, st);
    case 5: return launch_level1<5>(b, s, d_level1, st);
    case 7: return launch_level1<7>(b, s, d_level1, st);
    case 9: return launch_level1<9>(b, s, d_level1, st);
    case 11: return launch_level1<11>(b, s, d_level1, st);
    case 13: return launch_level1<13>(b, s, d_level1, st);
    case 15: return launch_level1<15>(b, s, d_level1, st);
    }
    return fail(DM_ERR_UNSUPPORTED, "window size %d", b->ws);
}

int dm_corr_level12(const dm_tiles *b, void *d_stats, double *d_level1, double *d_level2, void *stream)
{
    int rc = check_tiles(b);
    if (rc) return rc;
    if (!d_stats || !d_level2) return fail(DM_ERR_ARG, "null workspace / output");
    if (level1_variant(b) != 3)
        return fail(DM_ERR_UNSUPPORTED, "fused level-1/level-2 kernel needs h0 %% 4 == 0, w0 %% 32 == 0, w0 <= 256, ws <= 15 (got %dx%d, ws %d)",
                    b->h0, b->w0, b->ws);
    return launch_mfq<true>(b, d_stats, d_level1, d_level2, (hipStream_t)stream);
}

static int volume_f32(const dm_tiles *b, void *d_stats, float *d_l0, void *stream, int have_mm)
{
    int rc = check_tiles(b);
    if (rc) return rc;
    if (!d_stats || !d_l0) return fail(DM_ERR_ARG, "null workspace / output");
    const int P = b->h0 * b->w0;
    Stats s = stats_view(d_stats, b->T, P);
    dim3 grid(P, b->T);
    if (level1_variant(b) == 3) { // MFMA paths (the window layouts of dm_corr_stats / k_volume_ls)
        rc = launch_volume_ls<float>(b, d_stats, s, d_l0, (hipStream_t)stream, have_mm);
        if (rc != DM_ERR_UNSUPPORTED) return rc;
        rc = launch_volume_mfq<float>(b, d_stats, s, d_l0, (hipStream_t)stream);
        if (rc != DM_ERR_UNSUPPORTED) return rc;
    }
    k_minmax<<<grid, 256, 0, (hipStream_t)stream>>>(make_geo(b), s);
    HIP_TRY(hipGetLastError());
    k_volume<float><<<grid, 256, 0, (hipStream_t)stream>>>(make_geo(b), s, d_l0);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

static int volume_f16(const dm_tiles *b, void *d_stats, uint16_t *d_l0, void *stream, int have_mm)
{
    int rc = check_tiles(b);
    if (rc) return rc;
    if (!d_stats || !d_l0) return fail(DM_ERR_ARG, "null workspace / output");
    const int P = b->h0 * b->w0;
    Stats s = stats_view(d_stats, b->T, P);
    _Float16 *out = (_Float16 *)d_l0;
    hipStream_t st = (hipStream_t)stream;
    if (level1_variant(b) == 3) {
        rc = launch_volume_ls<_Float16>(b, d_stats, s, out, st, have_mm);
        if (rc != DM_ERR_UNSUPPORTED) return rc;
        rc = launch_volume_mfq<_Float16>(b, d_stats, s, out, st);
        if (rc != DM_ERR_UNSUPPORTED) return rc;
    }
    dim3 grid(P, b->T);
    k_minmax<<<grid, 256, 0, st>>>(make_geo(b), s);
    HIP_TRY(hipGetLastError());
    k_volume<_Float16><<<grid, 256, 0, st>>>(make_geo(b), s, out);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_corr_volume(const dm_tiles *b, void *d_stats, float *d_l0, void *stream)
{
    return volume_f32(b, d_stats, d_l0, stream, 0);
}

int dm_corr_volume_f16(const dm_tiles *b, void *d_stats, uint16_t *d_l0, void *stream)
{
    return volume_f16(b, d_stats, d_l0, stream, 0);
}

int dm_corr_volume_ex(const dm_tiles *b, void *d_stats, int32_t flags, void *d_l0, void *stream)
{
    if (flags & ~(DM_VOLUME_F16 | DM_VOLUME_MINMAX_KNOWN)) return fail(DM_ERR_ARG, "unknown volume flags 0x%x", flags);
    const int mm = (flags & DM_VOLUME_MINMAX_KNOWN) != 0;
    if (flags & DM_VOLUME_F16) return volume_f16(b, d_stats, (uint16_t *)d_l0, stream, mm);
    return volume_f32(b, d_stats, (float *)d_l0, stream, mm);
}

int dm_rectify_f16(const uint16_t *d_in, size_t n, double *d_out, void *stream)
{
    if (!d_in || !d_out) return fail(DM_ERR_ARG, "null pointer");
    if (n == 0) return DM_OK;
    k_rectify<_Float16><<<nblk(n, 256) > 8192 ? 8192 : nblk(n, 256), 256, 0, (hipStream_t)stream>>>(
        (const _Float16 *)d_in, n, d_out);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_rectify(const float *d_in, size_t n, double *d_out, void *stream)
{
    if (!d_in || !d_out) return fail(DM_ERR_ARG, "null pointer");
    if (n == 0) return DM_OK;
    k_rectify<float><<<nblk(n, 256) > 8192 ? 8192 : nblk(n, 256), 256, 0, (hipStream_t)stream>>>(d_in, n, d_out);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_pow14_variant(int32_t variant, const double *d_in, size_t n, double *d_out, void *stream)
{
    if ((!d_in || !d_out) && n) return fail(DM_ERR_ARG, "null input / output");
    if (!n) return DM_OK;
    const unsigned grid = nblk(n, 256) > 1024 ? 1024 : nblk(n, 256);
    hipStream_t st = (hipStream_t)stream;
    switch (variant) {
    case DM_POW_F32: k_pow_variant<DM_POW_F32><<<grid, 256, 0, st>>>(d_in, n, d_out); break;
    case DM_POW_Q4: k_pow_variant<DM_POW_Q4><<<grid, 256, 0, st>>>(d_in, n, d_out); break;
    case DM_POW_K: k_pow_variant<DM_POW_K><<<grid, 256, 0, st>>>(d_in, n, d_out); break;
    case DM_POW_Q4G: k_pow_variant<DM_POW_Q4G><<<grid, 256, 0, st>>>(d_in, n, d_out); break;
    case DM_POW_KG: k_pow_variant<DM_POW_KG><<<grid, 256, 0, st>>>(d_in, n, d_out); break;
    case DM_POW_FULL: k_pow_variant<DM_POW_FULL><<<grid, 256, 0, st>>>(d_in, n, d_out); break;
    default: return fail(DM_ERR_ARG, "unknown pow14 variant %d", variant);
    }
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_rectify64(const double *d_in, size_t n, double *d_out, void *stream)
{
    if (!d_in || !d_out) return fail(DM_ERR_ARG, "null pointer");
    if (n == 0) return DM_OK;
    k_rectify<double><<<nblk(n, 256) > 8192 ? 8192 : nblk(n, 256), 256, 0, (hipStream_t)stream>>>(d_in, n, d_out);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_aggregate(const double *d_in, int32_t T, int32_t h, int32_t w, int32_t rectify, double *d_out,
                 void *stream)
{
    if (!d_in || !d_out || T < 1 || h < 1 || w < 1) return fail(DM_ERR_ARG, "bad aggregate arguments");
    if ((h & 1) || (w & 1))
        return fail(DM_ERR_SHAPE, "could not broadcast: map side %d must halve (Correlation_map.py:96-103)", (h & 1) ? h : w);
    const int W2 = w / 2, h2 = h / 2;
    const char *ag = getenv("DM_AGGREGATE");
    if (W2 >= 16 && 4 * W2 <= 256 && !(ag && ag[0] == '0')) { // streaming kernel
        // band rows: what fits AGG_LDS_DOUBLES (8-row bands measured no faster at C3: the
        // extra input row per band offsets the occupancy)
        const int BR = AGG_LDS_DOUBLES / (4 * W2) < h2 ? AGG_LDS_DOUBLES / (4 * W2) : h2;
        const size_t nwg = (size_t)T * h2 * W2 * ((h2 + BR - 1) / BR);
        if (nwg <= 0x7fffffff) {
            const bool vec = ((uintptr_t)d_in & 15) == 0 && (W2 == 16 || W2 == 32 || W2 == 64);
            const size_t lds = (size_t)4 * BR * W2 * sizeof(double);
            if (vec) k_aggregate_rows<true><<<(unsigned)nwg, 4 * W2, lds, (hipStream_t)stream>>>(d_in, T, h, w, BR, rectify, d_out);
            else k_aggregate_rows<false><<<(unsigned)nwg, 4 * W2, lds, (hipStream_t)stream>>>(d_in, T, h, w, BR, rectify, d_out);
            HIP_TRY(hipGetLastError());
            return DM_OK;
        }
    }
    const size_t n = (size_t)T * (h / 2) * (w / 2) * (h / 2) * (w / 2);
    k_aggregate<<<nblk(n, 256) > 65536 ? 65536 : nblk(n, 256), 256, 0, (hipStream_t)stream>>>(d_in, T, h, w, rectify, d_out);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_match(const dm_tiles *b, const void *d_stats, const double *const *d_levels, int32_t nlev,
             int32_t T, int32_t h0, int32_t w0, int32_t sub_pix, int32_t filter_window,
             int32_t filter_num, int32_t filter_mode, double *d_scratch, double *d_out, void *stream)
{
    if (!d_levels || !d_scratch || !d_out) return fail(DM_ERR_ARG, "null pointer");
    if (T < 1 || h0 < 1 || w0 < 1) return fail(DM_ERR_ARG, "empty batch (T=%d, h0=%d, w0=%d)", T, h0, w0);
    if (nlev < 2) return fail(DM_ERR_SHAPE, "list index out of range: Matching._B needs >= 2 levels (got %d)", nlev);
    if (nlev > 31) return fail(DM_ERR_ARG, "too many levels %d", nlev);
    const int K = nlev - 1;
    if ((h0 >> K) << K != h0 || (w0 >> K) << K != w0)
        return fail(DM_ERR_SHAPE, "map sides %dx%d not divisible by 2^(nlev-1) (nlev=%d)", h0, w0, nlev);
    for (int l = 1; l < nlev; ++l) // level 1 may be on demand too (dm_corr_level12), below the top
        if (!d_levels[l] && !(l == 1 && nlev >= 3 && !d_levels[0]))
            return fail(DM_ERR_ARG, "null level pointer %d", l);
    if (filter_num > 0 && (filter_window < 1 || filter_window > 7))
        return fail(DM_ERR_UNSUPPORTED, "filter_window_size %d not in [1, 7]", filter_window);
    if (filter_mode != 0 && filter_mode != 1) return fail(DM_ERR_ARG, "invalid filtering mode %d", filter_mode);
    Geo g{};
    Stats s{};
    if (!d_levels[0]) {
        int rc = check_tiles(b);
        if (rc) return rc;
        if (!d_stats) return fail(DM_ERR_ARG, "level 0 on demand needs the statistics workspace");
        if (b->T != T || b->h0 != h0 || b->w0 != w0) return fail(DM_ERR_ARG, "tile batch does not match T/h0/w0");
        g = make_geo(b);
        s = stats_view((void *)d_stats, T, h0 * w0);
    }
    hipStream_t st = (hipStream_t)stream;
    // one launch per phase; the buffer parity is chosen so that the last phase writes d_out
    // (no copy): count the swaps (K steps + the filter passes that run)
    int swaps = K;
    {
        int fl = filter_num, hh = h0 >> K, ww = w0 >> K;
        for (int l = K; l >= 0; --l) {
            if (fl > 0) {
                if (hh >= filter_window && ww >= filter_window) ++swaps;
                --fl;
            }
            hh *= 2; ww *= 2;
        }
    }
    double *buf[2] = {d_out, d_scratch};
    int cur = swaps & 1;
    int h = h0 >> K, w = w0 >> K;
    int fleft = filter_num;
    auto filt = [&](int hh, int ww) -> int { // Matching._filter hook (:91-93, :136-138)
        if (fleft > 0) {
            if (hh >= filter_window && ww >= filter_window) {
                if (hh != ww) return fail(DM_ERR_UNSUPPORTED, "Matching._filter needs square maps (%dx%d): Matching.py:235-236", hh, ww);
                k_filter<<<nblk((size_t)T * hh * ww, 64), 64, 0, st>>>(buf[cur], buf[cur ^ 1], T, hh, ww, filter_window, filter_mode);
                HIP_TRY(hipGetLastError());
                cur ^= 1;
            }
            --fleft; // decremented even when the size check skips the filter
        }
        return DM_OK;
    };
    k_match_top<<<nblk((size_t)T * h * w, 64), 64, 0, st>>>(d_levels[K], T, h, w, buf[cur]);
    HIP_TRY(hipGetLastError());
    int rc = filt(h, w);
    if (rc) return rc;
    for (int l = K - 1; l >= 0; --l) {
        const size_t n = (size_t)T * (2 * h) * (2 * w);
        if (l == 1 && !d_levels[1]) { // level 1 on demand: dedicated 4-lanes-per-entry kernel
            const unsigned nb = nblk(4 * n, 256);
            switch (g.ws) {
            case 1: k_match_step_l1<1><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 3: k_match_step_l1<3><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 5: k_match_step_l1<5><<<nblk(4 * n, TAIL_WG), TAIL_WG, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 7: k_match_step_l1<7><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 9: k_match_step_l1<9><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 11: k_match_step_l1<11><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 13: k_match_step_l1<13><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 15: k_match_step_l1<15><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            default:
                k_match_step<<<nblk(n, 64), 64, 0, st>>>(g, s, d_levels[l], l, T, h, w, buf[cur], buf[cur ^ 1]);
            }
        } else if (l == 0 && !d_levels[0] && g.ws <= 15) { // level 0 on demand, taps in registers
            const unsigned nb = nblk(n, 256);
            switch (g.ws) {
            case 1: k_match_step_l0<1><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 3: k_match_step_l0<3><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 5: k_match_step_l0<5><<<nblk(n, TAIL_WG), TAIL_WG, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 7: k_match_step_l0<7><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 9: k_match_step_l0<9><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 11: k_match_step_l0<11><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            case 13: k_match_step_l0<13><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            default: k_match_step_l0<15><<<nb, 256, 0, st>>>(g, s, T, buf[cur], buf[cur ^ 1]); break;
            }
        } else {
            k_match_step<<<nblk(n, 64), 64, 0, st>>>(g, s, d_levels[l], l, T, h, w, buf[cur], buf[cur ^ 1]);
        }
        HIP_TRY(hipGetLastError());
        cur ^= 1;
        h *= 2; w *= 2;
        rc = filt(h, w);
        if (rc) return rc;
    }
    if (sub_pix) {
        const unsigned nb = nblk((size_t)T * h0 * w0, 256);
        if (!d_levels[0]) {
            switch (g.ws) {
            case 1: k_subpix_t<1><<<nb, 256, 0, st>>>(g, s, T, buf[cur]); break;
            case 3: k_subpix_t<3><<<nb, 256, 0, st>>>(g, s, T, buf[cur]); break;
            case 5: k_subpix_t<5><<<nblk((size_t)T * h0 * w0, TAIL_WG), TAIL_WG, 0, st>>>(g, s, T, buf[cur]); break;
            case 7: k_subpix_t<7><<<nb, 256, 0, st>>>(g, s, T, buf[cur]); break;
            case 9: k_subpix_t<9><<<nb, 256, 0, st>>>(g, s, T, buf[cur]); break;
            case 11: k_subpix_t<11><<<nb, 256, 0, st>>>(g, s, T, buf[cur]); break;
            case 13: k_subpix_t<13><<<nb, 256, 0, st>>>(g, s, T, buf[cur]); break;
            default: k_subpix_t<15><<<nb, 256, 0, st>>>(g, s, T, buf[cur]); break;
            }
        } else {
            k_subpix<<<nblk((size_t)T * h0 * w0, 64), 64, 0, st>>>(g, s, d_levels[0], T, h0, w0, h0, w0, buf[cur]);
        }
        HIP_TRY(hipGetLastError());
    }
    if (buf[cur] != d_out) // (the parity above makes this unreachable; kept as a guard)
        HIP_TRY(hipMemcpyAsync(d_out, buf[cur], sizeof(double) * 3 * (size_t)T * h0 * w0, hipMemcpyDeviceToDevice, st));
    return DM_OK;
}

int dm_subpix_map(const double *d_level0, int32_t T, int32_t h0, int32_t w0, int32_t hm, int32_t wm,
                  double *d_map, void *stream)
{
    if (!d_level0 || !d_map) return fail(DM_ERR_ARG, "dm_subpix_map needs level 0 and the map");
    if (T < 1 || h0 < 1 || w0 < 1 || hm < 1 || wm < 1 || hm > h0 || wm > w0)
        return fail(DM_ERR_ARG, "dm_subpix_map: T=%d level 0 %dx%d map %dx%d", T, h0, w0, hm, wm);
    const Geo g{};
    const Stats s{};
    k_subpix<<<nblk((size_t)T * hm * wm, 64), 64, 0, (hipStream_t)stream>>>(g, s, d_level0, T, h0, w0, hm, wm, d_map);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_subpix_map_tiles(const dm_tiles *b, const void *d_stats, int32_t hm, int32_t wm, double *d_map, void *stream)
{
    int rc = check_tiles(b);
    if (rc) return rc;
    if (!d_stats || !d_map) return fail(DM_ERR_ARG, "dm_subpix_map_tiles needs the statistics workspace and the map");
    if (hm < 1 || wm < 1 || hm > b->h0 || wm > b->w0)
        return fail(DM_ERR_ARG, "dm_subpix_map_tiles: map %dx%d for level 0 %dx%d", hm, wm, b->h0, b->w0);
    const Geo g = make_geo(b);
    const Stats s = stats_view((void *)d_stats, b->T, b->h0 * b->w0);
    k_subpix<<<nblk((size_t)b->T * hm * wm, 64), 64, 0, (hipStream_t)stream>>>(g, s, nullptr, b->T, b->h0, b->w0, hm, wm, d_map);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_sub_pix_cal(const double *d_arr, const double *d_score, int32_t h, int32_t w, int32_t direction,
                   double ratio, double *d_out, void *stream)
{
    if (!d_arr || !d_score || !d_out || h < 1 || w < 1) return fail(DM_ERR_ARG, "bad sub_pix_cal arguments");
    if (direction != 0 && direction != 1) return fail(DM_ERR_ARG, "direction must be 0 or 1 (got %d)", direction);
    const size_t n = (size_t)h * w;
    k_sub_pix_cal<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(d_arr, d_score, h, w, direction, ratio, d_out);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_cal_map(const double *d_map, int32_t T, int32_t h, int32_t w, int32_t mode, double *d_out, void *stream)
{
    if (!d_map || !d_out || T < 1 || h < 1 || w < 1) return fail(DM_ERR_ARG, "bad cal_map arguments");
    if (mode < 0 || mode > 2) return fail(DM_ERR_ARG, "please input valid mode! (%d)", mode);
    const size_t n = (size_t)T * h * w;
    k_cal_map<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(d_map, T, h, w, mode, d_out);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

int dm_stitch(const double *d_match, int32_t n0, int32_t n1, int32_t h0, int32_t w0, int32_t stride0,
              int32_t stride1, const int32_t *modes, int32_t nmodes, double *d_dmap, double *d_score,
              void *stream)
{
    if (!d_match || !d_dmap || !d_score || n0 < 1 || n1 < 1 || stride0 < 1 || stride1 < 1 ||
        nmodes < 0 || nmodes > 8 || (nmodes && !modes))
        return fail(DM_ERR_ARG, "bad stitch arguments");
    Modes m;
    for (int k = 0; k < 8; ++k) m.m[k] = k < nmodes ? modes[k] : 0;
    for (int k = 0; k < nmodes; ++k)
        if (m.m[k] < 0 || m.m[k] > 2) return fail(DM_ERR_ARG, "please input valid mode! (%d)", m.m[k]);
    const int Hout = stride0 * (n0 - 1) + h0, Wout = stride1 * (n1 - 1) + w0;
    const size_t n = (size_t)Hout * Wout;
    k_stitch<<<nblk(n, 256), 256, 0, (hipStream_t)stream>>>(d_match, n0, n1, h0, w0, stride0, stride1, m,
                                                            nmodes, d_dmap, d_score, Hout, Wout);
    HIP_TRY(hipGetLastError());
    return DM_OK;
}

} // extern "C"
