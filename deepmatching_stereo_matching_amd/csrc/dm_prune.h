// dm_prune.h -- the fused level-1 / level-2 kernel with PRUNED child pows (k_level12_prune,
// round 6), the C3 (S = 128) instance of k_level1_mfq's algorithm when level 1 is not stored.
// Included by dm_kernels.hip after dm_mfma.h (Geo, Stats, PowLdsG, pow14_zf / q4g / kg,
// fill_ptab, half_wave_minmax, mfma_tile, y_of_acc, pk_*, cellmax_d, k_prep_strips).
//
// Reference semantics (misc/Correlation_map.py:89-159): level 1 of cell i at position j is
// pow14(s_i[j] / 4), s_i[j] = sum over the 4 children of pow14(x_c[j]) (x the pooled, normalised
// level-0 value); level 2 = pow14 of the /4 sum over 4 cells of MaxPool(3, 2, 1) of level 1.
// On the matching path level 1 is never stored (the matching kernels re-derive it), so the
// level kernel needs s_i[j] only to find, for every level-2 window W (3 x 3 level-1 values at
// stride 2) and cell, max_{j in W} s_i[j] (pow14 is monotone: DESIGN.md section 2).  A value
// that is provably below another value of EVERY window it belongs to never decides a maximum,
// and its four float64 child pows -- 28 % of k_level1_mfq's issue cycles -- can be skipped.
//
// The proof uses a bin-centre approximation of each child pow: a_c = (1/c_i)^1.4 * 2^(1.4 E)
// (the hi parts of the pow tables' rows for x = M 2^E, i the top 9 bits of M; two LDS reads and a
// float64 multiply).  x^1.4 = a_c (1 + r)^1.4 (1 + O(2^-52)) with r = M c_i - 1, |r| <= 0.00145
// over all 512 table rows (10-bit c_i), so |a_c / pow14(x) - 1| <= e = 0.00204; the sum of the
// four (and its float32 rounding) keeps that relative bound, a(v) in [s(v)(1 - e), s(v)(1 + e)].
// Hence a(v) < K a(w) with K = 0.9955 <= (1 - e) / (1 + e) proves s(v) < s(w).  A value is a
// CANDIDATE unless, for every window containing it, some known value of that window proves it
// smaller; only candidates get their exact child sums (the same pow14_zf and the same ul, ur,
// ll, lr summation order as k_level1_mfq), the others -inf, and the window maxima -- hence
// level 2 -- are bit for bit k_level1_mfq's.  Each window's true maximum is always a candidate
// (no known value of its window proves it smaller), exact ties included.
//
// Schedule (lane (grp, c): cell grp, level-1 columns 2c, 2c + 1 of the wave's 32; level-2 window
// column c = columns 2c - 1 .. 2c + 1): level-1 rows are decided in pairs, rows 2i and 2i + 1 at
// row 2i + 2, when window i (rows 2i - 1 .. 2i + 1) is complete and window i + 1 (rows 2i + 1 ..
// 2i + 3) known up to row 2i + 2 (a partial window is still a valid proof: its known values).
// Windows a wave cannot see are never used to prune: the next wave's window 0 contains this
// wave's column 31, so lane 15's odd column is always a candidate (its exact value also goes to
// the next wave, as before); column -1 is left out of window 0's maximum (a smaller maximum,
// fewer values pruned).  The 4 x 64 decisions of a pair are compacted (ballot + mbcnt): each
// candidate's x (kept in LDS since its row) is evaluated by one lane -- 4 exact pows per lane
// per round, 64 candidates a round (~59 per pair on the bench's C3 pair: one round, 1.2 on
// average) -- instead of 16 pows per lane per pair.
// The gz rows of the pow tables are not held (PowLdsG: pow14_q4g / pow14_kg from the float32-
// exponent rows, bit for bit pow14_q4 / pow14_k), which keeps the x buffers within 40 KB of LDS
// per 4-wave workgroup: 4 workgroups per CU, 4 waves per SIMD, as k_level1_mfq.
#pragma once

// Measured (round 6, same box, interleaved, profiles/r06d_prune_ab.txt): bit-identical level 2
// (sha256 a2244402bf3721e5 both ways) but 7.03 / 7.08 ms against k_level1_mfq's 6.88 / 6.85 ms
// (+2.8 %).  The ISA model agrees: per row pair the 16 child pows removed from the rows save 660
// issue cycles, the approximations, the candidate bookkeeping (thresholds, ballots, mbcnt
// positions) and 1.2 compacted rounds of 4 exact pows per lane add 571 + 2 x 134.  So it is a
// compile-time switch, off (tools/abl_build.sh prune1 builds it).
#ifndef DM_PRUNE
#define DM_PRUNE 0   // 1: C3 k_level12_prune when level 1 is not stored (0: k_level1_mfq)
#endif

// lane c + 1 of the same 16-lane row (DPP row_shl:1); lane c == 15 gets `old`
__device__ __forceinline__ float dpp_next16_or(float v, float old)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x101, 0xf, 0xf, false));
}

// the bin-centre approximation of pow14(x) (see the header): (1/c_i)^y hi * 2^(yE) hi
__device__ __forceinline__ double pow14_bin(float x, const PowLdsG &t)
{
    const unsigned u = __float_as_uint(x);
    const unsigned ofp = (u >> 10) & 0x1FF0u, og = (u >> 19) & 0xFF0u;
    return (*(const double *)((const char *)t.fp + ofp)) * (*(const double *)((const char *)t.g32 + og));
}

template <int NWc, int NB, int MINW>
__global__ __launch_bounds__(64 * NWc * NB, MINW) void k_level12_prune(Geo g, Stats s, double *L2,
                                                                      const dm_v4i *__restrict__ Bw,
                                                                      const int2 *__restrict__ QS,
                                                                      const dm_v4i *__restrict__ Bs,
                                                                      const dm_v4i *__restrict__ Ss)
{
    constexpr int KS = 1, GW = 4, NW = NWc * NB, M = GW / 2;   // M = 2 pooled columns per lane
    static_assert(NWc > 1, "the column-split instance (C3): one 32-column group per wave");
    constexpr int XS = NWc + 1;
    constexpr int L2V = 4 * GW, L2B = 64 / L2V;                 // level-2 values per wave row; stash rows
    constexpr float K = 0.9955f;                                // <= (1 - e) / (1 + e), e = 0.00204
    struct Lds {
        PowLdsG pw;
        unsigned ptab[NB][16][16];
        float4 cst[NB][4][6];         // [block][cell][field][child]: a_p, lo, hi, rmin, den, rinv
        double stash[NW][64];         // [wave][row slot * L2V + column]: level-2 pow inputs
        float4 xb[NW][2][64][M];      // [wave][level-1 row parity][lane][column]: the 4 children's x
        int addr[NW][64];             // compaction: xb index (within the wave) of a candidate
        double res[NW][64];           // compaction: its exact child sum
    };
    struct Xch {                      // in the g32 rows no input reads (PowLdsG)
        float xch[NB][2][2][XS][4][4];  // [block][pair parity][row][slot][cell group][child]
        double xch2[NB][2][NWc][4];     // [block][level-1 row parity][wave][cell]: exact s at column 32 w + 31
    };
    static_assert(sizeof(Xch) <= G32_HOLE, "exchange arrays in the g32 hole");
    static_assert(sizeof(float) * NB * 2 * NWc * 16 <= sizeof(float4) * NW * 2 * 64 * M, "red fits in xb");
    __shared__ Lds L;
    Xch &X = *reinterpret_cast<Xch *>((char *)&L.pw.g32[128]);
    auto &xch = X.xch;
    auto &xch2 = X.xch2;
    // the per-wave partial min / max of sweep 1 (read before sweep 2 writes xb)
    auto &red = *reinterpret_cast<float (*)[NB][2][NWc][16]>(&L.xb[0][0][0][0]);
    const int tid = threadIdx.x;
    pow_lds_fill_g(L.pw, tid, 64 * NW);
    if (tid < 64 * NB)
        (&xch[tid >> 6][0][0][0][0][0])[((tid & 63) >> 4) * XS * 16 + (tid & 15)] = -INFINITY;
    {
        const int nbj_ = (g.w0 / 2) / 2, bpt_ = ((g.h0 / 2) / 2) * nbj_;
        if (g.ws == 5) fill_ptab<NB, 64 * NW, 5>(L.ptab, g, tid, bpt_, nbj_);
        else fill_ptab<NB, 64 * NW, 0>(L.ptab, g, tid, bpt_, nbj_);
    }
    __syncthreads();

    constexpr int G = GW * NWc;
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sb = wave / NWc, wc = wave % NWc;
    const int c = lane & 15, grp = lane >> 4;
    const int h0 = g.h0, w0 = g.w0, n = g.ws * g.ws, P = h0 * w0;
    const int nbj = (w0 / 2) / 2, bpt = ((h0 / 2) / 2) * nbj;
    const int blk = wg_logical() * NB + sb;
    const int t = blk / bpt;
    const int I0 = 2 * ((blk % bpt) / nbj), J0 = 2 * ((blk % bpt) % nbj);
    const size_t tb = (size_t)t * P;
    const int Ic = I0 + (grp >> 1), Jc = J0 + (grp & 1);

    // ---- sweep 1 on the row-pair strips (k_level1_mfq's S1 path) ----
    {
        const int c32 = lane & 31, hs = lane >> 5;
        const dm_v4i A32 = *(const dm_v4i *)&L.ptab[sb][lane & 15][8 * ((lane >> 4) & 1) + 4 * hs];
        float sTs[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int cell = 2 * (k >> 2) + hs, ch = k & 3;
            const int p = (2 * (I0 + (cell >> 1)) + (ch >> 1)) * w0 + 2 * (J0 + (cell & 1)) + (ch & 1);
            sTs[k] = (float)s.sT[tb + p];
        }
        float mn8[8], mx8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { mn8[k] = INFINITY; mx8[k] = -INFINITY; }
        const int h2 = h0 / 2, NT32 = w0 / 32;
        const __amdgpu_buffer_rsrc_t rS1 = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(Bs + ((size_t)t * h2 * NT32 + 2 * wc) * 64), 0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rS2 = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(Ss + (size_t)t * h2 * w0 + 64 * wc), 0, 0x7fffffff, 0x00020000);
        const unsigned voS = (unsigned)lane * 16u, voQ2 = (unsigned)c32 * 32u;
        struct StripFrag {
            dm_v4i b[2], q[2];
        };
        auto load_strip = [&](StripFrag &f, int rp) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f.b[j] = __builtin_amdgcn_raw_buffer_load_b128(rS1, voS, (unsigned)(rp * NT32 + j) * 1024u, 0);
                f.q[j] = __builtin_amdgcn_raw_buffer_load_b128(rS2, voQ2, (unsigned)(rp * w0 + j) * 16u, 0);
            }
        };
        const float nf = (float)n, nb = -nf * 12582912.0f;
        const dm_v16i acc32 = {DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS,
                               DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS};
        auto minmax_strip = [&](const StripFrag &f) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const dm_v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A32, f.b[j], acc32, 0, 0, 0);
                const dm_f2 qs0 = dm_f2{__int_as_float(f.q[j].x), __int_as_float(f.q[j].y)};
                const dm_f2 qs1 = dm_f2{__int_as_float(f.q[j].z), __int_as_float(f.q[j].w)};
                float y[16];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const int q = m >> 1, cs = q & 1, cp = m & 1;
                    const dm_f2 qs = (q >> 1) ? qs1 : qs0;
                    const dm_f2 a = dm_f2{__int_as_float(acc[2 * m]), __int_as_float(acc[2 * m + 1])};
                    const dm_f2 mm = __builtin_elementwise_fma(a, dm_f2{nf, nf}, dm_f2{nb, nb});
                    const dm_f2 nu = __builtin_elementwise_fma(dm_f2{sTs[4 * cs + 2 * cp], sTs[4 * cs + 2 * cp + 1]},
                                                               __builtin_shufflevector(qs, qs, 0, 0), mm);
                    const dm_f2 yy = pk_mul_bhi(qs, nu);
                    y[2 * m] = yy.x; y[2 * m + 1] = yy.y;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    mn8[k] = fminf(fminf(mn8[k], y[k]), y[8 + k]);
                    mx8[k] = fmaxf(fmaxf(mx8[k], y[k]), y[8 + k]);
                }
            }
        };
        StripFrag sa, sb2;
        load_strip(sa, 0);
        for (int rp = 0; rp < h2; rp += 2) {
            load_strip(sb2, rp + 1);
            minmax_strip(sa);
            load_strip(sa, rp + 2 < h2 ? rp + 2 : rp);
            minmax_strip(sb2);
        }
        half_wave_minmax(mn8, mx8);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int pl = 4 * (2 * (k >> 2) + hs) + (k & 3);
            if (c32 == 31) { red[sb][0][wc][pl] = mn8[k]; red[sb][1][wc][pl] = mx8[k]; }
        }
    }

    // sweep 2's operands: the spread 16 x 16 fragment of patch row c and the patch sums
    dm_v4i A[KS];
    int sTr[4];
    float sTf[4];
    {
        const dm_v2i tp = *(const dm_v2i *)&L.ptab[sb][c][2 * grp];
        A[0] = dm_v4i{tp.x, tp.y, 0, 0};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = (2 * Ic + (r >> 1)) * w0 + 2 * Jc + (r & 1);
            sTr[r] = s.sT[tb + p];
            sTf[r] = (float)sTr[r];
        }
    }
    const dm_v4i acc0 = {DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS};
    const unsigned mant = mant_mask_vgpr();
    const dm_v4i *Bt = Bw + ((size_t)t * h0 * G + wc * GW) * KS * 64;
    struct RowFrag {
        dm_v4i b[GW][KS];
    };
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void *)Bt, 0, 0x7fffffff, 0x00020000);
    const unsigned voB = (unsigned)lane * 16u;
    auto load_row = [&](RowFrag &f, int q0) {
#pragma unroll
        for (int tw = 0; tw < GW; ++tw)
            f.b[tw][0] = __builtin_amdgcn_raw_buffer_load_b128(rB, voB, ((unsigned)q0 * G + tw) * 1024u, 0);
    };
    RowFrag fa, fb;
    load_row(fa, 0);
    __syncthreads();
    // per-patch normalisation constants (k_level1_mfq's)
    if (wc == 0 && c < 4) {
        const int r = c;
        const int p = (2 * Ic + (r >> 1)) * w0 + 2 * Jc + (r & 1);
        const float ap = s.aP[tb + p];
        float a = red[sb][0][0][4 * grp + r], b = red[sb][1][0][4 * grp + r];
#pragma unroll
        for (int w = 1; w < NWc; ++w) { a = fminf(a, red[sb][0][w][4 * grp + r]); b = fmaxf(b, red[sb][1][w][4 * grp + r]); }
        const float rmn = r_of_y(a, ap, g.method), rmx = r_of_y(b, ap, g.method);
        const float den = __fsub_rn(rmx, rmn);
        const bool cc = g.method == DM_TM_CCOEFF;
        float *f = (float *)&L.cst[sb][grp][0];
        f[0 * 4 + r] = ap;
        f[1 * 4 + r] = cc ? -INFINITY : (ap == 0.0f ? 1.0f : -1.0f);
        f[2 * 4 + r] = cc ? INFINITY : 1.0f;
        f[3 * 4 + r] = rmn;
        f[4 * 4 + r] = den;
        f[5 * 4 + r] = __frcp_rn(den);
        s.rmn[tb + p] = rmn;
        s.rmx[tb + p] = rmx;
    }
    __syncthreads();

    // ---- sweep 2: pool on y -> normalise -> x (LDS) + approximate child sums; per row pair:
    // candidates, their exact child sums, level 2 ----
    const bool bflat = __builtin_amdgcn_readfirstlane((int)block_has_flat(L.cst[sb])) != 0;
    float Cprev[M][4];
    double Racc2 = 0.0, Cprev2 = 0.0;
    const int w2 = w0 / 4, P2 = (h0 / 4) * w2;
    double *L2row = L2 + ((size_t)t * P2 + (size_t)(I0 / 2) * w2 + J0 / 2) * P2;

    auto pool_cols = [&](const RowFrag &f, float (&Cm)[M][4], float (&last)[4]) {
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            const dm_v4i acc = mfma_tile<KS, true>(A, f.b[tw], acc0);
            float y[4];
            y_of_acc<true>(acc, sTr, sTf, qs_of_frag(f.b[tw][0]), n, y);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if ((tw & 1) == 0) Cm[tw / 2][r] = tw == 0 ? y[r] : fmaxf(last[r], y[r]);
                else Cm[tw / 2][r] = fmaxf(Cm[tw / 2][r], y[r]);
                last[r] = y[r];
            }
        }
    };

    // level 2 from level-1 row u's exact child sums (-inf where pruned): k_level1_mfq's level2_row
    // (M = 2: one level-2 column per lane) with the g32 pow forms
    auto level2_row = [&](int u, const double (&l1v)[M]) {
        const double lft = __shfl(l1v[M - 1], lane - 1);
        const double left = c != 0 ? lft : (wc == 0 ? l1v[0] : xch2[sb][u & 1][wc - 1][grp]);
        const double Cq = cellmax_d(cellmax_d(left, l1v[0]), l1v[1]);
        if ((u & 1) == 0) {
            Racc2 = u == 0 ? Cq : cellmax_d(Cprev2, Cq);
            return;
        }
        const int u2 = u >> 1, slot = u2 % L2B;
        const double R2 = pow14_q4g(cellmax_d(Racc2, Cq), L.pw);   // pooled child, rectified
        Cprev2 = Cq;
        const double s0 = __shfl(R2, c), s1 = __shfl(R2, c + 16), s2 = __shfl(R2, c + 32), s3 = __shfl(R2, c + 48);
        if (grp == 0) L.stash[wave][slot * L2V + c] = (((s0 + s1) + s2) + s3) / 4.0;
        if (slot == L2B - 1 || u2 == h0 / 4 - 1) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < (slot + 1) * L2V) {
                double l2 = pow14_kg(L.stash[wave][lane], L.pw);
                if (bflat) l2 = (double)NAN; // see norm_clamp
                L2row[(size_t)(u2 - slot + lane / L2V) * w2 + 4 * GW * wc + lane % L2V] = l2;
            }
            __builtin_amdgcn_wave_barrier();
        }
    };

    // the pair's decisions and exact sums: rows r0 (even, approximations ae, x in xb[0]) and
    // r0 + 1 (odd, ao, xb[1]); an: row r0 + 2's approximations (has_next) -- see the header
    float ae[M], ao[M], cAo_prev = -INFINITY;
    auto colmax = [&](const float (&a)[M]) {
        return fmaxf(fmaxf(dpp_prev16_or(a[1], -INFINITY), a[0]), a[1]);
    };
    auto decide = [&](int r0, bool has_next, const float (&an)[M]) {
        const float cAe = colmax(ae), cAo = colmax(ao);
        const float Wi = fmaxf(fmaxf(cAo_prev, cAe), cAo);             // window r0 / 2: complete
        const float Wn = has_next ? fmaxf(cAo, colmax(an)) : INFINITY;  // window r0 / 2 + 1: rows known
        const float Wo = fminf(Wi, Wn);
        cAo_prev = cAo;
        const float te1 = fminf(Wi, dpp_next16_or(Wi, -INFINITY));      // odd column: windows c, c + 1
        const float to1 = fminf(Wo, dpp_next16_or(Wo, -INFINITY));
        const bool k0 = ae[0] >= K * Wi, k1 = ae[1] >= K * te1, k2 = ao[0] >= K * Wo, k3 = ao[1] >= K * to1;
        const unsigned long long m0 = __builtin_amdgcn_ballot_w64(k0), m1 = __builtin_amdgcn_ballot_w64(k1);
        const unsigned long long m2 = __builtin_amdgcn_ballot_w64(k2), m3 = __builtin_amdgcn_ballot_w64(k3);
        const int b1 = __builtin_popcountll(m0), b2 = b1 + __builtin_popcountll(m1);
        const int b3 = b2 + __builtin_popcountll(m2), nc = b3 + __builtin_popcountll(m3);
        auto below = [&](unsigned long long m) {
            return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        };
        const int p0 = below(m0), p1 = b1 + below(m1), p2 = b2 + below(m2), p3 = b3 + below(m3);
        double ee[M] = {-INFINITY, -INFINITY}, eo[M] = {-INFINITY, -INFINITY};
        for (int base = 0; base < nc; base += 64) {   // wave-uniform: ceil(nc / 64) rounds
            // xb index within the wave: (parity * 64 + lane) * M + column
            if (k0 && (unsigned)(p0 - base) < 64u) L.addr[wave][p0 - base] = (0 * 64 + lane) * M + 0;
            if (k1 && (unsigned)(p1 - base) < 64u) L.addr[wave][p1 - base] = (0 * 64 + lane) * M + 1;
            if (k2 && (unsigned)(p2 - base) < 64u) L.addr[wave][p2 - base] = (1 * 64 + lane) * M + 0;
            if (k3 && (unsigned)(p3 - base) < 64u) L.addr[wave][p3 - base] = (1 * 64 + lane) * M + 1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < nc - base) {
                const float4 x4 = (&L.xb[wave][0][0][0])[L.addr[wave][lane]];
                double sum = pow14_zf(x4.x, L.pw, mant);       // ul, ur, ll, lr: left-to-right sum
                sum = sum + pow14_zf(x4.y, L.pw, mant);
                sum = sum + pow14_zf(x4.z, L.pw, mant);
                sum = sum + pow14_zf(x4.w, L.pw, mant);
                L.res[wave][lane] = sum;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (k0 && (unsigned)(p0 - base) < 64u) ee[0] = L.res[wave][p0 - base];
            if (k1 && (unsigned)(p1 - base) < 64u) ee[1] = L.res[wave][p1 - base];
            if (k2 && (unsigned)(p2 - base) < 64u) eo[0] = L.res[wave][p2 - base];
            if (k3 && (unsigned)(p3 - base) < 64u) eo[1] = L.res[wave][p3 - base];
            __builtin_amdgcn_wave_barrier();
        }
        // the wave's last column (always a candidate) to the next wave, then level 2 of both rows
        if (c == 15) { xch2[sb][0][wc][grp] = ee[1]; xch2[sb][1][wc][grp] = eo[1]; }
        __syncthreads();
        level2_row(r0, ee);
        level2_row(r0 + 1, eo);
    };

    for (int q0 = 0; q0 < h0; q0 += 2) {
        const int u = q0 >> 1, k = u & 1;
        load_row(fb, q0 + 1);
        float Ca[M][4], Cb[M][4], la[4], lb[4];
        pool_cols(fa, Ca, la);
        if (q0 > 0) {
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) Ca[m][r] = fmaxf(Cprev[m][r], Ca[m][r]);
        }
        pool_cols(fb, Cb, lb);
        if (c == 15) {
#pragma unroll
            for (int r = 0; r < 4; ++r) { xch[sb][k][0][wc + 1][grp][r] = la[r]; xch[sb][k][1][wc + 1][grp][r] = lb[r]; }
        }
        __syncthreads();
        {
            const float4 xa = *(const float4 *)&xch[sb][k][0][wc][grp][0];
            const float4 xb_ = *(const float4 *)&xch[sb][k][1][wc][grp][0];
            const float oa[4] = {xa.x, xa.y, xa.z, xa.w}, ob[4] = {xb_.x, xb_.y, xb_.z, xb_.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                Ca[0][r] = fmaxf(Ca[0][r], dpp_prev16_or(la[r], oa[r]));
                Cb[0][r] = fmaxf(Cb[0][r], dpp_prev16_or(lb[r], ob[r]));
            }
        }
        // normalise (the clamp bit, norm_clamp) -> x of the 4 children per column, and the
        // approximate child sums
        const float4 kap = L.cst[sb][grp][0], kmn = L.cst[sb][grp][3], kden = L.cst[sb][grp][4], kinv = L.cst[sb][grp][5];
        float4 xr[M];
        float an[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            float R[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                R[r] = fmaxf(Ca[m][r], Cb[m][r]);
                Cprev[m][r] = Cb[m][r];
            }
            const dm_f2 ra = dm_f2{R[0], R[1]} * dm_f2{kap.x, kap.y}, rb = dm_f2{R[2], R[3]} * dm_f2{kap.z, kap.w};
            const dm_f2 a01 = ra - dm_f2{kmn.x, kmn.y}, a23 = rb - dm_f2{kmn.z, kmn.w};
            const dm_f2 i01 = {kinv.x, kinv.y}, i23 = {kinv.z, kinv.w};
            const dm_f2 q01 = a01 * i01, q23 = a23 * i23;
            const dm_f2 e01 = __builtin_elementwise_fma(-q01, dm_f2{kden.x, kden.y}, a01);
            const dm_f2 e23 = __builtin_elementwise_fma(-q23, dm_f2{kden.z, kden.w}, a23);
            const dm_f2 x01 = pk_fma_clamp01(e01, i01, q01), x23 = pk_fma_clamp01(e23, i23, q23);
            xr[m] = make_float4(x01.x, x01.y, x23.x, x23.y);
            an[m] = (float)(((pow14_bin(x01.x, L.pw) + pow14_bin(x01.y, L.pw)) + pow14_bin(x23.x, L.pw)) +
                            pow14_bin(x23.y, L.pw));
        }
        if (k == 0) {
            if (u > 0) decide(u - 2, true, an);      // rows u - 2, u - 1 (their x in xb[0], xb[1])
#pragma unroll
            for (int m = 0; m < M; ++m) { L.xb[wave][0][lane][m] = xr[m]; ae[m] = an[m]; }
        } else {
#pragma unroll
            for (int m = 0; m < M; ++m) { L.xb[wave][1][lane][m] = xr[m]; ao[m] = an[m]; }
        }
        load_row(fa, q0 + 2 < h0 ? q0 + 2 : 0);
    }
    decide(h0 / 2 - 2, false, ae);   // the last pair (no row after it: window h0 / 4 is absent)
}
