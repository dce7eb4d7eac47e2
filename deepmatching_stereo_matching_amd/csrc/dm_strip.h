// dm_strip.h -- the fused level-1 / level-2 kernel with BOTH sweeps on row-pair strips
// (k_level12_strip).  Included by dm_kernels.hip after dm_mfma.h (Geo, Stats, PowLds, pow14_*,
// fill_ptab, half_wave_minmax, pk_mul_bhi, pk_fma_clamp01, cellmax_d, k_prep_strips).
//
// Reference semantics as k_level1_mfq (misc/Correlation_map.py:69-159, misc/Feature_value.py:
// 32-43): level 1 of cell (I, J) at (u, v) = pow14((R_ul + R_ur + R_ll + R_lr) / 4), R_c the
// MaxPool(3,2,1) of child c's rectified min-max level-0 map; level 2 the same one level up.
//
// k_level1_mfq sweeps the level-0 windows twice: sweep 1 (per-patch min / max of y) on the
// row-pair strips with v_mfma_i32_32x32x32_i8, sweep 2 (pool, normalise, rectify) on 16 x 16
// tiles with v_mfma_i32_16x16x32_i8 -- twice the matrix-core issue cycles per voxel, and a
// second window operand set (k_prep_windows16) read from memory.  Here sweep 2 runs on the
// same strips: one 32 x 32 x 32 MFMA gives a lane 8 patches (2 cells x 4 children) x 2 window
// rows of ONE window column, and the strips' columns are ordered so that lane c32 of strip
// tiles j = 0, 1 holds windows 2 c32 + j of the wave's 64 (k_prep_strips).  Then
//   - the row pooling of level-1 row u (window rows 2u - 1, 2u, 2u + 1) is in the lane: the two
//     rows of the pair and the previous pair's odd row (carried, 16 floats);
//   - the column pooling of level-1 column v = c32 (windows 2v - 1, 2v, 2v + 1) needs one value
//     from lane c32 - 1 (DPP row_shr:1); the first lane of each 16-lane row gets it through LDS
//     (lane 15 -> 16 and 47 -> 48 of the same wave, lanes 31 / 63 -> lanes 0 / 32 of the next);
//   - a lane's pooled values are the 4 children of 2 cells at one level-1 column: the child
//     sums stay in the lane, as before.
// Level 2 pools level-1 columns 2 v2 - 1 .. 2 v2 + 1 = lanes c32 - 1 .. c32 + 1 (even c32) and
// rectifies the 64 pooled children of a level-2 row with one pow per lane (LDS stash).
// Every value is formed by the same operations on the same operands as k_level1_mfq's (y, the
// pooling maxima, the Markstein quotient, pow14, the child sums in ul, ur, ll, lr order), so
// the two kernels agree bit for bit.
#pragma once

// LDS hand-over inside one cell block: a workgroup barrier when the block spans NWc > 1 waves,
// a wave barrier (with the LDS fences) when the block is one wave
#ifndef DM_STRIP_WAVESYNC
#define DM_STRIP_WAVESYNC 0   // 1: wave barriers for one-wave blocks (C2) -- A/B switch, measured neutral (round 6)
#endif
template <int NWc>
__device__ __forceinline__ void block_sync()
{
    if constexpr (NWc > 1 || !DM_STRIP_WAVESYNC) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int NWc, int NB, bool L2F, bool CL, int MINW>
__global__ __launch_bounds__(64 * NWc * NB, MINW) void k_level12_strip(Geo g, Stats s, double *L1, double *L2,
                                                                       const dm_v4i *__restrict__ Bs,
                                                                       const dm_v4i *__restrict__ Ss)
{
    DM_CLOCK_STAMP_HERE
    constexpr int NW = NWc * NB;
    constexpr bool RICH = MINW < 4;   // register budget of 3 waves / SIMD (or fewer)
    static_assert(!CL || L2F, "clamp-bit normalisation: NaN cells are restored at the level-2 / level-1 stores");
    __shared__ PowLds plds;
    // [block][pair parity][slot][16-lane row][patch slot]: the row-pooled y of window 2 c32 + 1
    // of the last lane of the 16-lane row before (slot w, rows 1 / 3: lanes 15 / 47 of wave w;
    // slot w + 1, rows 0 / 2: lanes 31 / 63 of wave w; slot 0 rows 0 / 2 = -inf, the padding)
    __shared__ __attribute__((aligned(16))) float xs[NB][2][NWc + 1][4][8];
    // [block][level-1 row parity][slot][half][cell slot]: level 1 at column 32 w + 31 of wave w - 1
    __shared__ double xch2[L2F ? NB : 1][2][NWc + 1][2][2];
    __shared__ double stash[L2F ? NW : 1][64];   // [wave][row slot * 16 + column]: level-2 pow inputs
    __shared__ double stash2[L2F ? NW : 1][64];  // [wave][cell * 16 + column]: pooled children
    __shared__ float red[NB][2][NWc][16];        // per-wave partial min / max per patch
    __shared__ float4 cst[NB][4][7];             // [block][cell][field][child]: a_p, lo, hi, rmin, den, rinv, f32(sT)
    __shared__ __attribute__((aligned(16))) unsigned ptab[NB][16][16];
    const int tid = threadIdx.x;
    pow_lds_fill(plds, tid, 64 * NW, false);
    if (tid < 32 * NB)
        xs[tid >> 5][(tid >> 4) & 1][0][2 * ((tid >> 3) & 1)][tid & 7] = -INFINITY;
    {
        const int nbj_ = (g.w0 / 2) / 2, bpt_ = ((g.h0 / 2) / 2) * nbj_;
        if (g.ws == 5) fill_ptab<NB, 64 * NW, 5>(ptab, g, tid, bpt_, nbj_);
        else fill_ptab<NB, 64 * NW, 0>(ptab, g, tid, bpt_, nbj_);
    }
    __syncthreads();

    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sb = NB > 1 ? wave / NWc : 0, wc = NB > 1 ? wave % NWc : wave;
    const int c32 = lane & 31, hs = lane >> 5, row16 = lane >> 4;
    // the lane index re-read where a rarely used address is formed (edge stores, level-2 stash):
    // the compiler would otherwise hoist those addresses out of sweep 2's loop and spill them
    auto laundered_lane = [&]() {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        return ln;
    };
    const int h0 = g.h0, w0 = g.w0, n = g.ws * g.ws, P = h0 * w0;
    const int h2 = h0 / 2, w1 = w0 / 2, P1 = h2 * w1, NT32 = w0 / 32;
    const int nbj = w1 / 2, bpt = (h2 / 2) * nbj;       // 2x2-cell blocks per tile
    const int blk = wg_logical() * NB + sb;
    const int t = blk / bpt;                             // whole workgroup in range (grid exact)
    const int I0 = 2 * ((blk % bpt) / nbj), J0 = 2 * ((blk % bpt) % nbj);
    const size_t tb = (size_t)t * P;

    // A rows (lane & 31): patch lane & 15 at strip row offset (lane >> 4) & 1, K bytes 16 hs ..
    // (read from the tap table where it is used: no registers held through sweep 2's pows)
    const dm_v4i *A32p = (const dm_v4i *)&ptab[sb][lane & 15][8 * ((lane >> 4) & 1) + 4 * hs];
    const dm_v4i A32 = *A32p;
    float sTs[8];   // [cell slot cs][child]: f32(sum T') of patch 4 (2 cs + hs) + child
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int cell = 2 * (k >> 2) + hs, ch = k & 3;
        const int p = (2 * (I0 + (cell >> 1)) + (ch >> 1)) * w0 + 2 * (J0 + (cell & 1)) + (ch & 1);
        sTs[k] = (float)s.sT[tb + p];
    }
    // strip tiles 2 wc, 2 wc + 1 of every row pair: lane c32 of tile j is window 64 wc + 2 c32 + j
    const __amdgpu_buffer_rsrc_t rS1 = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(Bs + ((size_t)t * h2 * NT32 + 2 * wc) * 64), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rS2 = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(Ss + (size_t)t * h2 * w0 + 64 * wc), 0, 0x7fffffff, 0x00020000);
    const unsigned voS = (unsigned)lane * 16u, voQ = (unsigned)c32 * 32u;
    struct StripFrag {
        dm_v4i b[2], q[2];
    };
    auto load_strip = [&](StripFrag &f, int rp) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f.b[j] = __builtin_amdgcn_raw_buffer_load_b128(rS1, voS, (unsigned)(rp * NT32 + j) * 1024u, 0);
            f.q[j] = __builtin_amdgcn_raw_buffer_load_b128(rS2, voQ, (unsigned)(rp * w0 + j) * 16u, 0);
        }
    };
    const float nf = (float)n, nb = -nf * 12582912.0f; // y_of_acc's exact steps
    const dm_v16i acc32 = {DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS,
                           DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS};
    // y of strip tile j: y[4 q + child], q = 2 (window row) + cell slot (y_of_acc's steps)
    auto acc_y = [&](const dm_v16i &acc, const dm_v4i &qv, const float (&sTs)[8], float (&y)[16]) {
        const dm_f2 qs0 = dm_f2{__int_as_float(qv.x), __int_as_float(qv.y)};
        const dm_f2 qs1 = dm_f2{__int_as_float(qv.z), __int_as_float(qv.w)};
#pragma unroll
        for (int m = 0; m < 8; ++m) { // register pair (2m, 2m + 1): row 8 (m >> 2) + 4 hs + 2 (m & 1) + {0, 1}
            const int q = m >> 1, cs = q & 1, cp = m & 1;
            const dm_f2 qs = (q >> 1) ? qs1 : qs0;  // window row q0 + (q >> 1)
            const dm_f2 a = dm_f2{__int_as_float(acc[2 * m]), __int_as_float(acc[2 * m + 1])};
            const dm_f2 mm = __builtin_elementwise_fma(a, dm_f2{nf, nf}, dm_f2{nb, nb});
            const dm_f2 nu = __builtin_elementwise_fma(dm_f2{sTs[4 * cs + 2 * cp], sTs[4 * cs + 2 * cp + 1]},
                                                       __builtin_shufflevector(qs, qs, 0, 0), mm);
            const dm_f2 yy = pk_mul_bhi(qs, nu);
            y[2 * m] = yy.x; y[2 * m + 1] = yy.y;
        }
    };
    auto strip_y = [&](const StripFrag &f, int j, const float (&sTs)[8], float (&y)[16]) {
        acc_y(__builtin_amdgcn_mfma_i32_32x32x32_i8(A32, f.b[j], acc32, 0, 0, 0), f.q[j], sTs, y);
    };

    // ---- sweep 1: min / max of y over this wave's windows, then over the waves ----
    {
        float mn8[8], mx8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { mn8[k] = INFINITY; mx8[k] = -INFINITY; }
        auto minmax_strip = [&](const StripFrag &f) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                float y[16];
                strip_y(f, j, sTs, y);
#pragma unroll
                for (int k = 0; k < 8; ++k) { // (cs, child): rows q0 (register k) and q0 + 1 (8 + k)
                    mn8[k] = fminf(fminf(mn8[k], y[k]), y[8 + k]);
                    mx8[k] = fmaxf(fmaxf(mx8[k], y[k]), y[8 + k]);
                }
            }
        };
        StripFrag sa, sb2;
        load_strip(sa, 0);
        for (int rp = 0; rp < h2; rp += 2) { // h2 even (h0 % 4 == 0)
            load_strip(sb2, rp + 1);
            minmax_strip(sa);
            load_strip(sa, rp + 2 < h2 ? rp + 2 : rp); // (the last one: in range, unused)
            minmax_strip(sb2);
        }
        half_wave_minmax(mn8, mx8);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int pl = 4 * (2 * (k >> 2) + hs) + (k & 3);  // patch of the block: 4 cell + child
            if (c32 == 31) { red[sb][0][wc][pl] = mn8[k]; red[sb][1][wc][pl] = mx8[k]; }
        }
    }
    StripFrag f2;
    load_strip(f2, 0); // sweep 2's first row pair, in flight through the reduction
    // the reduction's partial extremes: from the block's waves (a workgroup barrier), or with one
    // wave per block (NWc == 1: C2) from this wave alone -- a wave barrier, so the workgroup's
    // NB independent blocks do not wait for each other between the sweeps (round 6)
    block_sync<NWc>();
    // per-patch normalisation constants {a_p, lo, hi, rmin, den, RN(1/den)} -> LDS (k_level1_mfq's)
    if (wc == 0 && (lane & 15) < 4) {
        const int r = lane & 15, grp = lane >> 4;
        const int p = (2 * (I0 + (grp >> 1)) + (r >> 1)) * w0 + 2 * (J0 + (grp & 1)) + (r & 1);
        const float ap = s.aP[tb + p];
        float a = red[sb][0][0][4 * grp + r], b = red[sb][1][0][4 * grp + r];
#pragma unroll
        for (int w = 1; w < NWc; ++w) { a = fminf(a, red[sb][0][w][4 * grp + r]); b = fmaxf(b, red[sb][1][w][4 * grp + r]); }
        const float rmn = r_of_y(a, ap, g.method), rmx = r_of_y(b, ap, g.method);
        const float den = __fsub_rn(rmx, rmn);
        const bool cc = g.method == DM_TM_CCOEFF;
        float *f = (float *)&cst[sb][grp][0];
        f[0 * 4 + r] = ap;
        f[1 * 4 + r] = cc ? -INFINITY : (ap == 0.0f ? 1.0f : -1.0f);
        f[2 * 4 + r] = cc ? INFINITY : 1.0f;
        f[3 * 4 + r] = rmn;
        f[4 * 4 + r] = den;
        f[5 * 4 + r] = __frcp_rn(den);
        f[6 * 4 + r] = (float)s.sT[tb + p];
        s.rmn[tb + p] = rmn;
        s.rmx[tb + p] = rmx;
    }
    block_sync<NWc>();

    // ---- sweep 2: pool on y -> normalise + rectify -> children sum -> level 1 [-> level 2] ----
    const bool bflat = CL && __builtin_amdgcn_readfirstlane((int)(cell_flat(cst[sb][0][4]) || cell_flat(cst[sb][1][4]) ||
                                                                 cell_flat(cst[sb][2][4]) || cell_flat(cst[sb][3][4]))) != 0;
    const unsigned mant = mant_mask_vgpr();   // pow14_zf's mantissa mask, kept in a VGPR
    const int w2 = w0 / 4, P2 = (h0 / 4) * w2;
    // level 2 of the block's level-2 cell (I0 / 2, J0 / 2), stored through a buffer resource
    // (scalar base, 32-bit lane offsets: no 64-bit address held per lane)
    const __amdgpu_buffer_rsrc_t rL2 = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(L2F ? L2 + ((size_t)t * P2 + (size_t)(I0 / 2) * w2 + J0 / 2) * P2 : L2), 0, 0x7fffffff, 0x00020000);
    // level-1 rows of the lane's cells hs (I0, J0 + hs) and 2 + hs (I0 + 1, J0 + hs), column 32 wc + c32
    float po[2][8];           // the previous pair's odd-row y of windows 2 c32 + j
#pragma unroll
    for (int k = 0; k < 8; ++k) { po[0][k] = -INFINITY; po[1][k] = -INFINITY; }
    // carry2: level-2 row pooling state of the lane's two cells -- the pooled rows 2 u2 - 1 and
    // 2 u2 after an even level-1 row, the column-pooled row 2 u2 + 1 after an odd one (never
    // both live at once)
    double l1p[2] = {0.0, 0.0}, carry2[2];

    // level 2 of the block from level-1 row u (the values before rectification, l1v): MaxPool
    // over level-1 columns 2 v2 - 1 .. 2 v2 + 1 (lanes c32 - 1 .. c32 + 1, valid on even c32;
    // column -1 is padding: the value itself stands in, cellmax_d), rows over u; every second
    // row the 64 pooled children (2 cells x 32 lanes) are rectified with one pow per lane, summed
    // in ul, ur, ll, lr order, /4, stashed; every 4 level-2 rows one pow per lane -> level 2
    auto level2_row = [&](int u, const double (&l1v)[2]) {
        double Cq[2];
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) {
            const double lft = __shfl(l1v[cs], lane - 1), rgt = __shfl(l1v[cs], lane + 1);
            const double left = c32 != 0 ? lft : (wc == 0 ? l1v[cs] : xch2[sb][u & 1][wc][hs][cs]);
            Cq[cs] = cellmax_d(cellmax_d(left, l1v[cs]), rgt);
        }
        if ((u & 1) == 0) {
#pragma unroll
            for (int cs = 0; cs < 2; ++cs) carry2[cs] = u == 0 ? Cq[cs] : cellmax_d(carry2[cs], Cq[cs]);
            return;
        }
        const int u2 = u >> 1, slot = u2 & 3;
        if ((c32 & 1) == 0) {
            const int ln = laundered_lane();
#pragma unroll
            for (int cs = 0; cs < 2; ++cs) stash2[wave][(2 * cs + (ln >> 5)) * 16 + ((ln & 31) >> 1)] = cellmax_d(carry2[cs], Cq[cs]);
        }
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) carry2[cs] = Cq[cs];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double Pc = pow14_q4(stash2[wave][lane], plds);   // pooled child, rectified
        __builtin_amdgcn_wave_barrier();
        stash2[wave][lane] = Pc;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < 16) {
            const double *q = &stash2[wave][lane];
            stash[wave][slot * 16 + lane] = (((q[0] + q[16]) + q[32]) + q[48]) / 4.0;
        }
        if (slot == 3 || u2 == h0 / 4 - 1) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < (slot + 1) * 16) {
                const int ln = laundered_lane();
                double l2 = pow14_k(stash[wave][lane], plds);
                if (CL && bflat) l2 = (double)NAN; // see norm_clamp
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(dm_v2i, l2), rL2,
                                                      (unsigned)((ln >> 4) * w2 + 16 * wc + (ln & 15)) * 8u,
                                                      (unsigned)((u2 - slot) * w2) * 8u, 0);
            }
        }
        __builtin_amdgcn_wave_barrier();
    };

    // one row pair = level-1 row u: y of both strip tiles, row pooling in the lane, the edge
    // values through LDS (one barrier), column pooling, normalise, rectify, child sums.
    // One operand buffer: each fragment is reloaded with the next pair's as soon as it has been
    // used (B after its MFMA, the window stats after the y), which keeps 16 VGPRs fewer live
    // than a second buffer would
    auto pair = [&](StripFrag &f, int u) {
        // (the last one: in range, unused; wave-uniform for the buffer loads' scalar offsets)
        const int nx = __builtin_amdgcn_readfirstlane(u + 1 < h2 ? u + 1 : u);
        const int k = u & 1;
        float rm[2][8];
        // RICH (< 4 waves per SIMD): A and the patch sums stay in registers; otherwise they are
        // re-read from LDS here (no registers held through the pows)
        const dm_v4i A2 = RICH ? A32 : *A32p;
        float sT2[8];
        if constexpr (RICH) {
#pragma unroll
            for (int k = 0; k < 8; ++k) sT2[k] = sTs[k];
        } else {
            const float4 s0 = cst[sb][hs][6], s1 = cst[sb][2 + hs][6];
            sT2[0] = s0.x; sT2[1] = s0.y; sT2[2] = s0.z; sT2[3] = s0.w;
            sT2[4] = s1.x; sT2[5] = s1.y; sT2[6] = s1.z; sT2[7] = s1.w;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float y[16];
            const dm_v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A2, f.b[j], acc32, 0, 0, 0);
            f.b[j] = __builtin_amdgcn_raw_buffer_load_b128(rS1, voS, (unsigned)(nx * NT32 + j) * 1024u, 0);
            acc_y(acc, f.q[j], sT2, y);
            f.q[j] = __builtin_amdgcn_raw_buffer_load_b128(rS2, voQ, (unsigned)(nx * w0 + j) * 16u, 0);
#pragma unroll
            for (int kk = 0; kk < 8; ++kk) {
                rm[j][kk] = fmaxf(fmaxf(po[j][kk], y[kk]), y[8 + kk]);
                po[j][kk] = y[8 + kk];
            }
        }
        if ((lane & 15) == 15) {
            const int r16 = laundered_lane() >> 4;
            const int slot = (r16 & 1) ? wc + 1 : wc, row = (r16 & 1) ? r16 - 1 : r16 + 1;
            *(float4 *)&xs[sb][k][slot][row][0] = make_float4(rm[1][0], rm[1][1], rm[1][2], rm[1][3]);
            *(float4 *)&xs[sb][k][slot][row][4] = make_float4(rm[1][4], rm[1][5], rm[1][6], rm[1][7]);
            if (L2F && NWc > 1 && u > 0 && c32 == 31) {
                xch2[sb][k ^ 1][wc + 1][hs][0] = l1p[0];
                xch2[sb][k ^ 1][wc + 1][hs][1] = l1p[1];
            }
        }
        if constexpr (NWc > 1) {
            __syncthreads();
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        float R[8];
        {
            const float4 xa = *(const float4 *)&xs[sb][k][wc][row16][0];
            const float4 xb = *(const float4 *)&xs[sb][k][wc][row16][4];
            const float old[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
                R[kk] = fmaxf(fmaxf(rm[0][kk], rm[1][kk]), dpp_prev16_or(rm[1][kk], old[kk]));
        }
        // level 2 from level-1 row u - 1 first (its edge values came with this barrier): l1p is
        // then free for row u
        if constexpr (L2F) {
            if (u > 0) level2_row(u - 1, l1p);
        }
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) {
            const int cl = 2 * cs + hs;
            const float4 kap = cst[sb][cl][0], kmn = cst[sb][cl][3], kden = cst[sb][cl][4], kinv = cst[sb][cl][5];
            float r4[4];
            const dm_f2 ra = dm_f2{R[4 * cs], R[4 * cs + 1]} * dm_f2{kap.x, kap.y};
            const dm_f2 rb = dm_f2{R[4 * cs + 2], R[4 * cs + 3]} * dm_f2{kap.z, kap.w};
            r4[0] = ra.x; r4[1] = ra.y; r4[2] = rb.x; r4[3] = rb.y;
            if constexpr (!CL) {
                const float4 klo = cst[sb][cl][1], khi = cst[sb][cl][2];
                r4[0] = __builtin_amdgcn_fmed3f(ra.x, klo.x, khi.x); r4[1] = __builtin_amdgcn_fmed3f(ra.y, klo.y, khi.y);
                r4[2] = __builtin_amdgcn_fmed3f(rb.x, klo.z, khi.z); r4[3] = __builtin_amdgcn_fmed3f(rb.y, klo.w, khi.w);
            }
            const dm_f2 a01 = dm_f2{r4[0], r4[1]} - dm_f2{kmn.x, kmn.y}, a23 = dm_f2{r4[2], r4[3]} - dm_f2{kmn.z, kmn.w};
            const dm_f2 i01 = {kinv.x, kinv.y}, i23 = {kinv.z, kinv.w};
            const dm_f2 q01 = a01 * i01, q23 = a23 * i23;
            const dm_f2 e01 = __builtin_elementwise_fma(-q01, dm_f2{kden.x, kden.y}, a01);
            const dm_f2 e23 = __builtin_elementwise_fma(-q23, dm_f2{kden.z, kden.w}, a23);
            dm_f2 x01, x23;
            if constexpr (CL) {
                x01 = pk_fma_clamp01(e01, i01, q01);
                x23 = pk_fma_clamp01(e23, i23, q23);
            } else {
                x01 = __builtin_elementwise_fma(e01, i01, q01);
                x23 = __builtin_elementwise_fma(e23, i23, q23);
            }
            const float x[4] = {x01.x, x01.y, x23.x, x23.y};
            double sum = 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) { // ul, ur, ll, lr: left-to-right sum
                const double pv = pow14_zf(x[r], plds, mant);
                sum = r == 0 ? pv : sum + pv;
            }
            l1p[cs] = sum;
            if (L1) {
                const bool cflat = CL && cell_flat(kden);
                // (the address formed here: no 64-bit pointer held through the loop)
                L1[((size_t)t * P1 + (size_t)(I0 + cs) * w1 + J0 + hs) * P1 + (size_t)u * w1 + 32 * wc + c32] =
                    cflat ? (double)NAN : pow14_q4(sum, plds);
            }
        }
    };

    if constexpr (RICH) {
        for (int u = 0; u < h2; u += 2) { // h2 even: the carried rows alternate registers, no copies
            pair(f2, u);
            pair(f2, u + 1);
        }
    } else {
        for (int u = 0; u < h2; ++u) pair(f2, u);
    }
    if constexpr (L2F) {
        const int u = h2 - 1;
        if (NWc > 1 && c32 == 31) {
            xch2[sb][u & 1][wc + 1][hs][0] = l1p[0];
            xch2[sb][u & 1][wc + 1][hs][1] = l1p[1];
        }
        if constexpr (NWc > 1) __syncthreads();
        level2_row(u, l1p);
    }
}
