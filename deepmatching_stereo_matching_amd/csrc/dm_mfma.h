// dm_mfma.h -- MFMA path (gfx950 v_mfma_i32_16x16x64_i8) of the fused level-0 -> level-1
// kernel.  Included by dm_kernels.hip after Geo/Stats/r_of_y/norm_mk/pow14_fast_any.
//
// Reference semantics (misc/Correlation_map.py:69-159, misc/Feature_value.py:32-43): level 1
// cell (I,J), position (u,v) = pow14( (R_ul + R_ur + R_ll + R_lr) / 4 ), R_c = MaxPool(3,2,1)
// of the rectified min-max level-0 map of child patch c of the cell.
//
// GEMM view: num(p, q) = n * sum_k T'_k(p) I'_k(q) - sT(p) sI(q), k over the ws*ws taps (K
// zero padded to 64 per MFMA, KS = ceil(ws^2/64) MFMAs per tile).
// Sweep 1 computes y = f32(num) * b_q for every (p, q) and the per-patch min/max; sweep 2
// recomputes y, pools on y (monotone, see dm_kernels.hip header), normalises and rectifies
// only the pooled values, sums the children, rectifies, and stores level 1.
// (A 32x32x32 variant, 8 cells per wave, ran at 1 wave/SIMD: 41 ms vs 25 ms per C3 pair.)
#pragma once

typedef int dm_v4i __attribute__((ext_vector_type(4)));
typedef int dm_v2i __attribute__((ext_vector_type(2)));

// ===================================================================================
// 16x16x64 variant (default).  v_mfma_i32_16x16x64_i8: lane L holds A[row L&15][k = 64ks +
// 16(L>>4) + j] and B[k][col L&15]; acc[reg] = C[row 4(L>>4) + reg][col L&15].
// Rows: 16 patches = 4 level-1 cells (2x2 block = one level-2 cell) x 4 children, so lane
// group L>>4 holds ONE cell and acc[reg] is child reg (ul, ur, ll, lr).  Columns: 16
// windows of one image row, lane c = L&15 <-> q1 = G*c + tau, G = w0/16 tiles per row.
// 4 accumulators per lane instead of 16 keep the per-lane pooling state small enough for
// several waves per SIMD.
// ===================================================================================

// Bw16[t][q0][tau][ks][lane] (16 B): lane L = c + 16 hq holds taps k = 64 ks + 16 hq + j of
// window (q0, G*c + tau) -- or, spread layout (KS == 1, n <= 32), taps 8 hq + j (j < 8) in
// bytes 0..7 and the window's {qx, qy} in words 2, 3 (build_a places A's taps the same way);
// QS16[t][q0][tau][c] = { bits(f32(-sum(I'))), bits(b_q) }.
// Column groups: tile tau = w*GW + tw belongs to column group w (16*GW consecutive columns);
// lane c of that tile is window q1 = 16*GW*w + GW*c + tw.  GW = G/NW: one group per wave of
// k_level1_mfq; GW = 16 B of output per lane for k_volume_ls.
// WSC: window side known at compile time (0 = g.ws): the window's bytes are loaded once and
// serve both the sums and the fragments.
template <int WSC>
__global__ void k_prep_windows16(Geo g, int G, int GW, int KS, dm_v4i *Bw, int2 *QS)
{
    DM_TAIL_ENTRY();
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t total = (size_t)g.T * g.h0 * G * 16;
    if (idx >= total) return;
    const int c = (int)(idx % 16);
    const int tau = (int)((idx / 16) % G);
    const int q0 = (int)((idx / (16 * (size_t)G)) % g.h0);
    const int t = (int)(idx / (16 * (size_t)G * g.h0));
    const int q1 = 16 * GW * (tau / GW) + GW * c + (tau % GW);
    const int ws = WSC ? WSC : g.ws, n = ws * ws;
    const uint8_t *base = g.img2 + (size_t)(g.org[2 * t] + q0) * g.pitch2 + g.org[2 * t + 1] + q1;
    int pix[WSC ? WSC * WSC : 1];
    if constexpr (WSC != 0) {
#pragma unroll
        for (int k = 0; k < WSC * WSC; ++k) pix[k] = (int)base[(size_t)(k / WSC) * g.pitch2 + (k % WSC)] - 128;
    }
    // tap k of the window, k < n
    auto px = [&](int k) -> int {
        if constexpr (WSC != 0) return pix[k];
        else return (int)base[(size_t)(k / ws) * g.pitch2 + (k % ws)] - 128;
    };
    int s = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        const int b = px(k);
        s += b; s2 += b * b;
    }
    const long long dI = (long long)n * s2 - (long long)s * s;
    float bq;
    if (g.method == DM_TM_CCOEFF) bq = 1.0f;
    else bq = dI == 0 ? 0.0f : (float)(1.0 / sqrt((double)dI));
    const int qx = __float_as_int((float)-s), qy = __float_as_int(bq); // exact: |s| <= 225*128
    QS[idx] = make_int2(qx, qy);
    const size_t tile = idx / 16; // (t, q0, tau)
    // spread layout (KS == 1, n <= 32; build_a uses the same): lane c + 16 hq holds taps
    // 8 hq .. 8 hq + 7 in bytes 0..7 and the window's stats {qx, qy} in words 2, 3, which meet
    // A's zero bytes 8..15 -- every lane reads its own window's stats from its own fragment
    // (qs_of_frag), no cross-lane move
    const bool spread = KS == 1 && n <= 32;
    for (int ks = 0; ks < KS; ++ks)
        for (int hq = 0; hq < 4; ++hq) {
            int w[4] = {0, 0, 0, 0};
            if (spread) {
                for (int j = 0; j < 8; ++j) {
                    const int k = 8 * hq + j;
                    const int val = k < n ? px(k) : 0;
                    w[j >> 2] |= (val & 0xFF) << (8 * (j & 3));
                }
                w[2] = qx;
                w[3] = qy;
            } else {
                for (int j = 0; j < 16; ++j) {
                    const int k = 64 * ks + 16 * hq + j;
                    const int val = k < n ? px(k) : 0;
                    w[j >> 2] |= (val & 0xFF) << (8 * (j & 3));
                }
            }
            dm_v4i o;
            o.x = w[0]; o.y = w[1]; o.z = w[2]; o.w = w[3];
            Bw[(tile * KS + ks) * 64 + c + 16 * hq] = o;
        }
}

// ===================================================================================
// Row-pair strips for v_mfma_i32_32x32x32_i8 (sweep 1 of k_level1_mfq, ws <= 5).
// The window of (q0, q1) and the one below it, (q0 + 1, q1), lie in one strip of ws + 1 image
// rows x ws columns, (ws + 1) ws <= 30 taps: strip tap k = ws * row + col (k < 32; the rest
// zero).  A 32 x 32 i8 MFMA with K = the 32 strip taps then gives 16 patches x 2 window rows
// x 32 window columns in one instruction: A row i < 16 holds patch i's taps at strip rows
// 0 .. ws - 1, row 16 + i the same taps one strip row down, so C[i][j] is patch i against
// window (q0, q1_j) and C[16 + i][j] against (q0 + 1, q1_j).  Four times the products of a
// 16 x 16 x 32 tile for twice its issue cycles (tools/mfma32_probe.hip).  Operand layout of
// the gfx950 32x32x32 i8 MFMA: lane L holds row / column L & 31, bytes 16 (L >> 5) .. +15 of
// K (the same byte order for A and B, which is all a dot product needs); result register r
// of lane L is C[8 (r >> 2) + 4 (L >> 5) + (r & 3)][L & 31].
//   Bs[t][rp][tile][lane]     16 B: strip taps 16 (lane >> 5) .. +15 of window column
//                             q1 = 64 (tile / 2) + 2 (lane & 31) + (tile & 1), rows q0 = 2 rp ..
//                             q0 + ws: the two tiles of a 64-window group interleave their
//                             columns, so lane c32 holds windows 2 c32 and 2 c32 + 1 of the
//                             group (the column pooling of k_level12_strip stays in the lane)
//   Ss[t][rp][q1]             {qx, qy} of window (q0, q1), then of (q0 + 1, q1) -- the same
//                             bits as QS16's (k_prep_windows16)
// ===================================================================================
typedef int dm_v16i __attribute__((ext_vector_type(16)));
typedef float dm_f2 __attribute__((ext_vector_type(2)));

// {bits(f32(-sum I')), bits(b_q)} of a window from its taps (k_prep_windows16's arithmetic)
__device__ __forceinline__ int2 window_qs(int s, int s2, int n, int method)
{
    const long long dI = (long long)n * s2 - (long long)s * s;
    float bq;
    if (method == DM_TM_CCOEFF) bq = 1.0f;
    else bq = dI == 0 ? 0.0f : (float)(1.0 / sqrt((double)dI));
    return make_int2(__float_as_int((float)-s), __float_as_int(bq));
}

// buffer resource over a tile's image crop (origin of tile t, wave-uniform t): scalar, so the
// byte loads through it need no per-lane resource (no waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const uint8_t *img, int pitch, const Geo &g, int t)
{
    const int ro = __builtin_amdgcn_readfirstlane(g.org[2 * t]), co = __builtin_amdgcn_readfirstlane(g.org[2 * t + 1]);
    return __builtin_amdgcn_make_buffer_rsrc((void *)(img + (size_t)ro * pitch + co), 0, 0x7fffffff, 0x00020000);
}

// WSC: ws known at compile time (5), 0 = g.ws (<= 5)
template <int WSC>
__global__ void k_prep_strips(Geo g, dm_v4i *Bs, dm_v4i *Ss)
{
    DM_TAIL_ENTRY();
    const int ws = WSC ? WSC : g.ws, NS = (ws + 1) * ws;
    const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const int h2 = g.h0 / 2, w0 = g.w0;
    if (idx >= (size_t)g.T * h2 * w0) return;
    const int q1 = (int)(idx % w0);
    const int rp = (int)((idx / w0) % h2);
    const int t = (int)(idx / ((size_t)w0 * h2));
    const uint8_t *base = g.img2 + (size_t)(g.org[2 * t] + 2 * rp) * g.pitch2 + g.org[2 * t + 1] + q1;
    int pix[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) pix[k] = k < NS ? (int)base[(size_t)(k / ws) * g.pitch2 + (k % ws)] - 128 : 0;
    int2 qs[2];
#pragma unroll
    for (int o = 0; o < 2; ++o) {
        int s = 0, s2 = 0;
#pragma unroll
        for (int k = 0; k < 30; ++k) {
            if (k >= ws * ws) break;
            const int v = pix[o * ws + k];
            s += v; s2 += v * v;
        }
        qs[o] = window_qs(s, s2, ws * ws, g.method);
    }
    Ss[idx] = dm_v4i{qs[0].x, qs[0].y, qs[1].x, qs[1].y};
    // window q1 = 64 gq + 2 cc + j -> strip tile 2 gq + j, column cc (w0 % 64 == 0)
    const size_t tile = (idx / w0) * (w0 / 32) + 2 * (q1 / 64) + (q1 & 1);
    const int cc = (q1 % 64) >> 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        int w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j >> 2] |= (pix[16 * h + j] & 0xFF) << (8 * (j & 3));
        Bs[tile * 64 + cc + 32 * h] = dm_v4i{w[0], w[1], w[2], w[3]};
    }
}

// XCD-aware workgroup order (DM_XCD_MAP): workgroups are dealt round robin over the 8 XCDs
// (MI355X_MICROARCH.md, workgroup dispatch), so consecutive workgroups -- the cell blocks of one
// tile, which read the same window operands -- land on 8 different L2s.  With the grid a
// multiple of 8, workgroup b is given logical index (b % 8) * (grid / 8) + b / 8: each XCD then
// walks one contiguous range of blocks, i.e. whole tiles in order, and the tile's window
// operands stay in that XCD's L2 (placement only: any order is correct).
#ifndef DM_LATE
#define DM_LATE 1   // k_level1_mfq (L2F): the next even row's fragments loaded after the emission
#endif
#ifndef DM_XCD_MAP
#define DM_XCD_MAP 1
#endif
#ifndef DM_ABL_PAPPROX
#define DM_ABL_PAPPROX 0   // ablation builds only (tools/abl_build.sh papprox, papprox2)
#endif
// In-kernel clock of the level kernels (diagnostic builds only: tools/abl_build.sh clk,
// MI355X_MICROARCH.md 'DVFS give-back' item 6): wave 0 of every workgroup reads the shader
// clock counter and the 100 MHz real-time counter when the workgroup starts and when it
// ends, and writes the four values (vector stores) to dm_clock_stamps, which no other code
// reads; dm_diag_clock_stamps copies them out.  Clock = d(shader) / d(real) x 100 MHz.
#ifndef DM_CLOCK_STAMP
#define DM_CLOCK_STAMP 0
#endif
#if DM_CLOCK_STAMP
__device__ unsigned long long dm_clock_stamps[4 * 65536];
struct ClockStamp {
    long long t0, r0;
    __device__ ClockStamp() : t0(__builtin_amdgcn_s_memtime()), r0(__builtin_amdgcn_s_memrealtime()) {}
    __device__ ~ClockStamp()
    {
        const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            unsigned long long *p = dm_clock_stamps + 4 * (blockIdx.x & 65535u);
            p[0] = (unsigned long long)t0; p[1] = (unsigned long long)t1;
            p[2] = (unsigned long long)r0; p[3] = (unsigned long long)r1;
        }
    }
};
#define DM_CLOCK_STAMP_HERE ClockStamp dm_clock_stamp_;
#else
#define DM_CLOCK_STAMP_HERE
#endif
__device__ __forceinline__ int wg_logical()
{
    const int b = blockIdx.x, n = gridDim.x;
    if (!DM_XCD_MAP || (n & 7)) return b;
    return (b & 7) * (n >> 3) + (b >> 3);
}

// The workgroup's patch taps in LDS (S1 instances): ptab[sb][patch][0..7] = the 16 patches' taps
// 0 .. 31 as int8 (zero from n on), [8..15] the same shifted by ws bytes (ws zero bytes, then
// the taps): exactly the K bytes of the strip MFMA's A rows (offset 0 and 1), and the first copy
// holds build_a's spread fragments (taps 8 grp .. 8 grp + 7).  One pass of the workgroup's
// threads (a dword each: 4 byte loads through the tile's buffer resource) replaces every lane's
// own 16 + 8 byte loads and address arithmetic.
template <int NB, int NT, int WSC>
__device__ __forceinline__ void fill_ptab(unsigned (&ptab)[NB][16][16], const Geo &g, int tid, int bpt, int nbj)
{
    const int ws = WSC ? WSC : g.ws, n = ws * ws;
    const int blk0 = wg_logical() * NB;
    const int t = blk0 / bpt; // bpt % NB == 0: every block of the workgroup is in tile t
    const __amdgpu_buffer_rsrc_t rI = tile_rsrc(g.img1, g.pitch1, g, t);
#pragma unroll
    for (int e0 = 0; e0 < NB * 256; e0 += NT) {
        const int e = e0 + tid;
        if (NB * 256 % NT != 0 && e >= NB * 256) break;
        const int sb = e >> 8, pi = (e >> 4) & 15, d = e & 15;
        const int blk = blk0 + sb;
        const int I0 = 2 * ((blk % bpt) / nbj), J0 = 2 * ((blk % bpt) % nbj);
        const int cl = pi >> 2, ch = pi & 3;
        const int p0 = 2 * (I0 + (cl >> 1)) + (ch >> 1), p1 = 2 * (J0 + (cl & 1)) + (ch & 1);
        const unsigned pb = (unsigned)(p0 * g.pitch1 + p1);
        const int o = d >> 3, k0 = 4 * (d & 7);
        unsigned w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int tau = k0 + b - ws * o;
            const bool in = tau >= 0 && tau < n;
            const int tc = tau < 0 ? 0 : (tau >= n ? n - 1 : tau);
            const int v = (int)__builtin_amdgcn_raw_buffer_load_b8(rI, pb + (unsigned)((tc / ws) * g.pitch1 + tc % ws), 0, 0) - 128;
            w |= (unsigned)((in ? v : 0) & 0xFF) << (8 * b);
        }
        ptab[sb][pi][d] = w;
    }
}

// min of mn[k] / max of mx[k] over the 32 lanes of each half-wave by DPP: row rotations 8, 4, 2,
// 1 leave every lane of a 16-lane row with the row's extreme, then row_bcast:15 folds row 0 into
// row 1 and row 2 into row 3 -- lanes 31 and 63 hold the two halves' results.  Each step is one
// VOP2-DPP instruction (v = op(dpp(v), v), vdst tied to v: rows the row_mask excludes keep it),
// issued for all 2N values before the next step, so no instruction reads a VGPR the one just
// before it wrote (the DPP read-after-VALU-write hazard needs 2 wait states); the values are
// never NaN.  (Five DPP instructions per value instead of five ds_bpermute shuffles.)
// N >= 2 keeps a value's DPP read >= 3 instructions after its write inside the sequence.  The
// compiler cannot see DPP inside asm, so tests/test_profiles.py checks the built ISA: no VALU
// write of a VGPR within the 2 wait states before a DPP read of it, in every kernel of the
// library (__builtin_amdgcn_update_dpp + fminf is not folded into v_min_f32_dpp --
// fminf's canonicalising v_max x, x sits between -- and costs 256 VALU instructions per wave,
// and one asm block over all 16 values changes the register allocation into a spill).
template <int N>
__device__ __forceinline__ void half_wave_minmax(float (&mn)[N], float (&mx)[N])
{
    static_assert(N >= 2, "a value's next DPP read must come >= 2 wait states after its write");
#define DM_HWR(ctl, rm)                                                                                   \
    _Pragma("unroll") for (int k = 0; k < N; ++k) {                                                       \
        asm volatile("v_min_f32_dpp %0, %0, %0 " ctl " row_mask:" rm " bank_mask:0xf" : "+v"(mn[k]));      \
        asm volatile("v_max_f32_dpp %0, %0, %0 " ctl " row_mask:" rm " bank_mask:0xf" : "+v"(mx[k]));      \
    }
    asm volatile("s_nop 1" ::: "memory"); // the values' last VALU writes may be just before
    DM_HWR("row_ror:8", "0xf")
    DM_HWR("row_ror:4", "0xf")
    DM_HWR("row_ror:2", "0xf")
    DM_HWR("row_ror:1", "0xf")
    DM_HWR("row_bcast:15", "0xa")
#undef DM_HWR
}

// {q.y, q.y} * v as one v_pk_mul_f32 (op_sel broadcast of the high half: the compiler would
// copy q.y into an even register first)
__device__ __forceinline__ dm_f2 pk_mul_bhi(dm_f2 q, dm_f2 v)
{
    dm_f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(q), "v"(v));
    return r;
}

// Window stats of this lane's window from its own B fragment (spread layout: KS == 1,
// n <= 32, i8): words 2, 3 = {qx, qy}, qx = f32 bits of -sum(I'), qy = b_q of window c --
// an aligned register pair whose halves the packed y arithmetic broadcasts with op_sel.
// (Round 2 first carried them in lanes 32..63 only and moved them with two
// v_permlane32_swap per tile: 8 issue cycles each on gfx950, tools/valu_probe.hip.)
__device__ __forceinline__ dm_f2 qs_of_frag(const dm_v4i &b)
{
    return dm_f2{__int_as_float(b.z), __int_as_float(b.w)};
}
__device__ __forceinline__ dm_f2 qs_pair(int2 q) { return dm_f2{__int_as_float(q.x), __int_as_float(q.y)}; }
// (measured: the same through ds_bpermute -- LDS instead of VALU issue -- ran 4 % slower in
// the fused level kernel, whose pow tables keep the LDS busy; a separate 8-B stats load 2 %)

template <int KS>
__device__ __forceinline__ void load_frag(dm_v4i *f, const dm_v4i *__restrict__ Bt, int lane)
{
    // unsigned lane offset: uniform base + zero-extended 32-bit offset -> saddr loads, no
    // per-load 64-bit VALU address add
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) f[ks] = Bt[(unsigned)(ks * 64) + (unsigned)lane];
}

template <int KS>
__device__ __forceinline__ dm_v4i mfma16_frag(const dm_v4i *A, const dm_v4i *Bf)
{
    dm_v4i acc = {};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[ks], Bf[ks], acc, 0, 0, 0);
    return acc;
}

template <int KS>
__device__ __forceinline__ dm_v4i mfma16_tile(const dm_v4i *A, const dm_v4i *__restrict__ Bt, int lane)
{
    dm_v4i acc = {};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[ks], Bt[ks * 64 + lane], acc, 0, 0, 0);
    return acc;
}

// y = f32(num) * b_q for the 4 patches (acc[r]) of one lane against its window (qs).
// YF (n <= 25): acc was accumulated onto DM_YBIAS, so its bits read as the float
// A = 1.5*2^23 + acc (exact for |acc| <= 128^2 n < 2^22).  Three packed-f32 steps, each
// exact or rounding an exact integer once:
//   m   = fma(A, n, -n*1.5*2^23)  = n*acc        exact: |n acc| <= 128^2 n^2 < 2^24, and
//                                                -n*1.5*2^23 = -3n*2^22 is an f32 (3n <= 75)
//   num = fma(sT, -sI, m)         = n*acc - sT*sI, exact: |num| <= sqrt(dT dI) <= n^2 255^2/4
//                                                < 2^24 (Cauchy-Schwarz)
//   y   = num * b_q               the one rounding of the reference's f32(num) * b_q
// (sTf = f32(sum T'), qs.x = f32 bits of -sum(I')) -- the integer path's f32(num) in 1.5
// packed instructions per voxel instead of 2.
#define DM_YBIAS 0x4B400000

template <bool YF>
__device__ __forceinline__ void y_of_acc(const dm_v4i &acc, const int *sTr, const float *sTf, dm_f2 q2, int n,
                                         float *y)
{
    if constexpr (YF) {
        const float nf = (float)n;
        const float nb = -nf * 12582912.0f;   // exact (see above)
        const dm_f2 sI2 = __builtin_shufflevector(q2, q2, 0, 0);
        const dm_f2 a01 = dm_f2{__int_as_float(acc[0]), __int_as_float(acc[1])};
        const dm_f2 a23 = dm_f2{__int_as_float(acc[2]), __int_as_float(acc[3])};
        const dm_f2 m01 = __builtin_elementwise_fma(a01, dm_f2{nf, nf}, dm_f2{nb, nb});
        const dm_f2 m23 = __builtin_elementwise_fma(a23, dm_f2{nf, nf}, dm_f2{nb, nb});
        const dm_f2 n01 = __builtin_elementwise_fma(dm_f2{sTf[0], sTf[1]}, sI2, m01);
        const dm_f2 n23 = __builtin_elementwise_fma(dm_f2{sTf[2], sTf[3]}, sI2, m23);
        // b_q broadcast from the pair's high half by op_sel (no copy into an even register)
        const dm_f2 y01 = pk_mul_bhi(q2, n01), y23 = pk_mul_bhi(q2, n23);
        y[0] = y01.x; y[1] = y01.y; y[2] = y23.x; y[3] = y23.y;
    } else {
        const float b = q2.y;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            y[r] = __fmul_rn((float)(__mul24(acc[r], n) + __mul24(sTr[r], (int)q2.x)), b);
    }
}

// A operand of one lane: patch rows of a 2x2 cell block (row c: cell cl = c/4, child ch = c%4),
// int8 taps 64ks + 16grp + j (spread layout, KS == 1 and n <= 32: taps 8grp + j)
// (WSC: ws known at compile time, 0 = g.ws; spread layout: branch-free byte loads from clamped
// in-patch addresses, so they issue together)
template <int KS, int WSC = 0>
__device__ __forceinline__ void build_a(dm_v4i *A, const Geo &g, int t, int I0, int J0, int c, int grp)
{
    const int ws = WSC ? WSC : g.ws, n = ws * ws;
    const int cl = c >> 2, ch = c & 3;
    const int p0 = 2 * (I0 + (cl >> 1)) + (ch >> 1), p1 = 2 * (J0 + (cl & 1)) + (ch & 1);
    const uint8_t *base = g.img1 + (size_t)(g.org[2 * t] + p0) * g.pitch1 + g.org[2 * t + 1] + p1;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        int w[4] = {0, 0, 0, 0};
        if (KS == 1 && n <= 32) { // spread layout (k_prep_windows16): taps 8 grp + j
            const __amdgpu_buffer_rsrc_t rI = tile_rsrc(g.img1, g.pitch1, g, t);
            const unsigned pb = (unsigned)(p0 * g.pitch1 + p1);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 8 * grp + j, kc = k < n ? k : n - 1;
                const int v = (int)__builtin_amdgcn_raw_buffer_load_b8(rI, pb + (unsigned)((kc / ws) * g.pitch1 + (kc % ws)), 0, 0) - 128;
                w[j >> 2] |= ((k < n ? v : 0) & 0xFF) << (8 * (j & 3));
            }
        } else {
            for (int j = 0; j < 16; ++j) {
                const int k = 64 * ks + 16 * grp + j;
                int val = 0;
                if (k < n) val = (int)base[(size_t)(k / g.ws) * g.pitch1 + (k % g.ws)] - 128;
                w[j >> 2] |= (val & 0xFF) << (8 * (j & 3));
            }
        }
        A[ks].x = w[0]; A[ks].y = w[1]; A[ks].z = w[2]; A[ks].w = w[3];
    }
}

template <int KS>
__device__ __forceinline__ dm_v4i mfma16_frag_c(const dm_v4i *A, const dm_v4i *Bf, dm_v4i acc)
{
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[ks], Bf[ks], acc, 0, 0, 0);
    return acc;
}

// lane c-1 of the same 16-lane row (DPP row_shr:1, a VALU op; lane c == 0 gets 0)
__device__ __forceinline__ float dpp_prev16(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false));
}

// same, lane c == 0 gets `old`
__device__ __forceinline__ float dpp_prev16_or(float v, float old)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x111, 0xf, 0xf, false));
}

// one 16x16 tile: i8 MFMA onto acc0 (YF bias), returned as raw bits.
// K32 (spread layout: KS == 1, n <= 32): the taps sit in bytes 0..7 of every lane, 8 per
// lane group -- exactly v_mfma_i32_16x16x32_i8's operand layout (k = 8 (lane >> 4) + j) -- so
// the K = 32 instruction on the low 8 bytes gives the same exact sums as the K = 64 one (whose
// bytes 8..15 are A's zeros against the window stats).  On gfx950 an MFMA keeps its SIMD
// from issuing VALU while it runs (profiles/r03_valu_probe.txt), and the K = 32 form runs
// half as long.
template <int KS, bool K32 = false>
__device__ __forceinline__ dm_v4i mfma_tile(const dm_v4i *A, const dm_v4i *Bf, dm_v4i acc0)
{
    if constexpr (K32) {
        static_assert(KS == 1, "K = 32 form: one spread-layout fragment");
        const long a = (long)(((unsigned long)(unsigned)A[0].y << 32) | (unsigned)A[0].x);
        const long b = (long)(((unsigned long)(unsigned)Bf[0].y << 32) | (unsigned)Bf[0].x);
        return __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, acc0, 0, 0, 0);
    } else {
        return mfma16_frag_c<KS>(A, Bf, acc0);
    }
}

// ===================================================================================
// Column-split variant (default).  One workgroup = NW waves = ONE 2x2 block of level-1
// cells (16 patches, the same A operand in every wave); wave w sweeps only column group w
// (16*GW window columns), so a lane pools GW/2 output columns instead of G/2 and the
// per-lane state shrinks enough for more waves per SIMD.  Crossings: the per-patch
// min/max is reduced over the waves through LDS once; MaxPool's left neighbour of column
// group w (q1 = 16*GW*w - 1) comes from wave w-1 through LDS once per image row.
// ===================================================================================
// MaxPool of one level-1 CELL's map: a plain IEEE max (v_max_f64) is torch's NaN-propagating
// MaxPool here, because a cell's level-1 map is all-NaN or NaN-free.  x = (r - rmin) / den is
// NaN only for den == 0 (a constant child map: a = 0 and rinv = inf, for EVERY window), and
// every level-1 value of the cell sums all four children, so one such child makes every value
// of the cell NaN and otherwise none is (y, r, x, pow14 are finite).  Every operand of these
// maxima belongs to one cell (the lane group; the edge value of wave w-1 is the same cell), so
// they are all NaN (max = NaN) or all finite.  Out-of-range neighbours (padding) are replaced by
// the value itself instead of -inf, which keeps a NaN cell NaN.  (A NaN-aware max -- two
// float64 compares and two selects, 16 issue cycles -- becomes one 4-cycle instruction.)
// (inline asm: llvm.maxnum would add a canonicalising v_max_f64 x, x per operand)
__device__ __forceinline__ double cellmax_d(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// 16 B per lane global -> LDS (buffer_load_dwordx4 ... lds): LDS byte address m0 + 16 * lane;
// m0 is saved and restored around it (the compiler owns m0)
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, unsigned lds_byte, unsigned voff, unsigned soff)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_byte), "v"(voff), "s"(r), "s"(soff) : "memory");
}

// Normalisation with the clamp bit (k_level1_mfq<..., CL = true>, the fused level-1/level-2
// path): x = (med3(R a_p, lo, hi) - rmin) / den becomes clamp01((R a_p - rmin) / den), the
// quotient by norm_mk's Markstein steps (= RN(a / den), monotone in a), bit for bit:
//  - r inside [lo, hi]: same operands; x in [0, 1] already (rmin <= r <= rmax, a <= den), so the
//    clamp changes nothing.  CCOEFF (lo, hi = -inf, inf) is always this case.
//  - R a_p > 1: r = 1 = rmax (max_q y >= R), so a = RN(rmax - rmin) = den and x = 1 exactly;
//    unclamped a' >= den gives x' >= 1, clamped to 1.
//  - R a_p < -1: r = -1 = rmin, a = +0, x = +0; unclamped a' < 0 gives x' < 0, clamped to +0.
//  - den == 0 (a constant child map; also every a_p == 0 patch, where r == 1 throughout): the
//    reference's values are NaN (0/0), but the hardware clamp maps NaN to 0 (dx10_clamp).  Every
//    level-1 value of such a cell is NaN and every level-2 value of its block is NaN (each sums
//    all four cells), so the kernel writes NaN there itself: level 2 when any of the block's 16
//    patches is flat (block_has_flat), a stored level 1 when one of the cell's 4 is (cell_flat).
// Saves the four v_med3_f32 (4 issue cycles each) per four pooled values.
__device__ __forceinline__ dm_f2 pk_fma_clamp01(dm_f2 a, dm_f2 b, dm_f2 c)
{
    dm_f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ bool cell_flat(float4 den)
{
    return den.x == 0.0f || den.y == 0.0f || den.z == 0.0f || den.w == 0.0f;
}
__device__ __forceinline__ bool block_has_flat(const float4 (&cst)[4][6])
{
    return cell_flat(cst[0][4]) || cell_flat(cst[1][4]) || cell_flat(cst[2][4]) || cell_flat(cst[3][4]);
}

// storage of k_level1_mfq's exchange arrays: its own LDS, or (H) the pow tables' g32 hole at
// byte offset OFF
template <bool H, typename T, int OFF = 0>
struct XchOwn {
    __attribute__((aligned(16))) T v;
    __device__ T &get(PowLds &) { return v; }
};
template <typename T, int OFF>
struct XchOwn<true, T, OFF> {
    __device__ T &get(PowLds &p) { return *reinterpret_cast<T *>((char *)&p.g32[128] + OFF); }
};

// L1 may be null when L2F (level 1 then lives only on chip); L2 is written when L2F.
// NB 2x2-cell blocks per workgroup (NB = 2 where one wave spans a whole tile row, S = 64):
// waves sb * NWc .. sb * NWc + NWc - 1 split block sb's columns; the blocks share the pow
// tables, which is what a workgroup of more than one wave buys there.
// S1: sweep 1 on the row-pair strips (Bs, Ss: k_prep_strips) with the 32 x 32 x 32 i8 MFMA --
// half the matrix-core issue cycles of the 16 x 16 tiles per voxel (A rows from the LDS tap table,
// fill_ptab), and the window stats
// broadcast without copies; sweep 2 keeps the 16 x 16 layout its pooling needs.
template <int KS, int GW, int NW, int MINW, bool L2F, bool YF, int NB = 1, bool CL = false, bool S1 = false>
__global__ __launch_bounds__(64 * NW, MINW) void k_level1_mfq(Geo g, Stats s, const dm_v4i *__restrict__ Bw,
                                                        const int2 *__restrict__ QS, double *L1, double *L2,
                                                        const dm_v4i *__restrict__ Bs = nullptr,
                                                        const dm_v4i *__restrict__ Ss = nullptr)
{
    DM_CLOCK_STAMP_HERE
    constexpr bool EQ = KS == 1 && YF;           // window stats ride in the B tile (qs_of_frag)
    static_assert(NW % NB == 0, "blocks split the waves evenly");
    static_assert(!CL || L2F, "clamp-bit normalisation: NaN cells are restored at the level-2 / level-1 stores");
    constexpr int NWc = NW / NB;                 // waves per cell block
    constexpr int XS = NWc > 1 ? NWc + 1 : 1;    // exchange slots (unused with one wave per block)
    constexpr int XW = NWc > 1 ? NWc : 1;
    __shared__ PowLds plds;
    // exchange arrays; they live in the pow tables' unused g32 rows when they fit (PowLds),
    // which keeps the C3 instance (2 waves per workgroup) at <= 20 KB of LDS: 8 workgroups,
    // 4 waves per SIMD
    struct Xch {
        // [block][pair parity][row][slot][cell group][child]: slot w+1 = y of wave w at
        // q1 = 16*GW*(w+1)-1, slot 0 = -inf (no window left of column 0)
        float xch[NB][2][2][XS][4][4];
        double stash[L2F ? NW : 1][64];  // [wave][row slot * L2V + column]: level-2 pow inputs
        double xch2[NB][2][XW][4];       // [block][level-1 row parity][wave][cell]: level 1 at v = 8*GW*(w+1)-1
    };
    struct Red {
        float red[NB][2][NWc][16];       // per-wave partial min / max per patch row
    };
    constexpr bool HOLE = sizeof(Xch) <= G32_HOLE;
    constexpr bool HOLE_R = HOLE && sizeof(Xch) + sizeof(Red) <= G32_HOLE;
    __shared__ XchOwn<HOLE, Xch> xown;
    __shared__ XchOwn<HOLE_R, Red, (int)sizeof(Xch)> rown;
    Xch &X = xown.get(plds);
    auto &xch = X.xch;
    auto &stash = X.stash;
    auto &xch2 = X.xch2;
    auto &red = rown.get(plds).red;
    __shared__ float4 cst[NB][4][6];   // [block][cell][field][child]: a_p, lo, hi, rmin, den, rinv
    // LATE: the next even row's fragments are loaded after the level-1 emission instead of
    // before it (12 fewer live VGPRs through the emission, less latency cover)
    constexpr bool LATE = L2F && DM_LATE;
    constexpr int L2V = 4 * GW, L2B = 64 / L2V; // level-2 values per wave per row; rows per stash
    // M == 1 (one pooled column per lane, valid on even lanes): the pooled children of RB
    // level-2 rows, [wave][row * 4 * L2V + child * L2V + column], rectified 64 at a time
    constexpr int RB = 64 / (4 * L2V);
    __shared__ double stash2[L2F && GW == 2 ? NW : 1][L2F && GW == 2 ? 64 : 1];
    const int tid = threadIdx.x;
    pow_lds_fill(plds, tid, 64 * NW, HOLE);
    if (NWc > 1 && tid < 64 * NB)
        (&xch[tid >> 6][0][0][0][0][0])[((tid & 63) >> 4) * XS * 16 + (tid & 15)] = -INFINITY;
    __shared__ __attribute__((aligned(16))) unsigned ptab[S1 ? NB : 1][16][16];
    if constexpr (S1) {
        const int nbj_ = (g.w0 / 2) / 2, bpt_ = ((g.h0 / 2) / 2) * nbj_;
        if (g.ws == 5) fill_ptab<S1 ? NB : 1, 64 * NW, 5>(ptab, g, tid, bpt_, nbj_);
        else fill_ptab<S1 ? NB : 1, 64 * NW, 0>(ptab, g, tid, bpt_, nbj_);
    }
    __syncthreads();

    constexpr int G = GW * NWc;
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // cell block of the workgroup and wave in it (NB == 1: block 0, as the compiler cannot see
    // wave < NW)
    const int sb = NB > 1 ? wave / NWc : 0, wc = NB > 1 ? wave % NWc : wave;
    const int c = lane & 15, grp = lane >> 4;
    const int h0 = g.h0, w0 = g.w0, n = g.ws * g.ws, P = h0 * w0;
    const int w1 = w0 / 2, P1 = (h0 / 2) * w1;
    const int nbj = w1 / 2, bpt = ((h0 / 2) / 2) * nbj; // 2x2-cell blocks per tile
    const int blk = wg_logical() * NB + sb;
    const int t = blk / bpt;                             // whole workgroup in range (grid exact)
    const int I0 = 2 * ((blk % bpt) / nbj), J0 = 2 * ((blk % bpt) % nbj);
    const size_t tb = (size_t)t * P;
    const int ro = g.org[2 * t], co = g.org[2 * t + 1];

    dm_v4i A[KS];
    const int Ic = I0 + (grp >> 1), Jc = J0 + (grp & 1);
    int sTr[4];
    float sTf[4];
    // the 16 x 16 tiles' patch operand and sums (S1: built after the strip sweep, which does
    // not read them -- they would hold registers through it)
    auto init_a16 = [&]() {
        if constexpr (S1) { // the spread fragment: taps 8 grp .. 8 grp + 7 of patch row c (ptab)
            const dm_v2i tp = *(const dm_v2i *)&ptab[sb][c][2 * grp];
            A[0] = dm_v4i{tp.x, tp.y, 0, 0};
        } else {
            build_a<KS>(A, g, t, I0, J0, c, grp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = (2 * Ic + (r >> 1)) * w0 + 2 * Jc + (r & 1);
            sTr[r] = s.sT[tb + p];
            sTf[r] = (float)sTr[r];
        }
    };
    if constexpr (!S1) init_a16();
    const int ab = YF ? DM_YBIAS : 0;
    const dm_v4i acc0 = {ab, ab, ab, ab};
    const unsigned mant = mant_mask_vgpr();   // pow14_zf's mantissa mask, kept in a VGPR
    const dm_v4i *Bt = Bw + ((size_t)t * h0 * G + wc * GW) * KS * 64;
    const int2 *Qt = QS + ((size_t)t * h0 * G + wc * GW) * 16;

    // one image row of this wave's column group: GW tiles of B fragments + window stats.
    // Rows are software-pipelined in pairs: the next row's loads are in flight while the
    // current one is computed (prefetch row index clamped into range; its data is unused).
    struct RowFrag {
        dm_v4i b[GW][KS];
        int2 q[GW];
    };
    // buffer loads: wave-uniform resource + row offset in SGPRs, lane offset a constant
    // VGPR -- no per-load VALU address arithmetic
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void *)Bt, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rQ = __builtin_amdgcn_make_buffer_rsrc((void *)Qt, 0, 0x7fffffff, 0x00020000);
    const unsigned voB = (unsigned)lane * 16u, voQ = (unsigned)c * 8u;
    auto load_row = [&](RowFrag &f, int q0) {
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            const unsigned ti = (unsigned)q0 * G + tw;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                f.b[tw][ks] = __builtin_amdgcn_raw_buffer_load_b128(rB, voB, (ti * KS + ks) * 1024u, 0);
            if constexpr (!EQ) {
                const dm_v2i qv = __builtin_amdgcn_raw_buffer_load_b64(rQ, voQ, ti * 128u, 0);
                f.q[tw] = make_int2(qv.x, qv.y);
            }
        }
    };

    // ---- sweep 1: min / max of y over this wave's columns, then over the waves ----
    float mn[4], mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { mn[r] = INFINITY; mx[r] = -INFINITY; }
    auto minmax_row = [&](const RowFrag &f) {
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            const dm_v4i acc = mfma_tile<KS, EQ>(A, f.b[tw], acc0);
            float y[4];
            y_of_acc<YF>(acc, sTr, sTf, EQ ? qs_of_frag(f.b[tw][0]) : qs_pair(f.q[tw]), n, y);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                mn[r] = fminf(mn[r], y[r]);
                mx[r] = fmaxf(mx[r], y[r]);
            }
        }
    };
    RowFrag fa, fb;
    if constexpr (S1) {
        static_assert(YF && KS == 1 && GW == 4, "strip sweep: packed y, one 64-window column group per wave");
        // this wave's windows: strip tiles 2 wc, 2 wc + 1 (32 columns each) of every row pair;
        // lane (c32, hs) holds cells hs, 2 + hs of the block at window column c32, both rows
        const int c32 = lane & 31, hs = lane >> 5;
        const dm_v4i A32 = *(const dm_v4i *)&ptab[sb][lane & 15][8 * ((lane >> 4) & 1) + 4 * hs]; // row L & 31: offset (L >> 4) & 1
        float sTs[8]; // [cell slot cs][child]: cell 2 cs + hs
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
        // (lane c32 of tile j: window 64 wc + 2 c32 + j, k_prep_strips)
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
        const float nf = (float)n, nb = -nf * 12582912.0f; // y_of_acc's exact steps
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
        load_row(fa, 0); // sweep 2's first row, in flight through the reduction
        init_a16();
        half_wave_minmax(mn8, mx8);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int pl = 4 * (2 * (k >> 2) + hs) + (k & 3);  // patch row of the block: 4 cell + child
            if (c32 == 31) { red[sb][0][wc][pl] = mn8[k]; red[sb][1][wc][pl] = mx8[k]; }
        }
    } else {
    load_row(fa, 0);
    for (int q0 = 0; q0 < h0; q0 += 2) { // h0 % 4 == 0
        load_row(fb, q0 + 1);
        minmax_row(fa);
        load_row(fa, q0 + 2 < h0 ? q0 + 2 : 0); // the last prefetch is sweep 2's row 0
        minmax_row(fb);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        for (int off = 1; off < 16; off <<= 1) {
            mn[r] = fminf(mn[r], __shfl_xor(mn[r], off));
            mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], off));
        }
        if (c == 0) { red[sb][0][wc][4 * grp + r] = mn[r]; red[sb][1][wc][4 * grp + r] = mx[r]; }
    }
    }
    __syncthreads();
    // per-patch normalisation constants {a_p, rmin, rmax - rmin, RN(1/(rmax - rmin))} of the
    // 16 patches -> LDS (read back at each level-1 row instead of holding 16 VGPRs)
    // r_of_y as one med3(y * a_p, lo, hi): NORMED [-1, 1] ([1, 1] for a constant patch,
    // a_p = 0: OpenCV's 1), CCOEFF unclamped
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
        float *f = (float *)&cst[sb][grp][0];
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

    // ---- sweep 2: pool on y -> normalise + rectify -> children sum -> level 1 [-> level 2] ----
    // CL (norm_clamp): level 2 of a block with a flat patch is NaN (wave-uniform, an SGPR), as
    // is a stored level 1 of a cell with a flat child (a lane mask); both set once
    const bool bflat = CL && __builtin_amdgcn_readfirstlane((int)block_has_flat(cst[sb])) != 0;
    const bool cflat = CL && L1 && cell_flat(cst[sb][grp][4]);
    constexpr int M = GW / 2;                 // pooled columns per lane: v = 8*GW*wave + M*c + m
    constexpr int M2 = M >= 2 ? M / 2 : 1;    // level-2 columns per lane (M == 1: even lanes)
    float Cprev[M][4];
    double Racc2[M2], Cprev2[M2], l1p[M];
    double *Lrow = L1 ? L1 + ((size_t)t * P1 + (size_t)Ic * w1 + Jc) * P1 + 8 * GW * wc : nullptr;
    const int w2 = w0 / 4, P2 = (h0 / 4) * w2;
    double *L2row = L2F ? L2 + ((size_t)t * P2 + (size_t)(I0 / 2) * w2 + J0 / 2) * P2 : nullptr;

    // column MaxPool(3,2,1) of one row on y: Cm[m] over q1 = 2v, 2v+1 and (m >= 1) 2v-1;
    // the row's last tile comes back in last; the left neighbour of m = 0 (lane c-1's last
    // tile, or wave w-1's through LDS) is merged after the barrier.
    auto pool_cols = [&](const RowFrag &f, float (&Cm)[M][4], float (&last)[4]) {
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            const dm_v4i acc = mfma_tile<KS, EQ>(A, f.b[tw], acc0);
            float y[4];
            y_of_acc<YF>(acc, sTr, sTf, EQ ? qs_of_frag(f.b[tw][0]) : qs_pair(f.q[tw]), n, y);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if ((tw & 1) == 0) Cm[tw / 2][r] = tw == 0 ? y[r] : fmaxf(last[r], y[r]);
                else Cm[tw / 2][r] = fmaxf(Cm[tw / 2][r], y[r]);
                last[r] = y[r];
            }
        }
    };

    // level 2 of this workgroup's cell from level-1 row u: NaN-propagating MaxPool(3,2,1) of
    // the four level-1 maps (torch semantics, misc/Correlation_map.py:101-103), sum of the four
    // maps in ul, ur, ll, lr order (:109-122), /4, rectify; rows stream over u.  l1p holds the
    // level-1 values BEFORE their rectification (the child sums s, level 1 = pow14(s / 4)),
    // lane c == 15's of wave w-1 in xch2[u & 1]: pow14 is monotone non-decreasing (NaN in ->
    // NaN out), so MaxPool of pow14(s / 4) == pow14 of MaxPool(s) / 4 bit for bit, and only
    // the pooled value of each child is rectified -- one pow per lane per level-2 row instead
    // of one per level-1 value.
    auto level2_row = [&](int u, const double (&l1p)[M]) {
        const double lft = __shfl(l1p[M - 1], lane - 1);
        // column -1 is padding: the value itself stands in (cellmax_d)
        const double left = c != 0 ? lft : (wc == 0 ? l1p[0] : xch2[sb][u & 1][wc - 1][grp]);
        double Cq[M2];
        if constexpr (M == 1) { // L2 column 4*GW*w + c/2 on even lanes
            const double right = __shfl(l1p[0], lane + 1);
            Cq[0] = cellmax_d(cellmax_d(left, l1p[0]), right);
        } else {
#pragma unroll
            for (int j = 0; j < M2; ++j)
                Cq[j] = cellmax_d(cellmax_d(j == 0 ? left : l1p[2 * j - 1], l1p[2 * j]), l1p[2 * j + 1]);
        }
        if ((u & 1) == 0) {
#pragma unroll
            for (int j = 0; j < M2; ++j) Racc2[j] = u == 0 ? Cq[j] : cellmax_d(Cprev2[j], Cq[j]);
        } else {
            // the wave's 4*GW level-2 values of row u2 (cell sums on lanes of group 0) go to
            // the LDS stash; every L2B rows one pow per lane rectifies them all
            const int u2 = u >> 1, slot = u2 % L2B;
            if constexpr (M == 1) {
                // even lanes hold the pooled children: collect RB rows, rectify all 64 entries
                // with one pow per lane, then sum the children (ul, ur, ll, lr) per column
                const double R2 = cellmax_d(Racc2[0], Cq[0]);
                Cprev2[0] = Cq[0];
                const int rb = u2 % RB;
                if ((c & 1) == 0) stash2[wave][rb * 4 * L2V + grp * L2V + c / 2] = R2;
                if (rb == RB - 1 || u2 == h0 / 4 - 1) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    const double P = pow14_q4(stash2[wave][lane], plds); // stale entries: unused
                    __builtin_amdgcn_wave_barrier();
                    stash2[wave][lane] = P;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if (lane < (rb + 1) * L2V) {
                        const int r = lane / L2V, col = lane % L2V;
                        const double *q = &stash2[wave][r * 4 * L2V + col];
                        stash[wave][((u2 - rb + r) % L2B) * L2V + col] = (((q[0] + q[L2V]) + q[2 * L2V]) + q[3 * L2V]) / 4.0;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            } else {
#pragma unroll
                for (int j = 0; j < M2; ++j) {
                    const double R2 = pow14_q4(cellmax_d(Racc2[j], Cq[j]), plds); // pooled child, rectified
                    Cprev2[j] = Cq[j];
                    const double s0 = __shfl(R2, c), s1 = __shfl(R2, c + 16), s2 = __shfl(R2, c + 32),
                                 s3 = __shfl(R2, c + 48);
                    if (grp == 0) stash[wave][slot * L2V + M2 * c + j] = (((s0 + s1) + s2) + s3) / 4.0;
                }
            }
            if (slot == L2B - 1 || u2 == h0 / 4 - 1) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane < (slot + 1) * L2V) {
                    double l2 = pow14_k(stash[wave][lane], plds);
                    if (CL && bflat) l2 = (double)NAN; // see norm_clamp
                    L2row[(size_t)(u2 - slot + lane / L2V) * w2 + 4 * GW * wc + lane % L2V] = l2;
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
    };

    // rows in pairs (q0 even, q0 + 1 odd) = level-1 row u = q0 / 2; one barrier per pair
    // publishes both rows' edge values and the previous pair's level-1 edge value
    // (measured: two pairs per iteration with the parity at compile time models 2.7 % MORE
    // issue cycles -- the compiler splits and spreads the first pair's MFMA block)
    for (int q0 = 0; q0 < h0; q0 += 2) {
        const int u = q0 >> 1, k = u & 1;
        load_row(fb, q0 + 1);
        float Ca[M][4], Cb[M][4], la[4], lb[4];
        pool_cols(fa, Ca, la);
        // row pooling, first half: the even row q0 opens level-1 row u with the previous
        // pair's odd row (Cprev) -- folded in now (max is exact and order-free), so Cprev is
        // dead before Cb is born and the loop carries it without a copy
        if (q0 > 0) {
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) Ca[m][r] = fmaxf(Cprev[m][r], Ca[m][r]);
        }
        if constexpr (!LATE) load_row(fa, q0 + 2 < h0 ? q0 + 2 : 0);
        pool_cols(fb, Cb, lb);
        if (NWc > 1 && c == 15) {
#pragma unroll
            for (int r = 0; r < 4; ++r) { xch[sb][k][0][wc + 1][grp][r] = la[r]; xch[sb][k][1][wc + 1][grp][r] = lb[r]; }
            if (L2F && u > 0) xch2[sb][k ^ 1][wc][grp] = l1p[M - 1];
        }
        // publishes the edge values to wave w+1; with one wave per cell block (NWc == 1: C2,
        // NB = 2) no wave reads another's, and the blocks of a workgroup run unsynchronised
        if constexpr (NWc > 1) __syncthreads();
        {
            // left neighbour of pooled column 0: lane c-1's last tile (DPP row_shr:1); lane
            // c == 0 keeps the DPP "old" operand = wave w-1's edge value (slot w; -inf for w = 0)
            const float4 ninf = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
            const float4 xa = NWc > 1 ? *(const float4 *)&xch[sb][k][0][wc][grp][0] : ninf;
            const float4 xb = NWc > 1 ? *(const float4 *)&xch[sb][k][1][wc][grp][0] : ninf;
            const float oa[4] = {xa.x, xa.y, xa.z, xa.w}, ob[4] = {xb.x, xb.y, xb.z, xb.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                Ca[0][r] = fmaxf(Ca[0][r], dpp_prev16_or(la[r], oa[r]));
                Cb[0][r] = fmaxf(Cb[0][r], dpp_prev16_or(lb[r], ob[r]));
            }
        }
        double l1q[M]; // level-1 row u - 1, consumed by level2_row below
#pragma unroll
        for (int m = 0; m < M; ++m) l1q[m] = l1p[m];
        // row pooling: even row q0 (Cprev already folded in) and odd row q0 + 1 close row u
        // a constant child map (den == 0) makes its values NaN (0 * inf in the Markstein step,
        // the reference's 0/0): pow14_zf and pow14_q4 map NaN to NaN, so the sum and level 1
        // of its cell are NaN, as in the reference (CL: the clamp bit maps that NaN to 0, and
        // the stores write the NaN instead -- bflat / cflat, norm_clamp)
        const float4 kap = cst[sb][grp][0], kmn = cst[sb][grp][3], kden = cst[sb][grp][4], kinv = cst[sb][grp][5];
        float4 klo = kap, khi = kap;
        if constexpr (!CL) { klo = cst[sb][grp][1]; khi = cst[sb][grp][2]; }
#pragma unroll
        for (int m = 0; m < M; ++m) {
            float R[4], x[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                R[r] = fmaxf(Ca[m][r], Cb[m][r]);
                Cprev[m][r] = Cb[m][r];
            }
            // r = med3(R * a_p, lo, hi); x = (r - rmin) / den (Markstein, see norm_mk), packed.
            // CL: the med3 is the clamp bit of the last Markstein step instead (see norm_clamp)
            const dm_f2 ra = dm_f2{R[0], R[1]} * dm_f2{kap.x, kap.y}, rb = dm_f2{R[2], R[3]} * dm_f2{kap.z, kap.w};
            float r4[4] = {ra.x, ra.y, rb.x, rb.y};
            if constexpr (!CL) {
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
            x[0] = x01.x; x[1] = x01.y; x[2] = x23.x; x[3] = x23.y;
            double sum = 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) { // ul, ur, ll, lr: left-to-right sum
#if DM_ABL_PAPPROX
                // ABLATION ONLY (tools/abl_build.sh papprox / papprox2; results WRONG): the price of
                // pruning the child pows -- the bin-centre approximation (1/c_i)^y * 2^(yE) (two
                // table reads and a multiply, within 0.21 % of pow14) for every child, and with
                // DM_ABL_PAPPROX == 2 the exact pow for 2 of the lane's 8 children per row (4 per
                // level-2 window row: one exact level-1 value per window, the ideal pruned count)
                double pv;
                if (DM_ABL_PAPPROX == 2 && m == 0 && r < 2) pv = pow14_zf(x[r], plds, mant);
                else {
                    const unsigned u = __float_as_uint(x[r]);
                    const unsigned ofp = (u >> 10) & 0x1FF0u, og = (u >> 19) & 0xFF0u;
                    pv = (*(const dm_d2 *)((const char *)plds.fp + ofp)).x * (*(const dm_d2 *)((const char *)plds.g32 + og)).x;
                }
#else
                const double pv = pow14_zf(x[r], plds, mant);
#endif
                sum = r == 0 ? pv : sum + pv;
            }
            // level 1 = pow14(sum / 4), rectified where it is read: here when level 1 is
            // stored, after level 2's MaxPool otherwise (see level2_row)
            l1p[m] = sum;
            if (L1) Lrow[(size_t)u * w1 + M * c + m] = cflat ? (double)NAN : pow14_q4(sum, plds);
        }
        if constexpr (L2F) {
            if (u > 0) level2_row(u - 1, l1q);
        }
        if constexpr (LATE) load_row(fa, q0 + 2 < h0 ? q0 + 2 : 0);
    }
    if constexpr (L2F) {
        const int u = h0 / 2 - 1;
        if (NWc > 1 && c == 15) xch2[sb][u & 1][wc][grp] = l1p[M - 1];
        if constexpr (NWc > 1) __syncthreads();
        level2_row(u, l1p);
    }
}

// ===================================================================================
// Level-0 volume ("co_map", misc/Correlation_map.py:69-87 + Feature_value.min_max), MFMA
// path: one wave per 16 patches (a 2x2 block of level-1 cells, as k_level1_mfq), every wave
// independent (no LDS, no barrier).  Sweep 1: min/max of y over all windows; sweep 2:
// recompute y, r = med3(y a_p, lo, hi), x = (r - rmin)/den (Markstein), store float32.
// Windows use the column-group layout of k_prep_windows16 (q1 = 16 GW g + GW c + tw), so
// lane c's GW tiles of group g are GW consecutive floats: one GW-float vector store per
// patch, a 16-lane group writing 64*GW/... = 16*GW*4 contiguous bytes of the patch's row.
// ===================================================================================
// OT = float (co_map) or _Float16 (the binary16 volume: the float32 value rounded to nearest
// even, as np.float16(co_map)).  Used for the shapes k_volume_ls does not take (ws > 5).
template <int KS, int GW, bool YF, bool NT, bool LS, typename OT = float>
__global__ __launch_bounds__(256) void k_volume_mfq(Geo g, Stats s, const dm_v4i *__restrict__ Bw,
                                                    const int2 *__restrict__ QS, OT *vol)
{
    // LS: a row's 16 x w0 results are staged in LDS and stored as whole patch rows
    // (w0 * 4 contiguous bytes per patch, 16-B lanes) instead of GW-float pieces
    __shared__ __attribute__((aligned(16))) float stage[LS ? 4 : 1][LS ? 16 * 128 : 1];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane & 15, grp = lane >> 4;
    const int h0 = g.h0, w0 = g.w0, n = g.ws * g.ws, P = h0 * w0;
    const int G = w0 / 16, NG = G / GW; // tiles per row, column groups per row
    const int nbj = w0 / 4, bpt = (h0 / 4) * nbj;
    const int wid = blockIdx.x * 4 + wv;
    if (wid >= g.T * bpt) return; // whole wave (no barrier in this kernel)
    const int t = wid / bpt;
    const int I0 = 2 * ((wid % bpt) / nbj), J0 = 2 * ((wid % bpt) % nbj);
    const size_t tb = (size_t)t * P;
    const int ro = g.org[2 * t], co = g.org[2 * t + 1];

    dm_v4i A[KS];
    build_a<KS>(A, g, t, I0, J0, c, grp);
    const int Ic = I0 + (grp >> 1), Jc = J0 + (grp & 1);
    int sTr[4], pr[4];
    float sTf[4], ap[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        pr[r] = (2 * Ic + (r >> 1)) * w0 + 2 * Jc + (r & 1);
        sTr[r] = s.sT[tb + pr[r]];
        sTf[r] = (float)sTr[r];
        ap[r] = s.aP[tb + pr[r]];
    }
    const int ab = YF ? DM_YBIAS : 0;
    const dm_v4i acc0 = {ab, ab, ab, ab};
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void *)(Bw + (size_t)t * h0 * G * KS * 64), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rQ =
        __builtin_amdgcn_make_buffer_rsrc((void *)(QS + (size_t)t * h0 * G * 16), 0, 0x7fffffff, 0x00020000);
    const unsigned voB = (unsigned)lane * 16u, voQ = (unsigned)c * 8u;

    // unit = (row q0, column group gg): GW tiles; double-buffered loads
    struct Unit {
        dm_v4i b[GW][KS];
        int2 q[GW];
    };
    const int NU = h0 * NG;
    auto load_unit = [&](Unit &f, int uidx) {
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            const unsigned ti = (unsigned)uidx * GW + tw; // = q0 * G + gg * GW + tw
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                f.b[tw][ks] = __builtin_amdgcn_raw_buffer_load_b128(rB, voB, (ti * KS + ks) * 1024u, 0);
            const dm_v2i qv = __builtin_amdgcn_raw_buffer_load_b64(rQ, voQ, ti * 128u, 0);
            f.q[tw] = make_int2(qv.x, qv.y);
        }
    };

    float mn[4], mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { mn[r] = INFINITY; mx[r] = -INFINITY; }
    Unit fa, fb;
    load_unit(fa, 0);
    for (int ui = 0; ui < NU; ui += 2) { // NU even (h0 % 4 == 0)
        load_unit(fb, ui + 1);
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            float y[4];
            y_of_acc<YF>(mfma_tile<KS>(A, fa.b[tw], acc0), sTr, sTf, qs_pair(fa.q[tw]), n, y);
#pragma unroll
            for (int r = 0; r < 4; ++r) { mn[r] = fminf(mn[r], y[r]); mx[r] = fmaxf(mx[r], y[r]); }
        }
        load_unit(fa, ui + 2 < NU ? ui + 2 : 0); // last prefetch = sweep 2's first unit
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            float y[4];
            y_of_acc<YF>(mfma_tile<KS>(A, fb.b[tw], acc0), sTr, sTf, qs_pair(fb.q[tw]), n, y);
#pragma unroll
            for (int r = 0; r < 4; ++r) { mn[r] = fminf(mn[r], y[r]); mx[r] = fmaxf(mx[r], y[r]); }
        }
    }
    float lo[4], hi[4], rmn[4], den[4], rinv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        for (int off = 1; off < 16; off <<= 1) {
            mn[r] = fminf(mn[r], __shfl_xor(mn[r], off));
            mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], off));
        }
        rmn[r] = r_of_y(mn[r], ap[r], g.method);
        const float rmx = r_of_y(mx[r], ap[r], g.method);
        den[r] = __fsub_rn(rmx, rmn[r]);
        rinv[r] = __frcp_rn(den[r]);
        const bool cc = g.method == DM_TM_CCOEFF;
        lo[r] = cc ? -INFINITY : (ap[r] == 0.0f ? 1.0f : -1.0f);
        hi[r] = cc ? INFINITY : 1.0f;
        if (c == 0) {
            s.rmn[tb + pr[r]] = rmn[r];
            s.rmx[tb + pr[r]] = rmx;
        }
    }

    typedef float fv __attribute__((ext_vector_type(GW)));
    typedef OT ofv __attribute__((ext_vector_type(GW)));
    float *stg = &stage[LS ? wv : 0][0];
    const size_t pbase = tb + (size_t)(2 * I0) * w0 + 2 * J0; // patch (row 2*I0, col 2*J0)
    auto emit = [&](const Unit &f, int uidx) {
        const int q0 = uidx / NG, gg = uidx % NG;
        float xs[GW][4];
#pragma unroll
        for (int tw = 0; tw < GW; ++tw) {
            float y[4];
            y_of_acc<YF>(mfma_tile<KS>(A, f.b[tw], acc0), sTr, sTf, qs_pair(f.q[tw]), n, y);
            // r = med3(y * a_p, lo, hi); x = (r - rmin) / den (norm_mk's Markstein), packed
            const dm_f2 ya = dm_f2{y[0], y[1]} * dm_f2{ap[0], ap[1]};
            const dm_f2 yb = dm_f2{y[2], y[3]} * dm_f2{ap[2], ap[3]};
            const float rr[4] = {__builtin_amdgcn_fmed3f(ya.x, lo[0], hi[0]), __builtin_amdgcn_fmed3f(ya.y, lo[1], hi[1]),
                                 __builtin_amdgcn_fmed3f(yb.x, lo[2], hi[2]), __builtin_amdgcn_fmed3f(yb.y, lo[3], hi[3])};
            const dm_f2 a01 = dm_f2{rr[0], rr[1]} - dm_f2{rmn[0], rmn[1]};
            const dm_f2 a23 = dm_f2{rr[2], rr[3]} - dm_f2{rmn[2], rmn[3]};
            const dm_f2 i01 = {rinv[0], rinv[1]}, i23 = {rinv[2], rinv[3]};
            const dm_f2 q01 = a01 * i01, q23 = a23 * i23;
            const dm_f2 e01 = __builtin_elementwise_fma(-q01, dm_f2{den[0], den[1]}, a01);
            const dm_f2 e23 = __builtin_elementwise_fma(-q23, dm_f2{den[2], den[3]}, a23);
            const dm_f2 x01 = __builtin_elementwise_fma(e01, i01, q01);
            const dm_f2 x23 = __builtin_elementwise_fma(e23, i23, q23);
            xs[tw][0] = x01.x; xs[tw][1] = x01.y; xs[tw][2] = x23.x; xs[tw][3] = x23.y;
        }
        const int col = 16 * GW * gg + GW * c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            fv v;
#pragma unroll
            for (int tw = 0; tw < GW; ++tw) v[tw] = xs[tw][r];
            if constexpr (LS) {
                *(fv *)(stg + (4 * grp + r) * w0 + col) = v;
            } else {
                ofv ov;
#pragma unroll
                for (int tw = 0; tw < GW; ++tw) ov[tw] = (OT)v[tw];
                ofv *dst = (ofv *)(vol + (tb + pr[r]) * (size_t)P + (size_t)q0 * w0 + col);
                if constexpr (NT) __builtin_nontemporal_store(ov, dst);
                else *dst = ov;
            }
        }
        if constexpr (LS) {
            if (gg == NG - 1) { // the row is complete: 16 patch rows of w0 floats
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int per = w0 / 4;            // float4 per patch row
                const int rows_per = 64 / per;     // patch rows per store instruction
                for (int j = 0; j < 16; j += rows_per) {
                    const int pl = j + lane / per, k4 = lane % per; // local patch 4*cell + child
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    typedef OT o4v __attribute__((ext_vector_type(4)));
                    const f4v v4 = *(const f4v *)(stg + pl * w0 + 4 * k4);
                    const o4v o4 = {(OT)v4.x, (OT)v4.y, (OT)v4.z, (OT)v4.w};
                    const int pc = pl >> 2, pch = pl & 3;
                    const size_t prow = pbase + (size_t)(2 * (pc >> 1) + (pch >> 1)) * w0 + 2 * (pc & 1) + (pch & 1);
                    o4v *dst = (o4v *)(vol + prow * (size_t)P + (size_t)q0 * w0) + k4;
                    if constexpr (NT) __builtin_nontemporal_store(o4, dst);
                    else *dst = o4;
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
    };
    for (int ui = 0; ui < NU; ui += 2) {
        load_unit(fb, ui + 1);
        emit(fa, ui);
        load_unit(fa, ui + 2 < NU ? ui + 2 : 0);
        emit(fb, ui + 1);
    }
}

// ===================================================================================
// Level-0 volume with LDS-shared windows (k_volume_ls).
// The column-split kernels above are bound by the per-CU vector-memory pipe, not by the
// VALU: PMC TA_TA_BUSY / TD_TD_BUSY 0.98 of the cycles (profiles/r02_pmc_mem.txt), because
// every wave streams its own copy of the window fragments (1 KB of B + 512 B of window
// stats per 16x16 tile).  Here the NW waves of a workgroup hold DIFFERENT patches (16 each,
// a 2x2 block of level-1 cells) and sweep ALL windows of the tile; each image row's G
// window tiles and their stats are staged in LDS once per workgroup by LDS-DMA
// (buffer_load_dwordx4 ... lds), double-buffered with one barrier per row -- 1/NW of the
// load traffic per voxel.  A wave owns its patches over every window, so the per-patch
// min/max needs no cross-wave step.  The windows are laid out in column groups of GW = 16 B
// of output per lane (8 tiles binary16, 4 float32; dm_corr_volume preps this layout into a
// second region): lane c of tile tau is window q1 = 16 GW (tau / GW) + GW c + tau % GW, so
// after a group a lane holds GW consecutive windows of each of its 4 patches and writes them
// with one 16-B store straight from registers: 16 lanes = one contiguous 256-B patch-row
// run per store instruction, no LDS stage.
// Arithmetic per voxel is k_volume_mfq's (same y, r, Markstein x): bit-identical output.
// ===================================================================================
// the standalone volumes' strip min/max sweep with each unit staged in LDS once per workgroup (1)
// or read from L2 by every wave (0).  Same box, bit-identical (profiles/r05x_vs1lds_ab.txt):
// C3 float32 13.58/13.56 -> 12.64/12.70 ms, C5-size binary16 16.00/16.13 -> 15.78/15.79,
// C3 binary16 and C5-size float32 within 0.4 %
#ifndef DM_VS1_LDS
#define DM_VS1_LDS 1
#endif
template <int G, int NW, bool NT, typename OT, int TR = 0, int MW = 1, int GW = (16 / (int)sizeof(OT)) < G ? (16 / (int)sizeof(OT)) : G>
__global__ __launch_bounds__(64 * NW, MW) void k_volume_ls(Geo g, Stats s, const dm_v4i *__restrict__ Bw,
                                                   const int2 *__restrict__ QS, OT *vol, int have_mm,
                                                   const dm_v4i *__restrict__ Bs = nullptr,
                                                   const dm_v4i *__restrict__ Ss = nullptr)
{
    // have_mm: the per-patch rmin / rmax are already in the statistics workspace (written by
    // dm_corr_level1/12 or an earlier volume launch on the same stats): sweep 1 -- the MFMA,
    // y and min/max over every window, ~40 % of this kernel's issue cycles -- is skipped and
    // the normalisation constants are read back instead (bit-identical: the same rmin/rmax).
    constexpr int W0 = 16 * G;
    constexpr int BUF = G * 1024;          // one row: G B tiles (window stats inside, qs_of_frag)
    constexpr int NL = G;                  // LDS-DMA instructions per row per workgroup
    static_assert(G % 2 == 0, "tiles come in column-group pairs");
    __shared__ __attribute__((aligned(16))) char lds[2 * BUF]; // the only LDS object (glds rule)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, grp = lane >> 4;
    const int h0 = g.h0, n = g.ws * g.ws, P = h0 * W0;
    const int nbj = W0 / 4, bpt = (h0 / 4) * nbj;  // 16-patch blocks per tile (bpt % NW == 0)
    const int blk = blockIdx.x * NW + wave;
    const int t = blk / bpt;                       // the same tile for every wave of the block
    const int I0 = 2 * ((blk % bpt) / nbj), J0 = 2 * ((blk % bpt) % nbj);
    const size_t tb = (size_t)t * P;

    dm_v4i A[1];
    build_a<1>(A, g, t, I0, J0, c, grp);
    const int Ic = I0 + (grp >> 1), Jc = J0 + (grp & 1);
    int sTr[4];
    float sTf[4], ap[4];
    OT *out[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int p = (2 * Ic + (r >> 1)) * W0 + 2 * Jc + (r & 1);
        sTr[r] = s.sT[tb + p];
        sTf[r] = (float)sTr[r];
        ap[r] = s.aP[tb + p];
        out[r] = vol + (tb + p) * (size_t)P + GW * c;
    }
    const dm_v4i acc0 = {DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS};
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void *)(Bw + (size_t)t * h0 * G * 64), 0, 0x7fffffff, 0x00020000);

    // LDS-DMA of row q0 into buffer `buf`: instruction i of the row goes to wave i % NW.
    // Issued through inline asm so that the compiler's wait insertion does not treat every
    // later ds_read as dependent on it (it would wait vmcnt(0) -- the prefetch AND the
    // stores -- before the first read of each row); the waits are the explicit vmcnt(N)
    // before each row's barrier.
    const unsigned lds0 = (unsigned)(uintptr_t)&lds[0];
    auto fill = [&](int q0, int buf) {
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            if (i % NW != wave) continue;
            const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + (unsigned)(buf * BUF + i * 1024));
            lds_dma16(rB, dst, (unsigned)lane * 16u, (unsigned)(q0 * G + i) * 1024u);
        }
    };
    // tile tau of the row in buffer buf: MFMA + y of this lane's 4 patches (the window stats
    // ride in words 2, 3 of the lane's own fragment: spread layout, qs_of_frag)
    auto tile_y = [&](int buf, int tau, float *y) {
        const dm_v4i bf = *(const dm_v4i *)&lds[buf * BUF + tau * 1024 + lane * 16];
        const dm_f2 q2 = qs_of_frag(bf); // {qx, qy}
        dm_v4i bfr[1] = {bf};
        y_of_acc<true>(mfma_tile<1, true>(A, bfr, acc0), sTr, sTf, q2, n, y);
    };

    float lo[4], hi[4], rmn[4], den[4], rinv[4];
    bool clamp = false;   // does any r = y * a_p of this wave leave [-1, 1]?
    const bool cc = g.method == DM_TM_CCOEFF;
    if (have_mm) {
        // sweep 2 reads row 0 from buffer h0 & 1 (where sweep 1 would have left it)
        fill(0, h0 & 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = (2 * Ic + (r >> 1)) * W0 + 2 * Jc + (r & 1);
            rmn[r] = s.rmn[tb + p];
            const float rmx = s.rmx[tb + p];
            den[r] = __fsub_rn(rmx, rmn[r]);
            rinv[r] = __frcp_rn(den[r]);
            lo[r] = cc ? -INFINITY : (ap[r] == 0.0f ? 1.0f : -1.0f);
            hi[r] = cc ? INFINITY : 1.0f;
            // conservative: rmin / rmax are already clamped, so a bound at +-1 may hide an r
            // beyond it -- take the clamped sweep then (it is the exact formula either way)
            clamp = clamp || (!cc && (ap[r] == 0.0f || rmx >= 1.0f || rmn[r] <= -1.0f));
        }
        clamp = __builtin_amdgcn_ballot_w64(clamp) != 0;
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else if (Bs) {
        // ---- sweep 1 on the row-pair strips (dm_corr_stats' k_prep_strips, round 5): the
        // 32 x 32 x 32 i8 MFMA gives this wave's 16 patches x 2 window rows x 32 windows per
        // instruction (k_level1_mfq's strip sweep); the strips come from memory, so the LDS
        // window rows are not needed until sweep 2 ----
        const int c32 = lane & 31, hs = lane >> 5, h2 = h0 / 2;
        constexpr int NT32 = W0 / 32, NGR = W0 >= 64 ? W0 / 64 : 1;   // strip tiles, 64-window groups per row pair
        // A rows (lane & 31): patch lane & 15 shifted by ws taps for rows 16..31, K bytes 16 hs ..
        dm_v4i A32;
        {
            const __amdgpu_buffer_rsrc_t rI = tile_rsrc(g.img1, g.pitch1, g, t);
            const int pi = lane & 15, o = (lane >> 4) & 1, cl = pi >> 2, ch = pi & 3;
            const int p0 = 2 * (I0 + (cl >> 1)) + (ch >> 1), p1 = 2 * (J0 + (cl & 1)) + (ch & 1);
            const unsigned pb = (unsigned)(p0 * g.pitch1 + p1);
            const int ws = g.ws;
            int w[4] = {0, 0, 0, 0};
#pragma unroll
            for (int bb = 0; bb < 16; ++bb) {
                const int tau = 16 * hs + bb - ws * o;
                const bool in = tau >= 0 && tau < n;
                const int tc = tau < 0 ? 0 : (tau >= n ? n - 1 : tau);
                const int v = (int)__builtin_amdgcn_raw_buffer_load_b8(rI, pb + (unsigned)((tc / ws) * g.pitch1 + tc % ws), 0, 0) - 128;
                w[bb >> 2] |= ((in ? v : 0) & 0xFF) << (8 * (bb & 3));
            }
            A32 = dm_v4i{w[0], w[1], w[2], w[3]};
        }
        float sTs[8];   // [cell slot][child]: patch 4 (2 (k >> 2) + hs) + (k & 3)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int cell = 2 * (k >> 2) + hs, ch = k & 3;
            const int p = (2 * (I0 + (cell >> 1)) + (ch >> 1)) * W0 + 2 * (J0 + (cell & 1)) + (ch & 1);
            sTs[k] = (float)s.sT[tb + p];
        }
        const __amdgpu_buffer_rsrc_t rS1 =
            __builtin_amdgcn_make_buffer_rsrc((void *)(Bs + (size_t)t * h2 * NT32 * 64), 0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rS2 =
            __builtin_amdgcn_make_buffer_rsrc((void *)(Ss + (size_t)t * h2 * W0), 0, 0x7fffffff, 0x00020000);
        const unsigned voS = (unsigned)lane * 16u, voQ = (unsigned)c32 * 32u;
        struct StripFrag {
            dm_v4i b[2], q[2];
        };
        // unit k = (row pair k / NGR, 64-window group k % NGR): strip tiles 2 gr, 2 gr + 1
        auto load_unit = [&](StripFrag &f, int k) {
            const int rp = k / NGR, gr = k % NGR;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f.b[j] = __builtin_amdgcn_raw_buffer_load_b128(rS1, voS, (unsigned)(rp * NT32 + 2 * gr + j) * 1024u, 0);
                f.q[j] = __builtin_amdgcn_raw_buffer_load_b128(rS2, voQ, (unsigned)(rp * W0 + 64 * gr + j) * 16u, 0);
            }
        };
        const float nf = (float)n, nb = -nf * 12582912.0f; // y_of_acc's exact steps
        const dm_v16i acc32 = {DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS,
                               DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS, DM_YBIAS};
        float mn8[8], mx8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { mn8[k] = INFINITY; mx8[k] = -INFINITY; }
        const int NU = h2 * NGR;
        // one fragment buffer, each part reloaded with unit k + 1's as soon as it is used (the
        // volume kernels' sweep 2 keeps the registers of the 16 x 16 path)
        auto minmax_unit = [&](StripFrag &f, int k) {
            const int kn = __builtin_amdgcn_readfirstlane(k + 1 < NU ? k + 1 : k), rpn = kn / NGR, grn = kn % NGR;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const dm_v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A32, f.b[j], acc32, 0, 0, 0);
                f.b[j] = __builtin_amdgcn_raw_buffer_load_b128(rS1, voS, (unsigned)(rpn * NT32 + 2 * grn + j) * 1024u, 0);
                const dm_f2 qs0 = dm_f2{__int_as_float(f.q[j].x), __int_as_float(f.q[j].y)};
                const dm_f2 qs1 = dm_f2{__int_as_float(f.q[j].z), __int_as_float(f.q[j].w)};
                float y[16];
#pragma unroll
                for (int m = 0; m < 8; ++m) { // register pair (2m, 2m + 1): window row m >> 2
                    const int cs = (m >> 1) & 1, cp = m & 1;
                    const dm_f2 qs = (m >> 2) ? qs1 : qs0;
                    const dm_f2 a = dm_f2{__int_as_float(acc[2 * m]), __int_as_float(acc[2 * m + 1])};
                    const dm_f2 mm = __builtin_elementwise_fma(a, dm_f2{nf, nf}, dm_f2{nb, nb});
                    const dm_f2 nu = __builtin_elementwise_fma(dm_f2{sTs[4 * cs + 2 * cp], sTs[4 * cs + 2 * cp + 1]},
                                                               __builtin_shufflevector(qs, qs, 0, 0), mm);
                    const dm_f2 yy = pk_mul_bhi(qs, nu);
                    y[2 * m] = yy.x; y[2 * m + 1] = yy.y;
                }
                f.q[j] = __builtin_amdgcn_raw_buffer_load_b128(rS2, voQ, (unsigned)(rpn * W0 + 64 * grn + j) * 16u, 0);
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                    mn8[kk] = fminf(fminf(mn8[kk], y[kk]), y[8 + kk]);
                    mx8[kk] = fmaxf(fmaxf(mx8[kk], y[kk]), y[8 + kk]);
                }
            }
        };
        if constexpr (DM_VS1_LDS && BUF >= 4096) {
            // the workgroup's waves sweep the same units: each unit's 2 strip tiles (2 KB) and
            // window stats (1 KB) come into LDS once per workgroup by LDS-DMA (instruction i by
            // wave i % NW), double-buffered in the row buffers, one barrier per unit
            constexpr int STG = 4096;
            auto stage = [&](int k, int sb) {
                const int rp = k / NGR, gr = k % NGR;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if (i % NW != wave) continue;
                    const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + (unsigned)(sb * STG + i * 1024));
                    if (i < 2) lds_dma16(rS1, dst, voS, (unsigned)(rp * NT32 + 2 * gr + i) * 1024u);
                    else lds_dma16(rS2, dst, voS, (unsigned)(rp * W0 + 64 * gr) * 16u);
                }
            };
            stage(0, 0);
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            for (int k = 0; k < NU; ++k) {
                const int sb = k & 1;
                if (k + 1 < NU) stage(k + 1, sb ^ 1);
                const char *u = &lds[sb * STG];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const dm_v4i bj = *(const dm_v4i *)(u + j * 1024 + lane * 16);
                    const dm_v4i qj = *(const dm_v4i *)(u + 2048 + c32 * 32 + j * 16);
                    const dm_v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A32, bj, acc32, 0, 0, 0);
                    const dm_f2 qs0 = dm_f2{__int_as_float(qj.x), __int_as_float(qj.y)};
                    const dm_f2 qs1 = dm_f2{__int_as_float(qj.z), __int_as_float(qj.w)};
                    float y[16];
#pragma unroll
                    for (int m = 0; m < 8; ++m) {
                        const int cs = (m >> 1) & 1, cp = m & 1;
                        const dm_f2 qs = (m >> 2) ? qs1 : qs0;
                        const dm_f2 a = dm_f2{__int_as_float(acc[2 * m]), __int_as_float(acc[2 * m + 1])};
                        const dm_f2 mm = __builtin_elementwise_fma(a, dm_f2{nf, nf}, dm_f2{nb, nb});
                        const dm_f2 nu = __builtin_elementwise_fma(dm_f2{sTs[4 * cs + 2 * cp], sTs[4 * cs + 2 * cp + 1]},
                                                                   __builtin_shufflevector(qs, qs, 0, 0), mm);
                        const dm_f2 yy = pk_mul_bhi(qs, nu);
                        y[2 * m] = yy.x; y[2 * m + 1] = yy.y;
                    }
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk) {
                        mn8[kk] = fminf(fminf(mn8[kk], y[kk]), y[8 + kk]);
                        mx8[kk] = fmaxf(fmaxf(mx8[kk], y[kk]), y[8 + kk]);
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            }
        } else {
            StripFrag fa;
            load_unit(fa, 0);
            for (int k = 0; k < NU; ++k) minmax_unit(fa, k);
        }
        half_wave_minmax(mn8, mx8);
        // the 16 patches' extremes (lanes 31, 63) to the 16 x 16 layout (lane group = cell,
        // accumulator row = child) through the LDS row buffer sweep 2 fills last
        float *red = (float *)&lds[((h0 & 1) ^ 1) * BUF] + wave * 32;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int pl = 4 * (2 * (k >> 2) + hs) + (k & 3);
            if (c32 == 31) { red[pl] = mn8[k]; red[16 + pl] = mx8[k]; }
        }
        fill(0, h0 & 1);   // sweep 2's row 0, in flight through the reduction
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float mnr = red[4 * grp + r], mxr = red[16 + 4 * grp + r];
            rmn[r] = r_of_y(mnr, ap[r], g.method);
            const float rmx = r_of_y(mxr, ap[r], g.method);
            den[r] = __fsub_rn(rmx, rmn[r]);
            rinv[r] = __frcp_rn(den[r]);
            lo[r] = cc ? -INFINITY : (ap[r] == 0.0f ? 1.0f : -1.0f);
            hi[r] = cc ? INFINITY : 1.0f;
            clamp = clamp || (!cc && (ap[r] == 0.0f || __fmul_rn(mxr, ap[r]) > 1.0f ||
                                      __fmul_rn(mnr, ap[r]) < -1.0f));
            if (c == 0) {
                const int p = (2 * Ic + (r >> 1)) * W0 + 2 * Jc + (r & 1);
                s.rmn[tb + p] = rmn[r];
                s.rmx[tb + p] = rmx;
            }
        }
        clamp = __builtin_amdgcn_ballot_w64(clamp) != 0;   // wave-uniform
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
    fill(0, 0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

    // ---- sweep 1: min / max of y over every window (this wave's patches only) ----
    float mn[4], mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { mn[r] = INFINITY; mx[r] = -INFINITY; }
    for (int q0 = 0; q0 < h0; ++q0) {
        const int buf = q0 & 1;
        fill(q0 + 1 < h0 ? q0 + 1 : 0, buf ^ 1);     // the last prefetch is sweep 2's row 0
#pragma unroll
        for (int tau = 0; tau < G; tau += 2) {
            float y0[4], y1[4];
            tile_y(buf, tau, y0);
            tile_y(buf, tau + 1, y1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {   // v_min3 / v_max3
                mn[r] = fminf(fminf(mn[r], y0[r]), y1[r]);
                mx[r] = fmaxf(fmaxf(mx[r], y0[r]), y1[r]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        for (int off = 1; off < 16; off <<= 1) {
            mn[r] = fminf(mn[r], __shfl_xor(mn[r], off));
            mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], off));
        }
        rmn[r] = r_of_y(mn[r], ap[r], g.method);
        const float rmx = r_of_y(mx[r], ap[r], g.method);
        den[r] = __fsub_rn(rmx, rmn[r]);
        rinv[r] = __frcp_rn(den[r]);
        lo[r] = cc ? -INFINITY : (ap[r] == 0.0f ? 1.0f : -1.0f);
        hi[r] = cc ? INFINITY : 1.0f;
        // y * a_p is monotone in y (a_p >= 0), so every r of the patch lies in
        // [mn * a_p, mx * a_p]: the clamp can only act if those bounds leave [-1, 1] (or for a
        // constant patch, whose r is pinned to 1)
        clamp = clamp || (!cc && (ap[r] == 0.0f || __fmul_rn(mx[r], ap[r]) > 1.0f ||
                                  __fmul_rn(mn[r], ap[r]) < -1.0f));
        if (c == 0) {
            const int p = (2 * Ic + (r >> 1)) * W0 + 2 * Jc + (r & 1);
            s.rmn[tb + p] = rmn[r];
            s.rmx[tb + p] = rmx;
        }
    }
    clamp = __builtin_amdgcn_ballot_w64(clamp) != 0;   // wave-uniform
    }

    // ---- sweep 2: x of every window; lane c holds windows G c .. G c + G - 1 of each of its
    // 4 patches, stored in 16-B pieces (CH tiles) straight from registers ----
    constexpr int CH = GW;                 // tiles per column group = per store (16 B or the row)
    constexpr int STORES = 4 * (G / CH);   // store instructions per row per wave
    typedef OT ov __attribute__((ext_vector_type(CH)));
    // the sweep, with or without the clamp (wave-uniform choice; rare: perfect correlations and
    // constant patches need it)
    auto sweep2 = [&](auto clamp_tag) {
    constexpr bool CL = decltype(clamp_tag)::value;
    // x of tile tau's window column c for this lane's 4 patches, into element tw of v[0..3]
    auto x_tile = [&](int buf, int tau, ov *v, int tw) {
        float y[4];
        tile_y(buf, tau, y);
        const dm_f2 ya = dm_f2{y[0], y[1]} * dm_f2{ap[0], ap[1]};
        const dm_f2 yb = dm_f2{y[2], y[3]} * dm_f2{ap[2], ap[3]};
        dm_f2 r01 = ya, r23 = yb;
        if constexpr (CL) {
            r01 = dm_f2{__builtin_amdgcn_fmed3f(ya.x, lo[0], hi[0]), __builtin_amdgcn_fmed3f(ya.y, lo[1], hi[1])};
            r23 = dm_f2{__builtin_amdgcn_fmed3f(yb.x, lo[2], hi[2]), __builtin_amdgcn_fmed3f(yb.y, lo[3], hi[3])};
        }
        const dm_f2 a01 = r01 - dm_f2{rmn[0], rmn[1]};
        const dm_f2 a23 = r23 - dm_f2{rmn[2], rmn[3]};
        const dm_f2 i01 = {rinv[0], rinv[1]}, i23 = {rinv[2], rinv[3]};
        const dm_f2 q01 = a01 * i01, q23 = a23 * i23;
        const dm_f2 e01 = __builtin_elementwise_fma(-q01, dm_f2{den[0], den[1]}, a01);
        const dm_f2 e23 = __builtin_elementwise_fma(-q23, dm_f2{den[2], den[3]}, a23);
        const dm_f2 x01 = __builtin_elementwise_fma(e01, i01, q01);
        const dm_f2 x23 = __builtin_elementwise_fma(e23, i23, q23);
        v[0][tw] = (OT)x01.x; v[1][tw] = (OT)x01.y; v[2][tw] = (OT)x23.x; v[3][tw] = (OT)x23.y;
    };
    if constexpr (TR > 0) {
        // Runs of TR 256-B chunks: RB rows of NCG 256-B column groups are TR consecutive chunks
        // of each patch map (the maps' rows are consecutive).  Lane group g computed chunk i of
        // its own patches (g, r).  TR = 4: a 4 x 4 transpose over the lane groups (permlane32
        // then permlane16 swaps, per dword) leaves lane group g with chunk g of patch (s, r) in
        // X[r][s], so one store instruction writes 1 KB of ONE map instead of 256 B of four.
        // TR = 2: the permlane16 stage alone; lane groups 2h, 2h + 1 then hold chunks 0, 1 of
        // patch (2h + e, r) in X[r][e]: two 512-B runs per store, half the swaps and registers.
        constexpr int NCG = G / CH, RB = TR / NCG;
        static_assert((TR == 2 || TR == 4) && CH * sizeof(OT) == 16 && NCG <= TR && TR % NCG == 0,
                      "runs of 256-B chunks need 16-B lanes");
        OT *const pb = vol + (tb + (size_t)(2 * I0) * W0 + 2 * J0) * (size_t)P;   // patch (0, 0)
        const int sel = TR == 4 ? 0 : grp >> 1;         // TR = 2: the patch pair of this lane
        const int loff = (grp % TR) * 16 * CH + GW * c;
        for (int q0 = 0; q0 < h0; q0 += RB) {
            dm_v4i X[4][TR];   // [r][i]: chunk i = k NCG + j of the burst, patch (grp, r)
#pragma unroll
            for (int k = 0; k < RB; ++k) {
                const int q = q0 + k;
                const int buf = (h0 + q) & 1;
                if (q + 1 < h0) fill(q + 1, buf ^ 1);
#pragma unroll
                for (int j = 0; j < NCG; ++j) {
                    ov v[4];
#pragma unroll
                    for (int tw = 0; tw < CH; ++tw) x_tile(buf, j * CH + tw, v, tw);
#pragma unroll
                    for (int r = 0; r < 4; ++r) X[r][k * NCG + j] = __builtin_bit_cast(dm_v4i, v[r]);
                }
                if (k + 1 < RB) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    if constexpr (TR == 4) {
#pragma unroll
                        for (int a = 0; a < 2; ++a) {   // groups 2, 3 of chunk a <-> groups 0, 1 of chunk a + 2
                            const auto w = __builtin_amdgcn_permlane32_swap(X[r][a][d], X[r][a + 2][d], false, false);
                            X[r][a][d] = (int)w[0];
                            X[r][a + 2][d] = (int)w[1];
                        }
                    }
#pragma unroll
                    for (int a = 0; a < TR; a += 2) { // odd rows of 16 lanes of a <-> even rows of a + 1
                        const auto w = __builtin_amdgcn_permlane16_swap(X[r][a][d], X[r][a + 1][d], false, false);
                        X[r][a][d] = (int)w[0];
                        X[r][a + 1][d] = (int)w[1];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int e = 0; e < TR; ++e) {
                    // TR = 4: patch (e, r); TR = 2: patch (2 sel + e, r)
                    const int pofs = (2 * (e >> 1) + (r >> 1) + 2 * sel) * W0 + 2 * (e & 1) + (r & 1);
                    ov *dst = (ov *)(pb + (size_t)pofs * (size_t)P + (size_t)q0 * W0 + loff);
                    const ov o = __builtin_bit_cast(ov, X[r][e]);
                    if constexpr (NT) __builtin_nontemporal_store(o, dst);
                    else *dst = o;
                }
            }
            if (q0 + RB < h0) {
                if constexpr (TR == 4) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
            }
        }
    } else {
    for (int q0 = 0; q0 < h0; ++q0) {
        const int buf = (h0 + q0) & 1;
        if (q0 + 1 < h0) fill(q0 + 1, buf ^ 1);
#pragma unroll
        for (int t0 = 0; t0 < G; t0 += CH) {
            ov v[4];
#pragma unroll
            for (int tw = 0; tw < CH; ++tw) x_tile(buf, t0 + tw, v, tw);
            const int col = q0 * W0 + 16 * t0;    // column group t0 / GW starts at window 16 GW (t0 / GW)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if constexpr (NT) __builtin_nontemporal_store(v[r], (ov *)(out[r] + col));
                else *(ov *)(out[r] + col) = v[r];
            }
        }
        // this row's prefetch has landed once at most the row's own stores are outstanding
        if (q0 + 1 < h0) {
            if constexpr (STORES == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
            else if constexpr (STORES == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
            else if constexpr (STORES == 16) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
    }
    }
    };
    if (clamp) sweep2(std::true_type{});
    else sweep2(std::false_type{});
}

static bool mf16_eligible(const dm_tiles *b)
{
    // w0 in {32, 64, 128, 256}: the instantiated column-group counts G = w0/16 = 2, 4, 8, 16
    return b->h0 % 4 == 0 && b->w0 >= 32 && b->w0 <= 256 && (b->w0 & (b->w0 - 1)) == 0 && b->ws <= 15;
}

static size_t mf16_extra_bytes(const dm_tiles *b)
{
    const int G = b->w0 / 16, KS = (b->ws * b->ws + 63) / 64;
    return (size_t)b->T * b->h0 * G * KS * 1024 + (size_t)b->T * b->h0 * G * 16 * 8;
}
