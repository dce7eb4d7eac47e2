// dm_gs_pf.h -- pipelined Gauss-Seidel level walks (included by dm_postproc.hip after
// GsGeo / gs_cell / pyix).  Every optimize_loop sweep (misc/optimize_loop.py:15-37) and the
// bilateral sweeps (misc/opt_loop.py:16-58) with exclusion 1..5.
//
// With one update per lane, a level of k_optimize_loop / k_bilateral pays three dependent
// memory round trips between barriers: the schedule entry (ord), then the coefficient /
// colour weights it addresses, then the image.  Only the image depends on the sweep's own
// values, so here the schedule is fetched two levels ahead and the coefficient / weights
// one level ahead; the critical path of a level is one image round trip, the arithmetic,
// the store and the barrier.
//
// The bilateral kernel prefetches R rounds of NTHR/LPU updates per level (R*NTHR/LPU at
// least the usual level width, ~n/(e+1) for an n-wide map; fewer lanes leave more
// registers per lane for the two weight buffers).  Its sums use LPU lanes per update: lane u owns numpy's accumulators
// k = u*K .. u*K+K-1 (K = 8/LPU), each a sequential sum over m = k, k+8, ..., and the
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) tree is formed with xor shuffles (IEEE addition is
// commutative, so every lane of the group holds the same bits); the m = n-1 tail
// ((2e+1)^2 = 1 mod 8) is added last.  Same operations in the same order as np_pairwise in
// k_bilateral, so the maps stay bit-identical to the sequential loops.
#pragma once

__device__ __forceinline__ double gs_coef(const GsGeo &g, const double *coef, int wc, int s)
{
    int r, c;
    gs_cell(g, s, r, c);
    return coef[(size_t)r * wc + c];
}

__global__ __launch_bounds__(1024) void k_optimize_loop_pf(double *img, const double *coef, int wc, double alpha,
                                                           GsGeo gf, const int32_t *__restrict__ ford,
                                                           const int32_t *__restrict__ foff, int fnl, GsGeo gb,
                                                           const int32_t *__restrict__ bord,
                                                           const int32_t *__restrict__ boff, int bnl, double *diff)
{
    const int h = gf.h, w = gf.w, tid = (int)threadIdx.x, NT = (int)blockDim.x;
    for (int pass = 0; pass < 2; ++pass) {
        const GsGeo g = pass ? gb : gf;
        const int32_t *ord = pass ? bord : ford;
        const int32_t *off = pass ? boff : foff;
        const int nl = pass ? bnl : fnl;
        // loads of one update (issued before the prefetches, so waiting for them does not
        // wait for the prefetches: vmcnt retires in issue order) and its arithmetic + store
        struct Nb {
            double x, sum;
        };
        auto load = [&](int s) {
            int r, c;
            gs_cell(g, s, r, c);
            const double *row = img + (size_t)r * w;
            Nb q;
            q.x = row[c];
            q.sum = ((row[pyix(c - 1, w)] + row[c + 1]) + img[(size_t)pyix(r - 1, h) * w + c]) +
                    img[(size_t)(r + 1) * w + c];
            return q;
        };
        auto finish = [&](int s, double a, const Nb &q) {
            int r, c;
            gs_cell(g, s, r, c);
            const double d = ((-a) * q.x + alpha * q.sum) / ((-a) + 4.0 * alpha);
            if (pass) diff[s] = fabs(q.x - d);
            img[(size_t)r * w + c] = d;
        };
        int b = off[0], e = off[1], e2 = nl > 1 ? off[2] : e;
        int s_cur = b + tid < e ? ord[b + tid] : -1;
        double aA = gs_coef(g, coef, wc, s_cur >= 0 ? s_cur : 0), aB = 0.0;
        int s_nxt = e + tid < e2 ? ord[e + tid] : -1;
        // one level: uses a_c, prefetches the next level's coefficient into a_n.  Issue order
        // image loads -> schedule (two levels ahead) -> coefficient, so that neither the
        // update nor the end-of-level rotation of s waits for the coefficient; the
        // coefficients ping-pong between aA and aB (no register copy of a load in flight)
        auto level = [&](int l, double &a_c, double &a_n) {
            const int e3 = l + 2 < nl ? off[l + 3] : e2;
            // every lane issues its loads (update 0 is a valid cell) so the order holds
            const Nb q = load(s_cur >= 0 ? s_cur : 0);
            __builtin_amdgcn_sched_barrier(0);
            const int s_nn = e2 + tid < e3 ? ord[e2 + tid] : -1;
            __builtin_amdgcn_sched_barrier(0);
            a_n = gs_coef(g, coef, wc, s_nxt >= 0 ? s_nxt : 0);
            if (s_cur >= 0) finish(s_cur, a_c, q);
            for (int base = b + NT; base < e; base += NT) { // levels wider than the workgroup
                const int s = base + tid < e ? ord[base + tid] : -1;
                if (s >= 0) finish(s, gs_coef(g, coef, wc, s), load(s));
            }
            __syncthreads();
            b = e;
            e = e2;
            e2 = e3;
            s_cur = s_nxt;
            s_nxt = s_nn;
        };
        for (int l = 0; l < nl; l += 2) {
            level(l, aA, aB);
            if (l + 1 < nl) level(l + 1, aB, aA);
        }
    }
}

template <int E, int LPU, int R, int NTHR>
__global__ __launch_bounds__(NTHR) void k_bilateral_pf(double *img, const double *color, const double *gauss,
                                                       const double *coef, int hc, int wc, int vertical, GsGeo g,
                                                       const int32_t *__restrict__ ord,
                                                       const int32_t *__restrict__ off, int nl, double *diff)
{
    constexpr int W = 2 * E + 1, N = W * W, A = (N - 1) / 8, K = 8 / LPU, NT = K * A;
    static_assert((N - 1) % 8 == 0 && LPU * K == 8, "odd window: (2e+1)^2 = 1 mod 8");
    __shared__ double gs[N];
    const int tid = (int)threadIdx.x, u = tid % LPU, grp = tid / LPU, NG = (int)blockDim.x / LPU;
    const int w = g.w, cwc = g.s1 - E;
    for (int m = tid; m < N; m += (int)blockDim.x) gs[m] = gauss[m];
    const int er = pyix(E, hc), ec = pyix(E, wc);
    const double c0 = coef[(size_t)er * wc + ec];
    const double cp = vertical ? coef[(size_t)pyix(E + 1, hc) * wc + ec] : coef[(size_t)er * wc + pyix(E + 1, wc)];
    const double cm = vertical ? coef[(size_t)pyix(E - 1, hc) * wc + ec] : coef[(size_t)er * wc + pyix(E - 1, wc)];
    const double a = -(c0 - (cp + cm) / 2.0);
    const double Kc = (cp - cm) / 2.0 / (((-2.0) * c0 + cp) + cm);
    __syncthreads();

    // element of term t of this lane: accumulator k = u*K + t/A, m = k + 8*(t%A); t = NT: m = N-1
    auto mof = [&](int t) { return t == NT ? N - 1 : u * K + t / A + 8 * (t % A); };
    auto load_cw = [&](int s, double *cw) {
        int i, j;
        gs_cell(g, s, i, j);
        const double *p = color + ((size_t)(i - E) * cwc + (j - E)) * N;
#pragma unroll
        for (int t = 0; t <= NT; ++t) cw[t] = p[mof(t)];
    };
    // the image loads of an update (sv[0..NT], sv[NT+1] = centre) are issued before the
    // prefetches of the next level, so waiting for them does not wait for the prefetches
    // (vmcnt retires in issue order)
    auto load_sv = [&](int s, double *sv) {
        int i, j;
        gs_cell(g, s, i, j);
        const double *sub = img + (size_t)(i - E) * w + (j - E);
#pragma unroll
        for (int t = 0; t <= NT; ++t) {
            const int m = mof(t);
            sv[t] = sub[(size_t)(m / W) * w + (m % W)];
        }
        sv[NT + 1] = img[(size_t)i * w + j];
    };
    auto update = [&](int s, const double *cw, const double *sv) {
        int i, j;
        gs_cell(g, s, i, j);
        const double x = sv[NT + 1];
        double r1[K], r2[K];
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
            const int t0 = kk * A;
            const double g0 = gs[mof(t0)] * cw[t0];
            r1[kk] = g0 * sv[t0];
            r2[kk] = g0;
#pragma unroll
            for (int q = 1; q < A; ++q) {
                const double gq = gs[mof(t0 + q)] * cw[t0 + q];
                r1[kk] += gq * sv[t0 + q];
                r2[kk] += gq;
            }
        }
        double p1 = r1[0], p2 = r2[0];
        if constexpr (K == 2) { // lane u: r[2u] + r[2u+1]
            p1 = r1[0] + r1[1];
            p2 = r2[0] + r2[1];
        }
#pragma unroll
        for (int sh = 1; sh < LPU; sh <<= 1) {
            p1 = p1 + __shfl_xor(p1, sh);
            p2 = p2 + __shfl_xor(p2, sh);
        }
        const double gt = gs[N - 1] * cw[NT];
        const double S1 = p1 + gt * sv[NT];
        const double S2 = p2 + gt;
        const double bb = x - Kc;
        const double d = ((-a) * bb + S1) / ((-a) + S2);
        if (u == 0) {
            diff[s] = fabs(x - d);
            img[(size_t)i * w + j] = d;
        }
    };

    // R rounds of NG updates per level are prefetched (update b + grp + r*NG); lanes without
    // an update load update 0's data (a valid cell), so every lane issues the same loads in
    // the same order
    int b = off[0], e = off[1], e2 = nl > 1 ? off[2] : e;
    int s_cur[R], s_nxt[R];
    double cwA[R][NT + 1], cwB[R][NT + 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        s_cur[r] = b + grp + r * NG < e ? ord[b + grp + r * NG] : -1;
        load_cw(s_cur[r] >= 0 ? s_cur[r] : 0, cwA[r]);
        s_nxt[r] = e + grp + r * NG < e2 ? ord[e + grp + r * NG] : -1;
    }
    // one level: uses cwc, prefetches the next level's weights into cwn.  Issue order image
    // loads -> schedule (two levels ahead) -> weights, so that neither the updates nor the
    // end-of-level rotation of s wait for the weights; the weights ping-pong between cwA
    // and cwB (no register copy of a load in flight)
    auto level = [&](int l, double (&cwc)[R][NT + 1], double (&cwn)[R][NT + 1]) {
        const int e3 = l + 2 < nl ? off[l + 3] : e2;
        double sv[R][NT + 2];
#pragma unroll
        for (int r = 0; r < R; ++r) load_sv(s_cur[r] >= 0 ? s_cur[r] : 0, sv[r]);
        __builtin_amdgcn_sched_barrier(0);
        int s_nn[R];
#pragma unroll
        for (int r = 0; r < R; ++r) s_nn[r] = e2 + grp + r * NG < e3 ? ord[e2 + grp + r * NG] : -1;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < R; ++r) load_cw(s_nxt[r] >= 0 ? s_nxt[r] : 0, cwn[r]);
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (s_cur[r] >= 0) update(s_cur[r], cwc[r], sv[r]);
        for (int base = b + R * NG; base < e; base += NG) { // levels wider than R*NG updates
            const int s = base + grp < e ? ord[base + grp] : -1;
            if (s >= 0) {
                double cwv[NT + 1], svv[NT + 2];
                load_cw(s, cwv);
                load_sv(s, svv);
                update(s, cwv, svv);
            }
        }
        __syncthreads();
        b = e;
        e = e2;
        e2 = e3;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            s_cur[r] = s_nxt[r];
            s_nxt[r] = s_nn[r];
        }
    };
    for (int l = 0; l < nl; l += 2) {
        level(l, cwA, cwB);
        if (l + 1 < nl) level(l + 1, cwB, cwA);
    }
}

// pipelined kernels on (DM_GS_PF=0: the one-lane-per-update kernels, for A/B)
static bool gs_pf()
{
    const char *v = getenv("DM_GS_PF");
    return !(v && v[0] == '0');
}
