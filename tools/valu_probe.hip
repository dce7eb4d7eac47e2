// VALU issue-rate probe: wave64 throughput of f32 FMA, packed f32 FMA, f64 FMA, f64 mul,
// i32 ops and f32->f64 converts on gfx950, 8 independent chains per lane so the issue rate
// (not the latency) bounds each loop.  Prints ns per wave-instruction per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_probe.hip -o /tmp/valu_probe && /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096, CH = 8;

__device__ long long g_clk[4];

template <int K>
__global__ __launch_bounds__(256) void probe(float *out, float a, float b)
{
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    long long c0 = 0, w0 = 0;
    if (tid == 0) { c0 = clock64(); w0 = wall_clock64(); }
    if constexpr (K == 0) { // f32 fma
        float v[CH];
        for (int c = 0; c < CH; ++c) v[c] = tid * 1e-9f + c;
        for (int it = 0; it < ITER; ++it)
#pragma unroll
            for (int c = 0; c < CH; ++c) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[c]) : "v"(a), "v"(b));
        float s = 0; for (int c = 0; c < CH; ++c) s += v[c];
        out[tid] = s;
    } else if constexpr (K == 1) { // packed f32 fma
        f2 v[CH];
        for (int c = 0; c < CH; ++c) v[c] = f2{tid * 1e-9f + c, (float)c};
        const f2 A = {a, a}, B = {b, b};
        for (int it = 0; it < ITER; ++it)
#pragma unroll
            for (int c = 0; c < CH; ++c) v[c] = __builtin_elementwise_fma(v[c], A, B);
        float s = 0; for (int c = 0; c < CH; ++c) s += v[c].x + v[c].y;
        out[tid] = s;
    } else if constexpr (K == 2) { // f64 fma
        double v[CH];
        for (int c = 0; c < CH; ++c) v[c] = tid * 1e-9 + c;
        const double A = a, B = b;
        for (int it = 0; it < ITER; ++it)
#pragma unroll
            for (int c = 0; c < CH; ++c) v[c] = __builtin_fma(v[c], A, B);
        double s = 0; for (int c = 0; c < CH; ++c) s += v[c];
        out[tid] = (float)s;
    } else if constexpr (K == 3) { // f64 mul
        double v[CH];
        for (int c = 0; c < CH; ++c) v[c] = tid * 1e-9 + c;
        const double A = a;
        for (int it = 0; it < ITER; ++it)
#pragma unroll
            for (int c = 0; c < CH; ++c) v[c] = v[c] * A;
        double s = 0; for (int c = 0; c < CH; ++c) s += v[c];
        out[tid] = (float)s;
    } else if constexpr (K == 4) { // i32 xor/add chain
        unsigned v[CH];
        const unsigned A = __float_as_uint(a), B = __float_as_uint(b);
        for (int c = 0; c < CH; ++c) v[c] = tid + c;
        for (int it = 0; it < ITER; ++it)
#pragma unroll
            for (int c = 0; c < CH; ++c) v[c] = (v[c] ^ A) + B;
        unsigned s = 0; for (int c = 0; c < CH; ++c) s += v[c];
        out[tid] = (float)s;
    } else { // f32 -> f64 -> f32 converts
        float v[CH];
        for (int c = 0; c < CH; ++c) v[c] = tid * 1e-9f + c;
        for (int it = 0; it < ITER; ++it)
#pragma unroll
            for (int c = 0; c < CH; ++c) { double t; asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(t) : "v"(v[c])); asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(v[c]) : "v"(t)); }
        float s = 0; for (int c = 0; c < CH; ++c) s += v[c];
        out[tid] = s + a;
    }
    if (tid == 0) { g_clk[0] = clock64() - c0; g_clk[1] = wall_clock64() - w0; }
}

// one VALU instruction per chain step, 8 independent chains (v = op(v, a, b))
#define ASM_PROBE(NAME, INSN)                                                                    \
    __global__ __launch_bounds__(256) void NAME(float *out, float a, float b)                     \
    {                                                                                            \
        const int tid = blockIdx.x * blockDim.x + threadIdx.x;                                   \
        long long c0 = 0, w0 = 0;                                                                \
        if (tid == 0) { c0 = clock64(); w0 = wall_clock64(); }                                   \
        float v[CH];                                                                             \
        for (int c = 0; c < CH; ++c) v[c] = tid * 1e-9f + c;                                     \
        for (int it = 0; it < ITER; ++it)                                                        \
            _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(INSN : "+v"(v[c]) : "v"(a), "v"(b)); \
        float s = 0;                                                                             \
        for (int c = 0; c < CH; ++c) s += v[c];                                                  \
        out[tid] = s;                                                                            \
        if (tid == 0) { g_clk[0] = clock64() - c0; g_clk[1] = wall_clock64() - w0; }             \
    }
ASM_PROBE(p_mul_f32, "v_mul_f32 %0, %0, %1")
ASM_PROBE(p_add_f32, "v_add_f32 %0, %0, %1")
ASM_PROBE(p_max3_f32, "v_max3_f32 %0, %0, %1, %2")
ASM_PROBE(p_med3_f32, "v_med3_f32 %0, %0, %1, %2")
ASM_PROBE(p_max_f32, "v_max_f32 %0, %0, %1")
ASM_PROBE(p_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
ASM_PROBE(p_and_b32, "v_and_b32 %0, %0, %1")
ASM_PROBE(p_lshr_b32, "v_lshrrev_b32 %0, 3, %0")
ASM_PROBE(p_and_or_b32, "v_and_or_b32 %0, %0, %1, %2")
ASM_PROBE(p_lshl_add_u32, "v_lshl_add_u32 %0, %0, 2, %1")
ASM_PROBE(p_bfe_u32, "v_bfe_u32 %0, %0, 3, 9")
ASM_PROBE(p_mov_dpp, "v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
ASM_PROBE(p_permlane32, "v_permlane32_swap_b32 %0, %0")
ASM_PROBE(p_cvt_f32_i32, "v_cvt_f32_i32 %0, %0")
ASM_PROBE(p_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
ASM_PROBE(p_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
ASM_PROBE(p_and_lit, "v_and_b32 %0, 0xff0, %0")
ASM_PROBE(p_mul_inl, "v_mul_f32 %0, 0.5, %0")
ASM_PROBE(p_mov_b32, "v_mov_b32 %0, %1")
// round 3: candidates for the level kernel's pow and pooling
ASM_PROBE(p_frexp_mant, "v_frexp_mant_f32 %0, %0")
ASM_PROBE(p_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xc8")
ASM_PROBE(p_max_i32, "v_max_i32 %0, %0, %1")
ASM_PROBE(p_min_u32, "v_min_u32 %0, %0, %1")
ASM_PROBE(p_or_b32, "v_or_b32 %0, %0, %1")
ASM_PROBE(p_xor_b32, "v_xor_b32 %0, %0, %1")
ASM_PROBE(p_add_u32, "v_add_u32 %0, %0, %1")
ASM_PROBE(p_mul_i24, "v_mul_i32_i24 %0, %0, %1")
ASM_PROBE(p_max_dpp, "v_max_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf")
ASM_PROBE(p_cvt_pk_f16, "v_cvt_pk_f16_f32 %0, %0, %1")
ASM_PROBE(p_sub_f32, "v_sub_f32 %0, %0, %1")
ASM_PROBE(p_min_f32, "v_min_f32 %0, %0, %1")
ASM_PROBE(p_min3_f32, "v_min3_f32 %0, %0, %1, %2")
ASM_PROBE(p_ldexp_f32, "v_ldexp_f32 %0, %0, 1")
ASM_PROBE(p_cvt_u32_f32, "v_cvt_u32_f32 %0, %0")

// 64-bit operand probes: v = op(v, A, B) on VGPR pairs
#define ASM_PROBE64(NAME, INSN)                                                                  \
    __global__ __launch_bounds__(256) void NAME(float *out, float a, float b)                     \
    {                                                                                            \
        const int tid = blockIdx.x * blockDim.x + threadIdx.x;                                   \
        long long c0 = 0, w0 = 0;                                                                \
        if (tid == 0) { c0 = clock64(); w0 = wall_clock64(); }                                   \
        double v[CH];                                                                            \
        const double A = a, B = b;                                                               \
        for (int c = 0; c < CH; ++c) v[c] = tid * 1e-9 + c;                                      \
        for (int it = 0; it < ITER; ++it)                                                        \
            _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(INSN : "+v"(v[c]) : "v"(A), "v"(B)); \
        double s = 0; for (int c = 0; c < CH; ++c) s += v[c];                                    \
        out[tid] = (float)s;                                                                     \
        if (tid == 0) { g_clk[0] = clock64() - c0; g_clk[1] = wall_clock64() - w0; }             \
    }
ASM_PROBE64(p_max_f64, "v_max_f64 %0, %0, %1")
ASM_PROBE64(p_add_f64, "v_add_f64 %0, %0, %1")
ASM_PROBE64(p_mov_b64, "v_mov_b64 %0, %1")
ASM_PROBE64(p_fma_f64_v, "v_fma_f64 %0, %0, %1, %2")

// MFMA beside plain VALU: one v_mfma_i32_16x16x64_i8 (4 rotating accumulators) and NV
// independent v_fma_f32 per step; time per step against NV shows how many VALU issue cycles
// an MFMA takes from its SIMD
template <int NV>
__global__ __launch_bounds__(256) void p_mfma_mix(float *out, float a, float b)
{
    typedef int v4i __attribute__((ext_vector_type(4)));
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    long long c0 = 0, w0 = 0;
    if (tid == 0) { c0 = clock64(); w0 = wall_clock64(); }
    v4i A = {tid, tid + 1, tid + 2, tid + 3}, B = {3 * tid, 5, 7, 9};
    v4i acc[4] = {};
    float v[8];
    for (int c = 0; c < 8; ++c) v[c] = tid * 1e-9f + c;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            acc[k] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, acc[k], 0, 0, 0);
#pragma unroll
            for (int c = 0; c < NV; ++c) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[c % 8]) : "v"(a), "v"(b));
        }
    }
    float s = 0; for (int c = 0; c < 8; ++c) s += v[c];
    for (int k = 0; k < 4; ++k) s += (float)(acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3]);
    out[tid] = s;
    if (tid == 0) { g_clk[0] = clock64() - c0; g_clk[1] = wall_clock64() - w0; }
}

// the same with other MFMA shapes: K = 0 bf16 16x16x32, 1 f16 16x16x32, 2 i8 32x32x32,
// 3 bf16 32x32x16 (one instruction per step, 4 rotating accumulators)
template <int K, int NV>
__global__ __launch_bounds__(256) void p_mfma_mix2(float *out, float a, float b)
{
    typedef int v4i __attribute__((ext_vector_type(4)));
    typedef float v4f __attribute__((ext_vector_type(4)));
    typedef int v16i __attribute__((ext_vector_type(16)));
    typedef float v16f __attribute__((ext_vector_type(16)));
    typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
    typedef _Float16 v8h __attribute__((ext_vector_type(8)));
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    long long c0 = 0, w0 = 0;
    if (tid == 0) { c0 = clock64(); w0 = wall_clock64(); }
    v4i A = {tid, tid + 1, tid + 2, tid + 3}, B = {3 * tid, 5, 7, 9};
    v4f acc4[4] = {};
    v16i acci[4] = {};
    v16f accf[4] = {};
    float v[8];
    for (int c = 0; c < 8; ++c) v[c] = tid * 1e-9f + c;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (K == 0)
                acc4[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, A), __builtin_bit_cast(v8bf, B), acc4[k], 0, 0, 0);
            else if constexpr (K == 1)
                acc4[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, A), __builtin_bit_cast(v8h, B), acc4[k], 0, 0, 0);
            else if constexpr (K == 2)
                acci[k] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, acci[k], 0, 0, 0);
            else if constexpr (K == 4) {  // i8 16x16x32 (8-byte operands)
                typedef int v4i_ __attribute__((ext_vector_type(4)));
                v4i_ r = __builtin_bit_cast(v4i_, acc4[k]);
                r = __builtin_amdgcn_mfma_i32_16x16x32_i8(((long)A.y << 32) | (unsigned)A.x, ((long)B.y << 32) | (unsigned)B.x, r, 0, 0, 0);
                acc4[k] = __builtin_bit_cast(v4f, r);
            }
            else
                accf[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, A), __builtin_bit_cast(v8bf, B), accf[k], 0, 0, 0);
#pragma unroll
            for (int c = 0; c < NV; ++c) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[c % 8]) : "v"(a), "v"(b));
        }
    }
    float s = 0; for (int c = 0; c < 8; ++c) s += v[c];
    for (int k = 0; k < 4; ++k) {
        s += acc4[k][0] + accf[k][0] + accf[k][15] + (float)(acci[k][0] + acci[k][15]);
    }
    out[tid] = s;
    if (tid == 0) { g_clk[0] = clock64() - c0; g_clk[1] = wall_clock64() - w0; }
}

static void run_mix(const char *name, void (*k)(float *, float, float), float *d, int nv)
{
    const int blocks = 256 * 8 * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<<<blocks, 256>>>(d, 1.0000001f, 1e-7f);
    hipEventRecord(e0);
    k<<<blocks, 256>>>(d, 1.0000001f, 1e-7f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double steps = blocks * 4.0 * ITER * 4; // wave-steps (one MFMA + nv VALU each)
    long long clk[4];
    hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk));
    int wclk = 0;
    hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);
    const double ghz = (double)clk[0] / ((double)clk[1] / (wclk * 1e3)) / 1e9;
    const double ns = ms * 1e6 / (steps / 1024.0);
    printf("%-14s %8.3f ms  %.3f ns/step/SIMD  block-0 clock %.2f GHz -> %.2f cycles per (mfma + %d v_fma_f32)\n",
           name, ms, ns, ghz, ns * ghz, nv);
}

static void run_k(const char *name, void (*k)(float *, float, float), float *d)
{
    const int blocks = 256 * 8 * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<<<blocks, 256>>>(d, 1.0000001f, 1e-7f);
    hipEventRecord(e0);
    k<<<blocks, 256>>>(d, 1.0000001f, 1e-7f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double insts = blocks * 4.0 * ITER * CH;
    long long clk[4];
    hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk));
    int wclk = 0;
    hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);
    const double ghz = (double)clk[0] / ((double)clk[1] / (wclk * 1e3)) / 1e9;
    const double ns = ms * 1e6 / (insts / 1024.0);
    printf("%-14s %8.3f ms  %.3f ns/wave-inst/SIMD  block-0 clock %.2f GHz -> %.2f cycles\n", name, ms, ns, ghz,
           ns * ghz);
}

template <int K>
static void run(const char *name, int insts_per_iter_chain, float *d)
{
    const int blocks = 256 * 8 * 4; // 8 waves/CU-ish per SIMD mix: 2048*4 workgroups of 4 waves
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    probe<K><<<blocks, 256>>>(d, 1.0000001f, 1e-7f);
    hipEventRecord(e0);
    probe<K><<<blocks, 256>>>(d, 1.0000001f, 1e-7f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0, insts = waves * ITER * CH * insts_per_iter_chain;
    // 1024 SIMDs; per-SIMD ns per wave-instruction
    long long clk[4];
    hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk));
    int wclk = 0;
    hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0); // kHz
    const double ghz = (double)clk[0] / ((double)clk[1] / (wclk * 1e3)) / 1e9;
    const double ns = ms * 1e6 / (insts / 1024.0);
    printf("%-12s %8.3f ms  %.3f ns/wave-inst/SIMD  block-0 clock %.2f GHz -> %.2f cycles\n", name, ms, ns,
           ghz, ns * ghz);
}

int main()
{
    float *d;
    hipMalloc(&d, 256 * 8192 * sizeof(float) * 4);
    run<0>("f32_fma", 1, d);
    run<1>("pk_fma_f32", 1, d);
    run<2>("f64_fma", 1, d);
    run<3>("f64_mul", 1, d);
    run<4>("i32_xor_add", 2, d);
    run<5>("cvt_f32_f64", 2, d);
    run_k("mul_f32", p_mul_f32, d);
    run_k("add_f32", p_add_f32, d);
    run_k("max_f32", p_max_f32, d);
    run_k("max3_f32", p_max3_f32, d);
    run_k("med3_f32", p_med3_f32, d);
    run_k("cndmask_b32", p_cndmask, d);
    run_k("and_b32", p_and_b32, d);
    run_k("lshrrev_b32", p_lshr_b32, d);
    run_k("and_or_b32", p_and_or_b32, d);
    run_k("lshl_add_u32", p_lshl_add_u32, d);
    run_k("bfe_u32", p_bfe_u32, d);
    run_k("mov_b32_dpp", p_mov_dpp, d);
    run_k("permlane32_swap", p_permlane32, d);
    run_k("cvt_f32_i32", p_cvt_f32_i32, d);
    run_k("mul_lo_u32", p_mul_lo_u32, d);
    run_k("mad_u32_u24", p_mad_u32_u24, d);
    run_k("and_b32 lit", p_and_lit, d);
    run_k("mul_f32 inl", p_mul_inl, d);
    run_k("mov_b32", p_mov_b32, d);
    run_k("frexp_mant", p_frexp_mant, d);
    run_k("bitop3_b32", p_bitop3, d);
    run_k("max_i32", p_max_i32, d);
    run_k("min_u32", p_min_u32, d);
    run_k("or_b32", p_or_b32, d);
    run_k("xor_b32", p_xor_b32, d);
    run_k("add_u32", p_add_u32, d);
    run_k("mul_i32_i24", p_mul_i24, d);
    run_k("max_f32_dpp", p_max_dpp, d);
    run_k("cvt_pk_f16", p_cvt_pk_f16, d);
    run_k("sub_f32", p_sub_f32, d);
    run_k("min_f32", p_min_f32, d);
    run_k("min3_f32", p_min3_f32, d);
    run_k("ldexp_f32", p_ldexp_f32, d);
    run_k("cvt_u32_f32", p_cvt_u32_f32, d);
    run_k("max_f64", p_max_f64, d);
    run_k("add_f64", p_add_f64, d);
    run_k("mov_b64", p_mov_b64, d);
    run_k("fma_f64 vvv", p_fma_f64_v, d);
    run_mix("mfma+0", p_mfma_mix<0>, d, 0);
    run_mix("mfma+2", p_mfma_mix<2>, d, 2);
    run_mix("mfma+4", p_mfma_mix<4>, d, 4);
    run_mix("mfma+6", p_mfma_mix<6>, d, 6);
    run_mix("mfma+8", p_mfma_mix<8>, d, 8);
    run_mix("mfma+12", p_mfma_mix<12>, d, 12);
    const char *nm[5] = {"bf16_16x32", "f16_16x32", "i8_32x32x32", "bf16_32x16", "i8_16x16x32"};
    run_mix(nm[4], p_mfma_mix2<4, 0>, d, 0); run_mix(nm[4], p_mfma_mix2<4, 4>, d, 4); run_mix(nm[4], p_mfma_mix2<4, 8>, d, 8);
    run_mix(nm[0], p_mfma_mix2<0, 0>, d, 0); run_mix(nm[0], p_mfma_mix2<0, 4>, d, 4); run_mix(nm[0], p_mfma_mix2<0, 8>, d, 8);
    run_mix(nm[1], p_mfma_mix2<1, 0>, d, 0); run_mix(nm[1], p_mfma_mix2<1, 4>, d, 4); run_mix(nm[1], p_mfma_mix2<1, 8>, d, 8);
    run_mix(nm[2], p_mfma_mix2<2, 0>, d, 0); run_mix(nm[2], p_mfma_mix2<2, 8>, d, 8); run_mix(nm[2], p_mfma_mix2<2, 16>, d, 16);
    run_mix(nm[3], p_mfma_mix2<3, 0>, d, 0); run_mix(nm[3], p_mfma_mix2<3, 8>, d, 8); run_mix(nm[3], p_mfma_mix2<3, 16>, d, 16);
    hipFree(d);
    return 0;
}
