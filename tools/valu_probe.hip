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
    hipFree(d);
    return 0;
}
