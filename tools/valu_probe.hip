// VALU issue-rate probe: wave64 throughput of f32 FMA, packed f32 FMA, f64 FMA, f64 mul,
// i32 ops and f32->f64 converts on gfx950, 8 independent chains per lane so the issue rate
// (not the latency) bounds each loop.  Prints ns per wave-instruction per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_probe.hip -o /tmp/valu_probe && /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096, CH = 8;

template <int K>
__global__ __launch_bounds__(256) void probe(float *out, float a, float b)
{
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
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
    printf("%-10s %8.3f ms  %.3f ns/wave-inst/SIMD  (%.2f G wave-inst/s)\n", name, ms,
           ms * 1e6 / (insts / 1024.0), insts / (ms * 1e6));
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
    hipFree(d);
    return 0;
}
