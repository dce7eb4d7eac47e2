// Probe of v_mfma_i32_4x4x4_16b_i8 on gfx950: operand / result lane layout and the cycles
// one MFMA holds its SIMD (alone and beside independent VALU work), for the on-demand
// matching kernels' 4-children x 4-windows dot products (k_match_step_l1).
//
//   hipcc -O3 --offload-arch=gfx950 tools/mfma44_probe.hip -o /tmp/mfma44_probe && /tmp/mfma44_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));

// layout: lane l supplies A = a[l] (4 int8) and B = b[l]; D[l][0..3] out
__global__ void k_layout(const int *a, const int *b, v4i *d)
{
    const int l = threadIdx.x;
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_4x4x4i8(a[l], b[l], acc, 0, 0, 0);
    d[l] = acc;
}

// timing: N dependent-free MFMAs (4 accumulators round robin) + V independent v_fma per MFMA
template <int V>
__global__ void k_time(int a0, int b0, long long *cyc, v4i *sink, float *fs)
{
    v4i acc[4] = {{0, 0, 0, 0}, {1, 1, 1, 1}, {2, 2, 2, 2}, {3, 3, 3, 3}};
    float f[8];
    for (int i = 0; i < 8; ++i) f[i] = fs[threadIdx.x] + i;
    const int a = a0 + threadIdx.x, b = b0 - threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < 256; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            acc[k & 3] = __builtin_amdgcn_mfma_i32_4x4x4i8(a + k, b, acc[k & 3], 0, 0, 0);
#pragma unroll
            for (int v = 0; v < V; ++v) f[v & 7] = __builtin_fmaf(f[v & 7], 1.0001f, 0.5f);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
    fs[64 + threadIdx.x] = f[0] + f[1] + f[2] + f[3] + f[4] + f[5] + f[6] + f[7];
}

// the same with v_mfma_i32_16x16x32_i8 (reference point: 11.2 issue cycles beside VALU)
template <int V>
__global__ void k_time16(long a0, long b0, long long *cyc, v4i *sink, float *fs)
{
    v4i acc[4] = {{0, 0, 0, 0}, {1, 1, 1, 1}, {2, 2, 2, 2}, {3, 3, 3, 3}};
    float f[8];
    for (int i = 0; i < 8; ++i) f[i] = fs[threadIdx.x] + i;
    const long a = a0 + threadIdx.x, b = b0 - threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < 256; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            acc[k & 3] = __builtin_amdgcn_mfma_i32_16x16x32_i8(a + k, b, acc[k & 3], 0, 0, 0);
#pragma unroll
            for (int v = 0; v < V; ++v) f[v & 7] = __builtin_fmaf(f[v & 7], 1.0001f, 0.5f);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
    fs[64 + threadIdx.x] = f[0] + f[1] + f[2] + f[3] + f[4] + f[5] + f[6] + f[7];
}

// calibration: the same loop without the MFMA (V independent v_fma per step)
template <int V>
__global__ void k_valu(int a0, int b0, long long *cyc, v4i *sink, float *fs)
{
    float f[8];
    for (int i = 0; i < 8; ++i) f[i] = fs[threadIdx.x] + i + a0 + b0;
    __syncthreads();
#pragma unroll 1
    for (int it = 0; it < 256; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int v = 0; v < V; ++v) f[v & 7] = __builtin_fmaf(f[v & 7], 1.0001f, 0.5f);
        }
    }
    fs[64 + threadIdx.x] = f[0] + f[1] + f[2] + f[3] + f[4] + f[5] + f[6] + f[7];
    (void)cyc; (void)sink;
}

int main()
{
    int ha[64], hb[64];
    // A: lane l holds bytes (l*4 + k) small; B: lane l holds bytes (100 + l) in byte k = (l % 4 == k)
    for (int l = 0; l < 64; ++l) {
        ha[l] = 0;
        hb[l] = 0;
        for (int k = 0; k < 4; ++k) ha[l] |= ((l % 4) * 4 + k + 1) << (8 * k);   // A[i=l%4][k] = 4i+k+1
    }
    int *da, *db;
    v4i *dd;
    hipMalloc(&da, 256); hipMalloc(&db, 256); hipMalloc(&dd, 64 * 16);
    // B = identity-like per lane: lane l holds B[k][j] with j = l % 4 (hypothesis); set B[k][j] = 1 for k == j
    for (int l = 0; l < 64; ++l) hb[l] = 1 << (8 * (l % 4));
    hipMemcpy(da, ha, 256, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, 256, hipMemcpyHostToDevice);
    k_layout<<<1, 64>>>(da, db, dd);
    v4i hd[64];
    hipMemcpy(hd, dd, 64 * 16, hipMemcpyDeviceToHost);
    printf("layout (A[lane] bytes = 4*(lane%%4)+k+1, B[lane] = byte (lane%%4) set to 1):\n");
    for (int l = 0; l < 8; ++l) printf("  lane %2d: %4d %4d %4d %4d\n", l, hd[l][0], hd[l][1], hd[l][2], hd[l][3]);
    // second probe: B[lane] = (lane + 1) in byte 0 only, A[lane] = 1 in byte 0 only -> D = sum over k of A*B
    for (int l = 0; l < 64; ++l) { ha[l] = (l == 5) ? 1 : 0; hb[l] = 0x01010101 * ((l % 16) + 1); }
    hipMemcpy(da, ha, 256, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, 256, hipMemcpyHostToDevice);
    k_layout<<<1, 64>>>(da, db, dd);
    hipMemcpy(hd, dd, 64 * 16, hipMemcpyDeviceToHost);
    printf("probe 2 (A = 1 on lane 5 byte 0 only; B[lane] all bytes (lane%%16)+1):\n");
    for (int l = 0; l < 16; ++l) printf("  lane %2d: %4d %4d %4d %4d\n", l, hd[l][0], hd[l][1], hd[l][2], hd[l][3]);

    long long *dc, hc[1024];
    v4i *sink;
    float *fs;
    // sized for the largest grid below: 4096 one-wave blocks
    hipMalloc(&dc, 8 * 4096); hipMalloc(&sink, (size_t)4096 * 64 * 16); hipMalloc(&fs, 4096);
    hipMemset(fs, 0, 4096);
    auto run = [&](const char *name, auto kern, int waves_per_simd) {
        const int blocks = 256 * 4 * waves_per_simd;   // one-wave blocks spread over 1024 SIMDs
        if (blocks > 4096) { printf("grid too large\n"); return; }
        kern<<<blocks, 64>>>(3, 5, dc, sink, fs);       // warm
        if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed\n", name); return; }
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        kern<<<blocks, 64>>>(3, 5, dc, sink, fs);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(hc, dc, 8 * 1, hipMemcpyDeviceToHost);
        // memtime ticks at 100 MHz; per-MFMA issue cycles from the event time at the clock the
        // SIMD ran: cycles per MFMA per SIMD = ms * 1e-3 * clock / (waves_per_simd * 4096)
        printf("%-28s waves/SIMD %d: %.3f ms for %d MFMAs per wave (%.2f ns per MFMA per SIMD)\n", name,
               waves_per_simd, ms, 4096, ms * 1e6 / (4096.0 * waves_per_simd));
    };
    run("v_fma x8 only (calibration)", k_valu<8>, 4);
    run("4x4x4_16b alone", k_time<0>, 1);
    run("4x4x4_16b alone", k_time<0>, 4);
    run("4x4x4_16b + 2 v_fma", k_time<2>, 4);
    run("4x4x4_16b + 4 v_fma", k_time<4>, 4);
    run("4x4x4_16b + 8 v_fma", k_time<8>, 4);
    run("16x16x32 alone", k_time16<0>, 4);
    run("16x16x32 + 4 v_fma", k_time16<4>, 4);
    run("16x16x32 + 8 v_fma", k_time16<8>, 4);
    return 0;
}
