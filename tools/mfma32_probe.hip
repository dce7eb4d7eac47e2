// Operand / result layout of v_mfma_i32_32x32x32_i8 on gfx950, as k_level1_mfq's strip sweep
// (dm_mfma.h, "Row-pair strips") assumes it: lane L holds row (A) / column (B) L & 31 and
// K bytes 16 (L >> 5) .. +15 (the same K order for A and B); result register r of lane L is
// C[8 (r >> 2) + 4 (L >> 5) + (r & 3)][L & 31].  Random int8 operands, checked on the host.
//
//   hipcc -O2 --offload-arch=gfx950 tools/mfma32_probe.hip -o /tmp/mfma32_probe && /tmp/mfma32_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const signed char *A, const signed char *B, int *C)
{
    const int L = threadIdx.x, i = L & 31, h = L >> 5;
    v4i a, b;
    signed char *pa = (signed char *)&a, *pb = (signed char *)&b;
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[i * 32 + 16 * h + j];   // A[row i][k]
        pb[j] = B[(16 * h + j) * 32 + i]; // B[k][col i]
    }
    const v16i z = {};
    const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, z, 0, 0, 0);
    for (int r = 0; r < 16; ++r) C[(8 * (r >> 2) + 4 * h + (r & 3)) * 32 + i] = c[r];
}

int main()
{
    signed char hA[1024], hB[1024];
    int hC[1024];
    srand(7);
    for (int x = 0; x < 1024; ++x) { hA[x] = (signed char)(rand() & 255); hB[x] = (signed char)(rand() & 255); }
    signed char *dA, *dB;
    int *dC;
    if (hipMalloc(&dA, 1024) || hipMalloc(&dB, 1024) || hipMalloc(&dC, 4096)) return 2;
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipMemset(dC, 0, 4096);
    k<<<1, 64>>>(dA, dB, dC);
    hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int s = 0;
            for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[kk * 32 + j];
            if (s != hC[i * 32 + j] && bad++ < 5) printf("C[%d][%d] = %d, expected %d\n", i, j, hC[i * 32 + j], s);
        }
    printf("mfma32_probe: %d of 1024 results differ from the assumed layout\n", bad);
    return bad != 0;
}
