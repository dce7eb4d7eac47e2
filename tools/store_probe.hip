// Store-pattern probe for the level-0 volume kernels (k_volume_ls): how fast can 16-B-per-lane
// stores fill a 34 GB binary16 volume (64 tiles of S=128: 64 x 16384 patches x 32 KB maps) in
//   seq   : each wave streams its own contiguous slab, 1 KB per store instruction
//   vol   : k_volume_ls's pattern -- a wave owns 16 patches (4 lane groups x 4 accumulator rows),
//           per image row one store per accumulator row: 4 x 256 B at 4 patch maps, the maps
//           advancing 256 B per row (rows of one patch map are consecutive)
//   vol2  : the same with two image rows per store burst (512 B per patch map per burst)
//   vol4  : four image rows per burst (1 KB per patch map)
// each with plain or nontemporal stores, 8 waves per workgroup as k_volume_ls.  No compute:
// the rate each pattern allows the write path.
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o tools/store_probe.bin
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr int S = 128, P = S * S, T = 64;           // C3 batch
constexpr size_t MAPB = (size_t)P * 2;              // one patch map, binary16: 32 KB
constexpr size_t VOLB = (size_t)T * P * MAPB;       // 34.4 GB

template <bool NT>
__device__ __forceinline__ void st16(char *p, v4u v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, (v4u *)p);
    else *(v4u *)p = v;
}

// one wave = 16 patches x all rows; RB rows per store burst
template <int RB, bool NT>
__global__ __launch_bounds__(512) void k_vol(char *vol)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane & 15, grp = lane >> 4;
    const size_t blk = (size_t)blockIdx.x * 8 + wave;        // 16-patch block
    const size_t bpt = (size_t)(S / 4) * (S / 4);
    const size_t t = blk / bpt, bi = blk % bpt;
    const int I0 = 2 * (int)(bi / (S / 4)), J0 = 2 * (int)(bi % (S / 4));
    const int Ic = I0 + (grp >> 1), Jc = J0 + (grp & 1);
    char *out[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const size_t p = (size_t)(2 * Ic + (r >> 1)) * S + 2 * Jc + (r & 1);
        out[r] = vol + (t * P + p) * MAPB + c * 16;
    }
    const v4u v = {(unsigned)lane, 1u, 2u, 3u};
    for (int q0 = 0; q0 < S; q0 += RB) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < RB; ++k) st16<NT>(out[r] + (size_t)(q0 + k) * 256, v);
    }
}

// each wave streams a contiguous slab of 16 x 32 KB, 1 KB per store instruction
template <bool NT>
__global__ __launch_bounds__(512) void k_seq(char *vol)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t blk = (size_t)blockIdx.x * 8 + wave;
    char *base = vol + blk * 16 * MAPB + lane * 16;
    const v4u v = {(unsigned)lane, 1u, 2u, 3u};
    for (size_t o = 0; o < 16 * MAPB; o += 1024) st16<NT>(base + o, v);
}

int main()
{
    char *vol;
    if (hipMalloc(&vol, VOLB) != hipSuccess) { fprintf(stderr, "hipMalloc %zu failed\n", VOLB); return 1; }
    const unsigned grid = (unsigned)((size_t)T * (S / 4) * (S / 4) / 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct V { const char *name; void (*launch)(char *, unsigned); };
    auto run = [&](const char *name, auto fn) {
        float best = 1e30f, sum = 0.0f;
        for (int i = 0; i < 6; ++i) {
            hipEventRecord(e0, 0);
            fn();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (i) { best = ms < best ? ms : best; sum += ms; }
        }
        printf("%-10s best %7.3f ms  mean %7.3f ms  %6.2f TB/s (best)\n", name, best, sum / 5, VOLB / (best * 1e-3) / 1e12);
        fflush(stdout);
    };
    run("seq", [&] { k_seq<false><<<grid, 512>>>(vol); });
    run("seq-nt", [&] { k_seq<true><<<grid, 512>>>(vol); });
    run("vol", [&] { k_vol<1, false><<<grid, 512>>>(vol); });
    run("vol-nt", [&] { k_vol<1, true><<<grid, 512>>>(vol); });
    run("vol2", [&] { k_vol<2, false><<<grid, 512>>>(vol); });
    run("vol2-nt", [&] { k_vol<2, true><<<grid, 512>>>(vol); });
    run("vol4", [&] { k_vol<4, false><<<grid, 512>>>(vol); });
    run("vol4-nt", [&] { k_vol<4, true><<<grid, 512>>>(vol); });
    hipError_t err = hipDeviceSynchronize();
    if (err != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(err)); return 1; }
    hipFree(vol);
    return 0;
}
