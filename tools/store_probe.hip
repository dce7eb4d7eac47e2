// Store-pattern probe for the level-0 volume kernels (k_volume_ls): how fast 16-B-per-lane
// stores can fill a level-0 volume of T tiles of side S (T x S^2 patch maps of S^2 values of
// esz bytes) in
//   seq   : each wave streams its own contiguous slab of 16 maps, 1 KB per store instruction
//   vol   : k_volume_ls's pattern -- a wave owns 16 patches (4 lane groups x 4 accumulator rows);
//           per image row and accumulator row, S*esz/256 stores of 4 x 256 B into 4 patch maps,
//           the maps advancing S*esz bytes per row (rows of one map are consecutive)
//   vol4  : four image rows per burst
//   volx  : k_volume_ls's patches and order, but each store instruction 1 KB of ONE patch map
//           (lane group g writes the map's 256-B chunk 4k + g): the pattern a cross-lane-group
//           transpose of four rows' results would give
//   volh  : the same with 2 x 512 B per instruction (two lane groups per map)
// each with plain or nontemporal stores, 8 waves per workgroup as k_volume_ls.  No arithmetic:
// the rate each pattern allows the write path.  One JSON line per shape on stdout.
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o tools/store_probe.bin
//   ./tools/store_probe.bin [shape...]  (c3_f16, c3_f32, c5_f16, c5_f32; default all)
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

template <bool NT>
__device__ __forceinline__ void st16(char *p, v4u v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, (v4u *)p);
    else *(v4u *)p = v;
}

// one wave = 16 patches x all rows; RB image rows per store burst; ROT: each workgroup starts
// its row sweep at its own row ((block * 37) mod S) and wraps, so the workgroups of the chip
// are at different offsets inside their maps at any moment
template <int RB, bool NT, bool ROT = false>
__global__ __launch_bounds__(512) void k_vol(char *vol, int S, int esz)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane & 15, grp = lane >> 4;
    const size_t P = (size_t)S * S, mapb = P * esz, rowb = (size_t)S * esz;
    const size_t blk = (size_t)blockIdx.x * 8 + wave;        // 16-patch block (2x2 level-1 cells)
    const size_t bpt = (size_t)(S / 4) * (S / 4);
    const size_t t = blk / bpt, bi = blk % bpt;
    const int I0 = 2 * (int)(bi / (S / 4)), J0 = 2 * (int)(bi % (S / 4));
    const int Ic = I0 + (grp >> 1), Jc = J0 + (grp & 1);
    char *out[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const size_t p = (size_t)(2 * Ic + (r >> 1)) * S + 2 * Jc + (r & 1);
        out[r] = vol + (t * P + p) * mapb + c * 16;
    }
    const v4u v = {(unsigned)lane, 1u, 2u, 3u};
    const int per_row = (int)(rowb / 256);
    const int off = ROT ? (int)((blockIdx.x * 37u) % (unsigned)S) & ~(RB - 1) : 0;
    for (int q00 = 0; q00 < S; q00 += RB) {
        const int q0 = (q00 + off) % S;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            for (int k = 0; k < RB; ++k)
                for (int j = 0; j < per_row; ++j) st16<NT>(out[r] + (size_t)(q0 + k) * rowb + j * 256, v);
    }
}

template <bool NT, int RUN = 4>
__global__ __launch_bounds__(512) void k_volx(char *vol, int S, int esz)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane & 15, grp = lane >> 4;
    const size_t P = (size_t)S * S, mapb = P * esz;
    const size_t blk = (size_t)blockIdx.x * 8 + wave;
    const size_t bpt = (size_t)(S / 4) * (S / 4);
    const size_t t = blk / bpt, bi = blk % bpt;
    const int I0 = 2 * (int)(bi / (S / 4)), J0 = 2 * (int)(bi % (S / 4));
    const v4u v = {(unsigned)lane, 1u, 2u, 3u};
    const int chunks = (int)(mapb / 256);
    // RUN = 4: lane group g writes chunk q + g of patch pp (1 KB of one map per instruction);
    // RUN = 2: lane groups 2h, 2h + 1 write chunks q, q + 1 of patch (pp + h) (2 x 512 B)
    for (int q = 0; q < chunks; q += RUN) {
#pragma unroll
        for (int pp = 0; pp < 16; pp += 4 / RUN) {
            const int pq = RUN == 4 ? pp : pp + (grp >> 1);
            const int g = pq >> 2, r = pq & 3;
            const size_t p = (size_t)(2 * (I0 + (g >> 1)) + (r >> 1)) * S + 2 * (J0 + (g & 1)) + (r & 1);
            st16<NT>(vol + (t * P + p) * mapb + (size_t)(q + (grp % RUN)) * 256 + c * 16, v);
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(512) void k_seq(char *vol, size_t slab)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t blk = (size_t)blockIdx.x * 8 + wave;
    char *base = vol + blk * slab + lane * 16;
    const v4u v = {(unsigned)lane, 1u, 2u, 3u};
    for (size_t o = 0; o < slab; o += 1024) st16<NT>(base + o, v);
}

int main(int argc, char **argv)
{
    struct Shape { const char *name; int S, T, esz; };
    const Shape all[] = {{"c3_f16", 128, 64, 2}, {"c3_f32", 128, 64, 4}, {"c5_f16", 256, 8, 2},
                         {"c5_f32", 256, 4, 4}};
    // argv: shape names to run (default: all)
    Shape shapes[4];
    int ns = 0;
    for (const Shape &sh : all) {
        bool want = argc < 2;
        for (int i = 1; i < argc; ++i) want = want || strcmp(argv[i], sh.name) == 0;
        if (want) shapes[ns++] = sh;
    }
    size_t maxb = 0;
    for (int i = 0; i < ns; ++i) {
        const Shape &sh = shapes[i];
        const size_t b = (size_t)sh.T * sh.S * sh.S * sh.S * sh.S * sh.esz;
        maxb = b > maxb ? b : maxb;
    }
    char *vol;
    CK(hipMalloc(&vol, maxb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < ns; ++i) {
        const Shape &sh = shapes[i];
        const size_t P = (size_t)sh.S * sh.S, bytes = (size_t)sh.T * P * P * sh.esz;
        const unsigned grid = (unsigned)((size_t)sh.T * (sh.S / 4) * (sh.S / 4) / 8);
        const size_t slab = 16 * P * sh.esz;
        printf("{\"shape\": \"%s\", \"S\": %d, \"tiles\": %d, \"bytes\": %zu", sh.name, sh.S, sh.T, bytes);
        auto run = [&](const char *name, auto fn) {
            float best = 1e30f;
            for (int i = 0; i < 6; ++i) {
                CK(hipEventRecord(e0, 0));
                fn();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (i) best = ms < best ? ms : best;
            }
            printf(", \"%s\": {\"ms\": %.3f, \"gb_s\": %.1f}", name, best, bytes / (best * 1e-3) / 1e9);
        };
        run("seq", [&] { k_seq<false><<<grid, 512>>>(vol, slab); });
        run("seq_nt", [&] { k_seq<true><<<grid, 512>>>(vol, slab); });
        run("vol", [&] { k_vol<1, false><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("vol_nt", [&] { k_vol<1, true><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("vol_rot_nt", [&] { k_vol<1, true, true><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("vol_rot", [&] { k_vol<1, false, true><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("vol4", [&] { k_vol<4, false><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("vol4_nt", [&] { k_vol<4, true><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("volx", [&] { k_volx<false><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("volx_nt", [&] { k_volx<true><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("volh", [&] { k_volx<false, 2><<<grid, 512>>>(vol, sh.S, sh.esz); });
        run("volh_nt", [&] { k_volx<true, 2><<<grid, 512>>>(vol, sh.S, sh.esz); });
        printf("}\n");
        fflush(stdout);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(vol));
    return 0;
}
