// Microbenchmark: HBM bandwidth of the block access patterns behind config 5's
// reduce (4 004-B records read at random, 4 000-B shard rows read and written in
// order). Not part of the product; bounds what k_reduce_rows' DEPTH-3 path can
// reach.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_blocks.hip -o gpurun_out/ubench_blocks
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(4)));
#define GL __attribute__((address_space(1)))
__device__ inline u32x4 ld_nt(const uint8_t* p) { return __builtin_nontemporal_load((const GL u32x4_u*)p); }
__device__ inline u32x4 ld(const uint8_t* p) { return *(const GL u32x4_u*)p; }
__device__ inline void st_nt(uint8_t* p, u32x4 v) { __builtin_nontemporal_store(v, (GL u32x4_u*)p); }

// Each wave reads NB blocks (block ids idx[w*NB + k]) of `bsz` bytes at `stride`
// (4 x 1 KiB per lane group, like CPW = 4) and, if ROW, reads and writes row w of
// `rows` (rsz bytes). XOR-folds into sink so nothing is dead.
// Config 4 AdaGrad pattern (k_ada_flat's traffic, bare): a wave owns R = 5
// neighbouring 800-B rows; it reads data and delta, streams the W pushes' 5
// records, and writes data and delta back. SLOT: a dependent per-wave index load
// first (k_ada_flat reads its slot rows before the push loads); PERSIST: a fixed
// grid whose waves walk groups with the next group's index prefetched.
template <int W, bool SLOT, bool PERSIST>
__global__ __launch_bounds__(256) void k_ada(const uint8_t* __restrict__ pushes, int64_t push_bytes,
                                             uint8_t* __restrict__ data, uint8_t* __restrict__ delta,
                                             const int32_t* __restrict__ idx, int64_t nwaves) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t step = PERSIST ? (int64_t)gridDim.x * 4 : nwaves;
    constexpr int R = 5, REC = 804, ROW = 800, J = 4;  // 4 x 64 x 16 B >= 4 000 B
    int32_t nx = (SLOT && w0 < nwaves) ? idx[w0] : (int32_t)w0;
    for (int64_t w = w0; w < nwaves; w += step) {
        const int32_t g = nx;
        if (PERSIST && SLOT && w + step < nwaves) nx = idx[w + step];
        else if (PERSIST) nx = (int32_t)(w + step);
        u32x4 a[J], d[J];
        uint8_t* dp = data + w * (int64_t)(R * ROW);
        uint8_t* ep = delta + w * (int64_t)(R * ROW);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int o = (j * 64 + lane) * 16;
            a[j] = o < R * ROW ? ld_nt(dp + o) : u32x4{0, 0, 0, 0};
            d[j] = o < R * ROW ? ld_nt(ep + o) : u32x4{0, 0, 0, 0};
        }
        u32x4 raw[W][J];
#pragma unroll
        for (int b = 0; b < W; ++b) {
            const uint8_t* bp = pushes + b * push_bytes + (int64_t)g * (R * REC) + 4;
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int o = (j * 64 + lane) * 16;
                raw[b][j] = o < R * REC - 16 ? ld_nt(bp + o) : u32x4{0, 0, 0, 0};
            }
        }
#pragma unroll
        for (int b = 0; b < W; ++b)
#pragma unroll
            for (int j = 0; j < J; ++j) {
                a[j] += raw[b][j];
                d[j] += raw[b][j] * raw[b][j];
            }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int o = (j * 64 + lane) * 16;
            if (o < R * ROW) {
                st_nt(dp + o, a[j]);
                st_nt(ep + o, d[j]);
            }
        }
        if (!PERSIST) break;
    }
}

template <int NB, bool ROW, bool NT>
__global__ __launch_bounds__(128) void k_blocks(const uint8_t* __restrict__ src, const int32_t* __restrict__ idx,
                                                int64_t stride, int bsz, uint8_t* __restrict__ rows, int rsz,
                                                int64_t nwaves, uint32_t* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 2 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    u32x4 acc[4];
    uint8_t* rp = rows + w * (int64_t)rsz;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int o = (c * 64 + lane) * 16;
        acc[c] = (ROW && o < rsz) ? ld_nt(rp + o) : u32x4{0, 0, 0, 0};
    }
    u32x4 raw[NB > 0 ? NB : 1][4];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const uint8_t* bp = src + (int64_t)idx[w * NB + k] * stride + 4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int o = (c * 64 + lane) * 16;
            raw[k][c] = o < bsz ? (NT ? ld_nt(bp + o) : ld(bp + o)) : u32x4{0, 0, 0, 0};
        }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] += raw[k][c];
    if (ROW) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int o = (c * 64 + lane) * 16;
            if (o < rsz) st_nt(rp + o, acc[c]);
        }
    } else {
        uint32_t x = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) x ^= acc[c].x ^ acc[c].y ^ acc[c].z ^ acc[c].w;
        if (x == 0x12345678u) sink[0] = x;
    }
}

// Config 4's pattern (ascending full-range pushes): a wave owns R = 10 neighbouring
// 800-B shard rows; per push it streams the matching 10 records (8 040 contiguous
// bytes) with 16-B loads, then writes its 8 000 shard bytes back. Bare traffic: no
// slot table, no key checks, no ordering.
template <int W>
__global__ __launch_bounds__(256) void k_c4(const uint8_t* __restrict__ pushes, int64_t push_bytes,
                                            uint8_t* __restrict__ shard, int64_t nwaves, uint32_t* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    constexpr int R = 10, REC = 804, ROW = 800, J = 8;  // 8 x 64 x 16 B >= 8 040 B
    u32x4 acc[J];
    uint8_t* sp = shard + w * (int64_t)(R * ROW);
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int o = (j * 64 + lane) * 16;
        acc[j] = o < R * ROW ? ld_nt(sp + o) : u32x4{0, 0, 0, 0};
    }
    for (int b = 0; b < W; ++b) {
        const uint8_t* bp = pushes + b * push_bytes + w * (int64_t)(R * REC) + 4;
        u32x4 raw[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int o = (j * 64 + lane) * 16;
            raw[j] = o < R * REC - 16 ? ld_nt(bp + o) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < J; ++j) acc[j] += raw[j];
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int o = (j * 64 + lane) * 16;
        if (o < R * ROW) st_nt(sp + o, acc[j]);
    }
}

template <int NB, bool ROW, bool NT>
static float run(const char* name, const uint8_t* src, const int32_t* idx, int64_t stride, int bsz, uint8_t* rows,
                 int rsz, int64_t nwaves, uint32_t* sink, double bytes) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned grid = (unsigned)((nwaves + 1) / 2);
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_blocks<NB, ROW, NT>), dim3(grid), dim3(128), 0, 0, src, idx, stride, bsz, rows, rsz,
                           nwaves, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep) best = std::min(best, ms);
    }
    printf("%-44s %8.1f us  %7.1f GB/s\n", name, best * 1e3, bytes / (best * 1e-3) / 1e9);
    return best;
}

int main() {
    const int64_t nblk = 262144;  // config 5: 32 pushes x 8192 records
    const int64_t stride = 4004;
    const int bsz = 4000;
    const int64_t nrows = 125000;
    uint8_t *src, *rows;
    int32_t *iseq, *irnd, *i2;
    uint32_t* sink;
    CK(hipMalloc(&src, nblk * stride + 4096));
    CK(hipMalloc(&rows, nrows * 4000 + 4096));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, nblk * stride + 4096));
    CK(hipMemset(rows, 2, nrows * 4000 + 4096));
    std::vector<int32_t> h(nblk);
    std::iota(h.begin(), h.end(), 0);
    CK(hipMalloc(&iseq, nblk * 4));
    CK(hipMemcpy(iseq, h.data(), nblk * 4, hipMemcpyHostToDevice));
    std::mt19937 g(7);
    std::shuffle(h.begin(), h.end(), g);
    CK(hipMalloc(&irnd, nblk * 4));
    CK(hipMemcpy(irnd, h.data(), nblk * 4, hipMemcpyHostToDevice));
    // config-5 shape: each of 125 000 rows takes 2 random records (~2.1 in config 5)
    CK(hipMalloc(&i2, nrows * 2 * 4));
    CK(hipMemcpy(i2, h.data(), nrows * 2 * 4, hipMemcpyHostToDevice));
    const double rb = (double)nblk * bsz;
    run<1, false, true>("read 4000-B blocks, sequential, nt", src, iseq, stride, bsz, rows, 4000, nblk, sink, rb);
    run<1, false, true>("read 4000-B blocks, random, nt", src, irnd, stride, bsz, rows, 4000, nblk, sink, rb);
    run<1, false, false>("read 4000-B blocks, random, cached", src, irnd, stride, bsz, rows, 4000, nblk, sink, rb);
    run<4, false, true>("read 4 random blocks per wave, nt", src, irnd, stride, bsz, rows, 4000, nblk / 4, sink, rb);
    run<4, false, false>("read 4 random blocks per wave, cached", src, irnd, stride, bsz, rows, 4000, nblk / 4, sink,
                         rb);
    const double c5 = (double)nrows * 2 * bsz + 2.0 * nrows * 4000;
    run<2, true, true>("row RMW + 2 random blocks per wave, nt", src, i2, stride, bsz, rows, 4000, nrows, sink, c5);
    run<2, true, false>("row RMW + 2 random blocks per wave, cached", src, i2, stride, bsz, rows, 4000, nrows, sink,
                        c5);
    run<2, true, false>("row RMW + 2 sequential blocks per wave, cached", src, iseq, stride, bsz, rows, 4000, nrows,
                        sink, c5);
    const double cp = 2.0 * nrows * 4000;
    run<0, true, true>("row RMW only (sequential copy-in-place)", src, iseq, stride, bsz, rows, 4000, nrows, sink, cp);
    // config 4 shard: 8 pushes of 1 250 000 x 804 B, shard 1 250 000 x 800 B
    {
        const int64_t r4 = 1250000, pb = r4 * 804;
        uint8_t *pp, *sh;
        CK(hipMalloc(&pp, 8 * pb + 64));
        CK(hipMalloc(&sh, r4 * 800 + 64));
        CK(hipMemset(pp, 1, 8 * pb + 64));
        CK(hipMemset(sh, 2, r4 * 800 + 64));
        const int64_t nw = r4 / 10;
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        float best = 1e30f;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_c4<8>, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, pp, pb, sh, nw, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep) best = std::min(best, ms);
        }
        const double by = 8.0 * pb + 2.0 * r4 * 800;
        printf("%-44s %8.1f us  %7.1f GB/s\n", "config-4 shard pattern (8 asc pushes, R=10)", best * 1e3,
               by / (best * 1e-3) / 1e9);
    }
    // config 4 AdaGrad: 2 pushes of 10 000 000 x 804 B, data + delta 10 000 000 x 800 B
    {
        const int64_t r4 = 10000000, pb = r4 * 804;
        uint8_t *pp, *da, *de;
        int32_t* ix;
        CK(hipMalloc(&pp, 2 * pb + 64));
        CK(hipMalloc(&da, r4 * 800 + 64));
        CK(hipMalloc(&de, r4 * 800 + 64));
        const int64_t nw = r4 / 5;
        std::vector<int32_t> hi(nw);
        std::iota(hi.begin(), hi.end(), 0);
        CK(hipMalloc(&ix, nw * 4));
        CK(hipMemcpy(ix, hi.data(), nw * 4, hipMemcpyHostToDevice));
        CK(hipMemset(pp, 0, 2 * pb + 64));
        CK(hipMemset(da, 0, r4 * 800 + 64));
        CK(hipMemset(de, 0, r4 * 800 + 64));
        const double by = 2.0 * pb + 4.0 * r4 * 800;
        auto go = [&](const char* name, auto kern, unsigned grid) {
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, pp, pb, da, de, ix, nw);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep) best = std::min(best, ms);
            }
            printf("%-44s %8.1f us  %7.1f GB/s\n", name, best * 1e3, by / (best * 1e-3) / 1e9);
        };
        const unsigned full = (unsigned)((nw + 3) / 4);
        go("ada pattern: 2 pushes, one group per wave", k_ada<2, false, false>, full);
        go("ada pattern: + dependent index load", k_ada<2, true, false>, full);
        go("ada pattern: persistent 256x8 blocks", k_ada<2, false, true>, 2048u);
        go("ada pattern: persistent + index prefetch", k_ada<2, true, true>, 2048u);
        go("ada pattern: persistent 256x12 blocks + idx", k_ada<2, true, true>, 3072u);
        go("ada pattern: persistent 256x4 blocks + idx", k_ada<2, true, true>, 1024u);
    }
    return 0;
}
