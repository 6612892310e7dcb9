// Microbenchmark: HBM rate of streaming kernels by read:write mix, unroll, grid shape and
// cache policy — the ceilings k_ada_flat (4 reads : 2 writes per element), k_flat_ident
// (17 : 1) and a plain copy (1 : 1) run against. Not part of the
// product.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_mix.hip -o scripts/ubench_mix
//   scripts/ubench_mix [GiB per array = 2] [case filter substring]
// K_mix<NR, NO, U, LP, SP, INPLACE, PERSIST>: NR arrays read, NO written (in place: the
// first NO of the read arrays; else NO separate arrays); a thread owns U 16-B vectors
// 256 apart within its block's tile; LP / SP = buffer-instruction cache policy of the
// loads / stores (0 default, 2 nt, 16 sc1, 18 nt sc1); PERSIST: a grid of 2048 blocks
// walks the tiles, else one block per tile.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int MAXA = 20;
struct Arr {
    uint8_t* p[MAXA];
};
__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t n) {
    const uint64_t b = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}
__device__ inline u32x4 addu(u32x4 a, u32x4 b) {
    u32x4 r;
    r.x = __float_as_uint(__uint_as_float(a.x) + __uint_as_float(b.x));
    r.y = __float_as_uint(__uint_as_float(a.y) + __uint_as_float(b.y));
    r.z = __float_as_uint(__uint_as_float(a.z) + __uint_as_float(b.z));
    r.w = __float_as_uint(__uint_as_float(a.w) + __uint_as_float(b.w));
    return r;
}

__device__ inline int64_t xcd_remap();
template <int NR, int NO, int U, int LP, int SP, bool INPLACE, bool PERSIST, bool SYNC = false, bool XCD = false>
__global__ __launch_bounds__(256) void k_mix(Arr a, Arr o, int64_t ntiles) {
    constexpr uint32_t TILE = 256u * U * 16u;
    for (int64_t t = XCD ? xcd_remap() : (int64_t)blockIdx.x; t < ntiles; t += PERSIST ? gridDim.x : ntiles) {
        const int64_t base = t * (int64_t)TILE;
        u32x4 acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = u32x4{0u, 0u, 0u, 0u};
        u32x4 v[NR][U];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const auto rs = rsrc(a.p[r] + base, TILE);
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[r][u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((u * 256 + threadIdx.x) * 16), 0, LP);
        }
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = addu(acc[u], v[r][u]);
        if (SYNC) __syncthreads();
        if (NO == 0) {  // reads only: keep the loads live
            uint32_t x = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) x ^= acc[u].x ^ acc[u].y ^ acc[u].z ^ acc[u].w;
            if (x == 0x9e3779b9u) o.p[0][threadIdx.x] = 1;
        }
#pragma unroll
        for (int w = 0; w < NO; ++w) {
            const auto rs = rsrc((INPLACE ? a.p[w] : o.p[w]) + base, TILE);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u32x4 x = acc[u];
                x.x += (uint32_t)w;  // distinct bytes per output
                __builtin_amdgcn_raw_buffer_store_b128(x, rs, (int)((u * 256 + threadIdx.x) * 16), 0, SP);
            }
        }
    }
}

// AdaGrad-shaped stream: data += u0 + u1 and delta += u0^2 + u1^2 per element (two
// pushes, in place), with k_ada_flat's per-element bookkeeping (last strict rise, last
// delta above 1, maxDelta candidate with its position, reduced per wave) when BOOK; REC:
// the pushes are 804-B records ([4-B key][200 floats]) as in config 4, else flat arrays.
__device__ inline int64_t xcd_remap() {  // XCD x runs the x-th contiguous run of blocks
    const int64_t nbk = gridDim.x, b = blockIdx.x, per = (nbk + 7) / 8, x = b % 8, i = b / 8;
    const int64_t full = nbk - (per - 1) * 8;
    return x < full ? x * per + i : full * per + (x - full) * (per - 1) + i;
}
template <int U, bool BOOK, bool REC, bool XCD = false>
__global__ __launch_bounds__(256) void k_adalike(Arr a, Arr o, int64_t ntiles) {
    constexpr uint32_t TILE = 256u * U * 16u;
    const int64_t t = XCD ? xcd_remap() : (int64_t)blockIdx.x;
    const int64_t base = t * (int64_t)TILE;
    const auto rd = rsrc(a.p[0] + base, TILE), rl = rsrc(a.p[1] + base, TILE);
    // record layout: element index i = base/4 + (u*256 + tid)*4 -> row i / 200, col i % 200
    __amdgpu_buffer_rsrc_t rp[2];
    uint32_t poff[U];
    const int64_t e0 = base / 4, row0 = e0 / 200;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t e = e0 + (int64_t)(u * 256 + threadIdx.x) * 4;
        poff[u] = REC ? (uint32_t)((e / 200 - row0) * 804 + 4 + (e % 200) * 4) : (uint32_t)((u * 256 + threadIdx.x) * 16);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) rp[b] = REC ? rsrc(a.p[2 + b] + row0 * 804, TILE / 200 * 804 + 2 * 804) : rsrc(a.p[2 + b] + base, TILE);
    u32x4 d[U], l[U], q[2][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        d[u] = __builtin_amdgcn_raw_buffer_load_b128(rd, (int)((u * 256 + threadIdx.x) * 16), 0, 2);
        l[u] = __builtin_amdgcn_raw_buffer_load_b128(rl, (int)((u * 256 + threadIdx.x) * 16), 0, 2);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) q[b][u] = __builtin_amdgcn_raw_buffer_load_b128(rp[b], (int)poff[u], 0, 2);
    float cv = 0.f;
    uint64_t cp = ~0ull;
    bool cok = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        float acc[4], dl[4], lg[4] = {0, 0, 0, 0}, rv[4] = {0, 0, 0, 0};
        int rb[4] = {-1, -1, -1, -1};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            acc[e] = __uint_as_float(d[u][e]);
            dl[e] = __uint_as_float(l[u][e]);
        }
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = __uint_as_float(q[b][u][e]);
                acc[e] = __fadd_rn(acc[e], x);
                const float nd = __fadd_rn(dl[e], __fmul_rn(x, x));
                if (BOOK) {
                    if (nd > dl[e]) { rv[e] = nd; rb[e] = b; }
                    if (nd > 1.0f) lg[e] = nd;
                }
                dl[e] = nd;
            }
        u32x4 od, ol;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            od[e] = __float_as_uint(acc[e]);
            ol[e] = __float_as_uint(dl[e]);
        }
        __builtin_amdgcn_raw_buffer_store_b128(od, rd, (int)((u * 256 + threadIdx.x) * 16), 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(ol, rl, (int)((u * 256 + threadIdx.x) * 16), 0, 2);
        if (BOOK) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (lg[e] > 1.0f) o.p[0][(base + (u * 256 + threadIdx.x) * 16 + e * 4) & 0xFFFF] = 1;
                if (rb[e] < 0) continue;
                const uint64_t p = ((uint64_t)rb[e] << 40) | (uint64_t)(poff[u] + e * 4);
                if (!cok || rv[e] > cv || (rv[e] == cv && p < cp)) { cok = true; cv = rv[e]; cp = p; }
            }
        }
    }
    if (BOOK) {
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
            const float ov = __shfl_xor(cv, m);
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)cp, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(cp >> 32), m);
            const bool ook = __shfl_xor((int)cok, m) != 0;
            const uint64_t op = (uint64_t)lo | ((uint64_t)hi << 32);
            if (ook && (!cok || ov > cv || (ov == cv && op < cp))) { cok = true; cv = ov; cp = op; }
        }
        if ((threadIdx.x & 63) == 0) *(uint64_t*)(o.p[1] + (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16) = cp ^ __float_as_uint(cv);
    }
}

__global__ void k_fill(uint8_t* p, int64_t n, uint32_t seed) {
    for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 16; i < n; i += (int64_t)gridDim.x * blockDim.x * 16) {
        u32x4 v{seed ^ (uint32_t)i, 0x3f800000u, (uint32_t)(i >> 7), 0x3f000000u};
        *(u32x4*)(p + i) = v;
    }
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 2.0;
    const char* filt = argc > 2 ? argv[2] : "";
    const int64_t n = (int64_t)(gib * (1 << 30)) / (1 << 20) * (1 << 20);  // bytes per array, MiB multiple
    Arr a{}, o{};
    for (int i = 0; i < 17; ++i) {
        CK(hipMalloc(&a.p[i], n + n / 128 + (1 << 20)));  // room for 804-B records of n / 4 floats
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, a.p[i], n, 11u * i + 1u);
    }
    for (int i = 0; i < 2; ++i) CK(hipMalloc(&o.p[i], n));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto kern, int nr, int no, int U, bool persist) {
        if (!strstr(name, filt)) return;
        const int64_t tile = 256LL * U * 16;
        const int64_t ntiles = n / tile;
        const unsigned grid = persist ? 2048u : (unsigned)ntiles;
        const double bytes = (double)(nr + no) * ntiles * tile;
        float best = 1e30f, sum = 0.f;
        for (int it = 0; it < 7; ++it) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, o, ntiles);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 0) {
                sum += ms;
                if (ms < best) best = ms;
            }
        }
        printf("{\"kernel\": \"%s\", \"reads\": %d, \"writes\": %d, \"GiB_per_array\": %.2f, \"best_us\": %.1f, "
               "\"mean_us\": %.1f, \"GBps_best\": %.1f, \"frac_best\": %.4f}\n",
               name, nr, no, gib, best * 1e3, sum / 6 * 1e3, bytes / best / 1e6, bytes / best / 1e6 / 8000.0);
        fflush(stdout);
    };
    if (!strcmp(filt, "boundary")) {
        // Kernel boundary cost: 50 back-to-back launches of a 256 MiB read-only pass,
        // plain launches against hipExtLaunchKernelGGL carrying a completion event (the
        // store's per-chunk `applied`), and one carrying start + stop events.
        const int64_t nb = 256LL << 20, tiles = nb / (256 * 4 * 16);
        hipEvent_t ev[2];
        CK(hipEventCreate(&ev[0]));
        CK(hipEventCreate(&ev[1]));
        hipEvent_t evd;
        CK(hipEventCreateWithFlags(&evd, hipEventDisableTiming));
        for (int mode = 0; mode < 4; ++mode) {
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(e0));
                for (int i = 0; i < 50; ++i) {
                    if (mode == 0)
                        hipLaunchKernelGGL((k_mix<1, 0, 4, 2, 0, false, false>), dim3((unsigned)tiles), dim3(256), 0, 0, a, o, tiles);
                    else if (mode == 1)
                        hipExtLaunchKernelGGL((k_mix<1, 0, 4, 2, 0, false, false>), dim3((unsigned)tiles), dim3(256), 0, 0,
                                              nullptr, ev[i & 1], 0, a, o, tiles);
                    else if (mode == 2)
                        hipExtLaunchKernelGGL((k_mix<1, 0, 4, 2, 0, false, false>), dim3((unsigned)tiles), dim3(256), 0, 0,
                                              ev[0], ev[1], 0, a, o, tiles);
                    else {
                        hipLaunchKernelGGL((k_mix<1, 0, 4, 2, 0, false, false>), dim3((unsigned)tiles), dim3(256), 0, 0, a, o, tiles);
                        CK(hipEventRecord(evd, 0));
                    }
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            static const char* nm[] = {"plain launches", "ext launch + completion event", "ext launch + start/stop events",
                                       "plain launch + hipEventRecord (no timing)"};
            printf("{\"kernel\": \"boundary: %s\", \"launches\": 50, \"bytes_each\": %lld, \"us_per_launch\": %.2f}\n", nm[mode],
                   (long long)nb, best * 1e3 / 50);
            fflush(stdout);
        }
        return 0;
    }
    // reads only
    run("read1 U4 nt", k_mix<1, 0, 4, 2, 0, false, false>, 1, 0, 4, false);
    run("read1 U4 default", k_mix<1, 0, 4, 0, 0, false, false>, 1, 0, 4, false);
    // copy 1:1
    run("copy U1 ld def st def", k_mix<1, 1, 1, 0, 0, false, false>, 1, 1, 1, false);
    run("copy U4 ld def st def", k_mix<1, 1, 4, 0, 0, false, false>, 1, 1, 4, false);
    run("copy U4 ld nt st def", k_mix<1, 1, 4, 2, 0, false, false>, 1, 1, 4, false);
    run("copy U4 ld nt st nt", k_mix<1, 1, 4, 2, 2, false, false>, 1, 1, 4, false);
    run("copy U4 ld def st nt", k_mix<1, 1, 4, 0, 2, false, false>, 1, 1, 4, false);
    run("copy U4 ld nt st sc1", k_mix<1, 1, 4, 2, 16, false, false>, 1, 1, 4, false);
    run("copy U4 ld nt st ntsc1", k_mix<1, 1, 4, 2, 18, false, false>, 1, 1, 4, false);
    run("copy U8 ld nt st nt", k_mix<1, 1, 8, 2, 2, false, false>, 1, 1, 8, false);
    run("copy U4 ld nt st nt persist", k_mix<1, 1, 4, 2, 2, false, true>, 1, 1, 4, true);
    run("copy U4 ld def st def persist", k_mix<1, 1, 4, 0, 0, false, true>, 1, 1, 4, true);
    run("copy in place U4 ld nt st nt", k_mix<1, 1, 4, 2, 2, true, false>, 1, 1, 4, false);
    run("copy in place U4 ld def st def", k_mix<1, 1, 4, 0, 0, true, false>, 1, 1, 4, false);
    // 2 : 1 (a += b)
    run("r2w1 in place U4 nt nt", k_mix<2, 1, 4, 2, 2, true, false>, 2, 1, 4, false);
    run("r2w1 in place U4 def def", k_mix<2, 1, 4, 0, 0, true, false>, 2, 1, 4, false);
    run("r2w1 out U4 nt nt", k_mix<2, 1, 4, 2, 2, false, false>, 2, 1, 4, false);
    // 4 : 2 in place (AdaGrad: data, delta, two pushes -> data, delta)
    run("r4w2 in place U2 nt nt", k_mix<4, 2, 2, 2, 2, true, false>, 4, 2, 2, false);
    run("r4w2 in place U4 nt nt", k_mix<4, 2, 4, 2, 2, true, false>, 4, 2, 4, false);
    run("r4w2 in place U4 def def", k_mix<4, 2, 4, 0, 0, true, false>, 4, 2, 4, false);
    run("r4w2 in place U4 def nt", k_mix<4, 2, 4, 0, 2, true, false>, 4, 2, 4, false);
    run("r4w2 in place U4 nt def", k_mix<4, 2, 4, 2, 0, true, false>, 4, 2, 4, false);
    run("r4w2 in place U4 nt sc1", k_mix<4, 2, 4, 2, 16, true, false>, 4, 2, 4, false);
    run("r4w2 in place U4 nt nt sync", k_mix<4, 2, 4, 2, 2, true, false, true>, 4, 2, 4, false);
    run("r4w2 in place U4 nt nt persist", k_mix<4, 2, 4, 2, 2, true, true>, 4, 2, 4, true);
    run("r4w2 out U4 nt nt", k_mix<4, 2, 4, 2, 2, false, false>, 4, 2, 4, false);
    run("ada U4 plain", k_adalike<4, false, false>, 4, 2, 4, false);
    run("ada U4 book", k_adalike<4, true, false>, 4, 2, 4, false);
    run("ada U4 rec", k_adalike<4, false, true>, 4, 2, 4, false);
    run("ada U4 book rec", k_adalike<4, true, true>, 4, 2, 4, false);
    run("ada U2 book rec", k_adalike<2, true, true>, 4, 2, 2, false);
    run("ada U4 book rec xcd", k_adalike<4, true, true, true>, 4, 2, 4, false);
    run("ada U4 plain xcd", k_adalike<4, false, false, true>, 4, 2, 4, false);
    run("r4w2 in place U4 nt nt xcd", k_mix<4, 2, 4, 2, 2, true, false, false, true>, 4, 2, 4, false);
    run("r17w1 in place U2 nt nt xcd", k_mix<17, 1, 2, 2, 2, true, false, false, true>, 17, 1, 2, false);
    // 17 : 1 (sixteen pushes + shard -> shard)
    run("r17w1 in place U2 nt nt", k_mix<17, 1, 2, 2, 2, true, false>, 17, 1, 2, false);
    run("r17w1 in place U2 nt nt sync", k_mix<17, 1, 2, 2, 2, true, false, true>, 17, 1, 2, false);
    run("r17w1 out U2 nt nt", k_mix<17, 1, 2, 2, 2, false, false>, 17, 1, 2, false);
    run("r16 reads U2 nt", k_mix<16, 0, 2, 2, 0, false, false>, 16, 0, 2, false);
    return 0;
}
