// Microbenchmark: the dense push-reduce access pattern (shard += Σ W pushes, flat fp32
// arrays, 16-B non-temporal loads and stores) at config 2's and config 4's geometries
// and their crosses, in one process: which of stream count, stream
// spacing, write share, per-wave span and shard size takes config 2's 0.85 of 8 TB/s
// down to config 4's 0.75. Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_geom.hip -o scripts/ubench_geom
//   scripts/ubench_geom [case filter substring] [rounds = 3]
// A case: W pushes of K x S bytes each and an S-byte shard. A wave owns a contiguous
// U-KiB span of the shard and the K x U KiB at the same place of every push (K = 2:
// 16 push streams carrying twice the shard's bytes, i.e. config 2's 2.9 % write share
// at 16 streams); D pushes' loads in flight per wave (D x K x U KiB). Pushes are slices
// of one slab (config 2's receive slab) or one allocation each (config 4's buffers).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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
constexpr int MAXW = 32;
struct Ptrs {
    uint8_t* p[MAXW];
};
__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t n) {
    const uint64_t b = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}
__device__ inline u32x4 addf(u32x4 a, u32x4 b) {
    u32x4 r;
    r.x = __float_as_uint(__uint_as_float(a.x) + __uint_as_float(b.x));
    r.y = __float_as_uint(__uint_as_float(a.y) + __uint_as_float(b.y));
    r.z = __float_as_uint(__uint_as_float(a.z) + __uint_as_float(b.z));
    r.w = __float_as_uint(__uint_as_float(a.w) + __uint_as_float(b.w));
    return r;
}
__device__ inline int64_t xcd_remap() {  // XCD x runs the x-th contiguous run of blocks
    const int64_t nbk = gridDim.x, b = blockIdx.x, per = (nbk + 7) / 8, x = b % 8, i = b / 8;
    const int64_t full = nbk - (per - 1) * 8;
    return x < full ? x * per + i : full * per + (x - full) * (per - 1) + i;
}

// MODE 0: shard read + pushes, shard written in place; 1: pushes only (reads); 2: shard
// read + pushes, no write; 3: shard read + pushes, written to the second shard buffer
// (out of place: the product's speculative chunks, which keep their input for a re-run)
template <int U, int D, int K, int MODE, bool XCD>
__global__ __launch_bounds__(256) void k_geo(Ptrs p, int W, uint8_t* shard, uint8_t* sink) {
    const int64_t blk = XCD ? xcd_remap() : (int64_t)blockIdx.x;
    const int64_t g = blk * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    constexpr uint32_t SB = U * 1024u;
    const auto rs = rsrc(shard + g * SB, SB);
    const auto ro = rsrc((MODE == 3 ? sink : shard) + g * SB, SB);
    u32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        acc[u] = MODE == 1 ? u32x4{0u, 0u, 0u, 0u} : __builtin_amdgcn_raw_buffer_load_b128(rs, u * 1024 + lane * 16, 0, 2);
    for (int b = 0; b < W; b += D) {
        u32x4 v[D][K * U];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const auto rp = rsrc(p.p[b + d] + g * (SB * K), SB * K);
#pragma unroll
            for (int j = 0; j < K * U; ++j) v[d][j] = __builtin_amdgcn_raw_buffer_load_b128(rp, j * 1024 + lane * 16, 0, 2);
        }
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int j = 0; j < K * U; ++j) acc[j % U] = addf(acc[j % U], v[d][j]);
    }
    if (MODE == 0 || MODE == 3) {
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(acc[u], ro, u * 1024 + lane * 16, 0, 2);
    } else {
        uint32_t x = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) x ^= acc[u].x ^ acc[u].y ^ acc[u].z ^ acc[u].w;
        if (x == 0x9e3779b9u) sink[threadIdx.x] = 1;
    }
}

// Config 2's record layout: pushes of 16 384 records [key][1 024 floats], the values
// OFF bytes into a record of STRIDE bytes (the wire: 4 / 4 100, so every 16-B value load
// is 4-B aligned; a padded layout: 16 / 4 112, 16-B aligned); a wave owns 4 rows of
// 4 KiB (the product's k_reduce_rows span), D pushes in flight.
template <int OFF, int STRIDE, int D>
__global__ __launch_bounds__(256) void k_rec(Ptrs p, int W, uint8_t* shard, uint8_t* sink) {
    const int64_t blk = xcd_remap();
    const int64_t g = blk * 4 + (threadIdx.x >> 6);  // wave -> rows 4g .. 4g + 3
    const int lane = threadIdx.x & 63;
    const auto rs = rsrc(shard + g * 4 * 4096, 4 * 4096);
    u32x4 acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (j >> 2) * 4096 + ((j & 3) * 64 + lane) * 16, 0, 2);
    for (int b = 0; b < W; b += D) {
        u32x4 v[D][16];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const auto rp = rsrc(p.p[b + d] + g * 4 * STRIDE, 4 * STRIDE);
#pragma unroll
            for (int j = 0; j < 16; ++j)
                v[d][j] = __builtin_amdgcn_raw_buffer_load_b128(rp, (j >> 2) * STRIDE + OFF + ((j & 3) * 64 + lane) * 16, 0, 2);
        }
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] = addf(acc[j], v[d][j]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) __builtin_amdgcn_raw_buffer_store_b128(acc[j], rs, (j >> 2) * 4096 + ((j & 3) * 64 + lane) * 16, 0, 2);
}

__global__ void k_fill(uint8_t* p, int64_t n, uint32_t seed) {
    for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 16; i < n; i += (int64_t)gridDim.x * blockDim.x * 16) {
        u32x4 v{(seed ^ (uint32_t)(i >> 4)) & 0x3fffffffu | 0x30000000u, 0x33800000u, 0x34000000u, 0x2f800000u};
        *(u32x4*)(p + i) = v;
    }
}

typedef void (*KernFn)(Ptrs, int, uint8_t*, uint8_t*);
struct Kern {
    KernFn f;
    int U, D, K, mode;
    bool xcd;
};
#define KN(U, D, K, M, X) Kern{k_geo<U, D, K, M, X>, U, D, K, M, X}

struct Geo {  // one allocation set
    int W, K;
    int64_t S;
    bool slab;
    std::vector<uint8_t*> allocs;
    Ptrs p{};
    uint8_t* shard = nullptr;
    uint8_t* shard2 = nullptr;  // out-of-place output (MODE 3)
};

static void alloc_geo(Geo& g) {
    const int64_t P = g.S * g.K;
    if (g.slab) {
        uint8_t* s;
        CK(hipMalloc(&s, P * g.W));
        g.allocs.push_back(s);
        for (int b = 0; b < g.W; ++b) g.p.p[b] = s + P * b;
    } else {
        for (int b = 0; b < g.W; ++b) {
            CK(hipMalloc(&g.p.p[b], P));
            g.allocs.push_back(g.p.p[b]);
        }
    }
    CK(hipMalloc(&g.shard, g.S));
    g.allocs.push_back(g.shard);
    CK(hipMalloc(&g.shard2, g.S));
    g.allocs.push_back(g.shard2);
    for (int b = 0; b < g.W; ++b) hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, g.p.p[b], P, 17u * b + 3u);
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, g.shard, g.S, 99u);
    CK(hipDeviceSynchronize());
}
static void free_geo(Geo& g) {
    for (auto* a : g.allocs) CK(hipFree(a));
    g.allocs.clear();
}

static uint8_t* g_sink;
static hipEvent_t e0, e1;

// times `reps` launches one at a time; returns best and mean (us)
static void time_case(const Geo& g, const Kern& k, int reps, float& best, float& mean) {
    const int64_t spans = g.S / (k.U * 1024LL);
    const unsigned grid = (unsigned)(spans / 4);
    best = 1e30f;
    float sum = 0.f;
    for (int it = 0; it <= reps; ++it) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, g.p, g.W, g.shard, k.mode == 3 ? g.shard2 : g_sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0) {
            sum += ms;
            if (ms < best) best = ms;
        }
    }
    best *= 1e3f;
    mean = sum / reps * 1e3f;
}

static void report(const char* label, const Geo& g, const Kern& k, int round, float best, float mean) {
    const double P = (double)g.S * g.K;
    const double bytes = g.W * P + (k.mode != 1 ? g.S : 0) + (k.mode == 0 || k.mode == 3 ? g.S : 0);
    const double wshare = k.mode == 0 || k.mode == 3 ? g.S / bytes : 0.0;
    printf("{\"case\": \"%s\", \"round\": %d, \"W\": %d, \"push_bytes\": %.0f, \"shard_bytes\": %lld, \"layout\": \"%s\", "
           "\"U_KiB_per_wave\": %d, \"D\": %d, \"K\": %d, \"mode\": \"%s\", \"xcd\": %d, \"write_share\": %.4f, "
           "\"best_us\": %.1f, \"mean_us\": %.1f, \"frac_best\": %.4f, \"frac_mean\": %.4f}\n",
           label, round, g.W, P, (long long)g.S, g.slab ? "slab" : "separate", k.U, k.D, k.K,
           k.mode == 0 ? "rmw" : k.mode == 1 ? "push reads only" : k.mode == 2 ? "shard+push reads" : "out of place", (int)k.xcd, wshare, best, mean,
           bytes / best / 1e3 / 8000.0, bytes / mean / 1e3 / 8000.0);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const char* filt = argc > 1 ? argv[1] : "";
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    CK(hipMalloc(&g_sink, 4096));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t MiB = 1LL << 20;
    const Kern base = KN(4, 4, 1, 0, true), base16 = KN(4, 4, 2, 0, true);
    struct Case {
        const char* label;
        int W, K;
        int64_t S;
        bool slab;
        std::vector<Kern> kerns;
        int reps;
    };
    std::vector<Case> cases = {
        // config 2: 32 x 64 MiB pushes in one slab -> 64 MiB shard
        {"g2: 32 x 64 MiB slab", 32, 1, 64 * MiB, true,
         {base, KN(4, 4, 1, 3, true), KN(4, 4, 1, 1, true), KN(4, 4, 1, 2, true), KN(4, 4, 1, 0, false), KN(2, 8, 1, 0, true), KN(8, 2, 1, 0, true),
          KN(16, 1, 1, 0, true)},
         20},
        {"g2 separate: 32 x 64 MiB", 32, 1, 64 * MiB, false, {base}, 20},
        // per-wave span beyond k_reduce_rows' 16 KiB (4 rows x 4 KiB): 32 KiB, one push in flight
        {"span: 32 x 64 MiB slab", 32, 1, 64 * MiB, true, {KN(16, 1, 1, 0, true), KN(32, 1, 1, 0, true), KN(16, 1, 1, 0, true), KN(32, 1, 1, 0, true)}, 20},
        // the write share of config 4 (1/18) at config 2's footprint
        {"x: 16 x 64 MiB slab", 16, 1, 64 * MiB, true, {base, KN(4, 4, 1, 1, true)}, 20},
        // shard size sweep (the 256 MiB Infinity Cache), config 2's 32 pushes and write share
        {"mall: 32 x 128 MiB slab", 32, 1, 128 * MiB, true, {base}, 10},
        {"mall: 32 x 256 MiB slab", 32, 1, 256 * MiB, true, {base}, 10},
        {"mall: 32 x 512 MiB slab", 32, 1, 512 * MiB, true, {base, KN(4, 4, 1, 1, true)}, 6},
        {"mall: 32 x 1 GiB slab", 32, 1, 1024 * MiB, true, {base, KN(4, 4, 1, 3, true), KN(4, 4, 1, 1, true)}, 5},
        {"mall: 16 x 1 GiB slab", 16, 1, 1024 * MiB, true, {base, KN(4, 4, 1, 1, true)}, 5},
        // 16 streams at config 2's write share (each push twice the shard's bytes)
        {"x: 16 x 2 GiB slab, 1 GiB shard (K 2)", 16, 2, 1024 * MiB, true, {base16, KN(4, 4, 2, 1, true)}, 5},
        {"x: 16 x 128 MiB slab, 64 MiB shard (K 2)", 16, 2, 64 * MiB, true, {base16}, 20},
        // 32 streams spaced 4 GB apart (separate allocations)
        {"x: 32 x 4 GB separate", 32, 1, 4000 * MiB, false, {base, KN(4, 4, 1, 1, true)}, 3},
        // config 4: 16 x 8 GB separate allocations -> 8 GB shard
        {"g4: 16 x 8 GB separate", 16, 1, 7630 * MiB, false,
         {base, KN(4, 4, 1, 3, true), KN(4, 4, 1, 1, true), KN(4, 4, 1, 2, true), KN(4, 4, 1, 0, false), KN(2, 8, 1, 0, true), KN(8, 2, 1, 0, true),
          KN(16, 1, 1, 0, true)},
         3},
        {"g4 slab: 16 x 8 GB slab", 16, 1, 7630 * MiB, true, {base}, 3},
    };
    // config 2's record layouts against the flat stream, alternated in one process
    if (!strcmp(filt, "rec")) {
        const int64_t R = 16384;
        uint8_t *slab4, *slab16, *shard;
        CK(hipMalloc(&slab4, 32 * R * 4100 + 4096));
        CK(hipMalloc(&slab16, 32 * R * 4112 + 4096));
        CK(hipMalloc(&shard, R * 4096));
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, slab4, 32 * R * 4100 / 16 * 16, 5u);
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, slab16, 32 * R * 4112 / 16 * 16, 6u);
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, shard, R * 4096, 7u);
        Geo flat{32, 1, 64 << 20, true};
        alloc_geo(flat);
        Ptrs p4{}, p16{};
        for (int b = 0; b < 32; ++b) {
            p4.p[b] = slab4 + b * R * 4100;
            p16.p[b] = slab16 + b * R * 4112;
        }
        CK(hipDeviceSynchronize());
        const double bytes4 = 32.0 * R * 4100 + 2.0 * R * 4096, bytes16 = 32.0 * R * 4112 + 2.0 * R * 4096;
        const unsigned grid = (unsigned)(R / 16);
        auto timeit = [&](auto kern, const Ptrs& pp, double bytes, const char* name, int r) {
            float best = 1e30f;
            for (int it = 0; it <= 50; ++it) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, pp, 32, shard, g_sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it > 0 && ms < best) best = ms;
            }
            printf("{\"case\": \"%s\", \"round\": %d, \"best_us\": %.1f, \"frac_best\": %.4f}\n", name, r, best * 1e3,
                   bytes / (best * 1e-3) / 1e9 / 8000.0);
            fflush(stdout);
        };
        for (int r = 0; r < rounds; ++r) {
            timeit(k_rec<4, 4100, 2>, p4, bytes4, "rec: values 4 B into 4100-B records (wire), D 2", r);
            timeit(k_rec<16, 4112, 2>, p16, bytes16, "rec: values 16 B into 4112-B records (aligned), D 2", r);
            timeit(k_rec<4, 4100, 1>, p4, bytes4, "rec: values 4 B into 4100-B records (wire), D 1", r);
            float best, mean;
            const Kern wide = KN(16, 1, 1, 0, true);
            time_case(flat, wide, 50, best, mean);
            report("rec: flat 32 x 64 MiB slab", flat, wide, r, best, mean);
        }
        return 0;
    }
    // same-process alternation of the two geometries (both resident): g2, g4, g2, g4 ...
    if (!strcmp(filt, "alt")) {
        Geo a{32, 1, 64 * MiB, true}, b{16, 1, 7630 * MiB, false};
        alloc_geo(a);
        alloc_geo(b);
        const Kern wide = KN(16, 1, 1, 0, true);  // 16 KiB per wave per push (config 2's k_reduce_rows span)
        for (int r = 0; r < rounds; ++r) {
            float best, mean;
            time_case(a, base, 50, best, mean);
            report("alt g2: 32 x 64 MiB slab", a, base, r, best, mean);
            time_case(a, wide, 50, best, mean);
            report("alt g2: 32 x 64 MiB slab", a, wide, r, best, mean);
            time_case(b, wide, 4, best, mean);
            report("alt g4: 16 x 8 GB separate", b, wide, r, best, mean);
            time_case(b, base, 4, best, mean);
            report("alt g4: 16 x 8 GB separate", b, base, r, best, mean);
            const Kern oop = KN(4, 4, 1, 3, true);
            time_case(b, oop, 4, best, mean);
            report("alt g4: 16 x 8 GB separate", b, oop, r, best, mean);
        }
        free_geo(a);
        free_geo(b);
        return 0;
    }
    for (int r = 0; r < rounds; ++r) {
        for (auto& c : cases) {
            if (!strstr(c.label, filt)) continue;
            Geo g{c.W, c.K, c.S, c.slab};
            alloc_geo(g);
            for (auto& k : c.kerns) {
                if (g.S % (k.U * 4096LL)) {
                    fprintf(stderr, "case %s: shard not a multiple of the block span\n", c.label);
                    exit(2);
                }
                float best, mean;
                time_case(g, k, c.reps, best, mean);
                report(c.label, g, k, r, best, mean);
            }
            free_geo(g);
        }
    }
    return 0;
}
