// Microbenchmark: config 4's stream (shard += Σ 16 pushes, 8 GB shard, flat fp32, 16-B
// non-temporal loads and stores) with the shard writes of the whole chip gathered into
// phases. DESIGN.md §4.2 measured that writes interleaved with this read stream cost the
// DRAM ~2 TB/s marginal against ~7 for reads; k_flat_ident already bursts each block's
// writes behind a block barrier. Here every block of a co-resident grid (cooperative
// launch) reads its tile(s), waits at a grid barrier, then writes: between barriers the
// DRAM sees reads only, then writes only. Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_phase.hip -o scripts/ubench_phase
//   scripts/ubench_phase [rounds = 3]
// Cases (one JSON line each): tile (k_flat_ident's shape: 8 waves x 8 vectors per lane,
// a ring of 3 pushes, block barrier, burst store), phased T (persistent, T tiles per
// block per epoch: the first in registers, the others stashed in LDS), reads only,
// writes only. The grid barrier's spin is bounded: a timed-out wait sets an error flag
// and the kernel runs on (wrong values, no hang).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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
constexpr int W = 16, NW = 8, J = 8, D = 3;
constexpr uint32_t TILE = NW * J * 1024;  // bytes of shard per block tile (64 KiB)
struct Ptrs {
    const uint8_t* p[W];
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
__device__ inline int64_t xcd_remap() {
    const int64_t nbk = gridDim.x, b = blockIdx.x, per = (nbk + 7) / 8, x = b % 8, i = b / 8;
    const int64_t full = nbk - (per - 1) * 8;
    return x < full ? x * per + i : full * per + (x - full) * (per - 1) + i;
}

// one tile: the wave's 8 KiB of the shard plus the same 8 KiB of every push, pushes in
// order with a ring of D in flight
template <bool STORE_READS>
__device__ inline void tile_reduce(u32x4 (&acc)[J], const Ptrs& p, uint8_t* shard, int64_t t, int wid, int lane) {
    const int64_t off = t * TILE + (int64_t)wid * J * 1024;
    const auto rs = rsrc(shard + off, J * 1024);
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, j * 1024 + lane * 16, 0, 2);
    u32x4 ring[D][J];
    auto issue = [&](int b, u32x4 (&r)[J]) {
        const auto rp = rsrc(p.p[b] + off, J * 1024);
#pragma unroll
        for (int j = 0; j < J; ++j) r[j] = __builtin_amdgcn_raw_buffer_load_b128(rp, j * 1024 + lane * 16, 0, 2);
    };
#pragma unroll
    for (int d = 0; d < D - 1; ++d) issue(d, ring[d]);
#pragma unroll 1
    for (int b0 = 0; b0 < W; b0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int b = b0 + d, bn = b + D - 1;
            if (bn < W) issue(bn, ring[(d + D - 1) % D]);
            if (b < W)
#pragma unroll
                for (int j = 0; j < J; ++j) acc[j] = addf(acc[j], ring[d][j]);
        }
    }
}
__device__ inline void tile_store(const u32x4 (&acc)[J], uint8_t* shard, int64_t t, int wid, int lane) {
    const auto rs = rsrc(shard + t * TILE + (int64_t)wid * J * 1024, J * 1024);
#pragma unroll
    for (int j = 0; j < J; ++j) __builtin_amdgcn_raw_buffer_store_b128(acc[j], rs, j * 1024 + lane * 16, 0, 2);
}

// MODE 0: read + burst store (k_flat_ident's shape); 1: reads only; 2: stores only
template <int MODE>
__global__ __launch_bounds__(NW * 64) void k_tile(Ptrs p, uint8_t* shard, int64_t ntiles, uint32_t* sink) {
    const int64_t t = xcd_remap();
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    u32x4 acc[J];
    if (MODE == 2) {
#pragma unroll
        for (int j = 0; j < J; ++j) acc[j] = u32x4{(uint32_t)t, 0u, 0u, 0u};
    } else {
        tile_reduce<false>(acc, p, shard, t, wid, lane);
    }
    __syncthreads();
    if (MODE == 1) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) x ^= acc[j].x ^ acc[j].y ^ acc[j].z ^ acc[j].w;
        if (x == 0x9e3779b9u) sink[threadIdx.x] = x;
        return;
    }
    tile_store(acc, shard, t, wid, lane);
}

// grid barrier over a device counter (vector atomics and loads only); bounded spin
__device__ inline void grid_sync(uint32_t* cnt, uint32_t target, uint32_t* err) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t v = 0;
        for (int spin = 0; spin < (1 << 22); ++spin) {
            v = __hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (v >= target || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (v < target) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
}

// persistent, T tiles per block per epoch (tile 0 in registers, tiles 1.. in LDS), one
// grid barrier between each epoch's reads and its writes
template <int T>
__global__ __launch_bounds__(NW * 64) void k_phased(Ptrs p, uint8_t* shard, int64_t ntiles, uint32_t* cnt,
                                                      uint32_t* err) {
    extern __shared__ u32x4 stash[];  // (T - 1) x NW x J x 64 vectors
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int64_t G = gridDim.x, b = xcd_remap();
    const int64_t per_epoch = G * T, nepoch = (ntiles + per_epoch - 1) / per_epoch;
    for (int64_t e = 0; e < nepoch; ++e) {
        u32x4 acc[J];
        // tiles of this block in epoch e: e*G*T + k*G + b (k = 0..T-1)
        for (int k = T - 1; k >= 0; --k) {
            const int64_t t = e * per_epoch + (int64_t)k * G + b;
            if (t < ntiles) tile_reduce<false>(acc, p, shard, t, wid, lane);
            if (k > 0) {
#pragma unroll
                for (int j = 0; j < J; ++j) stash[(((k - 1) * NW + wid) * J + j) * 64 + lane] = acc[j];
            }
        }
        grid_sync(cnt, (uint32_t)(G * (e + 1)), err);
        for (int k = 0; k < T; ++k) {
            const int64_t t = e * per_epoch + (int64_t)k * G + b;
            if (t >= ntiles) continue;
            if (k > 0) {
#pragma unroll
                for (int j = 0; j < J; ++j) acc[j] = stash[(((k - 1) * NW + wid) * J + j) * 64 + lane];
            }
            tile_store(acc, shard, t, wid, lane);
        }
    }
}

__global__ void k_fill(uint8_t* p, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * blockDim.x)
        ((float*)p)[i] = (float)((i * 2654435761u + seed) % 1000u) * 1e-6f;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    const int64_t ntiles = 122070;  // 8 GB shard (7 999 979 520 B), 16 pushes of the same size
    const int64_t S = ntiles * TILE;
    uint8_t *slab, *shard;
    uint32_t *cnt, *err, *sink;
    CK(hipMalloc(&slab, S * W));
    CK(hipMalloc(&shard, S));
    CK(hipMalloc(&cnt, 4));
    CK(hipMalloc(&err, 4));
    CK(hipMalloc(&sink, 4096));
    Ptrs p;
    for (int b = 0; b < W; ++b) p.p[b] = slab + b * S;
    for (int b = 0; b < W; ++b) k_fill<<<4096, 256>>>(slab + b * S, S, b);
    k_fill<<<4096, 256>>>(shard, S, 99);
    CK(hipMemset(err, 0, 4));
    CK(hipDeviceSynchronize());
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double algo = (double)S * (W + 2);
    auto report = [&](int r, const char* name, int grid, float ms) {
        printf("{\"case\": \"%s\", \"round\": %d, \"grid\": %d, \"ms\": %.3f, \"frac\": %.4f}\n", name, r, grid, ms,
               algo / (ms * 1e-3) / 8e12);
        fflush(stdout);
    };
    auto timed = [&](auto launch) {
        launch();
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms;
    };
    int occ1 = 0, occ2 = 0, occ3 = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, k_phased<1>, NW * 64, 0));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_phased<2>, NW * 64, 1 * NW * J * 64 * 16));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ3, k_phased<3>, NW * 64, 2 * NW * J * 64 * 16));
    printf("{\"cus\": %d, \"blocks_per_cu\": [%d, %d, %d]}\n", prop.multiProcessorCount, occ1, occ2, occ3);
    auto coop = [&](auto kern, int occ, size_t shm) {
        const int grid = occ * prop.multiProcessorCount;
        void* args[] = {(void*)&p, (void*)&shard, (void*)&ntiles, (void*)&cnt, (void*)&err};
        CK(hipMemsetAsync(cnt, 0, 4, 0));
        CK(hipLaunchCooperativeKernel((const void*)kern, dim3(grid), dim3(NW * 64), args, shm, 0));
        return grid;
    };
    for (int r = 0; r < rounds; ++r) {
        report(r, "tile (k_flat_ident shape)", (int)ntiles,
               timed([&] { k_tile<0><<<(unsigned)ntiles, NW * 64>>>(p, shard, ntiles, sink); }));
        report(r, "reads only", (int)ntiles, timed([&] { k_tile<1><<<(unsigned)ntiles, NW * 64>>>(p, shard, ntiles, sink); }));
        report(r, "writes only", (int)ntiles, timed([&] { k_tile<2><<<(unsigned)ntiles, NW * 64>>>(p, shard, ntiles, sink); }));
        if (occ1 > 0) {
            int g = 0;
            const float ms = timed([&] { g = coop(k_phased<1>, occ1, 0); });
            report(r, "phased T=1", g, ms);
        }
        if (occ2 > 0) {
            int g = 0;
            const float ms = timed([&] { g = coop(k_phased<2>, occ2, (size_t)1 * NW * J * 64 * 16); });
            report(r, "phased T=2", g, ms);
        }
        if (occ3 > 0) {
            int g = 0;
            const float ms = timed([&] { g = coop(k_phased<3>, occ3, (size_t)2 * NW * J * 64 * 16); });
            report(r, "phased T=3", g, ms);
        }
        uint32_t herr = 0;
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        if (herr) printf("{\"error\": \"a grid barrier timed out\"}\n");
    }
    return 0;
}
