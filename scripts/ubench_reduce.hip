// Microbenchmark: HBM access orders for the config-2 multi-push reduce
// (32 buffers x 16384 records x 4 KiB values -> 64 MiB shard). Not part of the
// product; informs k_reduce's work decomposition.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_reduce.hip -o gpurun_out/ubench_reduce
#include <hip/hip_runtime.h>

#include <algorithm>
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
typedef u32x4 u32x4_u __attribute__((aligned(4)));
#define GL __attribute__((address_space(1)))
__device__ inline u32x4 ld_nt(const uint8_t* p) { return __builtin_nontemporal_load((const GL u32x4_u*)p); }
__device__ inline u32x4 ld(const uint8_t* p) { return *(const GL u32x4_u*)p; }
__device__ inline void st(void* p, u32x4 v) { *(GL u32x4_u*)p = v; }

constexpr int W = 32, ROWS = 16384, C = 1024;
struct Bufs {
    const uint8_t* b[W];
    int32_t pa[W], pc[W];  // record of row r in push b = (pa*r + pc) % ROWS
};
__device__ inline float addf(float a, uint32_t b) { return __fadd_rn(a, __uint_as_float(b)); }

// K1: one wave per row (CPW = 4 chunks), G pushes' loads in flight (the current k_reduce shape).
template <int G>
__global__ __launch_bounds__(256) void k_rowwave(float* shard, Bufs bf, int64_t stride, int voff) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    float acc[4][4];
    for (int c = 0; c < 4; ++c) {
        u32x4 t = ld((const uint8_t*)(shard + (int64_t)row * C + (c * 64 + lane) * 4));
        acc[c][0] = __uint_as_float(t.x); acc[c][1] = __uint_as_float(t.y);
        acc[c][2] = __uint_as_float(t.z); acc[c][3] = __uint_as_float(t.w);
    }
    for (int b0 = 0; b0 < W; b0 += G) {
        u32x4 raw[G][4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t rec = ((int64_t)bf.pa[b0 + g] * row + bf.pc[b0 + g]) % ROWS;
            const uint8_t* p = bf.b[b0 + g] + rec * stride + voff;
#pragma unroll
            for (int c = 0; c < 4; ++c) raw[g][c] = ld_nt(p + (c * 64 + lane) * 16);
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                acc[c][0] = addf(acc[c][0], raw[g][c].x); acc[c][1] = addf(acc[c][1], raw[g][c].y);
                acc[c][2] = addf(acc[c][2], raw[g][c].z); acc[c][3] = addf(acc[c][3], raw[g][c].w);
            }
    }
    for (int c = 0; c < 4; ++c) {
        u32x4 t;
        t.x = __float_as_uint(acc[c][0]); t.y = __float_as_uint(acc[c][1]);
        t.z = __float_as_uint(acc[c][2]); t.w = __float_as_uint(acc[c][3]);
        st(shard + (int64_t)row * C + (c * 64 + lane) * 4, t);
    }
}

// K2: one wave per RPW consecutive rows; per push all RPW records in flight
// (RPW x 4 KiB contiguous per push for ascending pushes).
template <int RPW, int G, bool IL = false, bool NTS = false>
__global__ __launch_bounds__(256) void k_multirow(float* shard, Bufs bf, int64_t stride, int voff) {
    const int lane = threadIdx.x & 63;
    // IL: the block's 4*RPW rows are dealt round-robin to its waves (row = base + r*4 + wave)
    const int rstep = IL ? 4 : 1;
    const int row0 = IL ? blockIdx.x * 4 * RPW + (threadIdx.x >> 6) : (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    float acc[RPW][4][4];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            u32x4 t = ld((const uint8_t*)(shard + (int64_t)(row0 + r * rstep) * C + (c * 64 + lane) * 4));
            acc[r][c][0] = __uint_as_float(t.x); acc[r][c][1] = __uint_as_float(t.y);
            acc[r][c][2] = __uint_as_float(t.z); acc[r][c][3] = __uint_as_float(t.w);
        }
    for (int b0 = 0; b0 < W; b0 += G) {
        u32x4 raw[G][RPW][4];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int64_t rec = ((int64_t)bf.pa[b0 + g] * (row0 + r * rstep) + bf.pc[b0 + g]) % ROWS;
                const uint8_t* p = bf.b[b0 + g] + rec * stride + voff;
#pragma unroll
                for (int c = 0; c < 4; ++c) raw[g][r][c] = ld_nt(p + (c * 64 + lane) * 16);
            }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < RPW; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    acc[r][c][0] = addf(acc[r][c][0], raw[g][r][c].x); acc[r][c][1] = addf(acc[r][c][1], raw[g][r][c].y);
                    acc[r][c][2] = addf(acc[r][c][2], raw[g][r][c].z); acc[r][c][3] = addf(acc[r][c][3], raw[g][r][c].w);
                }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            u32x4 t;
            t.x = __float_as_uint(acc[r][c][0]); t.y = __float_as_uint(acc[r][c][1]);
            t.z = __float_as_uint(acc[r][c][2]); t.w = __float_as_uint(acc[r][c][3]);
            if (NTS) __builtin_nontemporal_store(t, (GL u32x4_u*)(shard + (int64_t)(row0 + r * rstep) * C + (c * 64 + lane) * 4));
            else st(shard + (int64_t)(row0 + r * rstep) * C + (c * 64 + lane) * 4, t);
        }
}

// K3: pure read, push-major sweep: waves walk buffer 0 in grid-stride 4 KiB
// steps, then buffer 1, ... (no reduce; the multi-buffer streaming ceiling).
__global__ __launch_bounds__(256) void k_pushmajor(Bufs bf, int64_t bytes, uint32_t* sink) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t f = 0;
    for (int b = 0; b < W; ++b)
        for (int64_t o = wave * 4096; o + 4096 <= bytes; o += nw * 4096) {
            u32x4 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = ld_nt(bf.b[b] + o + (j * 64 + lane) * 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) f ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
        }
    if (f == 0x9E3779B9u) *sink = f;
}

// K4: one wave per row (as K1) but pure reads, no shard RMW (isolates the write cost).
template <int G>
__global__ __launch_bounds__(256) void k_rowread(Bufs bf, int64_t stride, int voff, uint32_t* sink) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t f = 0;
    for (int b0 = 0; b0 < W; b0 += G) {
        u32x4 raw[G][4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t rec = ((int64_t)bf.pa[b0 + g] * row + bf.pc[b0 + g]) % ROWS;
            const uint8_t* p = bf.b[b0 + g] + rec * stride + voff;
#pragma unroll
            for (int c = 0; c < 4; ++c) raw[g][c] = ld_nt(p + (c * 64 + lane) * 16);
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int c = 0; c < 4; ++c) f ^= raw[g][c].x ^ raw[g][c].y ^ raw[g][c].z ^ raw[g][c].w;
    }
    if (f == 0x9E3779B9u) *sink = f;
}

// K5: persistent waves, row-block tiles assigned so that the concurrently
// running waves cover a contiguous window of rows and step through the
// pushes together: tile t = rows [t*RPW, (t+1)*RPW); wave w takes tiles
// w, w + nw, ... (same per-wave work as K2).
template <int RPW>
__global__ __launch_bounds__(256) void k_persist(float* shard, Bufs bf, int64_t stride, int voff) {
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * 4;
    for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < ROWS / RPW; t += nw) {
        const int row0 = t * RPW;
        float acc[RPW][4][4];
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                u32x4 q = ld((const uint8_t*)(shard + (int64_t)(row0 + r) * C + (c * 64 + lane) * 4));
                acc[r][c][0] = __uint_as_float(q.x); acc[r][c][1] = __uint_as_float(q.y);
                acc[r][c][2] = __uint_as_float(q.z); acc[r][c][3] = __uint_as_float(q.w);
            }
        for (int b = 0; b < W; ++b) {
            u32x4 raw[RPW][4];
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int64_t rec = ((int64_t)bf.pa[b] * (row0 + r) + bf.pc[b]) % ROWS;
                const uint8_t* p = bf.b[b] + rec * stride + voff;
#pragma unroll
                for (int c = 0; c < 4; ++c) raw[r][c] = ld_nt(p + (c * 64 + lane) * 16);
            }
#pragma unroll
            for (int r = 0; r < RPW; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    acc[r][c][0] = addf(acc[r][c][0], raw[r][c].x); acc[r][c][1] = addf(acc[r][c][1], raw[r][c].y);
                    acc[r][c][2] = addf(acc[r][c][2], raw[r][c].z); acc[r][c][3] = addf(acc[r][c][3], raw[r][c].w);
                }
        }
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                u32x4 q;
                q.x = __float_as_uint(acc[r][c][0]); q.y = __float_as_uint(acc[r][c][1]);
                q.z = __float_as_uint(acc[r][c][2]); q.w = __float_as_uint(acc[r][c][3]);
                st(shard + (int64_t)(row0 + r) * C + (c * 64 + lane) * 4, q);
            }
    }
}

__global__ void k_fill(uint32_t* p, int64_t n, uint32_t s) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = ((uint32_t)(i * 2654435761u) ^ s) & 0x3c7fffffu;  // small finite floats
}

template <typename F>
static float time_best(F f, int reps = 7) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (i > 0) best = std::min(best, ms);
    }
    return best;
}

int main() {
    const int64_t strides[2] = {4096, 4100};
    const int64_t maxbytes = (int64_t)ROWS * 4100 + 64;
    Bufs bf{}, bp{};
    std::vector<uint8_t*> raw(W);
    // one 2.1 GB pool; buffer b at offset b * round_up(maxbytes, 2 MiB) (torch-allocator-like spacing)
    const int64_t span = (maxbytes + (2 << 20) - 1) / (2 << 20) * (2 << 20);
    uint8_t* pool;
    CK(hipMalloc(&pool, span * W));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (uint32_t*)pool, span * W / 4, 7u);
    float* shard;
    CK(hipMalloc(&shard, (size_t)ROWS * C * 4));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (uint32_t*)shard, (int64_t)ROWS * C, 9u);
    uint32_t* sink;
    CK(hipMalloc(&sink, 64));
    for (int b = 0; b < W; ++b) {
        bf.b[b] = bp.b[b] = pool + span * b;
        bf.pa[b] = 1; bf.pc[b] = 0;
        bp.pa[b] = (b % 2) ? ((((2 * b + 1) * 2654435761u) % ROWS) | 1) : 1;
        bp.pc[b] = (b % 2) ? (b * 7919) % ROWS : 0;
    }
    CK(hipDeviceSynchronize());
    auto report = [&](const char* name, int64_t s, int voff, float ms, int64_t bytes) {
        printf("{\"kernel\": \"%s\", \"stride\": %lld, \"voff\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", name,
               (long long)s, voff, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    const int64_t rmw = 2LL * ROWS * C * 4;
    const int nblk = ROWS / 4;
    for (int si = 0; si < 2; ++si) {
        const int64_t s = strides[si];
        const int voff = si == 0 ? 0 : 4;
        const int64_t rd = (int64_t)W * ROWS * s;
        for (int mix = 0; mix < 2; ++mix) {
            const Bufs& B = mix ? bp : bf;
            const char* tag = mix ? "mixed" : "asc";
            char nm[64];
#define RUN(NAME, BYTES, ...)                                 \
    snprintf(nm, sizeof nm, "%s/%s", NAME, tag);              \
    report(nm, s, voff, time_best([&] { __VA_ARGS__; }), BYTES);
            RUN("rowwave_G4", rd + rmw, k_rowwave<4><<<nblk, 256>>>(shard, B, s, voff));
            RUN("rowwave_G8", rd + rmw, k_rowwave<8><<<nblk, 256>>>(shard, B, s, voff));
            RUN("rowread_G4", rd, k_rowread<4><<<nblk, 256>>>(B, s, voff, sink));
            RUN("multirow_R2G1", rd + rmw, k_multirow<2, 1><<<nblk / 2, 256>>>(shard, B, s, voff));
            RUN("multirow_R2G2", rd + rmw, k_multirow<2, 2><<<nblk / 2, 256>>>(shard, B, s, voff));
            RUN("multirow_R4G1", rd + rmw, k_multirow<4, 1><<<nblk / 4, 256>>>(shard, B, s, voff));
            RUN("multirow_R4G1_il", rd + rmw, k_multirow<4, 1, true><<<nblk / 4, 256>>>(shard, B, s, voff));
            RUN("multirow_R4G1_nts", rd + rmw, k_multirow<4, 1, false, true><<<nblk / 4, 256>>>(shard, B, s, voff));
            RUN("multirow_R4G2", rd + rmw, k_multirow<4, 2><<<nblk / 4, 256>>>(shard, B, s, voff));
            RUN("multirow_R8G1", rd + rmw, k_multirow<8, 1><<<nblk / 8, 256>>>(shard, B, s, voff));
            RUN("multirow_R8G1_il", rd + rmw, k_multirow<8, 1, true><<<nblk / 8, 256>>>(shard, B, s, voff));
            RUN("persist_R1_g1024", rd + rmw, k_persist<1><<<1024, 256>>>(shard, B, s, voff));
            RUN("persist_R2_g1024", rd + rmw, k_persist<2><<<1024, 256>>>(shard, B, s, voff));
            RUN("persist_R4_g512", rd + rmw, k_persist<4><<<512, 256>>>(shard, B, s, voff));
            RUN("persist_R4_g1024", rd + rmw, k_persist<4><<<1024, 256>>>(shard, B, s, voff));
        }
        char nm[64];
        snprintf(nm, sizeof nm, "pushmajor_g4096");
        report(nm, s, 0, time_best([&] { k_pushmajor<<<4096, 256>>>(bf, (int64_t)ROWS * s, sink); }),
               (int64_t)W * (ROWS * s / 4096) * 4096);
        snprintf(nm, sizeof nm, "pushmajor_g1024");
        report(nm, s, 0, time_best([&] { k_pushmajor<<<1024, 256>>>(bf, (int64_t)ROWS * s, sink); }),
               (int64_t)W * (ROWS * s / 4096) * 4096);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
