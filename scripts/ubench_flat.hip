// Microbenchmark: config 4's narrow-row dense reduce (rows of 200 fp32 in 804-B
// records, 16 full-range identity pushes) — the loop shapes of k_reduce_flat
// (DESIGN.md §4.2). Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/ubench_flat.hip -o gpurun_out/ubench_flat
//   gpurun_out/ubench_flat [rows=1250000] [pushes=16]
// K_group<J, PB>:  a wave owns R = 64*J/50 rows as one flat run of 16-B vectors (lane l,
//                  step j -> vector 64j + l); PB pushes' loads in flight, then the adds
//                  (the previous product loop: the wave drains to zero at every round).
// K_roll<J, D>:    the same ownership; a ring of D pushes in flight (push b+D-1's loads
//                  are issued before push b's adds), 32-bit buffer offsets shared by
//                  every push (identity records: a wave-uniform base + per-lane offset).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
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
__device__ inline void st_nt(void* p, u32x4 v) { __builtin_nontemporal_store(v, (GL u32x4_u*)p); }
__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t n) {
    const uint64_t b = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}
__device__ inline u32x4 ldb_nt(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2);
}
__device__ inline void stb_nt(u32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 2);
}
constexpr uint32_t OFF = 0xFFFFFFF0u;
constexpr int MAXB = 64;
struct Bufs {
    const uint8_t* b[MAXB];
};
__device__ inline void addv(float (&a)[4], u32x4 t) {
    a[0] = __fadd_rn(a[0], __uint_as_float(t.x));
    a[1] = __fadd_rn(a[1], __uint_as_float(t.y));
    a[2] = __fadd_rn(a[2], __uint_as_float(t.z));
    a[3] = __fadd_rn(a[3], __uint_as_float(t.w));
}

template <int J, int PB>
__global__ __launch_bounds__(256) void k_group(const float* __restrict__ in, float* __restrict__ out, Bufs bf, int nb,
                                               int64_t rows, int cols, int R, int64_t stride) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t t0 = ((int64_t)blockIdx.x * 4 + wid) * R;
    if (t0 >= rows) return;
    const int nrow = (int)(rows - t0 < R ? rows - t0 : R);
    const int NV = cols / 4, nvec = nrow * NV;
    int rl[J], cv[J];
    float acc[J][4];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int v = j * 64 + lane;
        rl[j] = v < nvec ? v / NV : -1;
        cv[j] = v < nvec ? v - (v / NV) * NV : 0;
        u32x4 t = rl[j] >= 0 ? ld_nt((const uint8_t*)(in + (t0 + rl[j]) * cols + cv[j] * 4)) : u32x4{0, 0, 0, 0};
        acc[j][0] = __uint_as_float(t.x); acc[j][1] = __uint_as_float(t.y);
        acc[j][2] = __uint_as_float(t.z); acc[j][3] = __uint_as_float(t.w);
    }
#pragma unroll 1
    for (int b0 = 0; b0 < nb; b0 += PB) {
        u32x4 raw[PB][J];
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const uint8_t* bp = bf.b[b0 + p < nb ? b0 + p : nb - 1];
#pragma unroll
            for (int j = 0; j < J; ++j)
                raw[p][j] = rl[j] >= 0 ? ld_nt(bp + (t0 + rl[j]) * stride + 4 + cv[j] * 16) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int p = 0; p < PB; ++p)
            if (b0 + p < nb)
#pragma unroll
                for (int j = 0; j < J; ++j) addv(acc[j], raw[p][j]);
    }
#pragma unroll
    for (int j = 0; j < J; ++j)
        if (rl[j] >= 0)
            st_nt(out + (t0 + rl[j]) * cols + cv[j] * 4,
                  u32x4{__float_as_uint(acc[j][0]), __float_as_uint(acc[j][1]), __float_as_uint(acc[j][2]),
                        __float_as_uint(acc[j][3])});
}

// SH: bit 0 read the shard, bit 1 write it; WP: the store's cache policy (aux bits:
// 2 = nt, 0 = default, 16 = sc1 write-through, 17 = sc0|sc1)
template <int J, int D, bool SHARD = true, int SH = 3, int WP = 2>
__global__ __launch_bounds__(256) void k_roll(const float* __restrict__ in, float* __restrict__ out, Bufs bf, int nb,
                                              int64_t rows, int cols, int R, int64_t stride) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t t0 = ((int64_t)blockIdx.x * 4 + wid) * R;
    if (t0 >= rows) return;
    const int nrow = (int)(rows - t0 < R ? rows - t0 : R);
    const int NV = cols / 4, nvec = nrow * NV;
    uint32_t loff[J], soff[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int v = j * 64 + lane;
        const int r = v / NV, c = v - r * NV;
        loff[j] = v < nvec ? (uint32_t)(r * stride + 4 + c * 16) : OFF;
        soff[j] = v < nvec ? (uint32_t)((r * cols + c * 4) * 4) : OFF;
    }
    const uint32_t sbytes = (uint32_t)(nrow * cols * 4);
    const auto sin = rsrc(in + t0 * cols, sbytes);
    float acc[J][4];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const u32x4 t = (SHARD && (SH & 1)) ? ldb_nt(sin, soff[j]) : u32x4{0, 0, 0, 0};
        acc[j][0] = __uint_as_float(t.x); acc[j][1] = __uint_as_float(t.y);
        acc[j][2] = __uint_as_float(t.z); acc[j][3] = __uint_as_float(t.w);
    }
    const uint32_t rbytes = (uint32_t)(nrow * stride);
    u32x4 ring[D][J];
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        const auto rs = rsrc(bf.b[d < nb ? d : nb - 1] + t0 * stride, rbytes);
#pragma unroll
        for (int j = 0; j < J; ++j) ring[d][j] = ldb_nt(rs, loff[j]);
    }
#pragma unroll 1
    for (int b0 = 0; b0 < nb; b0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int b = b0 + d;
            const int bn = b + D - 1;  // issued now, into slot (d + D - 1) % D
            if (bn < nb) {
                const auto rs = rsrc(bf.b[bn] + t0 * stride, rbytes);
#pragma unroll
                for (int j = 0; j < J; ++j) ring[(d + D - 1) % D][j] = ldb_nt(rs, loff[j]);
            }
            if (b < nb)
#pragma unroll
                for (int j = 0; j < J; ++j) addv(acc[j], ring[d][j]);
        }
    }
    if (!SHARD || !(SH & 2)) {  // no shard write: one word per wave keeps the sums live
        float x = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) x += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
        if (x == 1.2345f) out[t0] = x;
        return;
    }
    const auto sout = rsrc(out + t0 * cols, sbytes);
#pragma unroll
    for (int j = 0; j < J; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(acc[j][0]), __float_as_uint(acc[j][1]),
                                                     __float_as_uint(acc[j][2]), __float_as_uint(acc[j][3])},
                                               sout, (int)soff[j], 0, WP);
}

// E2: a wave runs G consecutive row groups, stashing all but the last group's sums in
// LDS, and writes all G groups at its end (write bursts G x larger per wave).
template <int J, int D, int G>
__global__ __launch_bounds__(256) void k_roll2(const float* __restrict__ in, float* __restrict__ out, Bufs bf, int nb,
                                               int64_t rows, int cols, int R, int64_t stride) {
    __shared__ u32x4 stash[4][G > 1 ? G - 1 : 1][J][64];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NV = cols / 4;
    uint32_t loff[J], soff[J];
    int64_t tg[G];
    int nrg[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        tg[g] = (((int64_t)blockIdx.x * 4 + wid) * G + g) * R;
        nrg[g] = (int)(tg[g] >= rows ? 0 : rows - tg[g] < R ? rows - tg[g] : R);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (nrg[g] == 0) break;
        const int64_t t0 = tg[g];
        const int nrow = nrg[g], nvec = nrow * NV;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int v = j * 64 + lane;
            const int r = v / NV, c = v - r * NV;
            loff[j] = v < nvec ? (uint32_t)(r * stride + 4 + c * 16) : OFF;
            soff[j] = v < nvec ? (uint32_t)((r * cols + c * 4) * 4) : OFF;
        }
        const auto sin = rsrc(in + t0 * cols, (uint32_t)(nrow * cols * 4));
        float acc[J][4];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const u32x4 t = ldb_nt(sin, soff[j]);
            acc[j][0] = __uint_as_float(t.x); acc[j][1] = __uint_as_float(t.y);
            acc[j][2] = __uint_as_float(t.z); acc[j][3] = __uint_as_float(t.w);
        }
        const uint32_t rbytes = (uint32_t)(nrow * stride);
        u32x4 ring[D][J];
#pragma unroll
        for (int d = 0; d < D - 1; ++d) {
            const auto rs = rsrc(bf.b[d < nb ? d : nb - 1] + t0 * stride, rbytes);
#pragma unroll
            for (int j = 0; j < J; ++j) ring[d][j] = ldb_nt(rs, loff[j]);
        }
#pragma unroll 1
        for (int b0 = 0; b0 < nb; b0 += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int b = b0 + d, bn = b + D - 1;
                if (bn < nb) {
                    const auto rs = rsrc(bf.b[bn] + t0 * stride, rbytes);
#pragma unroll
                    for (int j = 0; j < J; ++j) ring[(d + D - 1) % D][j] = ldb_nt(rs, loff[j]);
                }
                if (b < nb)
#pragma unroll
                    for (int j = 0; j < J; ++j) addv(acc[j], ring[d][j]);
            }
        }
        if (g + 1 < G && nrg[g + 1] > 0) {
#pragma unroll
            for (int j = 0; j < J; ++j)
                stash[wid][g][j][lane] = u32x4{__float_as_uint(acc[j][0]), __float_as_uint(acc[j][1]),
                                               __float_as_uint(acc[j][2]), __float_as_uint(acc[j][3])};
            continue;
        }
        // last group: write the stashed groups, then this one
#pragma unroll
        for (int h = 0; h < G - 1; ++h) {
            if (h >= g) break;
            const int64_t th = tg[h];
            const int nvh = nrg[h] * NV;
            const auto so = rsrc(out + th * cols, (uint32_t)(nrg[h] * cols * 4));
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int v = j * 64 + lane;
                const int r = v / NV, c = v - r * NV;
                __builtin_amdgcn_raw_buffer_store_b128(stash[wid][h][j][lane], so,
                                                       (int)(v < nvh ? (uint32_t)((r * cols + c * 4) * 4) : OFF), 0, 2);
            }
        }
        const auto sout = rsrc(out + t0 * cols, (uint32_t)(nrow * cols * 4));
#pragma unroll
        for (int j = 0; j < J; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(acc[j][0]), __float_as_uint(acc[j][1]),
                                                         __float_as_uint(acc[j][2]), __float_as_uint(acc[j][3])},
                                                   sout, (int)soff[j], 0, 2);
    }
}

// E1: NW waves per block (NW x 64 threads), all of them finish reading before any
// stores (a block-wide barrier): a CU's writes leave in one burst.
template <int J, int D, int NW>
__global__ __launch_bounds__(NW * 64) void k_rollsync(const float* __restrict__ in, float* __restrict__ out, Bufs bf,
                                                      int nb, int64_t rows, int cols, int R, int64_t stride) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t t0 = ((int64_t)blockIdx.x * NW + wid) * R;
    const int nrow = (int)(t0 >= rows ? 0 : rows - t0 < R ? rows - t0 : R);
    const int NV = cols / 4, nvec = nrow * NV;
    uint32_t loff[J], soff[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int v = j * 64 + lane;
        const int r = v / NV, c = v - r * NV;
        loff[j] = v < nvec ? (uint32_t)(r * stride + 4 + c * 16) : OFF;
        soff[j] = v < nvec ? (uint32_t)((r * cols + c * 4) * 4) : OFF;
    }
    const int64_t tb = t0 < rows ? t0 : 0;
    const auto sin = rsrc(in + tb * cols, (uint32_t)(nrow * cols * 4));
    float acc[J][4];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const u32x4 t = ldb_nt(sin, soff[j]);
        acc[j][0] = __uint_as_float(t.x); acc[j][1] = __uint_as_float(t.y);
        acc[j][2] = __uint_as_float(t.z); acc[j][3] = __uint_as_float(t.w);
    }
    const uint32_t rbytes = (uint32_t)(nrow * stride);
    u32x4 ring[D][J];
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        const auto rs = rsrc(bf.b[d < nb ? d : nb - 1] + tb * stride, rbytes);
#pragma unroll
        for (int j = 0; j < J; ++j) ring[d][j] = ldb_nt(rs, loff[j]);
    }
#pragma unroll 1
    for (int b0 = 0; b0 < nb; b0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int b = b0 + d, bn = b + D - 1;
            if (bn < nb) {
                const auto rs = rsrc(bf.b[bn] + tb * stride, rbytes);
#pragma unroll
                for (int j = 0; j < J; ++j) ring[(d + D - 1) % D][j] = ldb_nt(rs, loff[j]);
            }
            if (b < nb)
#pragma unroll
                for (int j = 0; j < J; ++j) addv(acc[j], ring[d][j]);
        }
    }
    __syncthreads();
    const auto sout = rsrc(out + tb * cols, (uint32_t)(nrow * cols * 4));
#pragma unroll
    for (int j = 0; j < J; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(acc[j][0]), __float_as_uint(acc[j][1]),
                                                     __float_as_uint(acc[j][2]), __float_as_uint(acc[j][3])},
                                               sout, (int)soff[j], 0, 2);
}

__global__ void k_fill(uint8_t* p, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * blockDim.x)
        ((uint32_t*)p)[i] = (uint32_t)((i * 2654435761u) ^ seed) & 0x3F7FFFFFu;
}

int main(int argc, char** argv) {
    const int64_t rows = argc > 1 ? atoll(argv[1]) : 1250000;
    const int nb = argc > 2 ? atoi(argv[2]) : 16;
    const int64_t stag = argc > 3 ? atoll(argv[3]) : 0;  // push b's base offset: b * stag bytes
    const int slab = argc > 4 ? atoi(argv[4]) : 0;       // 1: the pushes as slices of one allocation
    const int cols = 200;
    const int64_t stride = 4 + 4 * cols;
    const int64_t pad = stag * nb + 4096;
    std::vector<uint8_t*> bufs(nb);
    uint8_t* slabp = nullptr;
    if (slab) CK(hipMalloc(&slabp, nb * (rows * stride + pad)));
    for (int b = 0; b < nb; ++b) {
        uint8_t* m = nullptr;
        if (slab) m = slabp + b * (rows * stride + pad);
        else CK(hipMalloc(&m, rows * stride + pad));
        bufs[b] = m + b * stag;
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, bufs[b], rows * stride, (uint32_t)b * 977u);
    }
    float *in, *out;
    CK(hipMalloc(&in, rows * cols * 4));
    CK(hipMalloc(&out, rows * cols * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint8_t*)in, rows * cols * 4, 7u);
    Bufs bf{};
    for (int b = 0; b < nb; ++b) bf.b[b] = bufs[b];
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ref;
    auto run = [&](const char* name, auto kern, int J, bool shard, int wpb = 4, int G = 1) {
        const double algo = (double)nb * rows * stride + (shard ? 2.0 * rows * cols * 4 : 0.0);
        const int R = std::min(16, J * 64 / (cols / 4));
        const int64_t nblk = ((rows + R - 1) / R + (int64_t)wpb * G - 1) / ((int64_t)wpb * G);
        float best = 1e30f;
        for (int it = 0; it < 6; ++it) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(64 * wpb), 0, 0, in, out, bf, nb, rows, cols, R, stride);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 0 && ms < best) best = ms;
        }
        bool same = true;
        if (shard) {
            std::vector<float> h((size_t)rows * cols);
            CK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
            if (ref.empty()) ref = h; else same = memcmp(ref.data(), h.data(), h.size() * 4) == 0;
        }
        printf("{\"kernel\": \"%s\", \"rows\": %ld, \"pushes\": %d, \"stagger\": %ld, \"slab\": %d, \"us\": %.1f, "
               "\"GBps\": %.1f, \"frac\": %.4f, \"same_as_first\": %s}\n",
               name, (long)rows, nb, (long)stag, slab, best * 1e3, algo / best / 1e6, algo / best / 1e6 / 8000.0,
               same ? "true" : "false");
        fflush(stdout);
    };
    const char* only = getenv("UB_ONLY");
    if (!only || !strcmp(only, "all")) {
        run("group<12,1>", k_group<12, 1>, 12, true);
        run("roll<12,2>", k_roll<12, 2>, 12, true);
        run("roll<8,3>", k_roll<8, 3>, 8, true);
    }
    run("roll<12,3>", k_roll<12, 3>, 12, true);
    run("roll<12,3> reads only", k_roll<12, 3, false>, 12, false);
    if (getenv("UB_BURST")) {
        run("roll2<12,3,2> LDS stash, 2 groups per wave", k_roll2<12, 3, 2>, 12, true);
        run("roll2<8,3,2> LDS stash, 2 groups per wave", k_roll2<8, 3, 2>, 8, true);
        run("roll2<8,3,3> LDS stash, 3 groups per wave", k_roll2<8, 3, 3>, 8, true);
        run("roll<4,4>", k_roll<4, 4>, 4, true);
        run("rollsync<4,4,16> 16-wave block, barrier", k_rollsync<4, 4, 16>, 4, true, 16);
        run("rollsync<4,4,8> 8-wave block, barrier", k_rollsync<4, 4, 8>, 4, true, 8);
        run("rollsync<12,3,4> 4-wave block, barrier", k_rollsync<12, 3, 4>, 12, true, 4);
        run("rollsync<8,3,8> 8-wave block, barrier", k_rollsync<8, 3, 8>, 8, true, 8);
    }
    if (getenv("UB_POLICY")) {
        ref.clear();
        run("roll<12,3> shard read, no write", k_roll<12, 3, true, 1>, 12, false);
        run("roll<12,3> shard write nt, no read", k_roll<12, 3, true, 2, 2>, 12, false);
        run("roll<12,3> rw, store default", k_roll<12, 3, true, 3, 0>, 12, true);
        run("roll<12,3> rw, store sc1", k_roll<12, 3, true, 3, 16>, 12, true);
        run("roll<12,3> rw, store sc0 sc1", k_roll<12, 3, true, 3, 17>, 12, true);
        run("roll<12,3> rw, store nt sc1", k_roll<12, 3, true, 3, 18>, 12, true);
        float* keep = out;
        out = in;  // in place
        run("roll<12,3> rw in place, nt", k_roll<12, 3, true, 3, 2>, 12, false);
        run("roll<12,3> rw in place, default", k_roll<12, 3, true, 3, 0>, 12, false);
        out = keep;
    }
    return 0;
}
