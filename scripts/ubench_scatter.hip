// Microbenchmark: scatter-add access patterns into a 1e9-float array (config 3 shape).
// Not part of the product; informs the sparse kernel design.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_scatter.hip -o gpurun_out/ubench_scatter
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ void k_atomic(float* a, const uint32_t* keys, const float* v, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&a[keys[i]], v[i]);
}
__global__ void k_plain(float* a, const uint32_t* keys, const float* v, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint32_t k = keys[i];
        a[k] = a[k] + v[i];
    }
}
// 4 independent RMWs per thread (more memory-level parallelism)
__global__ void k_plain4(float* a, const uint32_t* keys, const float* v, int64_t n) {
    int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    uint32_t k[4];
    float x[4], u[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int64_t i = i0 + j * stride;
        k[j] = i < n ? keys[i] : 0;
        u[j] = i < n ? v[i] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = a[k[j]];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (i0 + j * stride < n) a[k[j]] = x[j] + u[j];
}
// One thread per touched U-float unit (U = 8: 32-B sector, 16: 64 B, 32: 128-B line):
// load the whole unit, add the unit's records (a run of the globally sorted keys),
// store the whole unit — full-unit writes instead of one 4-B store per record.
template <int U>
__global__ void k_unit(float* a, const uint32_t* unit, const uint32_t* run, const uint32_t* keys, const float* v,
                       int64_t nu) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nu) return;
    float4 q[U / 4];
    float4* p = (float4*)(a + (int64_t)unit[i] * U);
#pragma unroll
    for (int j = 0; j < U / 4; ++j) q[j] = p[j];
    for (uint32_t r = run[i]; r < run[i + 1]; ++r) {
        const int e = keys[r] % U;
        float* f = (float*)q;
        f[e] += v[r];
    }
#pragma unroll
    for (int j = 0; j < U / 4; ++j) p[j] = q[j];
}
// the same with non-temporal shard load and store
__global__ void k_plain_nt(float* a, const uint32_t* keys, const float* v, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint32_t k = keys[i];
        __builtin_nontemporal_store(__builtin_nontemporal_load(&a[k]) + v[i], &a[k]);
    }
}
__global__ void k_read(const float4* p, int64_t n, float* out) {
    float s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float4 q = p[i];
        s += q.x + q.y + q.z + q.w;
    }
    if (s == 1234.5f) *out = s;
}

// Dense sweep: one block per region of RF floats. The region is read whole
// (coalesced 16-B loads) into LDS, the region's updates (a run of the globally
// sorted keys) are added there, and the region is written back whole (WB 0) or
// only its touched 32-B sectors (WB 1). Streams the 4 GB array instead of
// random 64-B reads: does HBM serve it faster than the random RMW?
template <int RF, int WB>
__global__ __launch_bounds__(256) void k_sweep(float* a, const uint32_t* run, const uint32_t* keys, const float* v) {
    __shared__ float4 reg[RF / 4];
    __shared__ uint8_t tsec[RF / 8];
    const int64_t base = (int64_t)blockIdx.x * RF;
    const float4* src = (const float4*)(a + base);
    for (int j = threadIdx.x; j < RF / 4; j += 256) reg[j] = src[j];
    for (int j = threadIdx.x; j < RF / 8; j += 256) tsec[j] = 0;
    __syncthreads();
    float* rf = (float*)reg;
    for (uint32_t r = run[blockIdx.x] + threadIdx.x; r < run[blockIdx.x + 1]; r += 256) {
        const uint32_t e = keys[r] - (uint32_t)base;
        atomicAdd(&rf[e], v[r]);
        if (WB) tsec[e / 8] = 1;
    }
    __syncthreads();
    float4* dst = (float4*)(a + base);
    if (WB == 0) {
        for (int j = threadIdx.x; j < RF / 4; j += 256) dst[j] = reg[j];
    } else {
        for (int j = threadIdx.x; j < RF / 4; j += 256)
            if (tsec[j / 2]) dst[j] = reg[j];
    }
}

static uint64_t sm(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

int main() {
    const int64_t rows = 1000000000, per = 1000000;
    const int W = 32;
    const int64_t N = per * W;
    float* a;
    CK(hipMalloc(&a, rows * 4));
    CK(hipMemset(a, 0, rows * 4));
    std::vector<uint32_t> hk(N), hs(N);
    std::vector<float> hv(N, 1e-3f);
    for (int b = 0; b < W; ++b) {
        uint64_t pa = (sm(2000 + b) % (rows - 1)) | 1, pc = sm(3000 + b) % rows;
        while (pa % 2 == 0 || pa % 5 == 0) pa += 2;  // coprime with 1e9
        for (int64_t r = 0; r < per; ++r) hk[b * per + r] = (uint32_t)((pa * (uint64_t)r + pc) % rows);
    }
    // per-push sorted copy and globally sorted copy
    hs = hk;
    for (int b = 0; b < W; ++b) std::sort(hs.begin() + b * per, hs.begin() + (b + 1) * per);
    std::vector<uint32_t> hg = hk;
    std::sort(hg.begin(), hg.end());
    uint32_t *dk, *ds, *dg;
    float *dv, *dout;
    CK(hipMalloc(&dk, N * 4));
    CK(hipMalloc(&ds, N * 4));
    CK(hipMalloc(&dg, N * 4));
    CK(hipMalloc(&dv, N * 4));
    CK(hipMalloc(&dout, 4));
    CK(hipMemcpy(dk, hk.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ds, hs.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, hg.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, hv.data(), N * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        printf("%-44s %8.3f ms  %7.2f Gupd/s\n", name, best, N / (best * 1e6));
    };
    const unsigned g1 = (unsigned)((per + 255) / 256);
    const unsigned gN = (unsigned)((N + 255) / 256);
    timeit("atomic, 32 launches x 1e6 random", [&] {
        for (int b = 0; b < W; ++b) k_atomic<<<g1, 256>>>(a, dk + b * per, dv + b * per, per);
    });
    timeit("plain RMW, 32 launches x 1e6 random", [&] {
        for (int b = 0; b < W; ++b) k_plain<<<g1, 256>>>(a, dk + b * per, dv + b * per, per);
    });
    timeit("plain RMW x4 ILP, 32 launches random", [&] {
        for (int b = 0; b < W; ++b) k_plain4<<<(g1 + 3) / 4, 256>>>(a, dk + b * per, dv + b * per, per);
    });
    timeit("plain RMW, 32 launches, per-push sorted", [&] {
        for (int b = 0; b < W; ++b) k_plain<<<g1, 256>>>(a, ds + b * per, dv + b * per, per);
    });
    timeit("atomic, 1 launch x 32e6 random", [&] { k_atomic<<<gN, 256>>>(a, dk, dv, N); });
    timeit("plain RMW, 1 launch, globally sorted 32e6", [&] { k_plain<<<gN, 256>>>(a, dg, dv, N); });
    timeit("plain RMW x4, 1 launch, globally sorted", [&] { k_plain4<<<(gN + 3) / 4, 256>>>(a, dg, dv, N); });
    timeit("atomic, 1 launch, globally sorted", [&] { k_atomic<<<gN, 256>>>(a, dg, dv, N); });
    timeit("plain RMW nt, 1 launch, globally sorted", [&] { k_plain_nt<<<gN, 256>>>(a, dg, dv, N); });
    auto unit_case = [&](auto tag, const char* name) {
        constexpr int U = decltype(tag)::value;
        std::vector<uint32_t> hu, hr;
        for (int64_t r = 0; r < N; ++r) {
            const uint32_t u = hg[r] / U;
            if (hu.empty() || hu.back() != u) { hu.push_back(u); hr.push_back((uint32_t)r); }
        }
        hr.push_back((uint32_t)N);
        uint32_t *du, *dr;
        CK(hipMalloc(&du, hu.size() * 4));
        CK(hipMalloc(&dr, hr.size() * 4));
        CK(hipMemcpy(du, hu.data(), hu.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dr, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
        const int64_t nu = (int64_t)hu.size();
        printf("  (%lld units of %d floats touched)\n", (long long)nu, U);
        timeit(name, [&] { k_unit<U><<<(unsigned)((nu + 255) / 256), 256>>>(a, du, dr, dg, dv, nu); });
        CK(hipFree(du));
        CK(hipFree(dr));
    };
    auto sweep_case = [&](auto tagr, auto tagw, const char* name) {
        constexpr int RF = decltype(tagr)::value, WB = decltype(tagw)::value;
        const int64_t nreg = rows / RF;  // 1e9 is a multiple of 8192 x 5^k? checked below
        if (nreg * RF != rows) { printf("  skip %s: rows %% %d\n", name, RF); return; }
        std::vector<uint32_t> hr(nreg + 1);
        int64_t r = 0;
        for (int64_t g = 0; g < nreg; ++g) {
            hr[g] = (uint32_t)r;
            while (r < N && hg[r] < (uint64_t)(g + 1) * RF) ++r;
        }
        hr[nreg] = (uint32_t)N;
        uint32_t* dr;
        CK(hipMalloc(&dr, hr.size() * 4));
        CK(hipMemcpy(dr, hr.data(), hr.size() * 4, hipMemcpyHostToDevice));
        timeit(name, [&] { k_sweep<RF, WB><<<(unsigned)nreg, 256>>>(a, dr, dg, dv); });
        CK(hipFree(dr));
    };
    sweep_case(std::integral_constant<int, 8000>{}, std::integral_constant<int, 0>{}, "sweep 32 KB regions, write all");
    sweep_case(std::integral_constant<int, 8000>{}, std::integral_constant<int, 1>{}, "sweep 32 KB regions, write touched 32 B");
    sweep_case(std::integral_constant<int, 16000>{}, std::integral_constant<int, 1>{}, "sweep 64 KB regions, write touched 32 B");
    sweep_case(std::integral_constant<int, 4000>{}, std::integral_constant<int, 1>{}, "sweep 16 KB regions, write touched 32 B");
    unit_case(std::integral_constant<int, 8>{}, "unit RMW 32 B, globally sorted");
    unit_case(std::integral_constant<int, 16>{}, "unit RMW 64 B, globally sorted");
    unit_case(std::integral_constant<int, 32>{}, "unit RMW 128 B, globally sorted");
    {
        float ms_best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            k_read<<<4096, 256>>>((const float4*)a, rows / 4, dout);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms_best = std::min(ms_best, ms);
        }
        printf("%-44s %8.3f ms  %7.1f GB/s\n", "stream read 4 GB", ms_best, rows * 4 / (ms_best * 1e6));
    }
    // partition cost: radix sort of 32e6 (u32 key, u64 payload) pairs on 16 / 30 key bits
    {
        uint32_t *kin, *kout;
        uint64_t *vin, *vout;
        CK(hipMalloc(&kin, N * 4));
        CK(hipMalloc(&kout, N * 4));
        CK(hipMalloc(&vin, N * 8));
        CK(hipMalloc(&vout, N * 8));
        CK(hipMemcpy(kin, hk.data(), N * 4, hipMemcpyHostToDevice));
        size_t tmp_bytes = 0;
        CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, vout, (int)N, 0, 30));
        void* tmp;
        CK(hipMalloc(&tmp, tmp_bytes));
        for (int bits : {16, 30}) {
            timeit(bits == 16 ? "hipcub SortPairs u32/u64, 16 bits (14..30)" : "hipcub SortPairs u32/u64, 30 bits",
                   [&] {
                       size_t tb = tmp_bytes;
                       CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin, vout, (int)N, 30 - bits, 30));
                   });
        }
        uint32_t* vin32;
        uint32_t* vout32;
        CK(hipMalloc(&vin32, N * 4));
        CK(hipMalloc(&vout32, N * 4));
        timeit("hipcub SortPairs u32/u32, 16 bits", [&] {
            size_t tb = tmp_bytes;
            CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin32, vout32, (int)N, 14, 30));
        });
        timeit("hipcub SortKeys u32, 16 bits", [&] {
            size_t tb = tmp_bytes;
            CK(hipcub::DeviceRadixSort::SortKeys(tmp, tb, kin, kout, (int)N, 14, 30));
        });
    }
    return 0;
}
