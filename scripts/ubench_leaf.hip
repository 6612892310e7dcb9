// Microbenchmark: is config 3's leaf slower than the random-RMW floor because of the
// order it issues its RMWs in, or because of what else the fused leaf does (the LDS
// sort, the ownership scan, the partition beside it)? The same 32 x 1e6 keys into a
// 1e9-float array (config 3 shape), every case alone on the GPU, no LDS anywhere:
//   floor      one plain RMW per thread over the globally sorted keys (k_rmw_floor)
//   leaf<T,S>  one block of T threads per big leaf of 2^16 rows, its sorted keys taken
//              S slots per thread at p = tid + k*T (the fused leaf's issue order), all
//              loads first, then the adds and stores (rot: the slot rotation by leaf)
//   leafrmw    the same order, each slot's store right after its load
// Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_leaf.hip -o scripts/ubench_leaf
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

__global__ __launch_bounds__(256) void k_floor(float* a, const uint32_t* keys, const float* v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t k = keys[i];
        a[k] = a[k] + v[i];
    }
}

template <int T, int S, bool ROT, bool IMM>
__global__ __launch_bounds__(T) void k_leaf(float* a, const uint32_t* keys, const float* v, const uint32_t* lb) {
    const int B = blockIdx.x;
    const uint32_t s = lb[B];
    const int n = (int)(lb[B + 1] - s);
    const int rot = ROT ? B % S : 0;
    const int tid = threadIdx.x;
    if (IMM) {
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int kk = k + rot >= S ? k + rot - S : k + rot;
            const int p = tid + kk * T;
            if (p < n) {
                const uint32_t q = keys[s + p];
                a[q] = a[q] + v[s + p];
            }
        }
        return;
    }
    uint32_t q[S];
    float x[S], u[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int kk = k + rot >= S ? k + rot - S : k + rot;
        const int p = min(tid + kk * T, n - 1);
        q[k] = keys[s + p];
        u[k] = v[s + p];
    }
#pragma unroll
    for (int k = 0; k < S; ++k) x[k] = a[q[k]];
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int kk = k + rot >= S ? k + rot - S : k + rot;
        if (tid + kk * T < n) a[q[k]] = x[k] + u[k];
    }
}

static uint64_t sm(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    const int64_t rows = 1000000000, per = 1000000;
    const int W = 32, BL = 16;
    const int64_t N = per * W;
    float* a;
    CK(hipMalloc(&a, rows * 4));
    CK(hipMemset(a, 0, rows * 4));
    std::vector<uint32_t> hg(N);
    std::vector<float> hv(N, 1e-3f);
    for (int b = 0; b < W; ++b) {
        uint64_t pa = (sm(2000 + b) % (rows - 1)) | 1, pc = sm(3000 + b) % rows;
        while (pa % 2 == 0 || pa % 5 == 0) pa += 2;  // coprime with 1e9
        for (int64_t r = 0; r < per; ++r) hg[b * per + r] = (uint32_t)((pa * (uint64_t)r + pc) % rows);
    }
    std::sort(hg.begin(), hg.end());
    const int64_t nleaf = (rows + (1 << BL) - 1) >> BL;
    std::vector<uint32_t> lb(nleaf + 1);
    int maxn = 0;
    {
        int64_t r = 0;
        for (int64_t B = 0; B < nleaf; ++B) {
            lb[B] = (uint32_t)r;
            while (r < N && (hg[r] >> BL) == (uint64_t)B) ++r;
            maxn = std::max(maxn, (int)(r - lb[B]));
        }
        lb[nleaf] = (uint32_t)N;
    }
    uint32_t *dg, *dlb;
    float* dv;
    CK(hipMalloc(&dg, N * 4));
    CK(hipMalloc(&dv, N * 4));
    CK(hipMalloc(&dlb, (nleaf + 1) * 4));
    CK(hipMemcpy(dg, hg.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, hv.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlb, lb.data(), (nleaf + 1) * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](int round, const char* name, int cap, auto fn) {
        if (cap && maxn > cap) {
            printf("{\"case\": \"%s\", \"skip\": \"leaf of %d keys > %d slots\"}\n", name, maxn, cap);
            return;
        }
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0;
        const int reps = 10;
        for (int rep = 0; rep < reps; ++rep) {
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
            sum += ms;
        }
        printf("{\"case\": \"%s\", \"round\": %d, \"best_us\": %.1f, \"mean_us\": %.1f}\n", name, round, best * 1e3,
               sum / reps * 1e3);
        fflush(stdout);
    };
    printf("{\"keys\": %lld, \"leaves\": %lld, \"max_keys_per_leaf\": %d, \"mean_keys_per_leaf\": %.1f}\n",
           (long long)N, (long long)nleaf, maxn, (double)N / nleaf);
    const unsigned gN = (unsigned)((N + 255) / 256), gL = (unsigned)nleaf;
    for (int r = 0; r < rounds; ++r) {
        timeit(r, "floor: sorted, 1 per thread", 0, [&] { k_floor<<<gN, 256>>>(a, dg, dv, N); });
        timeit(r, "leaf 512 x 8, rot, loads first", 4096,
               [&] { k_leaf<512, 8, true, false><<<gL, 512>>>(a, dg, dv, dlb); });
        timeit(r, "leaf 512 x 8, no rot, loads first", 4096,
               [&] { k_leaf<512, 8, false, false><<<gL, 512>>>(a, dg, dv, dlb); });
        timeit(r, "leaf 512 x 8, rot, rmw per slot", 4096,
               [&] { k_leaf<512, 8, true, true><<<gL, 512>>>(a, dg, dv, dlb); });
        timeit(r, "leaf 1024 x 4, no rot, loads first", 4096,
               [&] { k_leaf<1024, 4, false, false><<<gL, 1024>>>(a, dg, dv, dlb); });
        timeit(r, "leaf 256 x 16, no rot, loads first", 4096,
               [&] { k_leaf<256, 16, false, false><<<gL, 256>>>(a, dg, dv, dlb); });
    }
    return 0;
}
