// dml_split.hip — per-shard split of device-resident pushes (C-ABI dml_shard_split).
//
// The client side of a push splits its records by parameter-server partition
// before sending (SparseMatrix.push, SparseMatrix.java:46-60; SparseArray the
// same): each server receives, per push, exactly its own keys, in the push's
// record order, and applies them in arrival order. dml_shard_split is that split
// for pushes already in HBM (the multi-GPU exchange path): a
// stable partition of every push's records by owner shard under
// KeyRange.linearSplit(world) (KeyRange.java:68-80), written dest-major
// ([dest][push][records in push order]) so one all-to-all sends each owner its
// slices. Keys outside [0, total_rows) are dropped, like the client's
// `p.contains(k)` test.
//
// Kernels (HBM-bound byte moves, no arithmetic on values):
//   k_split_count    one thread per record: owner of the key -> per-block
//                    histogram in LDS -> blkcnt[push][block][dest]
//   k_split_scan     per (push, dest): exclusive scan of the block counts
//   k_split_scatter  per block: the owner and the stable rank of each of its 256
//                    records (LDS), then the block's records move as one flat run
//                    of 16-B chunks, stored as vectors where the output is contiguous
#include <algorithm>
#include <vector>

#include "distml_ps.h"
#include "dml_device.h"

using namespace dml;

namespace {

constexpr int kSplitBlock = 256;
constexpr int kMaxWorld = 64;

__device__ inline int owner_of(int64_t key, int64_t total_rows, int64_t step, int world) {
    if (key < 0 || key >= total_rows) return world;  // dropped
    const int64_t d = key / step;
    return d < world ? (int)d : world;
}

__global__ __launch_bounds__(kSplitBlock) void k_split_count(const Batch bt, int64_t stride, int K, int64_t total_rows,
                                                            int64_t step, int world, int64_t nblk,
                                                            int32_t* __restrict__ blkcnt) {
    __shared__ int32_t h[kMaxWorld + 1];
    const int b = blockIdx.y;
    if (threadIdx.x <= world) h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * kSplitBlock + threadIdx.x;
    if (r < bt.nrec[b]) atomicAdd(&h[owner_of(ld_key(bt.base[b] + r * stride, K), total_rows, step, world)], 1);
    __syncthreads();
    if (threadIdx.x <= world) blkcnt[((int64_t)b * nblk + blockIdx.x) * (world + 1) + threadIdx.x] = h[threadIdx.x];
}

// grid (n, world): blkoff[b][blk][d] = sum of blkcnt[b][0..blk)[d]; tot[b][d] = the sum over all blocks.
__global__ __launch_bounds__(256) void k_split_scan(const int32_t* __restrict__ blkcnt, int64_t nblk, int world,
                                                   int64_t* __restrict__ blkoff, int64_t* __restrict__ tot) {
    __shared__ int64_t part[256];
    const int b = blockIdx.x, d = blockIdx.y, W1 = world + 1;
    const int64_t per = (nblk + 255) / 256;
    const int64_t lo = threadIdx.x * per, hi = lo + per < nblk ? lo + per : nblk;
    int64_t s = 0;
    for (int64_t i = lo; i < hi; ++i) s += blkcnt[((int64_t)b * nblk + i) * W1 + d];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {  // 256 partial sums: a serial scan is cheaper than a tree here
        int64_t run = 0;
        for (int i = 0; i < 256; ++i) { const int64_t v = part[i]; part[i] = run; run += v; }
        tot[(int64_t)b * W1 + d] = run;
    }
    __syncthreads();
    int64_t run = part[threadIdx.x];
    for (int64_t i = lo; i < hi; ++i) {
        const int64_t at = ((int64_t)b * nblk + i) * W1 + d;
        blkoff[at] = run;
        run += blkcnt[at];
    }
}

__global__ __launch_bounds__(kSplitBlock) void k_split_scatter(const Batch bt, int64_t stride, int K, int64_t total_rows,
                                                              int64_t step, int world, int64_t nblk,
                                                              const int64_t* __restrict__ blkoff,
                                                              const int64_t* __restrict__ base,
                                                              uint8_t* __restrict__ out) {
    __shared__ int8_t dst[kSplitBlock];
    __shared__ int64_t pos[kSplitBlock];
    const int b = blockIdx.y;
    const int64_t r0 = (int64_t)blockIdx.x * kSplitBlock;
    const int64_t nrec = bt.nrec[b];
    const int64_t r = r0 + threadIdx.x;
    const uint8_t* src = bt.base[b];
    const int d = r < nrec ? owner_of(ld_key(src + r * stride, K), total_rows, step, world) : world;
    dst[threadIdx.x] = (int8_t)d;
    __syncthreads();
    if (d < world) {
        int rank = 0;  // records of this block before mine with the same owner (stable order)
        for (int i = 0; i < (int)threadIdx.x; ++i) rank += dst[i] == d;
        pos[threadIdx.x] = base[(int64_t)b * world + d] + blkoff[((int64_t)b * nblk + blockIdx.x) * (world + 1) + d] + rank;
    } else {
        pos[threadIdx.x] = -1;
    }
    __syncthreads();
    // Copy: the block's records are one contiguous source range; it moves as a flat
    // run of 16-B chunks (chunk c = dwords 4c..4c+3 of the range; U chunks per thread,
    // all loads in flight before the stores). A chunk spans at most two records
    // (records are >= 2 dwords); it is stored as one 16-B vector when its records are
    // neighbours in the output (the common case: a run of one owner's records), else
    // dword by dword. Records are 4-byte aligned only: unaligned vector accesses.
    const int64_t nw = stride / 4;  // records are whole dwords (K and V are 4 or 8 bytes)
    const int64_t nr = nrec - r0 < kSplitBlock ? nrec - r0 : kSplitBlock;
    const int64_t ndw = nr > 0 ? nr * nw : 0;
    const int64_t nch = (ndw + 3) / 4;
    const uint8_t* sb = src + r0 * stride;
    constexpr int U = 8;
    for (int64_t c0 = threadIdx.x; c0 < nch; c0 += (int64_t)kSplitBlock * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t c = c0 + (int64_t)u * kSplitBlock;
            if (c + 1 < nch || (c + 1 == nch && (ndw & 3) == 0)) {
                v[u] = ldg16_nt(sb + c * 16);
            } else if (c < nch) {  // the range's last, partial chunk: no read past its end
                v[u] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (4 * c + k < ndw) v[u][k] = ldg32(sb + (4 * c + k) * 4);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t c = c0 + (int64_t)u * kSplitBlock;
            if (c >= nch) break;
            const int64_t x = 4 * c;
            const int i0 = (int)(x / nw);
            const int64_t p0 = pos[i0];
            const int64_t last = x + 3 < ndw ? x + 3 : ndw - 1;
            const int i1 = (int)(last / nw);
            if (last == x + 3 && p0 >= 0 && (i1 == i0 || pos[i1] == p0 + 1)) {
                stg16(out + (p0 * nw + (x - (int64_t)i0 * nw)) * 4, v[u]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (x + k >= ndw) break;
                    const int i = (int)((x + k) / nw);
                    const int64_t p = pos[i];
                    if (p >= 0) *(DML_GLOBAL uint32_t*)(out + (p * nw + (x + k - (int64_t)i * nw)) * 4) = v[u][k];
                }
            }
        }
    }
}

}  // namespace

extern "C" int dml_shard_split(const dml_desc* desc, int32_t cols, int64_t total_rows, int32_t world,
                               const void* const* dev_bufs, const int64_t* lens, int32_t n, void* dev_out,
                               int64_t out_cap, int64_t* counts, void* stream) {
    if (!desc || total_rows <= 0 || world <= 0 || world > kMaxWorld || n < 0 || n > kMaxW ||
        (n > 0 && (!dev_bufs || !lens || !counts)))
        return set_error(DML_E_INVALID_ARG, "bad split arguments (world <= 64, n <= 64)");
    if (desc->data_type == DML_DATA_TYPE_MATRIX && !desc->dense_column)
        return set_error(DML_E_UNSUPPORTED, "sparse-column matrix pushes are not supported");
    const int K = desc->key_type == 0 ? 4 : 8;
    const int V = (desc->value_type == DML_ELEMENT_TYPE_INT || desc->value_type == DML_ELEMENT_TYPE_FLOAT) ? 4 : 8;
    const int64_t stride = desc->data_type == DML_DATA_TYPE_MATRIX ? K + (int64_t)V * cols : K + V;
    if (desc->data_type == DML_DATA_TYPE_MATRIX && cols <= 0) return set_error(DML_E_INVALID_ARG, "cols must be > 0");
    std::vector<int64_t> f((size_t)world), l((size_t)world);
    if (int rc = dml_linear_split(0, total_rows - 1, world, f.data(), l.data())) return rc;
    const int64_t step = l[0] - f[0] + 1;
    Batch bt{};
    int64_t max_nrec = 0;
    for (int b = 0; b < n; ++b) {
        if (lens[b] < 0 || lens[b] % stride) return set_error(DML_E_INVALID_ARG, "push length is not whole records");
        bt.base[b] = (const uint8_t*)dev_bufs[b];
        bt.len[b] = lens[b];
        bt.nrec[b] = lens[b] / stride;
        bt.bidx[b] = b;
        max_nrec = std::max(max_nrec, bt.nrec[b]);
    }
    const int W1 = world + 1;
    for (int64_t i = 0; i < (int64_t)n * world; ++i) counts[i] = 0;
    if (n == 0 || max_nrec == 0) return DML_OK;
    hipStream_t st = (hipStream_t)stream;
    const int64_t nblk = (max_nrec + kSplitBlock - 1) / kSplitBlock;
    const size_t cnt_bytes = (sizeof(int32_t) * (size_t)(n * nblk * W1) + 255) & ~(size_t)255;  // int64 arrays follow
    const size_t off_bytes = sizeof(int64_t) * (size_t)(n * nblk * W1);
    const size_t tot_bytes = sizeof(int64_t) * (size_t)(n * W1);
    const size_t base_bytes = sizeof(int64_t) * (size_t)(n * world);
    uint8_t* ws = nullptr;
    hipError_t e = hipMallocAsync((void**)&ws, cnt_bytes + off_bytes + tot_bytes + base_bytes, st);
    if (e != hipSuccess) return set_error(DML_E_HIP, std::string("split workspace: ") + hipGetErrorString(e));
    int32_t* blkcnt = (int32_t*)ws;
    int64_t* blkoff = (int64_t*)(ws + cnt_bytes);
    int64_t* tot = (int64_t*)(ws + cnt_bytes + off_bytes);
    int64_t* dbase = (int64_t*)(ws + cnt_bytes + off_bytes + tot_bytes);
    std::vector<int64_t> htot((size_t)(n * W1)), hbase((size_t)(n * world));
    int rc = DML_OK;
    auto hip = [&](hipError_t x, const char* what) {
        if (x != hipSuccess && rc == DML_OK) rc = set_error(DML_E_HIP, std::string(what) + ": " + hipGetErrorString(x));
        return rc == DML_OK;
    };
    // blocks past a shorter push's records write zero counts
    if (hip(hipMemsetAsync(blkcnt, 0, cnt_bytes, st), "memset")) {
        hipLaunchKernelGGL(k_split_count, dim3((unsigned)nblk, (unsigned)n), dim3(kSplitBlock), 0, st, bt, stride, K,
                           total_rows, step, world, nblk, blkcnt);
        hip(hipGetLastError(), "k_split_count");
    }
    if (rc == DML_OK) {
        hipLaunchKernelGGL(k_split_scan, dim3((unsigned)n, (unsigned)W1), dim3(256), 0, st, blkcnt, nblk, world, blkoff,
                           tot);
        hip(hipGetLastError(), "k_split_scan");
    }
    if (rc == DML_OK && hip(hipMemcpyAsync(htot.data(), tot, tot_bytes, hipMemcpyDeviceToHost, st), "D2H") &&
        hip(hipStreamSynchronize(st), "sync")) {
        // dest-major layout: dest d's slices of push 0, 1, ... n-1
        int64_t run = 0;
        for (int d = 0; d < world; ++d)
            for (int b = 0; b < n; ++b) {
                const int64_t c = htot[(size_t)(b * W1 + d)];
                counts[(int64_t)b * world + d] = c;
                hbase[(size_t)(b * world + d)] = run;
                run += c;
            }
        if (dev_out && run * stride > out_cap) rc = set_error(DML_E_CAPACITY, "split output buffer too small");
    }
    if (rc == DML_OK && dev_out &&
        hip(hipMemcpyAsync(dbase, hbase.data(), base_bytes, hipMemcpyHostToDevice, st), "H2D")) {
        hipLaunchKernelGGL(k_split_scatter, dim3((unsigned)nblk, (unsigned)n), dim3(kSplitBlock), 0, st, bt, stride, K,
                           total_rows, step, world, nblk, blkoff, dbase, (uint8_t*)dev_out);
        hip(hipGetLastError(), "k_split_scatter");
    }
    (void)hipFreeAsync(ws, st);
    // the H2D of hbase reads host memory: it must finish before hbase goes out of scope
    if (hipStreamSynchronize(st) != hipSuccess && rc == DML_OK) rc = set_error(DML_E_HIP, "split sync");
    return rc;
}
