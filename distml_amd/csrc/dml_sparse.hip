// dml_sparse.hip — ordered sparse scatter-add for the float / double array stores
// (FloatArrayStore.java:110-122, DoubleArrayStore.java:115-127) over a chunk of
// pushes, without atomics on the shard.
//
// The reference adds record after record: per shard element, the adds land in
// (push, record) order. Here every kept record becomes (comp, value) with
// comp = row << 32 | seq, seq = its (push, record) rank in the chunk. Records are
// partitioned by "leaf" = row >> SL (a key range holding ~1 K records on
// average) with two 256-way digit passes (count -> exclusive scan -> scatter,
// like one radix pass each; no ordering needed, seq travels along). A leaf
// kernel then orders its records by address in LDS (counting sort by shard
// line) and applies each row once: v = shard[row]; v += u_1; v += u_2 ... in
// sequence order; shard[row] = v. That is the reference's value bit for bit,
// also when one push repeats a key. Address-ordered lanes share DRAM rows,
// which is what makes this faster than per-push scattered atomics over the
// whole shard (scripts/ubench_scatter.hip).
//
// The level-1 count finds the chunk's cutoff (first key outside the shard, or
// the first truncated access): records at or past it keep their partition slot
// with the sequence kSpSkip and are never applied.
// A leaf with more than kSpLeafCap records, or a line bucket with more than
// kSpBucketMax (skewed keys), is not applied by the leaf kernel: it is flagged,
// Ctrl::no_dup is cleared, and the host replays the flagged leaves from a full
// device sort of the chunk (sparse_replay).
#include "dml_device.h"

#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <type_traits>

namespace dml {

namespace {

// Push of a level-1 tile: largest b with tile_base[b] <= tile (binary search over
// the <= 64 prefix entries; a linear walk is a chain of dependent scalar loads).
__device__ inline int push_of_tile(const SpPlan& pl, int64_t tile) {
    int lo = 0, hi = pl.nb;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pl.tile_base[mid] <= tile) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Records [lo, hi) of the chunk-wide first-level bin b: tile t of the bin, or
// (-1) when this block has no tile. Second-level tiles enumerate bins in order.
struct Tile2 {
    int bin;
    int64_t t, ntiles, lo, hi;
};
__device__ inline Tile2 tile2_of(const SpMeta* m, int nbins1, int64_t tile) {
    Tile2 r{-1, 0, 0, 0, 0};
    if (tile >= m->tile_start2[nbins1]) return r;
    int lo = 0, hi = nbins1;  // largest b with tile_start2[b] <= tile
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (m->tile_start2[mid] <= tile) lo = mid;
        else hi = mid;
    }
    while (lo + 1 < nbins1 && m->tile_start2[lo + 1] <= tile) ++lo;  // skip empty bins
    r.bin = lo;
    r.t = tile - m->tile_start2[lo];
    r.ntiles = m->tile_start2[lo + 1] - m->tile_start2[lo];
    r.lo = m->bin_start1[lo] + r.t * kSpTile;
    r.hi = min(r.lo + (int64_t)kSpTile, m->bin_start1[lo + 1]);
    return r;
}

}  // namespace


// LDS staging of a tile's scatter: records are first grouped by bin in LDS (a
// local counting sort), then each bin's run is written to its global segment
// by consecutive threads at consecutive addresses — full-line stores instead of
// one scattered 8-B + 4/8-B store per record (the level-1 / level-2 scatters
// measured 1.8–2.1 TB/s with per-record scattered stores).
template <typename T>
struct SpStage {
    uint64_t c[kSpTile];
    T v[kSpTile];
    uint32_t cnt[256];     // records per bin, then running local position
    uint32_t lstart[257];  // local start of each bin (exclusive scan), lstart[256] = total
    uint32_t gstart[256];  // global start of this tile's segment of each bin
    uint32_t wsum[4];
};
// Compact records (SpPlan::compact): the value travels inside the 8-B word.
struct SpStageC {
    uint64_t c[kSpTile];
    uint32_t cnt[256], lstart[257], gstart[256], wsum[4];
};

// Exclusive scan of st.cnt[0..255] into st.lstart (256 threads), cnt := lstart.
template <typename S>
__device__ inline void sp_stage_scan(S& st) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t a = st.cnt[tid];
    uint32_t x = a;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) st.wsum[wave] = x;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < wave; ++w) base += st.wsum[w];
    st.lstart[tid] = base + x - a;
    if (tid == 255) st.lstart[256] = base + x;
    st.cnt[tid] = base + x - a;
    __syncthreads();
}

// ---- level 1: first digit of the leaf, straight from the wire records -------
// COUNT pass: counts every record whose key lies in the shard and lowers
// ctrl->cutoff to the first record whose key does not (the validation the
// per-push path runs separately). SCATTER pass (cutoff final by then): writes
// every counted record; records at or past the cutoff keep their slot but carry
// the sequence kSpSkip and are never applied.
template <typename T, bool SCATTER>
__global__ __launch_bounds__(256) void k_sp_level1(const Batch bt, const SpPlan pl, int64_t stride, int K,
                                                   int64_t first, int64_t rows, Ctrl* __restrict__ ctrl,
                                                   uint64_t tail_cut, uint32_t* __restrict__ cnt1,
                                                   const uint32_t* __restrict__ off1, uint64_t* __restrict__ comp,
                                                   T* __restrict__ val) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.x;
    const int b = push_of_tile(pl, tile);
    if (!SCATTER && tile == 0 && tid == 0 && tail_cut != kNoPos)
        atomicMin(&ctrl->cutoff, (unsigned long long)tail_cut);
    // level 1 scatters each record straight to its bin (~34 records per bin and
    // tile at config 3); LDS staging as in level 2 measured 2.3x slower here (its
    // 53 KB of LDS cut the occupancy the strided wire-record loads need)
    h[tid] = SCATTER ? (tid < pl.nbins1 ? off1[(int64_t)tid * pl.ntiles1 + tile] : 0u) : 0u;
    __syncthreads();
    uint64_t cut = kNoPos;
    if (SCATTER) {
        cut = ctrl->cutoff;
        if (tail_cut < cut) cut = tail_cut;
    }
    const int64_t r0 = (tile - pl.tile_base[b]) * kSpTile + tid;
    const int64_t n = bt.nrec[b];
    const uint8_t* base = bt.base[b];
    constexpr int kPer = kSpTile / 256;
    int64_t key[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {  // all key loads in flight first
        const int64_t r = min(r0 + i * 256, n - 1);
        key[i] = ld_key(base + r * stride, K);
    }
    T u[kPer];
    if constexpr (SCATTER) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int64_t r = min(r0 + i * 256, n - 1);
            u[i] = Elem<T>::load(base + r * stride + K);
        }
    }
    uint64_t bad = kNoPos;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t r = r0 + i * 256;
        if (r >= n) continue;
        const int64_t row = row_index(key[i], first, rows);
        if (row < 0) {  // key outside the shard: the exception position
            if (!SCATTER) bad = min(bad, pos_of((uint64_t)bt.bidx[b], (uint64_t)(r * stride)));
            continue;
        }
        const uint32_t bin = (uint32_t)((row >> pl.SL) >> pl.D2);
        if constexpr (SCATTER) {
            const uint32_t p = atomicAdd(&h[bin], 1u);
            const bool skip = pos_of((uint64_t)bt.bidx[b], (uint64_t)(r * stride)) >= cut;
            comp[p] = ((uint64_t)row << 32) | (skip ? (uint64_t)kSpSkip : (uint64_t)(pl.rec_base[b] + r));
            val[p] = u[i];
        } else {
            atomicAdd(&h[bin], 1u);
        }
    }
    if constexpr (!SCATTER) {
        if (bad != kNoPos) atomicMin(&ctrl->cutoff, (unsigned long long)bad);
        __syncthreads();
        if (tid < pl.nbins1) cnt1[(int64_t)tid * pl.ntiles1 + tile] = h[tid];
    }
}

// ---- between the levels: bin bounds and the second-level tile table ---------
__global__ __launch_bounds__(256) void k_sp_plan2(const SpPlan pl, const uint32_t* __restrict__ cnt1,
                                                  const uint32_t* __restrict__ off1, SpMeta* __restrict__ m) {
    __shared__ int64_t wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t cells = (int64_t)pl.nbins1 * pl.ntiles1;
    const int64_t kept = cells ? (int64_t)off1[cells - 1] + cnt1[cells - 1] : 0;
    // bin b (one per thread, nbins1 <= 256): start, and its level-2 tile count
    int64_t start = 0, ntiles = 0;
    if (tid < pl.nbins1) {
        start = off1[(int64_t)tid * pl.ntiles1];
        const int64_t end = tid + 1 < pl.nbins1 ? (int64_t)off1[(int64_t)(tid + 1) * pl.ntiles1] : kept;
        ntiles = (end - start + kSpTile - 1) / kSpTile;
        m->bin_start1[tid] = start;
    }
    if (tid == 0) {
        m->bin_start1[pl.nbins1] = kept;
        m->kept = kept;
    }
    int64_t x = ntiles;  // inclusive scan of the tile counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int64_t base = 0;
    for (int w = 0; w < wave; ++w) base += wsum[w];
    if (tid < pl.nbins1) m->tile_start2[tid] = base + x - ntiles;
    if (tid == pl.nbins1 - 1) m->tile_start2[pl.nbins1] = base + x;
}

// ---- level 2: second digit, within each first-level bin ---------------------
template <typename T, bool SCATTER>
__global__ __launch_bounds__(256) void k_sp_level2(const SpPlan pl, const SpMeta* __restrict__ m,
                                                   uint32_t* __restrict__ cnt2, const uint32_t* __restrict__ off2,
                                                   const uint64_t* __restrict__ comp_in, const T* __restrict__ val_in,
                                                   uint64_t* __restrict__ comp_out, T* __restrict__ val_out) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x;
    const Tile2 tl = tile2_of(m, pl.nbins1, blockIdx.x);
    if (tl.bin < 0) return;  // uniform: spare block of the upper-bound grid
    const int nd = 1 << pl.D2;
    const int64_t cell0 = (m->tile_start2[tl.bin] << pl.D2) + tl.t;  // + d * ntiles
    h[tid] = 0u;
    __syncthreads();
    const uint32_t mask = (uint32_t)nd - 1u;
    constexpr int kPer = kSpTile / 256;
    uint64_t c[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t j = tl.lo + i * 256 + tid;
        c[i] = j < tl.hi ? comp_in[j] : 0;
    }
    T u[kPer];
    if constexpr (SCATTER) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int64_t j = tl.lo + i * 256 + tid;
            u[i] = j < tl.hi ? val_in[j] : T(0);
        }
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t j = tl.lo + i * 256 + tid;
        if (j >= tl.hi) continue;
        const uint32_t d = (uint32_t)(c[i] >> (32 + pl.SL)) & mask;
        atomicAdd(&h[d], 1u);
    }
    if constexpr (!SCATTER) {
        __syncthreads();
        if (tid < nd) cnt2[cell0 + (int64_t)tid * tl.ntiles] = h[tid];
    } else {
        __shared__ SpStage<T> st;  // LDS staging, scatter pass only
        __syncthreads();
        st.cnt[tid] = h[tid];
        st.gstart[tid] = tid < nd ? off2[cell0 + (int64_t)tid * tl.ntiles] : 0u;
        __syncthreads();
        sp_stage_scan(st);
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int64_t j = tl.lo + i * 256 + tid;
            if (j >= tl.hi) continue;
            const uint32_t d = (uint32_t)(c[i] >> (32 + pl.SL)) & mask;
            const uint32_t q = atomicAdd(&st.cnt[d], 1u);
            st.c[q] = c[i];
            st.v[q] = u[i];
        }
        __syncthreads();
        const uint32_t nloc = st.lstart[256];
        for (uint32_t i = tid; i < nloc; i += 256) {
            const uint64_t cc = st.c[i];
            const uint32_t d = (uint32_t)(cc >> (32 + pl.SL)) & mask;
            const uint32_t g = st.gstart[d] + (i - st.lstart[d]);
            comp_out[g] = cc;
            val_out[g] = st.v[i];
        }
    }
}

// First record of leaf L in the leaf-ordered arrays (L == nleaves: records kept).
__device__ inline int64_t leaf_start(const SpPlan& pl, const SpMeta* m, const uint32_t* off2, int64_t L) {
    if (L >= pl.nleaves) return m->kept;
    const int b = (int)(L >> pl.D2);
    const int64_t d = L & ((1 << pl.D2) - 1);
    const int64_t nt = m->tile_start2[b + 1] - m->tile_start2[b];
    return nt ? (int64_t)off2[(m->tile_start2[b] << pl.D2) + d * nt] : m->bin_start1[b];
}

// Leaf bounds, computed once on the index stream: bounds[L] .. bounds[L + 1].
__global__ __launch_bounds__(256) void k_sp_bounds(const SpPlan pl, const SpMeta* __restrict__ m,
                                                   const uint32_t* __restrict__ off2, int64_t* __restrict__ bounds) {
    const int64_t L = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (L <= pl.nleaves) bounds[L] = leaf_start(pl, m, off2, L);
}

// ---- leaf: records in address order, one ordered RMW per row ---------------
// A counting sort over kSpLines line buckets of the leaf's row range puts the
// leaf's records in ascending address order (bucket = 32 rows = one 128-B line
// at config-3 leaf sizes), so neighbouring lanes touch neighbouring shard lines
// and a wave's accesses share DRAM rows (random 4-B RMW is bound by row
// activations, scripts/ubench_scatter.hip). A record owns its row when no
// record of the same row (same bucket) has a smaller comp (= earlier sequence).
// Owners of single-record rows issue their shard loads together and add once;
// owners of repeated rows walk their bucket in ascending comp order. Buckets
// over kSpBucketMax records (adversarial keys) send the whole leaf to the exact
// replay before any of its rows is written.
constexpr int kSpLeafThreads = 512;  // 8 waves per leaf
// Every record's shard load is issued right after its comp is loaded (its row
// is known then), so the HBM round trip runs under the LDS counting sort and
// the ownership phase; owners then add and store in record order (measured:
// apply 1.53 -> 1.49 ms on config 3 against loads after the sort).
constexpr int kSpLines = 2 * kSpLeafThreads;
constexpr int kSpBucketMax = 64;

// int32 leaves (IntArrayStore): the negativity check after every add
template <typename T>
constexpr bool kIntLeaf = sizeof(T) == 4 && T(0.5) == T(0);

// A leaf record's fields. Full records: comp = row << 32 | sequence (+ value in
// val[]); compact records (CMP): row within the level-1 bin << 38 | push << 32 |
// value bits, ordered within a row by push.
template <bool CMP>
struct LeafRec {
    uint64_t rowb0;     // CMP: first row of the leaf's level-1 bin (or big leaf)
    uint32_t seq_cut;   // full records: sequences at / past it are never applied
    uint64_t kmask = ~0ull;  // CMP: the (row, push) bits of c >> 32 (a big leaf keeps flags above them)
    __device__ uint64_t row(uint64_t c) const { return CMP ? rowb0 + ((c >> 38) & (kmask >> 6)) : c >> 32; }
    __device__ uint64_t key(uint64_t c) const { return CMP ? (c >> 32) & kmask : c; }  // add order within a row
    __device__ bool applied(uint64_t c) const { return CMP || (uint32_t)c < seq_cut; }
};

// A repeated row's records in ascending key (= push / sequence) order, added to x.
// int32 (IntArrayStore): *neg receives the sequence of the first add that leaves
// the counter negative (IntArrayStore.java:108-110), if any.
template <typename T, bool CMP>
__device__ inline T leaf_chain(T x, uint64_t row, uint64_t row0, int bshift, const uint32_t* bstart,
                               const uint16_t* perm, const uint64_t* sc, const T* sv, const LeafRec<CMP>& lr,
                               uint32_t* neg) {
    const uint32_t b = (uint32_t)((row - row0) >> bshift);
    const uint32_t bs = bstart[b], be = bstart[b + 1];
    bool started = false;
    uint64_t last = 0;  // started: records up to key `last` are in x
    for (;;) {
        uint64_t best = ~0ull;
        int bj = -1;
        for (uint32_t q = bs; q < be; ++q) {
            const int j = perm[q];
            const uint64_t cj = sc[j], kj = lr.key(cj);
            if (lr.row(cj) == row && lr.applied(cj) && (!started || kj > last) && kj < best) {
                best = kj;
                bj = j;
            }
        }
        if (bj < 0) break;
        if constexpr (CMP) x = Elem<T>::add(x, __uint_as_float((uint32_t)sc[bj]));
        else x = Elem<T>::add(x, sv[bj]);
        if constexpr (kIntLeaf<T>)
            if (x < 0 && *neg == kSpSkip) *neg = (uint32_t)best;  // full records: key = row << 32 | sequence
        last = best;
        started = true;
    }
    return x;
}

template <typename T, bool CMP>
__global__ __launch_bounds__(kSpLeafThreads) void k_sp_leaf(T* __restrict__ shard, const int64_t* __restrict__ bounds,
                                                            const uint32_t* __restrict__ cnt2, int64_t cap2,
                                                            const uint64_t* __restrict__ comp,
                                                            const T* __restrict__ val, int SL, int D2, int bshift,
                                                            uint32_t seq_cut, uint8_t* __restrict__ leafflag,
                                                            Ctrl* __restrict__ ctrl, const Ctrl* __restrict__ prev) {
    constexpr int kT = kSpLeafThreads;
    constexpr int kPer = kSpLeafCap / kT;
    static_assert(kSpLines == 2 * kT, "the scan gives each thread two buckets");
    static_assert(!CMP || sizeof(T) == 4, "compact records carry fp32 values");
    __shared__ uint64_t sc[kSpLeafCap];
    __shared__ T sv[CMP ? 1 : kSpLeafCap];
    __shared__ uint16_t perm[kSpLeafCap];
    __shared__ uint32_t bstart[kSpLines + 1];
    __shared__ uint32_t cur[kSpLines];
    __shared__ uint32_t wsum[kT / 64];
    __shared__ int s_over;
    __shared__ uint8_t oflag[kSpLeafCap];  // record i: bit 0 owns its row, bit 1 row repeated
    if (prev && ctrl_abnormal(prev)) return;  // predecessor needs the host first
    const int tid = threadIdx.x;
    const int64_t L = blockIdx.x;
    // compact layout: the leaf's records are [bounds[L], bounds[L+1]); fixed-capacity
    // layout (single-pass partition): [L * cap2, L * cap2 + cnt2[L])
    const int64_t lo = cnt2 ? L * cap2 : bounds[L];
    const int64_t hi = cnt2 ? lo + (int64_t)cnt2[L] : bounds[L + 1];
    const int n = (int)(hi - lo);
    if (hi - lo <= 0) return;
    if (hi - lo > kSpLeafCap) {  // skewed leaf: exact replay on the host's request
        if (tid == 0) {
            leafflag[L] = 1;
            atomicAnd(&ctrl->no_dup, 0u);
        }
        return;
    }
    const uint64_t row0 = (uint64_t)L << SL;
    LeafRec<CMP> lr;
    lr.rowb0 = (uint64_t)(L >> D2) << (SL + D2);
    lr.seq_cut = seq_cut;
    for (int i = tid; i < kSpLines; i += kT) cur[i] = 0;
    if (tid == 0) s_over = 0;
    // loads from clamped in-range indices, all in flight before the first use
    // (a load under `if (i < n)` gets its own vmcnt(0) wait)
    uint64_t c[kPer];
    T u[kPer];
    uint32_t bk[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = min(tid + k * kT, n - 1);
        c[k] = comp[lo + i];
        if constexpr (!CMP) u[k] = val[lo + i];
    }
    T x0[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) x0[k] = shard[lr.row(c[k])];  // every record's row lies in this leaf
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = tid + k * kT;
        bk[k] = (uint32_t)((lr.row(c[k]) - row0) >> bshift);
        if constexpr (CMP) u[k] = __uint_as_float((uint32_t)c[k]);
        else if (i < n) sv[i] = u[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = tid + k * kT;
        if (i < n) {
            sc[i] = c[k];
            atomicAdd(&cur[bk[k]], 1u);
        }
    }
    __syncthreads();
    {  // exclusive scan of the bucket counts: thread t owns buckets 2t, 2t+1
        const uint32_t a0 = cur[2 * tid], a1 = cur[2 * tid + 1];
        uint32_t x = a0 + a1;
        const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t base = 0;
        for (int w = 0; w < wave; ++w) base += wsum[w];
        const uint32_t ex = base + x - (a0 + a1);
        bstart[2 * tid] = ex;
        bstart[2 * tid + 1] = ex + a0;
        __syncthreads();
        cur[2 * tid] = ex;
        cur[2 * tid + 1] = ex + a0;
        if (tid == 0) bstart[kSpLines] = (uint32_t)n;
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = tid + k * kT;
        if (i < n) perm[atomicAdd(&cur[bk[k]], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    // ownership, in address order: sorted position p = tid + k * kT
    int ri[kPer];
    bool own[kPer], multi[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int p = tid + k * kT;
        own[k] = multi[k] = false;
        ri[k] = 0;
        if (p >= n) continue;
        const int i = perm[p];
        ri[k] = i;
        const uint64_t ci = sc[i], row = lr.row(ci), ki = lr.key(ci);
        if (!lr.applied(ci)) continue;  // at / past the cutoff: never applied
        const uint32_t b = (uint32_t)((row - row0) >> bshift);
        const uint32_t bs = bstart[b], be = bstart[b + 1];
        if (be - bs > (uint32_t)kSpBucketMax) s_over = 1;
        bool first = true, dup = false;
        for (uint32_t q = bs; q < be; ++q) {
            const int j = perm[q];
            const uint64_t cj = sc[j];
            if (j != i && lr.row(cj) == row && lr.applied(cj)) {
                const uint64_t kj = lr.key(cj);
                dup = true;
                first &= kj > ki;
                // compact: one push lists the row twice; only the replay's full
                // sequence numbers order those adds
                if (CMP && kj == ki) s_over = 1;
            }
        }
        own[k] = first;
        multi[k] = dup;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k)
        if (tid + k * kT < n) oflag[ri[k]] = (uint8_t)((own[k] ? 1 : 0) | (multi[k] ? 2 : 0));
    __syncthreads();
    if (s_over) {  // uniform
        if (tid == 0) {
            leafflag[L] = 1;
            atomicAnd(&ctrl->no_dup, 0u);
        }
        return;
    }
    uint32_t neg = kSpSkip;  // int32: sequence of this thread's first add that left a counter negative
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = tid + k * kT;
        if (i >= n) continue;
        const uint8_t f = oflag[i];
        if (!(f & 1)) continue;
        const uint64_t row = lr.row(sc[i]);
        T x = x0[k];
        if (!(f & 2)) {
            x = Elem<T>::add(x, u[k]);
            if constexpr (kIntLeaf<T>)
                if (x < 0) neg = min(neg, (uint32_t)sc[i]);
        } else {
            uint32_t rn = kSpSkip;
            x = leaf_chain<T, CMP>(x, row, row0, bshift, bstart, perm, sc, sv, lr, &rn);
            neg = min(neg, rn);
        }
        shard[row] = x;
    }
    // the chunk's first negative counter (min sequence); the host undoes every add
    // after it, so the store holds what the reference's does when it throws
    if constexpr (kIntLeaf<T>)
        if (neg != kSpSkip) atomicMin(&ctrl->neg_pos, (unsigned long long)neg);
}

// Replay of flagged leaves from the fully sorted chunk (comp ascending).
template <typename T>
__global__ __launch_bounds__(256) void k_sp_runs(T* __restrict__ shard, const uint64_t* __restrict__ comp,
                                                 const T* __restrict__ val, int64_t n, int SL,
                                                 const uint8_t* __restrict__ leafflag, uint32_t seq_cut,
                                                 Ctrl* __restrict__ ctrl) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t row = comp[p] >> 32;
    if (!leafflag[row >> SL]) return;
    if (p > 0 && (comp[p - 1] >> 32) == row) return;
    if ((uint32_t)comp[p] >= seq_cut) return;  // the row's only records are at / past the cutoff
    T v = shard[row];
    // the row's run in sequence order; records past the cutoff sort last
    bool neg = false;
    for (int64_t q = p; q < n && (comp[q] >> 32) == row && (uint32_t)comp[q] < seq_cut; ++q) {
        v = Elem<T>::add(v, val[q]);
        if constexpr (kIntLeaf<T>)
            if (!neg && v < 0) {  // this row's first negative counter (int32 arrays)
                neg = true;
                atomicMin(&ctrl->neg_pos, (unsigned long long)(uint32_t)comp[q]);
            }
    }
    shard[row] = v;
}

// ---- single-pass partition (no count passes, no scans) -------------------------
// Level 1 (k_sp_l1_fast): a tile's records are counted per bin in LDS (the
// returned count is each record's rank), one global cursor reservation per (tile,
// bin), then every record is written at its bin's reserved slot of a
// fixed-capacity region (cap1 records per bin: twice the mean + one tile; config
// 3's lattice keys put up to 1.4x the mean into one bin). Level 2 (k_sp_l2_fast):
// one block per 4096-record tile of a bin's filled part, records grouped by leaf
// in LDS and each leaf's run written at a slot reserved with one cursor atomic per
// (tile, leaf) in the leaf's fixed region (cap2 records). Any overflow (skewed
// keys) sets the status and the host runs the counted partition instead, before
// the leaf kernel. Level 1 also finds the cutoff (first key outside the shard),
// which the leaf applies as a sequence cut. Measured against the counted
// partition (same box, 2 rounds): config 3 step 1.46 / 1.56 ms vs 1.69 / 1.62 ms;
// a count-free variant with tile-local level-1 output and a gathering level 2:
// 1.64 / 1.75 ms.
template <typename T, bool CMP>
__global__ __launch_bounds__(256) void k_sp_l1_fast(const Batch bt, const SpPlan pl, int64_t stride, int K,
                                                    int64_t first, int64_t rows, Ctrl* __restrict__ ctrl,
                                                    uint64_t tail_cut, uint32_t* __restrict__ cur1,
                                                    uint64_t* __restrict__ comp, T* __restrict__ val,
                                                    SpStat* __restrict__ stat) {
    __shared__ uint32_t h[256];
    __shared__ uint32_t base[256];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.x;
    const int b = push_of_tile(pl, tile);
    if (tile == 0 && tid == 0 && tail_cut != kNoPos) atomicMin(&ctrl->cutoff, (unsigned long long)tail_cut);
    h[tid] = 0u;
    __syncthreads();
    const int64_t r0 = (tile - pl.tile_base[b]) * kSpTile + tid;
    const int64_t n = bt.nrec[b];
    const uint8_t* base_b = bt.base[b];
    constexpr int kPer = kSpTile / 256;
    int64_t key[kPer];
    T u[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t r = min(r0 + i * 256, n - 1);
        key[i] = ld_key(base_b + r * stride, K);
        u[i] = Elem<T>::load(base_b + r * stride + K);
    }
    uint64_t bad = kNoPos;
    int64_t row[kPer];
    uint32_t rank[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t r = r0 + i * 256;
        row[i] = -1;
        if (r >= n) continue;
        row[i] = row_index(key[i], first, rows);
        if (row[i] < 0) {
            bad = min(bad, pos_of((uint64_t)bt.bidx[b], (uint64_t)(r * stride)));
            continue;
        }
        rank[i] = atomicAdd(&h[(uint32_t)((row[i] >> pl.SL) >> pl.D2)], 1u);
    }
    if (bad != kNoPos) atomicMin(&ctrl->cutoff, (unsigned long long)bad);
    __syncthreads();
    if (tid < pl.nbins1 && h[tid]) {
        const uint32_t at = atomicAdd(&cur1[tid], h[tid]);
        base[tid] = at;
        if ((int64_t)at + h[tid] > pl.cap1) stat->overflow = 1u;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        if (row[i] < 0) continue;
        const uint32_t bin = (uint32_t)((row[i] >> pl.SL) >> pl.D2);
        const int64_t q = (int64_t)base[bin] + rank[i];
        if (q >= pl.cap1) continue;
        const int64_t at = (int64_t)bin * pl.cap1 + q;
        if constexpr (CMP) {
            const int64_t rb = (int64_t)bin << (pl.SL + pl.D2);
            comp[at] = ((uint64_t)(row[i] - rb) << 38) | ((uint64_t)b << 32) | (uint64_t)__float_as_uint(u[i]);
        } else {
            comp[at] = ((uint64_t)row[i] << 32) | (uint64_t)(pl.rec_base[b] + r0 + i * 256);
            val[at] = u[i];
        }
    }
}
template <typename T, bool CMP>
__global__ __launch_bounds__(256) void k_sp_l2_fast(const SpPlan pl, const uint32_t* __restrict__ cur1,
                                                    const uint64_t* __restrict__ comp_in,
                                                    const T* __restrict__ val_in, uint32_t* __restrict__ cur2,
                                                    uint64_t* __restrict__ comp_out, T* __restrict__ val_out,
                                                    SpStat* __restrict__ stat) {
    using Stage = std::conditional_t<CMP, SpStageC, SpStage<T>>;
    __shared__ Stage st;
    constexpr int kRowShift = CMP ? 38 : 32;  // the record's row (within its level-1 bin if CMP)
    const int tid = threadIdx.x;
    // Every tile of a level-1 bin runs on one XCD (blocks b and b + 8 share one; the
    // grid is padded to a multiple of 8 bins): the runs that neighbouring tiles write
    // into one leaf region meet in that XCD's L2 instead of leaving partial lines in
    // two. Config-3 step 1.406-1.409 -> 1.369-1.372 ms against bin-major tiles (same
    // box, 3 rounds).
    const int64_t s8 = blockIdx.x / 8u;
    const int bin = (int)(blockIdx.x % 8u) + 8 * (int)(s8 / pl.tiles2_per_bin);
    const int64_t t = s8 % pl.tiles2_per_bin;
    if (bin >= pl.nbins1) return;
    const int64_t nbin = min((int64_t)cur1[bin], pl.cap1);
    const int64_t lo = t * kSpTile;
    if (lo >= nbin) return;
    const int64_t hi = min(lo + (int64_t)kSpTile, nbin);
    const int nd = 1 << pl.D2;
    const uint32_t mask = (uint32_t)nd - 1u;
    const int64_t src0 = (int64_t)bin * pl.cap1;
    constexpr int kPer = kSpTile / 256;
    uint64_t c[kPer];
    T u[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t j = lo + i * 256 + tid;
        c[i] = j < hi ? comp_in[src0 + j] : 0;
        if constexpr (!CMP) u[i] = j < hi ? val_in[src0 + j] : T(0);
    }
    st.cnt[tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPer; ++i)
        if (lo + i * 256 + tid < hi) atomicAdd(&st.cnt[(uint32_t)(c[i] >> (kRowShift + pl.SL)) & mask], 1u);
    __syncthreads();
    {
        const uint32_t cn = st.cnt[tid];
        uint32_t g = 0;
        if (tid < nd && cn) {
            g = atomicAdd(&cur2[((int64_t)bin << pl.D2) + tid], cn);
            if ((int64_t)g + cn > pl.cap2) stat->overflow = 1u;
        }
        st.gstart[tid] = g;
    }
    __syncthreads();
    sp_stage_scan(st);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        if (lo + i * 256 + tid >= hi) continue;
        const uint32_t d = (uint32_t)(c[i] >> (kRowShift + pl.SL)) & mask;
        const uint32_t q = atomicAdd(&st.cnt[d], 1u);
        st.c[q] = c[i];
        if constexpr (!CMP) st.v[q] = u[i];
    }
    __syncthreads();
    const uint32_t nloc = st.lstart[256];
    for (uint32_t i = tid; i < nloc; i += 256) {
        const uint64_t cc = st.c[i];
        const uint32_t d = (uint32_t)(cc >> (kRowShift + pl.SL)) & mask;
        const int64_t q = (int64_t)st.gstart[d] + (i - st.lstart[d]);
        if (q >= pl.cap2) continue;
        const int64_t at = (((int64_t)bin << pl.D2) + d) * pl.cap2 + q;
        comp_out[at] = cc;
        if constexpr (!CMP) val_out[at] = st.v[i];
    }
}

// Records of the leaves the leaf kernel flagged (fixed-capacity layout), packed
// into one array for the exact replay (sort + runs).
template <typename T>
__global__ __launch_bounds__(256) void k_sp_pack_flagged(const uint32_t* __restrict__ cnt2, int64_t cap2,
                                                         const uint8_t* __restrict__ leafflag,
                                                         const uint64_t* __restrict__ comp, const T* __restrict__ val,
                                                         unsigned long long* __restrict__ packed_n,
                                                         uint64_t* __restrict__ comp_out, T* __restrict__ val_out) {
    __shared__ unsigned long long at;
    const int64_t L = blockIdx.x;
    if (!leafflag[L]) return;
    const int64_t n = min((int64_t)cnt2[L], cap2);
    if (threadIdx.x == 0) at = atomicAdd(packed_n, (unsigned long long)n);
    __syncthreads();
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        comp_out[at + i] = comp[L * cap2 + i];
        val_out[at + i] = val[L * cap2 + i];
    }
}

// ---- one-level partition: big leaves sorted in LDS (no second pass) -------------
// k_sp_l1_big: as k_sp_l1_fast, with up to kSpBigBins big leaves of 2^BL rows as its
// bins (the LDS histogram holds them all) and one region per (big leaf, slice). The
// grid is slice-major: block b runs on XCD b % 8 (the dispatcher deals blocks round
// robin) and takes the (b / 8)-th tile of the pushes p with p % 8 == b % 8, so every
// region is written from one XCD and the runs that tiles append to it meet in that
// XCD's L2 (scripts/ubench_l1.hip: 3 815 bins x 8 slices 303 us against 440 us with
// one region per bin written from every XCD, for 32 M random keys).
__global__ __launch_bounds__(256) void k_sp_l1_big(const Batch bt, const SpPlan pl, int64_t stride, int K,
                                                   int64_t first, int64_t rows, Ctrl* __restrict__ ctrl,
                                                   uint64_t tail_cut, uint32_t* __restrict__ curS,
                                                   uint64_t* __restrict__ comp, SpStat* __restrict__ stat) {
    // records per big leaf, then this tile's base in its region: two 16-bit halves a
    // word (counts <= kSpTile, bases < capS < 2^16), 32 KB, so one partition block
    // fits beside two leaf blocks on a CU
    __shared__ uint32_t h[kSpBigBins / 2];
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && tid == 0 && tail_cut != kNoPos) atomicMin(&ctrl->cutoff, (unsigned long long)tail_cut);
    const int x = (int)(blockIdx.x % kSpSlices);
    const int64_t ti = blockIdx.x / kSpSlices;
    int b = -1;
    int64_t tin = 0;
    for (int p = x; p < pl.nb; p += kSpSlices) {  // <= 8 pushes per slice
        const int64_t t = pl.tile_base[p + 1] - pl.tile_base[p];
        if (ti < pl.sbase[p] + t) {
            b = p;
            tin = ti - pl.sbase[p];
            break;
        }
    }
    if (b < 0) return;  // uniform: past this slice's tiles
    for (int j = tid; j < (pl.nbig + 1) / 2; j += 256) h[j] = 0u;
    __syncthreads();
    const int64_t r0 = tin * kSpTile + tid;
    const int64_t n = bt.nrec[b];
    const uint8_t* base_b = bt.base[b];
    constexpr int kPer = kSpTile / 256;
    int64_t key[kPer];
    float u[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t r = min(r0 + i * 256, n - 1);
        key[i] = ld_key(base_b + r * stride, K);
        u[i] = Elem<float>::load(base_b + r * stride + K);
    }
    uint64_t bad = kNoPos;
    int64_t row[kPer];
    uint32_t rank[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int64_t r = r0 + i * 256;
        row[i] = -1;
        if (r >= n) continue;
        row[i] = row_index(key[i], first, rows);
        if (row[i] < 0) {
            bad = min(bad, pos_of((uint64_t)bt.bidx[b], (uint64_t)(r * stride)));
            continue;
        }
        const uint32_t B = (uint32_t)(row[i] >> pl.BL), sh = 16u * (B & 1u);
        rank[i] = (atomicAdd(&h[B >> 1], 1u << sh) >> sh) & 0xFFFFu;
    }
    if (bad != kNoPos) atomicMin(&ctrl->cutoff, (unsigned long long)bad);
    __syncthreads();
    for (int j = tid; j < (pl.nbig + 1) / 2; j += 256) {  // both halves of a word in one thread
        const uint32_t w = h[j];
        uint32_t o = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const uint32_t c = (w >> (16 * e)) & 0xFFFFu;
            const int64_t B = 2 * (int64_t)j + e;
            if (!c || B >= pl.nbig) continue;
            const uint32_t at = atomicAdd(&curS[(int64_t)x * pl.nbig + B], c);
            if ((int64_t)at + c > pl.capS) stat->overflow = 1u;
            o |= min(at, 0xFFFFu) << (16 * e);  // an overflowing base is not used (q >= capS)
        }
        h[j] = o;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        if (row[i] < 0) continue;
        const int64_t B = row[i] >> pl.BL;
        const int64_t q = (int64_t)((h[B >> 1] >> (16 * (B & 1))) & 0xFFFFu) + rank[i];
        if (q >= pl.capS) continue;
        comp[(B * kSpSlices + x) * pl.capS + q] = ((uint64_t)(row[i] - (B << pl.BL)) << 38) | ((uint64_t)b << 32) |
                                                  (uint64_t)__float_as_uint(u[i]);
    }
}

// k_sp_leaf_big: k_sp_leaf's ordered apply for one big leaf (up to kSpBigCap compact
// records from its 8 slice regions): counting sort over kSpBigLines line buckets,
// then each thread takes sorted positions p = tid + k * 512 — its shard loads are
// issued in address order (a round of the block covers 1/8 of the big leaf's range,
// which keeps the DRAM rows the chip touches at once few: loads in record order,
// across a 1 MB big leaf, ran the kernel 1.61 ms against 1.36 ms in address order)
// and run under the ownership scan of the same positions. 8-wave blocks of 48 KB of
// LDS, up to three per CU. Big leaves of 2^16 rows (<= 4 096 records) run config 3's
// step 1.32-1.33 ms against 1.39 ms for 2^17 rows (<= 6 144 records, 68 KB, two per
// CU) and 1.40 ms for 2^15 (<= 2 048: the partition's 64 KB histogram), 3 rounds on
// one box; one 16-wave block of 12 K records per CU ran 1.36 ms.
constexpr int kSpBigThreads = 512;
constexpr int kSpBigLines = 2 * kSpBigThreads;
__global__ __launch_bounds__(kSpBigThreads) void k_sp_leaf_big(float* __restrict__ shard,
                                                               const uint32_t* __restrict__ curS, int64_t nbig,
                                                               int64_t capS, const uint64_t* __restrict__ comp, int BL,
                                                               int bshift, uint8_t* __restrict__ leafflag,
                                                               Ctrl* __restrict__ ctrl, const Ctrl* __restrict__ prev) {
    constexpr int kT = kSpBigThreads;
    constexpr int kPer = kSpBigCap / kT;
    __shared__ uint64_t sc[kSpBigCap];
    __shared__ uint16_t perm[kSpBigCap];
    __shared__ uint32_t bstart[kSpBigLines + 1];
    __shared__ uint32_t cur[kSpBigLines];
    __shared__ uint32_t wsum[kT / 64];
    __shared__ int s_over;
    if (prev && ctrl_abnormal(prev)) return;  // predecessor needs the host first
    const int tid = threadIdx.x;
    const int64_t B = blockIdx.x;
    int64_t pre[kSpSlices + 1];
    pre[0] = 0;
#pragma unroll
    for (int x = 0; x < kSpSlices; ++x) pre[x + 1] = pre[x] + min((int64_t)curS[(int64_t)x * nbig + B], capS);
    const int n = (int)pre[kSpSlices];
    if (n <= 0) return;
    if (n > kSpBigCap) {  // skewed big leaf: exact replay on the host's request
        if (tid == 0) {
            leafflag[B] = 1;
            atomicAnd(&ctrl->no_dup, 0u);
        }
        return;
    }
    const uint64_t row0 = (uint64_t)B << BL;
    LeafRec<true> lr;
    lr.rowb0 = row0;
    lr.seq_cut = kSpSkip;
    for (int i = tid; i < kSpBigLines; i += kT) cur[i] = 0;
    if (tid == 0) s_over = 0;
    uint64_t c[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = min(tid + k * kT, n - 1);
        int x = 0;
#pragma unroll
        for (int y = 1; y < kSpSlices; ++y) x += i >= pre[y] ? 1 : 0;
        // read once: non-temporal, out of the L2 the shard's RMW lines use (-0.5 %,
        // 3 of 3 same-box rounds)
        c[k] = __builtin_nontemporal_load(&comp[(B * kSpSlices + x) * capS + (i - pre[x])]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = tid + k * kT;
        if (i < n) {
            sc[i] = c[k];
            atomicAdd(&cur[(uint32_t)((lr.row(c[k]) - row0) >> bshift)], 1u);
        }
    }
    __syncthreads();
    {  // exclusive scan of the bucket counts: thread t owns buckets 2t, 2t+1
        const uint32_t a0 = cur[2 * tid], a1 = cur[2 * tid + 1];
        uint32_t x = a0 + a1;
        const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t base = 0;
        for (int w = 0; w < wave; ++w) base += wsum[w];
        const uint32_t ex = base + x - (a0 + a1);
        bstart[2 * tid] = ex;
        bstart[2 * tid + 1] = ex + a0;
        __syncthreads();
        cur[2 * tid] = ex;
        cur[2 * tid + 1] = ex + a0;
        if (tid == 0) bstart[kSpBigLines] = (uint32_t)n;
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = tid + k * kT;  // the word from LDS: c[] is dead by now (fewer live VGPRs)
        if (i < n) perm[atomicAdd(&cur[(uint32_t)((lr.row(sc[i]) - row0) >> bshift)], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    // sorted positions p = tid + k * kT: the shard loads first (address order), then
    // the ownership scan of the same positions while they are in flight
    // slot k takes the sorted twelfth (k + rot) % kPer: with rot = B % kPer, the blocks'
    // concurrent rounds do not all sit at the same offset of their big leaves (-0.5 %,
    // 3 rounds on one box)
    const int rot = (int)(B % kPer);
    // only the shard values stay in registers; the words are re-read from LDS where
    // needed (109 -> fewer VGPRs, so a partition block fits beside two leaf blocks)
    float x0[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int kk = k + rot >= kPer ? k + rot - kPer : k + rot;
        x0[k] = shard[lr.row(sc[perm[min(tid + kk * kT, n - 1)]])];
    }
    uint32_t fl = 0;  // bit 2k: owns its row, bit 2k+1: row repeated
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int p = tid + (k + rot >= kPer ? k + rot - kPer : k + rot) * kT;
        if (p >= n) continue;
        const int i = perm[p];
        const uint64_t ci = sc[i], row = lr.row(ci), ki = lr.key(ci);
        const uint32_t b = (uint32_t)((row - row0) >> bshift);
        const uint32_t bs = bstart[b], be = bstart[b + 1];
        if (be - bs > (uint32_t)kSpBucketMax) s_over = 1;
        bool first = true, dup = false;
        for (uint32_t q = bs; q < be; ++q) {
            const int j = perm[q];
            const uint64_t cj = sc[j];
            if (j != i && lr.row(cj) == row) {
                const uint64_t kj = lr.key(cj);
                dup = true;
                first &= kj > ki;
                if (kj == ki) s_over = 1;  // one push lists the row twice: the replay orders it
            }
        }
        fl |= ((first ? 1u : 0u) | (dup ? 2u : 0u)) << (2 * k);
    }
    __syncthreads();
    if (s_over) {  // uniform: nothing of a flagged big leaf is written
        if (tid == 0) {
            leafflag[B] = 1;
            atomicAnd(&ctrl->no_dup, 0u);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t f = fl >> (2 * k);
        if (!(f & 1u)) continue;  // not an owner (or past n)
        const uint64_t ci = sc[perm[tid + (k + rot >= kPer ? k + rot - kPer : k + rot) * kT]];
        const uint64_t row = lr.row(ci);
        float xv = x0[k];
        if (!(f & 2u)) {
            xv = Elem<float>::add(xv, __uint_as_float((uint32_t)ci));
        } else {
            uint32_t rn = kSpSkip;
            xv = leaf_chain<float, true>(xv, row, row0, bshift, bstart, perm, sc, (const float*)nullptr, lr, &rn);
        }
        shard[row] = xv;
    }
}

// ---- host side ----------------------------------------------------------------
static int ceil_log2(int64_t x) {
    int r = 0;
    while ((int64_t)1 << r < x) ++r;
    return r;
}

// The SL-dependent fields of a plan (leaf = row >> SL; two 256-way digits).
static void plan_leaves(SpPlan& pl, int64_t rows, int SL) {
    pl.SL = SL;
    pl.nleaves = (rows + ((int64_t)1 << SL) - 1) >> SL;
    pl.D2 = std::min(8, ceil_log2(pl.nleaves));
    pl.nbins1 = (int)((pl.nleaves + ((int64_t)1 << pl.D2) - 1) >> pl.D2);
    pl.max_tiles2 = (pl.nrec + kSpTile - 1) / kSpTile + pl.nbins1;
    // single-pass layout: cap1 records per level-1 bin (twice the mean + one tile;
    // config 3's lattice keys put up to 1.4x the mean into one bin, skewed keys
    // overflow and take the counted partition), cap2 per leaf (twice the mean + 256,
    // at most what the leaf kernel orders)
    pl.cap1 = (pl.nrec / std::max(pl.nbins1, 1)) * 2 + kSpTile;
    pl.cap2 = std::min<int64_t>(kSpLeafCap, 2 * (pl.nrec / std::max<int64_t>(pl.nleaves, 1)) + 256);
    pl.tiles2_per_bin = (pl.cap1 + kSpTile - 1) / kSpTile;
}

SpPlan sparse_plan(const Batch& bt, int nb, int64_t rows) {
    SpPlan pl{};
    pl.nb = nb;
    int64_t nrec = 0, ntiles = 0;
    for (int b = 0; b < nb; ++b) {
        pl.tile_base[b] = ntiles;
        pl.rec_base[b] = nrec;
        ntiles += (bt.nrec[b] + kSpTile - 1) / kSpTile;
        nrec += bt.nrec[b];
    }
    pl.tile_base[nb] = ntiles;
    pl.rec_base[nb] = nrec;
    pl.ntiles1 = ntiles;
    pl.nrec = nrec;
    // leaves of ~kSpLeafCap/2 records on average, at most 65536 (two 256-way digits)
    const double span = (double)(kSpLeafCap / 2) * (double)rows / (double)std::max<int64_t>(nrec, 1);
    int SL = 0;
    while (SL < 31 && (double)((int64_t)1 << (SL + 1)) <= span) ++SL;
    while (SL < 31 && ((rows + ((int64_t)1 << SL) - 1) >> SL) > 65536) ++SL;
    plan_leaves(pl, rows, SL);
    pl.fast = 1;
    pl.seq_cut = kSpSkip;
    return pl;
}

// One-level partition: big leaves of 2^BL rows, as few as fit the
// one-level pass's LDS histogram (<= kSpBigBins), holding 0.68 K - 2.9 K records on
// average (kSpBigCap orders up to 4 096: config 3's lattice keys put 1.41x the
// mean, 2 959 of 2 097, into its fullest big leaf of 2^16 rows; fuller ones take the
// exact replay). The 8 slices (pushes p % 8) must carry near-equal shares, since
// slice x's tiles all run on one XCD.
void sparse_plan_big(SpPlan& pl, const Batch& bt, int64_t rows) {
    pl.big = 0;
    if (!pl.compact || pl.nb < kSpSlices || pl.nrec <= 0) return;
    int BL = 0;
    while (BL < 24 && ((rows + ((int64_t)1 << BL) - 1) >> BL) > kSpBigBins) ++BL;
    const int64_t nbig = (rows + ((int64_t)1 << BL) - 1) >> BL;
    const int64_t mean = pl.nrec / nbig;
    // the compact word: value | push << 32 | row within the big leaf << 38
    if (BL > 24 || mean < kSpBigCap / 6 || mean > kSpBigCap * 17 / 24) return;
    // the exact replay re-plans a big leaf's chunk with BL inside the layout sized for
    // the two-level plan (SL): in bounds only while big leaves are at least as large
    // (fewer, larger leaves), so refuse the one-level pass otherwise
    if (BL < pl.SL) return;
    int64_t srec[kSpSlices] = {0}, stile[kSpSlices] = {0};
    for (int b = 0; b < pl.nb; ++b) {
        pl.sbase[b] = stile[b % kSpSlices];
        stile[b % kSpSlices] += pl.tile_base[b + 1] - pl.tile_base[b];
        srec[b % kSpSlices] += bt.nrec[b];
    }
    int64_t smax = 0, tmax = 0;
    for (int x = 0; x < kSpSlices; ++x) {
        smax = std::max(smax, srec[x]);
        tmax = std::max(tmax, stile[x]);
    }
    if (smax * kSpSlices > pl.nrec * 5 / 4) return;  // unbalanced slices: one XCD would do most of the work
    pl.BL = BL;
    pl.nbig = nbig;
    pl.tiles_per_slice = tmax;
    // a region holds twice the slice's mean share of a big leaf + 512 (pushes spread
    // their keys: config 3's regions peak at 1.1x the mean); overflow -> counted partition
    pl.capS = 2 * (smax / nbig) + 512;
    if (pl.capS >= 0xFFFF) return;  // the one-level pass keeps region bases in 16 bits
    pl.big = 1;
}

uint32_t sparse_seq_cut(const SpPlan& pl, const Batch& bt, uint64_t cut, int64_t stride) {
    if (cut == kNoPos) return kSpSkip;
    const int gb = (int)(cut >> 40);
    const int64_t off = (int64_t)(cut & kOffMask);
    for (int b = 0; b < pl.nb; ++b)
        if (bt.bidx[b] == gb) return (uint32_t)(pl.rec_base[b] + off / stride);
    return 0u;
}

SpLayout sparse_layout(const SpPlan& pl, int vbytes) {
    SpLayout l{};
    auto take = [&](size_t bytes) {
        const size_t o = l.total;
        l.total += (bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t n = (size_t)std::max<int64_t>(pl.nrec, 1);
    const size_t cells1 = (size_t)pl.nbins1 * (size_t)pl.ntiles1 + 1;
    const size_t cells2 = ((size_t)pl.max_tiles2 << pl.D2) + 1;
    // the fixed-capacity layout (single pass) is larger than the compact one (counted)
    const size_t n1 = std::max(n, (size_t)pl.nbins1 * (size_t)pl.cap1);
    const size_t n2 = std::max(n, (size_t)pl.nleaves * (size_t)pl.cap2);
    l.meta = take(sizeof(SpMeta));
    l.comp1 = take(n1 * 8);
    l.val1 = take(n1 * (size_t)vbytes);
    l.comp2 = take(n2 * 8);
    l.val2 = take(n2 * (size_t)vbytes);
    l.cur1 = take(256 * 4);
    l.cur2 = take((size_t)pl.nleaves * 4);
    l.stat = take(sizeof(SpStat) + sizeof(unsigned long long));  // + the replay's pack counter
    l.cnt1 = take(cells1 * 4);
    l.off1 = take(cells1 * 4);
    l.cnt2 = take(cells2 * 4);
    l.off2 = take(cells2 * 4);
    l.leafflag = take((size_t)pl.nleaves);
    l.bounds = take(((size_t)pl.nleaves + 1) * 8);
    if (pl.big) {
        l.big = take((size_t)pl.nbig * kSpSlices * (size_t)pl.capS * 8);
        l.curS = take((size_t)pl.nbig * kSpSlices * 4);
    }
    size_t t1 = 0, t2 = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t1, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)cells1);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)cells2);
    l.scan_tmp_bytes = std::max(t1, t2);
    l.scan_tmp = take(l.scan_tmp_bytes);
    return l;
}

template <typename T>
static hipError_t partition_t(const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws, int64_t stride,
                              int K, int64_t first, int64_t rows, Ctrl* ctrl, uint64_t tail_cut, hipStream_t st,
                              bool clear_flags = true) {
    SpMeta* m = (SpMeta*)(ws + l.meta);
    uint64_t* comp1 = (uint64_t*)(ws + l.comp1);
    uint64_t* comp2 = (uint64_t*)(ws + l.comp2);
    T* val1 = (T*)(ws + l.val1);
    T* val2 = (T*)(ws + l.val2);
    uint32_t* cnt1 = (uint32_t*)(ws + l.cnt1);
    uint32_t* off1 = (uint32_t*)(ws + l.off1);
    uint32_t* cnt2 = (uint32_t*)(ws + l.cnt2);
    uint32_t* off2 = (uint32_t*)(ws + l.off2);
    const int cells1 = (int)((int64_t)pl.nbins1 * pl.ntiles1 + 1);
    const int cells2 = (int)((pl.max_tiles2 << pl.D2) + 1);
    hipError_t e = clear_flags ? hipMemsetAsync(ws + l.leafflag, 0, (size_t)pl.nleaves, st) : hipSuccess;
    if (e == hipSuccess) e = hipMemsetAsync(cnt1, 0, (size_t)cells1 * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(cnt2, 0, (size_t)cells2 * 4, st);
    if (e != hipSuccess) return e;
    if (pl.ntiles1 > 0) {
        hipLaunchKernelGGL((k_sp_level1<T, false>), dim3((unsigned)pl.ntiles1), dim3(256), 0, st, bt, pl, stride, K,
                           first, rows, ctrl, tail_cut, cnt1, (const uint32_t*)nullptr, (uint64_t*)nullptr, (T*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else if (tail_cut != kNoPos) {  // no complete record: only the truncation position
        if ((e = hipMemcpyAsync(&ctrl->cutoff, &tail_cut, sizeof tail_cut, hipMemcpyHostToDevice, st)) != hipSuccess)
            return e;
    }
    size_t tb = l.scan_tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(ws + l.scan_tmp, tb, cnt1, off1, cells1, st)) != hipSuccess) return e;
    if (pl.ntiles1 > 0) {
        hipLaunchKernelGGL((k_sp_level1<T, true>), dim3((unsigned)pl.ntiles1), dim3(256), 0, st, bt, pl, stride, K,
                           first, rows, ctrl, tail_cut, (uint32_t*)nullptr, (const uint32_t*)off1, comp1, val1);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_sp_plan2, dim3(1), dim3(256), 0, st, pl, (const uint32_t*)cnt1, (const uint32_t*)off1, m);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (pl.max_tiles2 > 0) {
        hipLaunchKernelGGL((k_sp_level2<T, false>), dim3((unsigned)pl.max_tiles2), dim3(256), 0, st, pl,
                           (const SpMeta*)m, cnt2, (const uint32_t*)nullptr, (const uint64_t*)comp1, (const T*)val1,
                           (uint64_t*)nullptr, (T*)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    tb = l.scan_tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(ws + l.scan_tmp, tb, cnt2, off2, cells2, st)) != hipSuccess) return e;
    if (pl.max_tiles2 > 0) {
        hipLaunchKernelGGL((k_sp_level2<T, true>), dim3((unsigned)pl.max_tiles2), dim3(256), 0, st, pl,
                           (const SpMeta*)m, (uint32_t*)nullptr, (const uint32_t*)off2, (const uint64_t*)comp1,
                           (const T*)val1, comp2, val2);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_sp_bounds, dim3((unsigned)((pl.nleaves + 1 + 255) / 256)), dim3(256), 0, st, pl,
                       (const SpMeta*)m, (const uint32_t*)off2, (int64_t*)(ws + l.bounds));
    return hipGetLastError();
}

// Status + the partition's cutoff for the host (read before the leaf launch).
static hipError_t finish_fast(uint8_t* ws, const SpLayout& l, Ctrl* ctrl, SpStat* hstat, hipStream_t st) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = hipMemcpyAsync(hstat, ws + l.stat, sizeof(unsigned int), hipMemcpyDeviceToHost, st)) != hipSuccess)
        return e;
    return hipMemcpyAsync(&hstat->cutoff, &ctrl->cutoff, sizeof(unsigned long long), hipMemcpyDeviceToHost, st);
}

template <typename T>
static hipError_t partition_fast_t(const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws, int64_t stride,
                                   int K, int64_t first, int64_t rows, Ctrl* ctrl, uint64_t tail_cut, SpStat* hstat,
                                   hipStream_t st) {
    uint32_t* cur1 = (uint32_t*)(ws + l.cur1);
    uint32_t* cur2 = (uint32_t*)(ws + l.cur2);
    SpStat* stat = (SpStat*)(ws + l.stat);
    hipError_t e = hipMemsetAsync(ws + l.leafflag, 0, (size_t)pl.nleaves, st);
    if (e == hipSuccess) e = hipMemsetAsync(cur1, 0, 256 * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(cur2, 0, (size_t)pl.nleaves * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(stat, 0, sizeof(SpStat), st);
    if (e != hipSuccess) return e;
    if (pl.ntiles1 > 0) {
        const dim3 g1((unsigned)pl.ntiles1), g2((unsigned)((pl.nbins1 + 7) / 8 * 8 * pl.tiles2_per_bin));
        uint64_t* c1 = (uint64_t*)(ws + l.comp1);
        uint64_t* c2 = (uint64_t*)(ws + l.comp2);
        if constexpr (sizeof(T) == 4) {
            if (pl.compact) {
                hipLaunchKernelGGL((k_sp_l1_fast<T, true>), g1, dim3(256), 0, st, bt, pl, stride, K, first, rows, ctrl,
                                   tail_cut, cur1, c1, (T*)nullptr, stat);
                hipLaunchKernelGGL((k_sp_l2_fast<T, true>), g2, dim3(256), 0, st, pl, (const uint32_t*)cur1,
                                   (const uint64_t*)c1, (const T*)nullptr, cur2, c2, (T*)nullptr, stat);
                return finish_fast(ws, l, ctrl, hstat, st);
            }
        }
        hipLaunchKernelGGL((k_sp_l1_fast<T, false>), g1, dim3(256), 0, st, bt, pl, stride, K, first, rows, ctrl,
                           tail_cut, cur1, c1, (T*)(ws + l.val1), stat);
        hipLaunchKernelGGL((k_sp_l2_fast<T, false>), g2, dim3(256), 0, st, pl, (const uint32_t*)cur1,
                           (const uint64_t*)c1, (const T*)(ws + l.val1), cur2, c2, (T*)(ws + l.val2), stat);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else if (tail_cut != kNoPos) {  // no complete record: only the truncation position
        if ((e = hipMemcpyAsync(&ctrl->cutoff, &tail_cut, sizeof tail_cut, hipMemcpyHostToDevice, st)) != hipSuccess)
            return e;
    }
    return finish_fast(ws, l, ctrl, hstat, st);
}

hipError_t launch_sparse_partition_big(const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws,
                                       int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl,
                                       uint64_t tail_cut, SpStat* hstat, hipStream_t st) {
    uint32_t* curS = (uint32_t*)(ws + l.curS);
    SpStat* stat = (SpStat*)(ws + l.stat);
    hipError_t e = hipMemsetAsync(ws + l.leafflag, 0, (size_t)pl.nbig, st);
    if (e == hipSuccess) e = hipMemsetAsync(curS, 0, (size_t)pl.nbig * kSpSlices * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(stat, 0, sizeof(SpStat), st);
    if (e != hipSuccess) return e;
    const dim3 g((unsigned)(pl.tiles_per_slice * kSpSlices));
    hipLaunchKernelGGL(k_sp_l1_big, g, dim3(256), 0, st, bt, pl, stride, K, first, rows, ctrl, tail_cut, curS,
                       (uint64_t*)(ws + l.big), stat);
    return finish_fast(ws, l, ctrl, hstat, st);
}

hipError_t launch_sparse_partition_fast(int vtype, const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws,
                                        int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl,
                                        uint64_t tail_cut, SpStat* hstat, hipStream_t st) {
    if (vtype == kF32) return partition_fast_t<float>(bt, pl, l, ws, stride, K, first, rows, ctrl, tail_cut, hstat, st);
    if (vtype == kF64) return partition_fast_t<double>(bt, pl, l, ws, stride, K, first, rows, ctrl, tail_cut, hstat, st);
    if (vtype == kI32) return partition_fast_t<int32_t>(bt, pl, l, ws, stride, K, first, rows, ctrl, tail_cut, hstat, st);
    return hipErrorInvalidValue;
}

hipError_t launch_sparse_partition(int vtype, const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws,
                                   int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl,
                                   uint64_t tail_cut, hipStream_t st) {
    if (vtype == kF32) return partition_t<float>(bt, pl, l, ws, stride, K, first, rows, ctrl, tail_cut, st);
    if (vtype == kF64) return partition_t<double>(bt, pl, l, ws, stride, K, first, rows, ctrl, tail_cut, st);
    if (vtype == kI32) return partition_t<int32_t>(bt, pl, l, ws, stride, K, first, rows, ctrl, tail_cut, st);
    return hipErrorInvalidValue;
}

// Leaf blocks per CU: 2. Unused dynamic LDS on top of the kernel's static arrays
// keeps a third leaf block off a CU, so the next chunk's partition blocks (on the
// index stream) find wave slots and LDS beside the running leaf: same box, 3
// rounds, config-3 step 1.455 -> 1.422 ms and 1.348 -> 1.328 ms on a second box;
// 3 blocks 1.443, 1 block 1.67 (all 4 fit otherwise: 8-wave blocks, 32 waves).
template <typename T, bool CMP>
constexpr unsigned leaf_lds_pad() {
    constexpr unsigned kLds = 160u * 1024u, kBlocks = 2;
    constexpr unsigned stat = 8u * kSpLeafCap + (CMP ? 4u : (unsigned)sizeof(T) * kSpLeafCap) + 2u * kSpLeafCap +
                              4u * (kSpLines + 1) + 4u * kSpLines + 4u * (kSpLeafThreads / 64) + 4u + kSpLeafCap;
    return kLds / (kBlocks + 1) + 256u - stat;
}

hipError_t launch_sparse_leaf(int vtype, void* shard, const SpPlan& pl, const SpLayout& l, uint8_t* ws, Ctrl* ctrl,
                              const Ctrl* prev, hipStream_t st, LaunchEv ev) {
    if (pl.big) {
        if (vtype != kF32) return hipErrorInvalidValue;
        g_kernel_name = "dml::k_sp_leaf_big";
        int bshift = 0;  // kSpBigLines line buckets over the big leaf's rows
        while ((((int64_t)1 << pl.BL) >> bshift) > kSpBigLines) ++bshift;
        hipExtLaunchKernelGGL(k_sp_leaf_big, dim3((unsigned)pl.nbig), dim3(kSpBigThreads), 0, st, ev.start, ev.stop, 0,
                              (float*)shard, (const uint32_t*)(ws + l.curS), pl.nbig, pl.capS,
                              (const uint64_t*)(ws + l.big), pl.BL, bshift, ws + l.leafflag, ctrl, prev);
        return hipGetLastError();
    }
    if (pl.nleaves <= 0) return hipSuccess;
    const int64_t* bounds = (const int64_t*)(ws + l.bounds);
    const uint32_t* cnt2 = pl.fast ? (const uint32_t*)(ws + l.cur2) : nullptr;  // fixed-capacity layout
    const uint64_t* comp2 = (const uint64_t*)(ws + l.comp2);
    uint8_t* flag = ws + l.leafflag;
    const dim3 grid((unsigned)pl.nleaves);
    // line buckets: leaf rows >> bshift < kSpLines
    int bshift = 0;
    while ((((int64_t)1 << pl.SL) >> bshift) > kSpLines) ++bshift;
    g_kernel_name = vtype == kF64   ? "dml::k_sp_leaf<double, false>"
                    : vtype == kI32 ? "dml::k_sp_leaf<int, false>"
                    : pl.compact    ? "dml::k_sp_leaf<float, true>"
                                    : "dml::k_sp_leaf<float, false>";
    if (vtype == kF32 && pl.compact)
        hipExtLaunchKernelGGL((k_sp_leaf<float, true>), grid, dim3(kSpLeafThreads), leaf_lds_pad<float, true>(), st,
                              ev.start, ev.stop, 0,
                              (float*)shard, bounds, cnt2, pl.cap2, comp2, (const float*)nullptr, pl.SL, pl.D2, bshift,
                              pl.seq_cut, flag, ctrl, prev);
    else if (vtype == kF32)
        hipExtLaunchKernelGGL((k_sp_leaf<float, false>), grid, dim3(kSpLeafThreads), leaf_lds_pad<float, false>(), st,
                              ev.start, ev.stop, 0,
                              (float*)shard, bounds, cnt2, pl.cap2, comp2, (const float*)(ws + l.val2), pl.SL, pl.D2,
                              bshift, pl.seq_cut, flag, ctrl, prev);
    else if (vtype == kF64)
        hipExtLaunchKernelGGL((k_sp_leaf<double, false>), grid, dim3(kSpLeafThreads), leaf_lds_pad<double, false>(), st,
                              ev.start, ev.stop, 0,
                              (double*)shard, bounds, cnt2, pl.cap2, comp2, (const double*)(ws + l.val2), pl.SL, pl.D2,
                              bshift, pl.seq_cut, flag, ctrl, prev);
    else if (vtype == kI32)
        hipExtLaunchKernelGGL((k_sp_leaf<int32_t, false>), grid, dim3(kSpLeafThreads), leaf_lds_pad<int32_t, false>(),
                              st, ev.start, ev.stop, 0,
                              (int32_t*)shard, bounds, cnt2, pl.cap2, comp2, (const int32_t*)(ws + l.val2), pl.SL,
                              pl.D2, bshift, pl.seq_cut, flag, ctrl, prev);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// Flagged (oversized) leaves, exactly: sort every kept record by (row, seq) and
// run-apply the rows of flagged leaves. Synchronous; a rare path (skewed keys).
hipError_t sparse_replay(int vtype, void* shard, const SpPlan& pl_in, const SpLayout& l, uint8_t* ws, const Batch& bt,
                         int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl, uint64_t tail_cut,
                         hipStream_t st) {
    hipError_t e = hipSuccess;
    SpPlan pl = pl_in;
    if (pl.big) {  // the flags are per big leaf: re-partition with leaves of 2^BL rows
        plan_leaves(pl, rows, pl.BL);
        pl.big = 0;
    }
    if (pl.compact) {
        // compact words order a row's adds by push only: re-partition the chunk with
        // full sequence numbers (counted, compact layout), keeping the leaf flags
        pl.compact = 0;
        pl.fast = 0;
        pl.seq_cut = kSpSkip;
        if ((e = partition_t<float>(bt, pl, l, ws, stride, K, first, rows, ctrl, tail_cut, st, false)) != hipSuccess)
            return e;
    }
    int64_t nk = 0;
    uint64_t* kin = (uint64_t*)(ws + l.comp2);
    uint64_t* kout = (uint64_t*)(ws + l.comp1);
    void* vin_p = ws + l.val2;
    void* vout_p = ws + l.val1;
    if (pl.fast) {
        // fixed-capacity layout: pack the flagged leaves' records (comp1 / val1 are
        // free by now), then sort them back into comp2 / val2
        unsigned long long* packed = (unsigned long long*)(ws + l.stat + sizeof(SpStat));
        e = hipMemsetAsync(packed, 0, sizeof *packed, st);
        if (e == hipSuccess) {
            if (vtype == kF32 || vtype == kI32)  // 4-B values, moved as bits
                hipLaunchKernelGGL(k_sp_pack_flagged<float>, dim3((unsigned)pl.nleaves), dim3(256), 0, st,
                                   (const uint32_t*)(ws + l.cur2), pl.cap2, (const uint8_t*)(ws + l.leafflag),
                                   (const uint64_t*)kin, (const float*)vin_p, packed, kout, (float*)vout_p);
            else
                hipLaunchKernelGGL(k_sp_pack_flagged<double>, dim3((unsigned)pl.nleaves), dim3(256), 0, st,
                                   (const uint32_t*)(ws + l.cur2), pl.cap2, (const uint8_t*)(ws + l.leafflag),
                                   (const uint64_t*)kin, (const double*)vin_p, packed, kout, (double*)vout_p);
            e = hipGetLastError();
        }
        unsigned long long hp = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(&hp, packed, sizeof hp, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess || hp == 0) return e;
        nk = (int64_t)hp;
        std::swap(kin, kout);
        std::swap(vin_p, vout_p);
    } else {
        SpMeta hm;
        e = hipMemcpyAsync(&hm, ws + l.meta, sizeof hm, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess || hm.kept <= 0) return e;
        nk = hm.kept;
    }
    const int n = (int)nk;
    size_t tmp = 0;
    void* dtmp = nullptr;
    if (vtype == kF32 || vtype == kI32) {
        uint32_t* vin = (uint32_t*)vin_p;
        uint32_t* vout = (uint32_t*)vout_p;
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kin, kout, vin, vout, n, 0, 64, st);
        if (e == hipSuccess) e = hipMallocAsync(&dtmp, tmp, st);
        if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(dtmp, tmp, kin, kout, vin, vout, n, 0, 64, st);
        if (e == hipSuccess && vtype == kF32)
            hipLaunchKernelGGL(k_sp_runs<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (float*)shard,
                               (const uint64_t*)kout, (const float*)vout, (int64_t)n, pl.SL,
                               (const uint8_t*)(ws + l.leafflag), pl.seq_cut, ctrl);
        else if (e == hipSuccess)
            hipLaunchKernelGGL(k_sp_runs<int32_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                               (int32_t*)shard, (const uint64_t*)kout, (const int32_t*)vout, (int64_t)n, pl.SL,
                               (const uint8_t*)(ws + l.leafflag), pl.seq_cut, ctrl);
    } else {
        uint64_t* vin = (uint64_t*)vin_p;
        uint64_t* vout = (uint64_t*)vout_p;
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kin, kout, vin, vout, n, 0, 64, st);
        if (e == hipSuccess) e = hipMallocAsync(&dtmp, tmp, st);
        if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(dtmp, tmp, kin, kout, vin, vout, n, 0, 64, st);
        if (e == hipSuccess)
            hipLaunchKernelGGL(k_sp_runs<double>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (double*)shard,
                               (const uint64_t*)kout, (const double*)vout, (int64_t)n, pl.SL,
                               (const uint8_t*)(ws + l.leafflag), pl.seq_cut, ctrl);
    }
    if (e == hipSuccess) e = hipGetLastError();
    if (dtmp) (void)hipFreeAsync(dtmp, st);
    const hipError_t s2 = hipStreamSynchronize(st);
    return e != hipSuccess ? e : s2;
}

}  // namespace dml
