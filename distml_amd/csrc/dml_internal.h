// dml_internal.h — types shared by the HIP kernels (dml_kernels.hip) and the
// C-ABI host implementation (dml_store.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace dml {

// One ordered batch chunk holds at most this many pushes (the slot table is
// [rows][kMaxW] int32); longer batches run as consecutive chunks, in order.
constexpr int kMaxW = 64;
// Row stride of a chunk's slot table: its push count rounded up to 8 (scalar slot
// loads read 8 entries at a time). [rows][stride] instead of [rows][64]: an
// 8-push chunk of config 4's 1.25 M rows indexes into 40 MB (stays in the 256 MB
// MALL) instead of 320 MB. Allocations stay rows x kMaxW.
__host__ __device__ inline int slot_stride(int nb) { return (nb + 7) & ~7; }

// Position of a byte in the batch, in reference processing order:
// bucket-major, then byte offset inside the bucket (the order in which
// handlePush's while-loop reads bytes, FloatMatrixStore.java:202-207).
__host__ __device__ inline uint64_t pos_of(uint64_t bucket, uint64_t off) { return (bucket << 40) | off; }
constexpr uint64_t kNoPos = ~0ull;
constexpr uint64_t kOffMask = (1ull << 40) - 1;

// Per-batch control block. Lives at the head of the workspace
// [Ctrl | slot rows x kMaxW int32 | rowflag rows x uint32]: one hipMemsetAsync(0xFF)
// resets Ctrl and the slot table (-1 = no record); rowflag is zeroed separately.
struct Ctrl {
    unsigned long long cutoff;   // first key-out-of-shard position (exclusive apply limit)
    unsigned long long neg_pos;  // first add that left an int32 counter negative
    unsigned long long ident;    // speculative chunk: bit b = push b verified in the reduce (identity: record r is row r; or slot reuse)
    unsigned int no_dup;         // 0xFFFFFFFF = no row repeated inside one push; 0 = repeat seen
    unsigned int spec_ok;        // speculative chunk: 0xFFFFFFFF = every identity record verified; 0 = not
    // Slot-table column of push b (0xFF, the reset value: column b). k_index writes a
    // push's records there and the reduce reads them from there. In a speculative
    // chunk a push whose `ident` bit is set takes slot = row when its column is 0xFF
    // (identity) and otherwise reads the kept column k_ident_check matched it to
    // (slot reuse, whatever position the push arrived at).
    unsigned char col[kMaxW];
};
static_assert(sizeof(Ctrl) == 96, "Ctrl layout (a multiple of 32 B: the slot table after it stays aligned)");
__host__ __device__ inline int ctrl_col(const Ctrl* c, int b) {
    const unsigned v = c->col[b];
    return v == 0xFFu ? b : (int)v;
}
// A speculative chunk's push b verified as identity (record r holds row r).
__host__ __device__ inline bool ctrl_identity(const Ctrl* c, unsigned long long ident, int b) {
    return ((ident >> b) & 1ull) && c->col[b] == 0xFFu;
}

// Bucket table passed by value as a kernel argument (scalar-loaded).
struct Batch {
    const uint8_t* base[kMaxW];
    int64_t len[kMaxW];
    int64_t nrec[kMaxW];  // records whose key is complete (a truncated tail record included)
    int32_t bidx[kMaxW];  // global push index of each column (positions use it; columns ascend)
    const Ctrl* prev;     // control block of the chunk enqueued just before (pipelining), or null
    // Identity speculation (full-range chunks of plain sums): pushes
    // whose sampled keys say "record r holds row r" skip the key index; the reduce
    // takes slot = row for them and verifies every such record's key, reading the
    // input shard at `src` and writing the output buffer (the host keeps the input
    // until the chunk retires, so a failed verification re-runs it exactly).
    const void* src;      // input shard (null: in place)
    int64_t first;        // key of row 0 (KeyRange first), for the verification
    int32_t spec;         // 1: speculative chunk
    // Slot reuse (speculative chunks): bit c = column c of the workspace's slot table
    // still holds the permutation a push of the workspace's previous chunk listed
    // (verified there). A push whose sampled keys match one of these columns, at any
    // position, skips the key index (k_ident_check sets Ctrl::col); the reduce reads
    // its slots from that column and verifies every record's key.
    uint64_t kept_cols;
    // 1: such a chunk (its table may hold kept columns, so a stale entry is no
    // repeat): the key index does not look for repeated rows, and the reduce
    // verifies the record of every row of every push instead (all pushes are
    // full-range, so a repeat leaves another row without its record).
    int32_t keeps;
    // 1: the Ctrl::ident pushes were verified record by record before this launch
    // (k_ident_full; the sharded pre-reduce, whose partial the reduce-scatter takes
    // before a speculative verdict could be read): the reduce takes slot = row for
    // them and verifies nothing.
    int32_t ident_ok;
    // Rows any push of the chunk lists (byte per row, written by the key index; null:
    // not tracked). Sparse-row chunks of k_reduce_rows (LDA's 65 536-row pushes into a
    // 1 M-row table, config 5) leave ~11 % of the rows untouched: their shard rows are
    // then neither read nor written.
    const uint8_t* listed;
};

// A chunk whose predecessor ended abnormally (error, rows to replay, or a failed
// identity speculation) must not run ahead of the host's fix-up: its kernels
// turn into no-ops and the host relaunches (replay) or drops (error) it.
// Every field is read and the tests combined without short-circuit: in a kernel the
// four loads issue together (one wait) instead of as a chain of dependent round trips
// ahead of the block's first data load.
__host__ __device__ inline bool ctrl_abnormal(const Ctrl* c) {
    const unsigned long long cut = c->cutoff, neg = c->neg_pos;
    const unsigned int nd = c->no_dup, ok = c->spec_ok;
    return (cut != kNoPos) | (neg != kNoPos) | (nd == 0u) | (ok == 0u);
}

// Per-block AdaGrad candidate: the largest final delta of an element whose
// delta rose in this batch, and the position where it last rose.
struct DeltaCand {
    float value;
    int32_t valid;
    unsigned long long pos;
};
// Running AdaGrad maxDelta state (FloatMatrixStoreAdaGrad.java:27-29), device
// resident, plus the chunk's best candidate while it waits for the rows a push
// repeats (replayed in layers): the chunk's candidates are finalized once, so a
// tie between a repeated and a non-repeated row goes to the earlier position.
struct MaxDelta {
    float value;
    int32_t row;
    int32_t col;
    int32_t pad;
    DeltaCand pend;
};
// k_maxdelta finalize modes
enum MdMode : int {
    kMdApply = 0,          // merge with the pending candidate, apply (strict >), clear it
    kMdDefer = 1,          // merge into the pending candidate only
    kMdDeferIfRepeat = 2,  // kMdDefer when the chunk's index saw a repeated row (ctrl->no_dup == 0)
};

// Optional row map of a reduce launch (multi-GPU pre-reduce pieces): task row t
// reduces shard row  (t / block) * stride + off + t % block  (block == 0: row = t)
// and writes it to out + t*cols (out == null: in place). Rows >= rows_total are
// padding of linearSplit's short last shard: written as zeros.
struct RowMap {
    int64_t block = 0, stride = 0, off = 0;
    int64_t rows_total = 0;
    void* out = nullptr;
    // model row of task row t (rows <= INT32_MAX, a Java array: 32-bit division)
    __host__ __device__ inline int64_t row(int64_t t) const {
        if (!block) return t;
        const uint32_t q = (uint32_t)t / (uint32_t)block;
        return (int64_t)q * stride + off + (int64_t)((uint32_t)t - q * (uint32_t)block);
    }
};

struct AdaArgs {
    float* alpha;
    float* delta;
    DeltaCand* cand;      // one per reduce block
    float initial_alpha, min_alpha, factor;
};

enum ReduceMode : int {
    kAdd = 0,          // f32 / f64 / i32-without-check
    kAddCheckI32 = 1,  // IntMatrixStore dense: negativity check after each add
    kAdaGrad = 2,      // FloatMatrixStoreAdaGrad dense
    kRollbackI32 = 3,  // undo adds after the first negative (exact mod 2^32)
    kPreReduce = 4,    // multi-GPU pre-reduce: acc starts at 0, every row written
};

enum VType : int { kI32 = 0, kF32 = 1, kF64 = 3 };

// Optional start/stop events carried in the dispatch packet (hipExtLaunchKernel):
// kernel timing and cross-stream dependencies without extra marker packets.
struct LaunchEv {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
};

// ---- launchers (dml_kernels.hip) ----
hipError_t launch_index(const Batch& bt, int nb, int64_t max_nrec, int64_t stride, int K,
                        int64_t first, int64_t rows, int32_t* slot, uint32_t* rowflag, Ctrl* ctrl,
                        uint64_t tail_cut, hipStream_t st);
// Identity speculation: clears ctrl->ident bit b unless push b is full-range and
// every sampled record r of it has row_index(key) == r (Ctrl reset to all ones).
hipError_t launch_ident_check(const Batch& bt, int nb, int64_t stride, int K, int64_t first, int64_t rows,
                              const int32_t* slot, Ctrl* ctrl, hipStream_t st);
// After k_ident_check of a chunk offered kept columns: gives every push that is
// neither identity nor matched a slot-table column no matched push reads
// (Ctrl::col), so its key index does not overwrite a reused permutation.
hipError_t launch_assign_cols(Ctrl* ctrl, int nb, hipStream_t st);
// Complete identity check (Ctrl::ident reset to all ones, or as k_ident_check left
// it): clears ctrl->ident bit b unless every record r of push b has row_index(key) == r.
hipError_t launch_ident_full(const Batch& bt, int nb, int64_t max_nrec, int64_t stride, int K, int64_t first,
                             int64_t rows, Ctrl* ctrl, hipStream_t st);
hipError_t launch_reduce(int vtype, int mode, void* shard, int64_t rows, int32_t cols, const Batch& bt,
                         int nb, int64_t stride, int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl,
                         uint64_t tail_cut, const AdaArgs& ada, hipStream_t st, int64_t* nblocks_out,
                         LaunchEv ev = {}, RowMap rm = {});
hipError_t launch_rollback_i32(int32_t* shard, int64_t rows, int32_t cols, const Batch& bt, int nb,
                               int64_t stride, int K, const int32_t* slot, const uint32_t* rowflag, Ctrl* ctrl,
                               uint64_t tail_cut, hipStream_t st);
// `cand` holds n candidates plus kMdParts entries of scratch after them.
constexpr int kMdParts = 256;
hipError_t launch_maxdelta_finalize(DeltaCand* cand, int64_t n, MaxDelta* md, const Batch& bt, int nb,
                                    int64_t stride, int K, int V, hipStream_t st, int mode = kMdApply,
                                    const Ctrl* ctrl = nullptr);
hipError_t launch_array_rollback_i32(int32_t* shard, int64_t rows, const uint8_t* base, int64_t nrec,
                                     int b_global, int64_t stride, int K, int64_t first, Ctrl* ctrl,
                                     uint64_t tail_cut, hipStream_t st);
hipError_t launch_fill(int vtype, void* p, int64_t n, double v, hipStream_t st);
hipError_t launch_fill_f32(float* p, int64_t n, float v, hipStream_t st);
hipError_t launch_apply_dense(int vtype, void* shard, const void* src, int64_t n, hipStream_t st);
hipError_t launch_apply_dense_i32chk(int32_t* shard, const int32_t* src, int64_t n, unsigned long long* neg,
                                     hipStream_t st);
hipError_t launch_fetch(int vtype, const void* shard, const float* alpha, int32_t cols, const int64_t* keys,
                        int64_t key_lo, int64_t n, int64_t first, uint8_t* out, int64_t rec, int K, int value_slot,
                        hipStream_t st);
hipError_t launch_bswap(int V, const void* src, void* dst, int64_t n, hipStream_t st);
hipError_t launch_synth_dense(uint8_t* out, int K, int vtype, int64_t first, int64_t shard_rows, int64_t nrec,
                              int32_t cols, uint64_t s0, uint64_t pa, uint64_t pc, hipStream_t st);
hipError_t launch_synth_sparse(uint8_t* out, int K, int vtype, int value_stride, int64_t first,
                               int64_t key_space, int64_t nrec, uint64_t s0, uint64_t pa, uint64_t pc,
                               hipStream_t st);
// ---- ordered sparse scatter-add (dml_sparse.hip), float / double array stores ----
constexpr int kSpTile = 4096;      // records per partition tile (256 threads x 16)
constexpr int kSpLeafCap = 2048;   // records one leaf orders in LDS
constexpr uint32_t kSpSkip = 0xFFFFFFFFu;  // sequence of a record at or past the cutoff (never applied)
constexpr int kSpBigCap = 4096;    // records a big leaf orders in LDS (one-level partition)
constexpr int kSpBigBins = 16384;  // big leaves per chunk, at most (the one-level pass's LDS histogram)
constexpr int kSpSlices = 8;       // regions per big leaf: slice x holds the pushes p with p % 8 == x
// Shape of one chunk's partition (host-computed, passed by value).
struct SpPlan {
    int64_t tile_base[kMaxW + 1];  // first level-1 tile of push b (prefix of ceil(nrec / kSpTile))
    int64_t rec_base[kMaxW + 1];   // first sequence number of push b (prefix of nrec)
    int64_t nrec, ntiles1, nleaves, max_tiles2;
    int nb, SL, D2, nbins1;        // leaf = row >> SL; 2^D2 leaves per level-1 bin
    // single-pass partition (no count passes): fixed-capacity bins (cap1 records
    // per level-1 bin, cap2 per leaf) filled through atomic cursors; an overflow
    // falls back to the counted partition before the leaf runs
    int64_t cap1, cap2, tiles2_per_bin;
    int fast;                      // the leaf reads the fixed-capacity layout
    // compact records (fp32, single-pass, no cutoff): one 8-B word per record,
    // row within its level-1 bin << 38 | chunk push << 32 | value bits; the push
    // index orders a row's adds (a push listing a row twice sends its leaf to the
    // exact replay, which re-partitions with full sequence numbers)
    int compact;
    uint32_t seq_cut;              // records with sequence >= seq_cut are at / past the cutoff
    // one-level partition (compact fp32, pushes balanced over the 8 slices): "big
    // leaves" of 2^BL rows, one region of capS records per (big leaf, slice), filled
    // by the slice's tiles (pushes p % 8 == x, run by the blocks of XCD x); the leaf
    // kernel orders a big leaf's records in LDS, so there is no second pass
    int big, BL;
    int64_t nbig, capS, tiles_per_slice;
    int64_t sbase[kMaxW];          // tiles of the earlier pushes of push b's slice
};
constexpr int kSpCompactRowBits = 26;  // SL + D2 limit of the compact word
// Pinned status of a single-pass partition, read by the host before the leaf launch.
struct SpStat {
    unsigned int overflow;         // a bin or leaf exceeded its capacity
    unsigned int pad;
    unsigned long long cutoff;     // Ctrl::cutoff after the partition (first key outside the shard)
};
// Device-side results of level 1 (bin bounds, level-2 tile table).
struct SpMeta {
    int64_t kept;                  // records before the cutoff
    int64_t bin_start1[257];
    int64_t tile_start2[257];
};
// Byte offsets of the partition buffers inside one workspace allocation.
struct SpLayout {
    size_t meta, comp1, val1, comp2, val2, cnt1, off1, cnt2, off2, leafflag, bounds, scan_tmp, scan_tmp_bytes,
        cur1, cur2, stat, big, curS, total;
};
SpPlan sparse_plan(const Batch& bt, int nb, int64_t rows);
// The one-level partition where it applies (compact fp32 plan, >= 8 pushes balanced
// over the slices, big leaves of 2 K - 8.7 K records on average): sets pl.big.
void sparse_plan_big(SpPlan& pl, const Batch& bt, int64_t rows);
hipError_t launch_sparse_partition_big(const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws,
                                       int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl,
                                       uint64_t tail_cut, SpStat* hstat, hipStream_t st);
SpLayout sparse_layout(const SpPlan& pl, int vbytes);
hipError_t launch_sparse_partition(int vtype, const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws,
                                   int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl,
                                   uint64_t tail_cut, hipStream_t st);
// Single-pass partition into the fixed-capacity layout; copies its SpStat to `hstat` (pinned).
hipError_t launch_sparse_partition_fast(int vtype, const Batch& bt, const SpPlan& pl, const SpLayout& l, uint8_t* ws,
                                        int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl,
                                        uint64_t tail_cut, SpStat* hstat, hipStream_t st);
// Sequence number of the first record at / past `cut` (a record-start position, or kNoPos).
uint32_t sparse_seq_cut(const SpPlan& pl, const Batch& bt, uint64_t cut, int64_t stride);
hipError_t launch_sparse_leaf(int vtype, void* shard, const SpPlan& pl, const SpLayout& l, uint8_t* ws, Ctrl* ctrl,
                              const Ctrl* prev, hipStream_t st, LaunchEv ev);
// Exact replay of the leaves the leaf kernel flagged. A compact chunk is first
// re-partitioned (counted, full sequence numbers) from its pushes.
hipError_t sparse_replay(int vtype, void* shard, const SpPlan& pl, const SpLayout& l, uint8_t* ws, const Batch& bt,
                         int64_t stride, int K, int64_t first, int64_t rows, Ctrl* ctrl, uint64_t tail_cut,
                         hipStream_t st);

// Two-moment AdaGrad (sharded path): per-rank [row][Σu | Σu²]
// pre-reduce pieces (flat shapes: cols % 4 == 0, rows under 4 KiB), and the owner
// apply of the reduce-scattered moments (+ maxDelta finalize; ada.cand holds
// kMomentBlocks entries).
constexpr int kMomentBlocks = 2048;
hipError_t launch_moments(int64_t ntask, int32_t cols, const Batch& bt, int nb, int64_t stride, int K, int32_t* slot,
                          const Ctrl* ctrl, RowMap rm, hipStream_t st, LaunchEv ev);
hipError_t launch_ada_moments(float* shard, const float* src, int64_t rows, int32_t cols, const AdaArgs& ada,
                              MaxDelta* md, int64_t first, hipStream_t st, LaunchEv ev);

hipError_t launch_stream(bool copy, void* dst, const void* src, int64_t n16, hipStream_t st, LaunchEv ev);
hipError_t launch_rmw_floor(float* a, const uint32_t* idx, const float* v, int64_t n, hipStream_t st, LaunchEv ev);
hipError_t launch_dense_floor(const float* data, float* out, float* delta, const Batch& bt, int nb, int64_t stride,
                              int K, int32_t cols, int64_t elems, hipStream_t st, LaunchEv ev);
hipError_t launch_gather_floor(int32_t* shard, int32_t cols, const int32_t* trow, const int32_t* tptr,
                               const uint64_t* addr, int64_t ntouched, hipStream_t st, LaunchEv ev);
hipError_t launch_rand(int vtype, void* p, int64_t rows, int32_t cols, uint64_t s0, hipStream_t st);
hipError_t launch_synth_fill(int vtype, void* p, int64_t n, uint64_t s0, hipStream_t st);
hipError_t launch_key_rows(const uint8_t* base, int64_t nrec, int64_t stride, int K, int64_t first, int64_t rows,
                           int32_t* out, hipStream_t st);
int64_t reduce_blocks(int vtype, int64_t rows, int32_t cols);
// True when launch_reduce(vtype, mode, cols) runs k_reduce_rows in a plain-sum mode,
// which rewrites every slot it reads to -1 (the next batch's index then needs no memset).
bool reduce_clears_slots(int vtype, int mode, int32_t cols);
// The chunk's plain-sum reduce is k_reduce_flat (narrow dense rows), not k_reduce_rows.
bool use_flat(int vtype, int mode, int32_t cols, const Batch& bt, int nb, int64_t rows);
// k_flat_ident (dml_kernels.hip): a flat-shape chunk (use_flat, kAdd / kPreReduce)
// the host has seen, after its index, to be all identity — every push lists every
// row as record r = row r (flat_ident_ok), no cutoff, no repeated row. Its waves
// verify every key; a mismatch clears ctrl->spec_ok as k_reduce_flat does.
constexpr int kFlatIdentWaves = 8;  // waves per block (their rows written after one block barrier)
hipError_t launch_ada_ident(void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb, int64_t stride, int K,
                            const AdaArgs& ada, hipStream_t st, int64_t* ncand_out, LaunchEv ev = {});
hipError_t launch_flat_ident(int vtype, int mode, void* shard, int64_t rows, int32_t cols, const Batch& bt, int nb,
                             int64_t stride, int K, Ctrl* ctrl, hipStream_t st, int64_t* nblocks_out,
                             LaunchEv ev = {}, RowMap rm = {});
// Whether a chunk of nb pushes may run k_flat_ident, from the host's copy of its
// Ctrl after the index (hctrl) and the pushes' record counts (`need` per push: the
// model rows).
bool flat_ident_ok(const Ctrl& hctrl, const Batch& bt, int nb, int64_t need, uint64_t tail_cut);
// One rank's ring reduce-scatter footprint (diagnostic): one kernel of `channels` blocks.
hipError_t launch_ring_rs(int vtype, const void* part, void* recv, void* land, int64_t chunk_bytes, int world,
                          int rank, int channels, hipStream_t st);
// Task rows per wave of k_flat_ident at this width (a row map's blocks must hold whole waves).
int flat_ident_rows_per_wave(int vtype, int32_t cols);
// row shapes whose reduce runs identity-speculative chunks (k_reduce_rows FULL, k_reduce_flat)
bool spec_shape(int vtype, int32_t cols);

uint64_t splitmix64(uint64_t x);

// Name of the dominant kernel (reduce / flat / AdaGrad / sparse leaf) the calling
// thread launched last, in rocprof's form, e.g.
// "dml::k_reduce_rows<float, 0, 4, 4, true, true, 1, 4, 0>": bench.py ties a profile's
// counted HBM bytes to the instantiation that ran (dml_store_kernel_name).
extern thread_local const char* g_kernel_name;
inline std::string kname_arg(bool v) { return v ? "true" : "false"; }
inline std::string kname_arg(int v) { return std::to_string(v); }
inline std::string kname_arg(const char* v) { return v; }
template <typename... A>
std::string kname(const char* base, A... a) {
    std::string s = std::string("dml::") + base + "<";
    bool first = true;
    ((s += (first ? "" : ", ") + kname_arg(a), first = false), ...);
    return s + ">";
}
template <typename T>
inline const char* type_name() {
    if constexpr (sizeof(T) == 8) return "double";
    else if constexpr (T(0.5) == T(0)) return "int";
    else return "float";
}

// Records `msg` as the calling thread's dml_last_error() and returns `code`
// (dml_store.hip; shared by the C-ABI translation units).
int set_error(int code, const std::string& msg);

}  // namespace dml
