// dml_store.hip — host implementation of the C-ABI in include/distml_ps.h.
//
// One dml_store = one DataStore shard (DataStore.java:17-38) resident in HBM on
// one device, with its own HIP stream, a mutex (the reference calls a store
// from three threads: PSAgent.java:278, PSActor.java:171-251, PSSync.java:131),
// and a workspace: [Ctrl | slot table rows x kMaxW int32].
//
// A push batch runs per chunk of <= kMaxW pushes:
//   memset(Ctrl+slots) -> k_index -> k_reduce (matrix)   or
//   memset(Ctrl) -> two-level partition by leaf -> k_sp_leaf (array; dml_sparse.hip)
// and is "retired" later (next call, flush, or immediately in sync mode):
// sync, read Ctrl, replay pushes that repeat a row (exact layered path), undo
// int32 adds past the first negative counter (exact mod 2^32), and turn the
// first failing position into the status code, key and column the reference's
// exception carries.
#include "distml_ps.h"
#include "dml_internal.h"
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

using namespace dml;

constexpr size_t kSmallStoreBytes = (size_t)1 << 20;  // shards up to 1 MiB: high-priority streams

static thread_local std::string g_err;

static int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int dml::set_error(int code, const std::string& msg) { return set_err(code, msg); }

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) return set_err(DML_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)


namespace {

// java.util.Random as its specification defines it: 48-bit LCG (multiplier
// 0x5DEECE66D, addend 0xB), setSeed's scramble, nextDouble from 26 + 27 bits, and
// nextGaussian by the polar method with StrictMath.log (fdlibm's e_log.c, below)
// and StrictMath.sqrt (IEEE). Used by dml_store_rand for DoubleMatrixStore.rand().
struct JavaRandom {
    uint64_t x;
    bool have = false;
    double spare = 0.0;
    explicit JavaRandom(int64_t seed) : x(((uint64_t)seed ^ 0x5DEECE66DULL) & kMask) {}
    static constexpr uint64_t kMask = (1ULL << 48) - 1;
    int32_t next(int bits) {
        x = (x * 0x5DEECE66DULL + 0xBULL) & kMask;
        return (int32_t)(uint32_t)(x >> (48 - bits));
    }
    double next_double() {
        const int64_t hi = next(26);
        return (double)((hi << 27) + next(27)) * 0x1.0p-53;
    }
    static double strict_log(double v);
    double next_gaussian() {
        if (have) {
            have = false;
            return spare;
        }
        double a, b, q;
        do {
            a = 2 * next_double() - 1;
            b = 2 * next_double() - 1;
            q = a * a + b * b;
        } while (q >= 1 || q == 0);
        const double m = std::sqrt(-2 * strict_log(q) / q);
        spare = b * m;
        have = true;
        return a * m;
    }
};

// fdlibm __ieee754_log: reduce to x = 2^k (1 + f) with sqrt(2)/2 < 1 + f < sqrt(2),
// then log(1 + f) = f - f^2/2 + s (f^2/2 + R(s^2)), s = f / (2 + f), R a degree-14
// minimax polynomial in s (its published coefficients Lg1..Lg7).
double JavaRandom::strict_log(double v) {
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                     two54 = 1.80143985094819840000e+16;
    constexpr double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
                     L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                     L7 = 1.479819860511658591e-01;
    uint64_t u;
    memcpy(&u, &v, 8);
    int32_t hx = (int32_t)(u >> 32), k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | (int32_t)(uint32_t)u) == 0) return -std::numeric_limits<double>::infinity();
        if (hx < 0) return std::numeric_limits<double>::quiet_NaN();
        k = -54;
        v *= two54;
        memcpy(&u, &v, 8);
        hx = (int32_t)(u >> 32);
    }
    if (hx >= 0x7ff00000) return v + v;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i0 = (hx + 0x95f64) & 0x100000;
    u = ((uint64_t)(uint32_t)(hx | (i0 ^ 0x3ff00000)) << 32) | (u & 0xffffffffULL);
    memcpy(&v, &u, 8);
    k += i0 >> 20;
    const double f = v - 1.0, dk = (double)k;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f), z = s * s, w = z * z;
    const double t1 = w * (L2 + w * (L4 + w * L6));
    const double t2 = z * (L1 + w * (L3 + w * (L5 + w * L7)));
    const double R = t2 + t1;
    if (((hx - 0x6147a) | (0x6b851 - hx)) > 0) {
        const double hfsq = 0.5 * f * f;
        return k == 0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// One row of DoubleMatrixStore.rand() (DoubleMatrixStore.java:196-206).
void java_unit_abs_gaussian_row(JavaRandom& jr, double* row, int64_t cols) {
    double sum = 0.0;
    for (int64_t j = 0; j < cols; ++j) {
        row[j] = std::fabs(jr.next_gaussian());
        sum += row[j] * row[j];
    }
    sum = std::sqrt(sum);
    for (int64_t j = 0; j < cols; ++j) row[j] = row[j] / sum;
}


struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

struct Chunk {
    Batch bt{};
    int nb = 0;
    int64_t max_nrec = 0;
    uint64_t tail_cut = kNoPos;
    bool sorted = false;  // array store: partitioned + per-leaf ordered apply (dml_sparse.hip)
    SpPlan sp{};
    SpLayout spl{};
    bool spec = false;     // identity speculation (full-range plain-sum chunk, Batch::spec)
    bool keeps = false;    // speculative chunk: its slot table is kept for the next chunk here (Batch::kept_cols)
    uint64_t seq = 0;      // number of the push call the chunk belongs to (dml_store_push_seq)
    void* in = nullptr;    // matrix shard the chunk reads (the previous chunk's output)
    void* out = nullptr;   // and writes: == in, or the other buffer of a speculative chunk
};

int vtype_of(const dml_desc& d) { return d.value_type; }

}  // namespace

// One workspace of the pipeline: [Ctrl | slot rows x kMaxW | rowflag rows].
// Ring of kRing, at most kRing-1 chunks pending: chunk j's index reuses chunk
// j-3's workspace, whose Ctrl chunk j-2 read as `prev` — and chunk j-2 has been
// retired before chunk j launches.
constexpr int kRing = 3;
struct Workspace {
    uint8_t* base = nullptr;
    Ctrl* ctrl = nullptr;
    int32_t* slot = nullptr;
    uint32_t* rowflag = nullptr;
    Ctrl* hctrl = nullptr;            // pinned copy of ctrl, written by the chunk's last DMA
    hipEvent_t idx_done = nullptr;    // side stream: index of the chunk built
    hipEvent_t kstart = nullptr;      // main stream: reduce dispatch start (in-packet timestamp)
    hipEvent_t applied = nullptr;     // main stream: chunk applied (in-packet stop of its last kernel)
    hipEvent_t done = nullptr;        // copy stream: ctrl copied out (chunk retired-able)
    uint8_t* sp = nullptr;            // sparse partition buffers (SpLayout), grown on demand
    size_t sp_cap = 0;
    SpStat* hsp = nullptr;            // pinned status of the single-pass sparse partition
    Ctrl* hidx = nullptr;             // pinned copy of ctrl right after the index (flat speculative chunks)
    bool flat_ident = false;          // the chunk's apply runs k_flat_ident (chosen from hidx)
    uint8_t* listed = nullptr;        // rows the chunk's pushes list (Batch::listed), grown on first use
    bool clears = false;              // the chunk's reduce leaves its slot table all -1
    bool clean = false;               // slot table all -1 and rowflags 0: only the Ctrl needs a reset
    // Kept slot table (the last chunk here was a verified speculative chunk): rowflags
    // 0, and column c of [rows][slot_stride(kept_nb)] is the verified permutation of
    // one of that chunk's pushes (indexed or reused, not identity) when bit c of
    // `perm` is set; other columns hold no meaning
    bool kept = false;
    int kept_nb = 0;
    uint64_t perm = 0;
};

struct Pending {
    Chunk c;
    int w = 0;  // workspace index
};

struct dml_store {
    std::mutex mu;
    int device = 0;
    int64_t ident_full_min = (int64_t)64 << 20;  // DML_KNOB_IDENT_FULL_MIN_BYTES
    hipStream_t stream = nullptr;     // applies (reduce / scatter-add), in push order
    hipStream_t istream = nullptr;    // key index of the next chunk, overlapping the current apply
    hipStream_t cstream = nullptr;    // ctrl read-back, off the apply stream
    dml_desc desc{};
    uint32_t flags = 0;
    bool is_matrix = false, adagrad = false;
    int K = 4, V = 4;           // DataDesc keySize / valueSize (DataDesc.java:50-51)
    int array_vs = 4;           // array record value stride
    int64_t first = 0, last = 0, rows = 0;
    int32_t cols = 1;
    int64_t stride = 0;         // record stride
    void* data = nullptr;       // rows*cols values, as of the last retired chunk
    void* data_alt = nullptr;   // second buffer of speculative chunks (allocated on first use)
    float* alpha = nullptr;     // AdaGrad (FloatMatrixStoreAdaGrad.java:23-24)
    float* delta = nullptr;
    DeltaCand* cand = nullptr;
    int64_t cand_n = 0;
    MaxDelta* md = nullptr;
    float initial_alpha = 0.f, min_alpha = 0.f, factor = 1.5f;  // :22, :26
    Workspace ws[kRing];
    size_t slot_bytes = 0, ws_bytes = 0;
    int next_ws = 0;
    uint64_t call_seq = 0;      // push calls accepted so far (dml_store_push_seq)
    dml_store_counters st{};    // pipeline counters (dml_store_stats), counted at retire
    bool no_spec = false;       // DML_FLAG_NO_SPECULATION, or no HBM headroom for data_alt
    std::deque<Pending> pend;   // launched, not yet retired (oldest first), at most kRing-1
    // staging for host-memory pushes
    uint8_t* hstage = nullptr;
    uint8_t* dstage = nullptr;
    size_t stage_cap = 0;
    // fetch / checkpoint transfers: device scratch (encoded records, swapped
    // rows) and two pinned bounce buffers that overlap DMA with the host copy
    uint8_t* dscr = nullptr;
    size_t dscr_cap = 0;
    uint8_t* xbuf[2] = {nullptr, nullptr};
    hipEvent_t xev[2] = {nullptr, nullptr};
    // sticky error (first failure)
    int err = 0;
    int64_t err_key = 0;
    int32_t err_col = -1;
    // int32 owner apply (dml_store_apply_dense_device): first negative final counter
    unsigned long long* neg_dev = nullptr;   // sticky, kNoPos until an apply leaves a negative
    unsigned long long* neg_host = nullptr;  // pinned copy, DMA'd behind every checked apply
    hipEvent_t neg_ev = nullptr;
    bool neg_pending = false;
    // timing of the dominant kernel
    const char* kname = nullptr;  // its instantiation, as last launched (dml_store_kernel_name)
    bool timing = false;
    int32_t timing_every = 1;  // time one matrix chunk in timing_every (dml_store_set_timing)
    int64_t timing_k = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used, ev_free;
    double timed_ms = 0.0;
    int64_t timed_n = 0;
};

namespace {

int value_read_bytes(const dml_store* s) { return s->V; }

std::pair<hipEvent_t, hipEvent_t> ev_pair(dml_store* s) {
    if (!s->ev_free.empty()) {
        auto p = s->ev_free.back();
        s->ev_free.pop_back();
        return p;
    }
    std::pair<hipEvent_t, hipEvent_t> p{nullptr, nullptr};
    (void)hipEventCreate(&p.first);
    (void)hipEventCreate(&p.second);
    return p;
}

// Collect elapsed times of the completed event pairs (recorded in stream order:
// stop at the first pair still in flight).
void ev_collect(dml_store* s) {
    size_t i = 0;
    for (; i < s->ev_used.size(); ++i) {
        auto& p = s->ev_used[i];
        if (hipEventQuery(p.second) != hipSuccess) break;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
            s->timed_ms += ms;
            s->timed_n += 1;
        }
        bool ring = false;
        for (const Workspace& W : s->ws) ring |= p.first == W.kstart;
        if (!ring) s->ev_free.push_back(p);
    }
    s->ev_used.erase(s->ev_used.begin(), s->ev_used.begin() + (std::ptrdiff_t)i);
}

int ensure_stage(dml_store* s, size_t bytes) {
    if (bytes <= s->stage_cap) return DML_OK;
    if (s->hstage) (void)hipHostFree(s->hstage);
    if (s->dstage) (void)hipFree(s->dstage);
    s->hstage = nullptr;
    s->dstage = nullptr;
    s->stage_cap = 0;
    size_t cap = std::max<size_t>(bytes, 1 << 20);
    HIPCHK(hipHostMalloc((void**)&s->hstage, cap, hipHostMallocDefault));
    HIPCHK(hipMalloc((void**)&s->dstage, cap));
    s->stage_cap = cap;
    return DML_OK;
}

// ---- host <-> device transfers for fetch / checkpoint ----------------------
// Pageable destinations go through two pinned bounce buffers: the DMA of chunk
// i+1 runs while the host copies chunk i out (several threads per chunk).
// Pinned destinations (dml_host_alloc, hipHostRegister) are DMA'd directly.
constexpr size_t kXferChunk = 16u << 20;

bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    const bool pinned = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // a pageable pointer leaves an error from the attribute query
    return pinned;
}

int ensure_scratch(dml_store* s, size_t bytes) {
    if (bytes <= s->dscr_cap) return DML_OK;
    HIPCHK(hipStreamSynchronize(s->stream));  // queued work may still read the old scratch
    if (s->dscr) (void)hipFree(s->dscr);
    s->dscr = nullptr;
    s->dscr_cap = 0;
    HIPCHK(hipMalloc((void**)&s->dscr, bytes));
    s->dscr_cap = bytes;
    return DML_OK;
}

int ensure_xfer(dml_store* s) {
    for (int i = 0; i < 2; ++i) {
        if (!s->xbuf[i]) HIPCHK(hipHostMalloc((void**)&s->xbuf[i], kXferChunk, hipHostMallocDefault));
        if (!s->xev[i]) HIPCHK(hipEventCreateWithFlags(&s->xev[i], hipEventDisableTiming));
    }
    return DML_OK;
}

void host_copy(uint8_t* d, const uint8_t* src, size_t n) {
    constexpr size_t kPart = 2u << 20;
    constexpr size_t kMaxThreads = 4;
    const size_t parts = std::min(kMaxThreads, n / kPart);
    if (parts < 2) {
        std::memcpy(d, src, n);
        return;
    }
    const size_t per = (n / parts + 63) & ~(size_t)63;
    std::thread th[kMaxThreads];
    for (size_t i = 1; i < parts; ++i) {
        const size_t lo = i * per;
        if (lo >= n) break;
        th[i] = std::thread([=] { std::memcpy(d + lo, src + lo, std::min(per, n - lo)); });
    }
    std::memcpy(d, src, std::min(per, n));
    for (size_t i = 1; i < parts; ++i)
        if (th[i].joinable()) th[i].join();
}

// Device -> host after everything queued on s->stream; returns with the bytes in `dst`.
int d2h(dml_store* s, uint8_t* dst, const uint8_t* src, size_t bytes) {
    if (bytes <= (256u << 10) || host_pinned(dst)) {
        if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        return DML_OK;
    }
    if (int rc = ensure_xfer(s)) return rc;
    const size_t n = (bytes + kXferChunk - 1) / kXferChunk;
    auto issue = [&](size_t i) -> hipError_t {
        const size_t off = i * kXferChunk, len = std::min(kXferChunk, bytes - off);
        hipError_t e = hipMemcpyAsync(s->xbuf[i & 1], src + off, len, hipMemcpyDeviceToHost, s->stream);
        return e == hipSuccess ? hipEventRecord(s->xev[i & 1], s->stream) : e;
    };
    HIPCHK(issue(0));
    if (n > 1) HIPCHK(issue(1));
    for (size_t i = 0; i < n; ++i) {
        HIPCHK(hipEventSynchronize(s->xev[i & 1]));
        const size_t off = i * kXferChunk;
        host_copy(dst + off, s->xbuf[i & 1], std::min(kXferChunk, bytes - off));
        if (i + 2 < n) HIPCHK(issue(i + 2));
    }
    return DML_OK;
}

// Host -> device, queued on s->stream; returns once `src` may be reused.
int h2d(dml_store* s, uint8_t* dst, const uint8_t* src, size_t bytes) {
    if (bytes <= (256u << 10) || host_pinned(src)) {
        if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        return DML_OK;
    }
    if (int rc = ensure_xfer(s)) return rc;
    const size_t n = (bytes + kXferChunk - 1) / kXferChunk;
    for (size_t i = 0; i < n; ++i) {
        if (i >= 2) HIPCHK(hipEventSynchronize(s->xev[i & 1]));  // bounce buffer drained by its DMA
        const size_t off = i * kXferChunk, len = std::min(kXferChunk, bytes - off);
        host_copy(s->xbuf[i & 1], src + off, len);
        HIPCHK(hipMemcpyAsync(dst + off, s->xbuf[i & 1], len, hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipEventRecord(s->xev[i & 1], s->stream));
    }
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

// Per-push record accounting: records with a complete key, and the position of
// the first truncated access of a ragged tail (DataDesc.readInt past data.length).
void plan_bucket(const dml_store* s, int64_t len, int gb, int64_t* nrec, uint64_t* tail_cut) {
    const int64_t nfull = len / s->stride, tail = len % s->stride;
    *nrec = nfull;
    *tail_cut = kNoPos;
    if (tail == 0) return;
    const int64_t t0 = nfull * s->stride;
    if (s->is_matrix) {
        if (tail < s->K) {
            *tail_cut = pos_of((uint64_t)gb, (uint64_t)t0);
        } else {
            *nrec = nfull + 1;  // key complete: the index sees it (an out-of-shard key is reported first)
            const int64_t nvals = (tail - s->K) / s->V;
            *tail_cut = pos_of((uint64_t)gb, (uint64_t)(t0 + s->K + nvals * s->V));
        }
    } else if (tail >= s->K + value_read_bytes(s)) {
        *nrec = nfull + 1;  // readable record (FloatArrayStore 8-byte stride, short last slot)
    } else {
        *tail_cut = pos_of((uint64_t)gb, (uint64_t)t0);
    }
}

int reduce_mode(const dml_store* s) {
    if (s->adagrad) return kAdaGrad;
    if (s->desc.value_type == DML_ELEMENT_TYPE_INT && s->desc.dense_column) return kAddCheckI32;
    return kAdd;
}

AdaArgs ada_args(dml_store* s) { return AdaArgs{s->alpha, s->delta, s->cand, s->initial_alpha, s->min_alpha, s->factor}; }

// Apply part of a chunk on the main stream (after its index is ready), then
// copy its Ctrl out and record `done`. `prev` = Ctrl of the chunk enqueued before.
int launch_apply(dml_store* s, Chunk& c, Workspace& W, const Ctrl* prev) {
    c.bt.prev = prev;
    g_kernel_name = nullptr;
    struct NameOnExit {
        dml_store* s;
        ~NameOnExit() {
            if (g_kernel_name) s->kname = g_kernel_name;
        }
    } name_on_exit{s};
    if (s->is_matrix) {
        // Boundary between consecutive reduces (measured): the chunk's
        // completion event rides in the reduce's dispatch packet (a marker packet after
        // it cost ~7 µs); a timed chunk also carries its start event there (start/stop
        // in every packet ~10 µs, so the bench times a sample of the chunks). AdaGrad's
        // finalize kernels follow the reduce: marker events around both.
        const bool inpacket = !s->adagrad;
        const bool timed = s->timing && (s->adagrad || s->timing_every <= 1 || s->timing_k++ % s->timing_every == 0);
        LaunchEv ev = inpacket ? LaunchEv{timed ? W.kstart : nullptr, W.applied} : LaunchEv{};
        if (timed && !inpacket) HIPCHK(hipEventRecord(W.kstart, s->stream));
        int64_t nblk = 0;
        W.clears = reduce_clears_slots(vtype_of(s->desc), reduce_mode(s), s->cols);
        c.bt.src = c.in != c.out ? c.in : nullptr;
        if (W.flat_ident) s->st.ident_launches += 1;
        if (W.flat_ident && s->adagrad)  // every push verified-identity (the host's Ctrl copy)
            HIPCHK(launch_ada_ident(c.out, s->rows, s->cols, c.bt, c.nb, s->stride, s->K, ada_args(s), s->stream,
                                    &nblk, ev));
        else if (W.flat_ident)
            HIPCHK(launch_flat_ident(vtype_of(s->desc), reduce_mode(s), c.out, s->rows, s->cols, c.bt, c.nb,
                                     s->stride, s->K, W.ctrl, s->stream, &nblk, ev));
        else
            HIPCHK(launch_reduce(vtype_of(s->desc), reduce_mode(s), c.out, s->rows, s->cols, c.bt, c.nb, s->stride,
                                 s->K, W.slot, W.rowflag, W.ctrl, c.tail_cut, ada_args(s), s->stream, &nblk, ev));
        if (s->adagrad)
            // finalized here unless the index saw a repeated row: then after its replay
            HIPCHK(launch_maxdelta_finalize(s->cand, nblk, s->md, c.bt, c.nb, s->stride, s->K, s->V, s->stream,
                                            kMdDeferIfRepeat, W.ctrl));
        if (!inpacket || nblk <= 0) HIPCHK(hipEventRecord(W.applied, s->stream));  // (no dispatch: a marker)
        if (timed && nblk > 0) s->ev_used.emplace_back(W.kstart, W.applied);
    } else {
        // the leaf launch carries the chunk's completion event (and, when timed, its start)
        const bool launched = c.sp.nleaves > 0;
        const bool timed = launched && s->timing && (s->timing_every <= 1 || s->timing_k++ % s->timing_every == 0);
        const LaunchEv ev = launched ? LaunchEv{timed ? W.kstart : nullptr, W.applied} : LaunchEv{};
        HIPCHK(launch_sparse_leaf(vtype_of(s->desc), s->data, c.sp, c.spl, W.sp, W.ctrl, prev, s->stream, ev));
        if (!launched) HIPCHK(hipEventRecord(W.applied, s->stream));
        if (timed) s->ev_used.emplace_back(W.kstart, W.applied);
    }
    // ctrl read-back on its own stream, so the next chunk's apply follows this one directly
    HIPCHK(hipStreamWaitEvent(s->cstream, W.applied, 0));
    HIPCHK(hipMemcpyAsync(W.hctrl, W.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, s->cstream));
    HIPCHK(hipEventRecord(W.done, s->cstream));
    return DML_OK;
}

// Index on the side stream (overlaps the previous chunk's apply), then apply.
int launch_chunk(dml_store* s, Chunk& c, Workspace& W, const Ctrl* prev) {
    hipStream_t is = s->istream;
    // A workspace whose last chunk retired normally through a slot-clearing reduce
    // (k_reduce_rows, plain-sum modes) already holds an all -1 slot table and zero
    // rowflags: only its Ctrl is reset (the 4 MiB-class memsets otherwise compete
    // with the running reduce).
    const bool clean = W.clean, kept = W.kept;
    W.clean = W.kept = false;
    // A speculative chunk after a kept table needs no -1 table either: its pushes
    // are full-range, so the index rewrites every row of each column it builds (a
    // push that is no permutation fails the chunk's verification, and the re-run
    // starts from a memset), and identity / reused columns are not rebuilt.
    const bool slots_ok = clean || (kept && c.keeps);
    HIPCHK(hipMemsetAsync(W.base, 0xFF, sizeof(Ctrl) + (slots_ok ? 0 : s->slot_bytes), is));
    if (s->is_matrix) {
        if (!(clean || kept)) HIPCHK(hipMemsetAsync(W.rowflag, 0, (size_t)s->rows * sizeof(uint32_t), is));
        if (c.spec) {
            HIPCHK(launch_ident_check(c.bt, c.nb, s->stride, s->K, s->first, s->rows, W.slot, W.ctrl, is));
            // pushes matched to kept columns: the indexed ones take columns nobody reads
            if (c.bt.kept_cols) HIPCHK(launch_assign_cols(W.ctrl, c.nb, is));
        }
        // AdaGrad chunks of k_ada_flat (no speculation: the apply cannot be undone):
        // full-range pushes whose records are rows in order skip the key index after a
        // complete key check, when the slot table is beyond the caches (its atomics go
        // to DRAM; see dml_prereduce_begin)
        c.bt.ident_ok = 0;
        if (s->adagrad && c.tail_cut == kNoPos &&
            (int64_t)s->rows * slot_stride(c.nb) * 4 > s->ident_full_min &&
            use_flat(vtype_of(s->desc), reduce_mode(s), s->cols, c.bt, c.nb, s->rows)) {
            bool full = c.nb > 0;
            for (int j = 0; j < c.nb && full; ++j) full = c.bt.nrec[j] == s->rows;
            if (full) {
                HIPCHK(launch_ident_full(c.bt, c.nb, c.max_nrec, s->stride, s->K, s->first, s->rows, W.ctrl, is));
                c.bt.ident_ok = 1;
            }
        }
        // Sparse-row chunks of k_reduce_rows (some push lists only part of the rows): the
        // index marks the rows any push lists, and the reduce skips the others' shard rows
        c.bt.listed = nullptr;
        if (!c.spec && !s->adagrad && (reduce_mode(s) == kAdd || reduce_mode(s) == kAddCheckI32) &&
            !use_flat(vtype_of(s->desc), reduce_mode(s), s->cols, c.bt, c.nb, s->rows)) {
            bool part = false;
            for (int j = 0; j < c.nb && !part; ++j) part = c.bt.nrec[j] < s->rows;
            if (part) {
                if (!W.listed) HIPCHK(hipMalloc((void**)&W.listed, (size_t)s->rows));
                HIPCHK(hipMemsetAsync(W.listed, 0, (size_t)s->rows, is));
                c.bt.listed = W.listed;
            }
        }
        HIPCHK(launch_index(c.bt, c.nb, c.max_nrec, s->stride, s->K, s->first, s->rows, W.slot, W.rowflag, W.ctrl,
                            c.tail_cut, is));
        // A speculative chunk of the flat shape: its Ctrl (identity / kept columns,
        // cutoff, repeats) is final here; a pinned copy lets the host pick the lean
        // all-identity kernel after the wait below (k_flat_ident)
        W.flat_ident = false;
        // AdaGrad chunks checked record by record (ident_ok) likewise pick k_ada_ident
        if (((c.spec && reduce_mode(s) == kAdd) || (s->adagrad && c.bt.ident_ok)) &&
            c.tail_cut == kNoPos && use_flat(vtype_of(s->desc), reduce_mode(s), s->cols, c.bt, c.nb, s->rows)) {
            if (!W.hidx) HIPCHK(hipHostMalloc((void**)&W.hidx, sizeof(Ctrl), hipHostMallocDefault));
            W.hidx->cutoff = 0;  // not all-identity unless the copy lands
            HIPCHK(hipMemcpyAsync(W.hidx, W.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, is));
            W.flat_ident = true;  // provisional: decided after idx_done
        }
    } else {
        // arrays: partition the chunk by leaf (row range) for the ordered per-leaf
        // apply (its first pass also finds the cutoff); int32 leaves check every add
        // (IntArrayStore.java:108-110) and report the chunk's first negative counter
        const int vt = vtype_of(s->desc);
        c.sorted = true;
        {
            c.sp = sparse_plan(c.bt, c.nb, s->rows);
            // one 8-B word per fp32 record through the partition
            c.sp.compact = vt == kF32 && c.sp.SL + c.sp.D2 <= kSpCompactRowBits && c.tail_cut == kNoPos;
            // big leaves sorted in LDS where they apply: no second partition pass (§4)
            sparse_plan_big(c.sp, c.bt, s->rows);
            c.spl = sparse_layout(c.sp, s->V);
            if (W.sp_cap < c.spl.total) {
                HIPCHK(hipStreamSynchronize(s->stream));  // W's previous chunk is retired; be safe
                (void)hipFree(W.sp);
                W.sp = nullptr;
                W.sp_cap = 0;
                HIPCHK(hipMalloc((void**)&W.sp, c.spl.total));
                W.sp_cap = c.spl.total;
            }
            if (!W.hsp) HIPCHK(hipHostMalloc((void**)&W.hsp, sizeof(SpStat), hipHostMallocDefault));
            if (c.sp.big)
                HIPCHK(launch_sparse_partition_big(c.bt, c.sp, c.spl, W.sp, s->stride, s->K, s->first, s->rows,
                                                   W.ctrl, c.tail_cut, W.hsp, is));
            else
                HIPCHK(launch_sparse_partition_fast(vt, c.bt, c.sp, c.spl, W.sp, s->stride, s->K, s->first, s->rows,
                                                    W.ctrl, c.tail_cut, W.hsp, is));
        }
    }
    HIPCHK(hipEventRecord(W.idx_done, is));
    // The index (tens of µs) finishes while the previous chunk's reduce (hundreds
    // of µs) still runs: wait for it on the host and enqueue this chunk's apply
    // directly behind that reduce. A cross-queue barrier packet instead costs
    // ~16 µs of idle GPU between the two reduces (measured).
    HIPCHK(hipEventSynchronize(W.idx_done));
    if (W.flat_ident) W.flat_ident = flat_ident_ok(*W.hidx, c.bt, c.nb, s->rows, c.tail_cut);
    if (c.sorted && c.sp.fast) {
        const uint64_t pcut = std::min<uint64_t>(W.hsp->cutoff, c.tail_cut);
        if (W.hsp->overflow || (c.sp.compact && pcut != kNoPos)) {
            // a bin or leaf of the single-pass partition overflowed (skewed keys), or
            // compact records met a cutoff (they carry no sequence to cut at): the
            // counted partition, compact layout (still beside the running apply)
            c.sp.fast = 0;
            c.sp.compact = 0;
            c.sp.big = 0;
            c.sp.seq_cut = kSpSkip;
            HIPCHK(launch_sparse_partition(vtype_of(s->desc), c.bt, c.sp, c.spl, W.sp, s->stride, s->K, s->first,
                                           s->rows, W.ctrl, c.tail_cut, is));
            HIPCHK(hipEventRecord(W.idx_done, is));
            HIPCHK(hipEventSynchronize(W.idx_done));
        } else {
            c.sp.seq_cut = sparse_seq_cut(c.sp, c.bt, pcut, s->stride);
        }
    }
    return launch_apply(s, c, W, prev);
}

int read_ctrl(dml_store* s, Workspace& W, Ctrl* out) {
    HIPCHK(hipMemcpyAsync(W.hctrl, W.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    *out = *W.hctrl;
    return DML_OK;
}

// Exact replay of the rows some push lists twice (rowflag set; the reduce left
// them untouched): split each push into layers (k-th occurrence of each flagged
// row) and apply layers in (push, layer) order, so per element the adds keep
// their reference order. Other rows are final already (rows are independent).
int replay_rows(dml_store* s, const Chunk& c, Workspace& W, Ctrl* ctl) {
    std::vector<uint32_t> flag((size_t)s->rows);
    HIPCHK(hipMemcpyAsync(flag.data(), W.rowflag, flag.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    struct VCol { int src_b; std::vector<std::pair<int32_t, int32_t>> rr; };
    std::vector<VCol> cols;
    int32_t* drows = nullptr;
    HIPCHK(hipMalloc((void**)&drows, sizeof(int32_t) * std::max<int64_t>(c.max_nrec, 1)));
    std::vector<int32_t> hrows;
    for (int b = 0; b < c.nb; ++b) {
        const int64_t n = c.bt.nrec[b];
        hrows.resize((size_t)n);
        if (n > 0) {
            hipError_t e = launch_key_rows(c.bt.base[b], n, s->stride, s->K, s->first, s->rows, drows, s->stream);
            if (e == hipSuccess) e = hipMemcpyAsync(hrows.data(), drows, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
            if (e != hipSuccess) { (void)hipFree(drows); return set_err(DML_E_HIP, hipGetErrorString(e)); }
        }
        std::unordered_map<int32_t, int32_t> occ;
        std::vector<VCol> layers;
        for (int64_t r = 0; r < n; ++r) {
            const int32_t row = hrows[(size_t)r];
            if (row < 0 || !flag[(size_t)row]) continue;  // out of shard (cutoff covers it) or already applied
            const int32_t l = occ[row]++;
            if ((int)layers.size() <= l) layers.push_back(VCol{b, {}});
            layers[(size_t)l].rr.emplace_back(row, (int32_t)r);
        }
        for (auto& L : layers) cols.push_back(std::move(L));
    }
    (void)hipFree(drows);
    std::vector<int32_t> hslot((size_t)s->rows * kMaxW);
    auto upload = [&](size_t v0, Chunk& vc) -> int {
        vc.nb = (int)std::min<size_t>(kMaxW, cols.size() - v0);
        vc.tail_cut = c.tail_cut;
        vc.bt.prev = nullptr;
        std::fill(hslot.begin(), hslot.end(), -1);
        for (int j = 0; j < vc.nb; ++j) {
            const VCol& col = cols[v0 + (size_t)j];
            vc.bt.base[j] = c.bt.base[col.src_b];
            vc.bt.len[j] = c.bt.len[col.src_b];
            vc.bt.nrec[j] = c.bt.nrec[col.src_b];
            vc.bt.bidx[j] = c.bt.bidx[col.src_b];
            for (auto& pr : col.rr) hslot[(size_t)pr.first * (size_t)slot_stride(vc.nb) + (size_t)j] = pr.second;
        }
        HIPCHK(hipMemcpy(W.slot, hslot.data(), hslot.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        return DML_OK;
    };
    for (size_t v0 = 0; v0 < cols.size(); v0 += kMaxW) {
        Chunk vc;
        if (int rc = upload(v0, vc)) return rc;
        int64_t nblk = 0;
        HIPCHK(launch_reduce(vtype_of(s->desc), reduce_mode(s), s->data, s->rows, s->cols, vc.bt, vc.nb, s->stride,
                             s->K, W.slot, nullptr, W.ctrl, vc.tail_cut, ada_args(s), s->stream, &nblk));
        if (s->adagrad)  // the layers' candidates join the chunk's pending one
            HIPCHK(launch_maxdelta_finalize(s->cand, nblk, s->md, vc.bt, vc.nb, s->stride, s->K, s->V, s->stream,
                                            kMdDefer));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    if (s->adagrad) {  // one finalize over the whole chunk: the reference's first position wins a tie
        HIPCHK(launch_maxdelta_finalize(s->cand, 0, s->md, c.bt, c.nb, s->stride, s->K, s->V, s->stream, kMdApply));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    if (int rc = read_ctrl(s, W, ctl)) return rc;
    if (ctl->neg_pos != kNoPos) {
        // undo every add after the first negative: the unflagged rows (rebuilt slot
        // table of the chunk) and every layer of the replayed rows
        Chunk mc = c;
        mc.bt.prev = nullptr;
        HIPCHK(hipMemsetAsync(W.slot, 0xFF, s->slot_bytes, s->stream));
        HIPCHK(launch_index(mc.bt, mc.nb, mc.max_nrec, s->stride, s->K, s->first, s->rows, W.slot, W.rowflag, W.ctrl,
                            kNoPos, s->stream));
        HIPCHK(launch_rollback_i32((int32_t*)s->data, s->rows, s->cols, mc.bt, mc.nb, s->stride, s->K, W.slot,
                                   W.rowflag, W.ctrl, mc.tail_cut, s->stream));
        for (size_t v0 = 0; v0 < cols.size(); v0 += kMaxW) {
            Chunk vc;
            HIPCHK(hipStreamSynchronize(s->stream));
            if (int rc = upload(v0, vc)) return rc;
            HIPCHK(launch_rollback_i32((int32_t*)s->data, s->rows, s->cols, vc.bt, vc.nb, s->stride, s->K, W.slot,
                                       nullptr, W.ctrl, vc.tail_cut, s->stream));
        }
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    return DML_OK;
}

int64_t read_key_at(dml_store* s, const uint8_t* dev_rec) {
    uint8_t kb[8] = {0};
    if (hipMemcpy(kb, dev_rec, (size_t)s->K, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    if (s->K == 4) {
        int32_t k;
        std::memcpy(&k, kb, 4);
        return k;
    }
    int64_t k;
    std::memcpy(&k, kb, 8);
    return k;
}

const uint8_t* base_of(const Chunk& c, int gb) {
    for (int b = 0; b < c.nb; ++b)
        if (c.bt.bidx[b] == gb) return c.bt.base[b];
    return nullptr;
}

int record_error(dml_store* s, int code, int64_t key, int32_t col) {
    if (!s->err) {
        s->err = code;
        s->err_key = key;
        s->err_col = col;
    }
    static const char* names[] = {"", "IllegalArgumentException", "ArrayIndexOutOfBoundsException (key outside shard)",
                                  "ArrayIndexOutOfBoundsException (truncated push)", "IllegalStateException (negative counter)"};
    char buf[160];
    std::snprintf(buf, sizeof buf, "%s: key=%lld col=%d", names[code], (long long)key, col);
    return set_err(code, buf);
}

// A chunk's input and output shard buffers: it reads `in` (the output of the
// chunk before it); a speculative chunk writes the other buffer, so the input
// survives until its identity records are verified.
void set_buffers(dml_store* s, Chunk& c, void* in) {
    c.in = in;
    c.out = c.spec ? (in == s->data ? s->data_alt : s->data) : in;
}

// Failed identity speculation: redo the chunk without it, in place on its input
// (== s->data: every chunk before it has retired), on the apply stream, and
// return the new Ctrl. The workspace's slot table / rowflags are rebuilt.
int rerun_unspeculated(dml_store* s, Chunk& c, Workspace& W, Ctrl* ctl) {
    c.spec = false;
    c.bt.spec = 0;
    c.keeps = false;
    c.bt.kept_cols = 0;
    c.bt.keeps = 0;
    c.bt.prev = nullptr;
    set_buffers(s, c, s->data);
    HIPCHK(hipMemsetAsync(W.base, 0xFF, sizeof(Ctrl) + s->slot_bytes, s->stream));
    HIPCHK(hipMemsetAsync(W.rowflag, 0, (size_t)s->rows * sizeof(uint32_t), s->stream));
    HIPCHK(launch_index(c.bt, c.nb, c.max_nrec, s->stride, s->K, s->first, s->rows, W.slot, W.rowflag, W.ctrl,
                        c.tail_cut, s->stream));
    c.bt.src = nullptr;
    int64_t nblk = 0;
    HIPCHK(launch_reduce(vtype_of(s->desc), reduce_mode(s), c.out, s->rows, s->cols, c.bt, c.nb, s->stride, s->K,
                         W.slot, W.rowflag, W.ctrl, c.tail_cut, ada_args(s), s->stream, &nblk));
    W.clears = reduce_clears_slots(vtype_of(s->desc), reduce_mode(s), s->cols);
    return read_ctrl(s, W, ctl);
}

// Turn the oldest pending chunk's Ctrl into final state + status: replay rows a
// push repeats, undo int32 adds past the first negative counter, map the first
// failing position to (code, key, col). If it ended abnormally, the chunk queued
// after it ran as a no-op: relaunch it (replay only) or drop it (error: the
// reference's PS loop has ended, PSAgent.java:188-191).
int retire_front(dml_store* s) {
    if (s->pend.empty()) return DML_OK;
    Pending p = s->pend.front();
    s->pend.pop_front();
    Workspace& W = s->ws[p.w];
    Chunk& c = p.c;
    HIPCHK(hipEventSynchronize(W.done));
    Ctrl ctl = *W.hctrl;
    if (s->timing) ev_collect(s);
    const bool abnormal = ctrl_abnormal(&ctl);  // the chunk queued behind it ran as a no-op
    W.clean = s->is_matrix && !abnormal && W.clears;
    s->st.chunks += 1;
    if (!s->is_matrix && c.sp.big) s->st.sparse_big_chunks += 1;
    if (c.spec && ctl.spec_ok != 0u) {
        std::swap(s->data, s->data_alt);  // every identity record verified: the output is the shard
        s->st.spec_chunks += 1;
        uint64_t perm = 0;
        for (int b = 0; b < c.nb; ++b) {
            if (ctrl_identity(&ctl, ctl.ident, b)) {
                s->st.identity_pushes += 1;
                continue;
            }
            if ((ctl.ident >> b) & 1ull) s->st.reused_pushes += 1;
            else s->st.indexed_pushes += 1;
            perm |= 1ull << ctrl_col(&ctl, b);  // a verified permutation (indexed or reused)
        }
        if (c.keeps) {  // the reduce left the slot table as built: the next chunk here may reuse it
            W.clean = false;
            W.kept = true;
            W.kept_nb = c.nb;
            W.perm = perm;
        }
    } else if (c.spec) {
        // An identity push was not (or the chunk met a cutoff / repeated row): the
        // output is discarded and the chunk re-runs exactly, in place on its input
        // (the shard as of the chunks before it), with the full key index.
        s->st.spec_chunks += 1;
        s->st.spec_reruns += 1;
        s->st.indexed_pushes += c.nb;
        if (int r2 = rerun_unspeculated(s, c, W, &ctl)) return r2;
        W.clean = !ctrl_abnormal(&ctl) && W.clears;
    } else if (s->is_matrix) {
        // non-speculative: AdaGrad chunks may have skipped the index for pushes checked
        // completely (Batch::ident_ok)
        for (int b = 0; b < c.nb; ++b) {
            if (c.bt.ident_ok && ((ctl.ident >> b) & 1ull)) s->st.identity_pushes += 1;
            else s->st.indexed_pushes += 1;
        }
    }
    int rc = DML_OK;
    if (s->is_matrix && ctl.no_dup == 0u) {
        rc = replay_rows(s, c, W, &ctl);
        if (rc) return rc;
    } else if (!s->is_matrix && ctl.no_dup == 0u) {
        // leaves too large for the LDS sort were skipped by the leaf kernel: apply them
        // exactly (an int32 replay may find an earlier negative counter)
        s->st.sparse_replays += 1;
        HIPCHK(sparse_replay(vtype_of(s->desc), s->data, c.sp, c.spl, W.sp, c.bt, s->stride, s->K, s->first, s->rows,
                             W.ctrl, c.tail_cut, s->stream));
        HIPCHK(hipMemcpyAsync(&ctl.neg_pos, &W.ctrl->neg_pos, sizeof(ctl.neg_pos), hipMemcpyDeviceToHost,
                              s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    if (!s->is_matrix && ctl.neg_pos != kNoPos) {
        // int32 array: the leaves reported the sequence of the chunk's first add that left
        // a counter negative; as a position (push, record) it bounds the rollback of every
        // later add (exact mod 2^32), the state the reference leaves when it throws
        const uint64_t seq = ctl.neg_pos;
        int b = 0;
        while (b + 1 < c.nb && (uint64_t)c.sp.rec_base[b + 1] <= seq) ++b;
        const int64_t r = (int64_t)(seq - (uint64_t)c.sp.rec_base[b]);
        ctl.neg_pos = pos_of((uint64_t)c.bt.bidx[b], (uint64_t)(r * s->stride + s->K));
        HIPCHK(hipMemcpyAsync(&W.ctrl->neg_pos, &ctl.neg_pos, sizeof(ctl.neg_pos), hipMemcpyHostToDevice, s->stream));
        for (int j = 0; j < c.nb; ++j)
            HIPCHK(launch_array_rollback_i32((int32_t*)s->data, s->rows, c.bt.base[j], c.bt.nrec[j], c.bt.bidx[j],
                                             s->stride, s->K, s->first, W.ctrl, c.tail_cut, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    } else if (s->is_matrix && ctl.neg_pos != kNoPos && ctl.no_dup != 0u) {
        // (a chunk with repeated rows rolled back inside replay_rows) the reduce handed
        // its slot rows back clean: rebuild the table (no row repeats here, so the
        // rowflags stay zero; the index leaves neg_pos alone), then undo past neg_pos
        HIPCHK(hipMemsetAsync(W.slot, 0xFF, s->slot_bytes, s->stream));
        HIPCHK(launch_index(c.bt, c.nb, c.max_nrec, s->stride, s->K, s->first, s->rows, W.slot, W.rowflag, W.ctrl,
                            c.tail_cut, s->stream));
        HIPCHK(launch_rollback_i32((int32_t*)s->data, s->rows, s->cols, c.bt, c.nb, s->stride, s->K, W.slot, W.rowflag,
                                   W.ctrl, c.tail_cut, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    const uint64_t cut = std::min<uint64_t>(ctl.cutoff, c.tail_cut);
    if (ctl.neg_pos != kNoPos && ctl.neg_pos < cut) {
        const int gb = (int)(ctl.neg_pos >> 40);
        const int64_t off = (int64_t)(ctl.neg_pos & kOffMask);
        const int64_t r = off / s->stride;
        const int32_t col = s->is_matrix ? (int32_t)((off - r * s->stride - s->K) / s->V) : -1;
        rc = record_error(s, DML_E_NEGATIVE_COUNTER, read_key_at(s, base_of(c, gb) + r * s->stride), col);
    } else if (cut != kNoPos) {
        const int gb = (int)(cut >> 40);
        const int64_t off = (int64_t)(cut & kOffMask);
        const int64_t r = off / s->stride;
        const uint8_t* rec = base_of(c, gb) + r * s->stride;
        if (ctl.cutoff < c.tail_cut) {
            rc = record_error(s, DML_E_KEY_OUT_OF_SHARD, read_key_at(s, rec), -1);
        } else {
            // truncated: the key is known when the record's key bytes were complete
            int64_t len = 0;
            for (int b = 0; b < c.nb; ++b)
                if (c.bt.bidx[b] == gb) len = c.bt.len[b];
            const bool key_ok = len - r * s->stride >= s->K;
            int32_t col = -1;
            if (s->is_matrix && key_ok) col = (int32_t)((off - r * s->stride - s->K) / s->V);
            rc = record_error(s, DML_E_TRUNCATED, key_ok ? read_key_at(s, rec) : 0, col);
        }
    }
    if (abnormal && !s->pend.empty()) {
        if (rc != DML_OK) {
            for (auto& q : s->pend) (void)hipEventSynchronize(s->ws[q.w].done);
            s->pend.clear();  // their kernels were no-ops; the store stops here like the reference
        } else {
            Pending& q = s->pend.front();  // relaunch its apply; its index is still valid
            HIPCHK(hipEventSynchronize(s->ws[q.w].done));
            set_buffers(s, q.c, s->data);
            if (int r2 = launch_apply(s, q.c, s->ws[q.w], nullptr)) return r2;
        }
    }
    return rc;
}

int retire_all(dml_store* s) {
    while (!s->pend.empty()) {
        int rc = retire_front(s);
        if (rc) {
            s->pend.clear();
            return rc;
        }
    }
    return DML_OK;
}

// Run `n` device-resident pushes (global indices 0..n-1) as ordered chunks of
// <= kMaxW; up to two chunks stay in flight (retired later, in order).
int collect_apply_check(dml_store* s, bool block);

int run_batch(dml_store* s, const uint8_t* const* dptr, const int64_t* lens, int n) {
    if (int rc = collect_apply_check(s, false)) return rc;  // an int32 owner apply failed earlier
    const uint64_t seq = ++s->call_seq;
    for (int c0 = 0; c0 < n; c0 += kMaxW) {
        Chunk c;
        c.seq = seq;
        c.nb = std::min(kMaxW, n - c0);
        for (int j = 0; j < c.nb; ++j) {
            const int gb = c0 + j;
            int64_t nrec;
            uint64_t tcut;
            plan_bucket(s, lens[gb], gb, &nrec, &tcut);
            c.bt.base[j] = dptr[gb];
            c.bt.len[j] = lens[gb];
            c.bt.nrec[j] = nrec;
            c.bt.bidx[j] = gb;
            c.max_nrec = std::max(c.max_nrec, nrec);
            c.tail_cut = std::min(c.tail_cut, tcut);
        }
        if (c.max_nrec == 0 && c.tail_cut == kNoPos) continue;  // empty pushes: nothing to apply
        while ((int)s->pend.size() >= kRing - 1) {  // see Workspace
            int rc = retire_front(s);
            if (rc) { s->pend.clear(); return rc; }
        }
        if (s->err) return set_err(s->err, "store is in a failed state (see dml_store_error_state)");
        // Identity speculation: plain-sum matrices of the spec_shape
        // widths, when every push of the chunk is full-range (one record per row, no
        // ragged tail): no key index, the reduce verifies every record's key.
        if (s->is_matrix && reduce_mode(s) == kAdd && !s->no_spec && spec_shape(vtype_of(s->desc), s->cols) &&
            c.tail_cut == kNoPos) {
            bool full = true;
            for (int j = 0; j < c.nb && full; ++j) full = c.bt.nrec[j] == s->rows && c.bt.len[j] == s->rows * s->stride;
            if (full && !s->data_alt) {
                // the second shard buffer, only with headroom left for the caller's
                // buffers (exchange slices, partials): 1/8 of the device or 4 GiB
                const size_t need = (size_t)s->rows * (size_t)s->cols * (size_t)s->V;
                size_t free_b = 0, total_b = 0;
                const bool room = hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
                                  free_b > need + std::max<size_t>(total_b / 8, (size_t)4 << 30);
                if (!room || hipMalloc(&s->data_alt, need) != hipSuccess) {
                    (void)hipGetLastError();
                    s->data_alt = nullptr;
                    s->no_spec = true;  // no room for a second buffer: no speculation
                }
            }
            c.spec = full && s->data_alt;
        }
        c.bt.spec = c.spec ? 1 : 0;
        // Slot reuse: a speculative chunk may take a push's slots from
        // any column its workspace kept (a verified permutation of the workspace's
        // previous chunk), when that push's sampled keys match it (k_ident_check)
        c.bt.kept_cols = 0;
        c.keeps = c.spec;
        c.bt.keeps = c.keeps ? 1 : 0;
        if (c.keeps) {
            const Workspace& Wn = s->ws[s->next_ws];
            if (Wn.kept && slot_stride(Wn.kept_nb) == slot_stride(c.nb)) c.bt.kept_cols = Wn.perm;
        }
        c.bt.first = s->first;
        const Ctrl* prev = s->pend.empty() ? nullptr : s->ws[s->pend.back().w].ctrl;
        set_buffers(s, c, s->pend.empty() ? s->data : s->pend.back().c.out);
        Pending p;
        p.c = c;
        p.w = s->next_ws;
        s->next_ws = (s->next_ws + 1) % kRing;
        int rc = launch_chunk(s, p.c, s->ws[p.w], prev);
        if (rc) return rc;
        s->pend.push_back(p);
    }
    return DML_OK;
}

int check_store(dml_store* s) {
    if (!s) return set_err(DML_E_INVALID_ARG, "null store");
    return DML_OK;
}

// Result of the int32 owner applies (dml_store_apply_dense_device): the first
// negative counter becomes the store's IllegalStateException. `block` waits for
// the last apply; otherwise only a finished one is read.
int collect_apply_check(dml_store* s, bool block) {
    if (!s->neg_pending) return DML_OK;
    if (!block && hipEventQuery(s->neg_ev) == hipErrorNotReady) return DML_OK;
    HIPCHK(hipEventSynchronize(s->neg_ev));
    s->neg_pending = false;
    const unsigned long long idx = *s->neg_host;
    if (idx == kNoPos) return DML_OK;
    return record_error(s, DML_E_NEGATIVE_COUNTER, s->first + (int64_t)(idx / (unsigned long long)s->cols),
                        (int32_t)(idx % (unsigned long long)s->cols));
}

// Entry of every reading / non-push call: all accepted pushes applied and
// checked (read-your-writes).
int begin_call(dml_store* s) {
    int rc = retire_all(s);
    int rc2 = collect_apply_check(s, true);
    return rc ? rc : rc2;
}

}  // namespace

// ===========================================================================
extern "C" {

const char* dml_last_error(void) { return g_err.c_str(); }
const char* dml_version(void) { return "distml_amd 0.1 (gfx950)"; }

int dml_linear_split(int64_t first_key, int64_t last_key, int32_t n, int64_t* first_out, int64_t* last_out) {
    if (n <= 0 || !first_out || !last_out) return set_err(DML_E_INVALID_ARG, "bad linear_split args");
    // KeyRange.linearSplit (KeyRange.java:68-80)
    int64_t start = first_key;
    const int64_t step = (last_key - first_key + n) / n;
    for (int32_t i = 0; i < n; ++i) {
        const int64_t end = std::min(start + step - 1, last_key);
        first_out[i] = start;
        last_out[i] = end;
        start += step;
    }
    return DML_OK;
}

int dml_store_create_range(const dml_desc* desc, int64_t first_key, int64_t last_key, int32_t cols, int32_t device,
                           uint32_t flags, dml_store** out) {
    if (!desc || !out) return set_err(DML_E_INVALID_ARG, "null argument");
    *out = nullptr;
    const dml_desc d = *desc;
    // DataStore.createStore dispatch (DataStore.java:50-92)
    if ((d.data_type != 0 && d.data_type != 1) || (d.key_type != 0 && d.key_type != 1) ||
        (d.value_type != DML_ELEMENT_TYPE_INT && d.value_type != DML_ELEMENT_TYPE_FLOAT &&
         d.value_type != DML_ELEMENT_TYPE_DOUBLE))
        return set_err(DML_E_BAD_DESC, "Unrecognized matrix type (DataStore.createStore)");
    if (d.data_type == 1 && !d.dense_column)
        return set_err(DML_E_UNSUPPORTED, "sparse-column matrix pushes are not supported (SURVEY defect 3)");
    if (last_key < first_key) return set_err(DML_E_INVALID_ARG, "empty KeyRange shard");
    if (d.data_type == 1 && cols <= 0) return set_err(DML_E_INVALID_ARG, "cols must be > 0");
    const int64_t rows = last_key - first_key + 1;
    if (rows > INT32_MAX) return set_err(DML_E_INVALID_ARG, "shard larger than a Java array");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return set_err(DML_E_HIP, "no HIP device");
    if (device < 0 || device >= ndev) return set_err(DML_E_INVALID_ARG, "bad device ordinal");
    DeviceGuard g(device);

    auto* s = new (std::nothrow) dml_store();
    if (!s) return set_err(DML_E_NOMEM, "out of host memory");
    s->device = device;
    s->desc = d;
    s->flags = flags;
    s->no_spec = (flags & DML_FLAG_NO_SPECULATION) != 0;
    s->is_matrix = d.data_type == 1;
    s->adagrad = s->is_matrix && d.value_type == DML_ELEMENT_TYPE_FLOAT && d.ada_grad;
    s->K = d.key_type == 0 ? 4 : 8;
    s->V = (d.value_type == DML_ELEMENT_TYPE_INT || d.value_type == DML_ELEMENT_TYPE_FLOAT) ? 4 : 8;
    s->array_vs = s->V;
    if (!s->is_matrix && d.value_type == DML_ELEMENT_TYPE_FLOAT && (flags & DML_FLAG_FLOAT_ARRAY_REF_STRIDE))
        s->array_vs = 8;  // FloatArrayStore.VALUE_SIZE (FloatArrayStore.java:15)
    s->first = first_key;
    s->last = last_key;
    s->rows = rows;
    s->cols = s->is_matrix ? cols : 1;
    s->stride = s->is_matrix ? s->K + (int64_t)s->V * s->cols : s->K + s->array_vs;

    auto fail = [&](hipError_t e, const char* what) {
        dml_store_destroy(s);
        return set_err(DML_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    hipError_t e;
    const size_t nbytes = (size_t)rows * (size_t)s->cols * (size_t)s->V;
    // A small shard's pushes are latency-bound (a few blocks for microseconds): its
    // streams take the high priority, so that on a GPU shared with a large store (LDA's
    // doc-topic totals beside the word-topic rows, LightLDA.scala:238-239) its kernels
    // are dispatched between the large store's reduce blocks instead of queueing
    // behind the whole reduce, which would hold up the caller's next push.
    int prio_lo = 0, prio_hi = 0;
    if ((e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi)) != hipSuccess) return fail(e, "stream priorities");
    const int prio = nbytes <= kSmallStoreBytes ? prio_hi : 0;
    auto mkstream = [&](hipStream_t* st) { return hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio); };
    if ((e = mkstream(&s->stream)) != hipSuccess) return fail(e, "stream");
    if ((e = hipMalloc(&s->data, nbytes)) != hipSuccess) return fail(e, "shard alloc");
    if ((e = hipMemsetAsync(s->data, 0, nbytes, s->stream)) != hipSuccess) return fail(e, "shard zero");
    if (s->adagrad) {
        const size_t n = (size_t)rows * (size_t)s->cols;
        if ((e = hipMalloc((void**)&s->alpha, n * 4)) != hipSuccess) return fail(e, "alpha alloc");
        if ((e = hipMalloc((void**)&s->delta, n * 4)) != hipSuccess) return fail(e, "delta alloc");
        if ((e = hipMemsetAsync(s->alpha, 0, n * 4, s->stream)) != hipSuccess) return fail(e, "alpha zero");
        if ((e = hipMemsetAsync(s->delta, 0, n * 4, s->stream)) != hipSuccess) return fail(e, "delta zero");
        s->cand_n = reduce_blocks(d.value_type, rows, s->cols);
        if ((e = hipMalloc((void**)&s->cand, sizeof(DeltaCand) * (size_t)(s->cand_n + kMdParts))) != hipSuccess)
            return fail(e, "cand alloc");
        if ((e = hipMalloc((void**)&s->md, sizeof(MaxDelta))) != hipSuccess) return fail(e, "md alloc");
        if ((e = hipMemsetAsync(s->md, 0, sizeof(MaxDelta), s->stream)) != hipSuccess) return fail(e, "md zero");
    }
    s->slot_bytes = s->is_matrix ? (size_t)rows * kMaxW * sizeof(int32_t) : 0;
    s->ws_bytes = sizeof(Ctrl) + s->slot_bytes + (s->is_matrix ? (size_t)rows * sizeof(uint32_t) : 0);
    if ((e = mkstream(&s->istream)) != hipSuccess) return fail(e, "index stream");
    if ((e = mkstream(&s->cstream)) != hipSuccess) return fail(e, "copy stream");
    for (Workspace& W : s->ws) {
        if ((e = hipMalloc((void**)&W.base, s->ws_bytes)) != hipSuccess) return fail(e, "workspace alloc");
        W.ctrl = (Ctrl*)W.base;
        W.slot = (int32_t*)(W.base + sizeof(Ctrl));
        W.rowflag = (uint32_t*)(W.base + sizeof(Ctrl) + s->slot_bytes);
        if ((e = hipHostMalloc((void**)&W.hctrl, sizeof(Ctrl), hipHostMallocDefault)) != hipSuccess) return fail(e, "ctrl");
        if ((e = hipEventCreateWithFlags(&W.idx_done, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
        if ((e = hipEventCreateWithFlags(&W.done, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
        if ((e = hipEventCreate(&W.applied)) != hipSuccess) return fail(e, "event");
        if ((e = hipEventCreate(&W.kstart)) != hipSuccess) return fail(e, "event");
    }
    if ((e = hipStreamSynchronize(s->stream)) != hipSuccess) return fail(e, "init sync");
    *out = s;
    return DML_OK;
}

void dml_store_destroy(dml_store* s) {
    if (!s) return;
    {
        std::lock_guard<std::mutex> lk(s->mu);
        DeviceGuard g(s->device);
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (s->istream) (void)hipStreamSynchronize(s->istream);
        if (s->cstream) (void)hipStreamSynchronize(s->cstream);
        for (auto& p : s->ev_used) {
            bool ring = false;
            for (const Workspace& W : s->ws) ring |= p.first == W.kstart;
            if (!ring) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
        }
        for (auto& p : s->ev_free) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
        for (Workspace& W : s->ws) {
            (void)hipFree(W.base);
            (void)hipFree(W.sp);
            if (W.hsp) (void)hipHostFree(W.hsp);
            if (W.hidx) (void)hipHostFree(W.hidx);
            if (W.listed) (void)hipFree(W.listed);
            if (W.hctrl) (void)hipHostFree(W.hctrl);
            if (W.idx_done) (void)hipEventDestroy(W.idx_done);
            if (W.done) (void)hipEventDestroy(W.done);
            if (W.applied) (void)hipEventDestroy(W.applied);
            if (W.kstart) (void)hipEventDestroy(W.kstart);
        }
        (void)hipFree(s->data);
        (void)hipFree(s->data_alt);
        (void)hipFree(s->alpha);
        (void)hipFree(s->delta);
        (void)hipFree(s->cand);
        (void)hipFree(s->md);
        (void)hipFree(s->neg_dev);
        if (s->neg_host) (void)hipHostFree(s->neg_host);
        if (s->neg_ev) (void)hipEventDestroy(s->neg_ev);
        (void)hipFree(s->dstage);
        if (s->hstage) (void)hipHostFree(s->hstage);
        (void)hipFree(s->dscr);
        for (int i = 0; i < 2; ++i) {
            if (s->xbuf[i]) (void)hipHostFree(s->xbuf[i]);
            if (s->xev[i]) (void)hipEventDestroy(s->xev[i]);
        }
        if (s->stream) (void)hipStreamDestroy(s->stream);
        if (s->istream) (void)hipStreamDestroy(s->istream);
        if (s->cstream) (void)hipStreamDestroy(s->cstream);
    }
    delete s;
}

static int push_host(dml_store* s, const uint8_t* const* bufs, const int64_t* lens, int32_t n) {
    if (n < 0 || (n > 0 && (!bufs || !lens))) return set_err(DML_E_INVALID_ARG, "bad push arguments");
    int rc = begin_call(s);
    if (rc) return rc;
    if (s->err) return set_err(s->err, "store is in a failed state (see dml_store_error_state)");
    size_t total = 0;
    std::vector<size_t> offs((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        if (lens[i] < 0 || (lens[i] > 0 && !bufs[i])) return set_err(DML_E_INVALID_ARG, "bad push buffer");
        offs[(size_t)i] = total;
        total += ((size_t)lens[i] + 255) & ~(size_t)255;
    }
    // Pinned caller buffers (hipHostMalloc / hipHostRegister) DMA straight into HBM;
    // pageable ones are copied into pinned staging push by push, each push's DMA
    // overlapping the CPU copy of the next. All on the index stream (the index
    // reads the bytes first; the apply waits for the index).
    bool all_pinned = true;
    for (int32_t i = 0; i < n && all_pinned; ++i) {
        if (lens[i] == 0) continue;
        hipPointerAttribute_t attr;
        all_pinned = hipPointerGetAttributes(&attr, bufs[i]) == hipSuccess && attr.type == hipMemoryTypeHost;
    }
    (void)hipGetLastError();  // a pageable pointer leaves an error from the attribute query
    rc = ensure_stage(s, total);
    if (rc) return rc;
    for (int32_t i = 0; i < n; ++i) {
        if (lens[i] == 0) continue;
        const uint8_t* src = bufs[i];
        if (!all_pinned) {
            std::memcpy(s->hstage + offs[(size_t)i], bufs[i], (size_t)lens[i]);
            src = s->hstage + offs[(size_t)i];
        }
        HIPCHK(hipMemcpyAsync(s->dstage + offs[(size_t)i], src, (size_t)lens[i], hipMemcpyHostToDevice, s->istream));
    }
    if (all_pinned && (s->flags & DML_FLAG_ASYNC)) HIPCHK(hipStreamSynchronize(s->istream));  // borrowed bytes
    std::vector<const uint8_t*> dptr((size_t)n);
    for (int32_t i = 0; i < n; ++i) dptr[(size_t)i] = s->dstage + offs[(size_t)i];
    rc = run_batch(s, dptr.data(), lens, n);
    if (rc) return rc;
    if (!(s->flags & DML_FLAG_ASYNC)) return retire_all(s);
    return DML_OK;  // async: the caller's bytes are in staging or already DMA'd
}

int dml_store_push(dml_store* s, const uint8_t* data, int64_t len) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    const uint8_t* bufs[1] = {data};
    return push_host(s, bufs, &len, 1);
}

int dml_store_push_batch(dml_store* s, const uint8_t* const* bufs, const int64_t* lens, int32_t n) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    return push_host(s, bufs, lens, n);
}

int dml_store_push_batch_device(dml_store* s, const void* const* dev_bufs, const int64_t* lens, int32_t n) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (n < 0 || (n > 0 && (!dev_bufs || !lens))) return set_err(DML_E_INVALID_ARG, "bad push arguments");
    // no retire-all here: run_batch keeps up to kRing-1 chunks in flight
    if (s->err) return set_err(s->err, "store is in a failed state (see dml_store_error_state)");
    for (int32_t i = 0; i < n; ++i)
        if (lens[i] < 0 || (lens[i] > 0 && !dev_bufs[i])) return set_err(DML_E_INVALID_ARG, "bad push buffer");
    return run_batch(s, (const uint8_t* const*)dev_bufs, lens, n);
}

int dml_store_flush(dml_store* s) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    int rc = begin_call(s);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_store_push_seq(dml_store* s, uint64_t* seq) {
    if (int rc = check_store(s)) return rc;
    if (!seq) return set_err(DML_E_INVALID_ARG, "null out");
    std::lock_guard<std::mutex> lk(s->mu);
    *seq = s->call_seq;
    return DML_OK;
}

int dml_store_retire(dml_store* s, uint64_t seq) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    while (!s->pend.empty() && s->pend.front().c.seq <= seq) {
        if (int rc = retire_front(s)) {
            s->pend.clear();
            return rc;
        }
    }
    return DML_OK;
}

int dml_store_stats(dml_store* s, dml_store_counters* out, int32_t reset) {
    if (int rc = check_store(s)) return rc;
    if (!out) return set_err(DML_E_INVALID_ARG, "null out");
    std::lock_guard<std::mutex> lk(s->mu);
    *out = s->st;
    if (reset) s->st = dml_store_counters{};
    return DML_OK;
}

int dml_store_error_state(dml_store* s, int64_t* bad_key, int32_t* bad_col) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    if (bad_key) *bad_key = s->err_key;
    if (bad_col) *bad_col = s->err_col;
    return s->err;
}

void dml_store_clear_error(dml_store* s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(s->mu);
    s->err = 0;
    s->err_key = 0;
    s->err_col = -1;
    if (s->neg_dev) {  // int32 owner applies resume
        DeviceGuard g(s->device);
        (void)hipStreamSynchronize(s->stream);
        s->neg_pending = false;
        (void)hipMemsetAsync(s->neg_dev, 0xFF, sizeof(unsigned long long), s->stream);
        (void)hipStreamSynchronize(s->stream);
    }
}

int dml_store_shape(dml_store* s, int64_t* rows, int32_t* cols) {
    if (int rc = check_store(s)) return rc;
    if (rows) *rows = s->rows;
    if (cols) *cols = s->cols;
    return DML_OK;
}

int dml_store_value_type(dml_store* s, int32_t* value_type, int32_t* adagrad) {
    if (int rc = check_store(s)) return rc;
    if (value_type) *value_type = s->desc.value_type;
    if (adagrad) *adagrad = s->adagrad ? 1 : 0;
    return DML_OK;
}

int dml_store_read_dense(dml_store* s, void* host_dst, int64_t bytes) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    const int64_t need = s->rows * s->cols * s->V;
    if (!host_dst || bytes < need) return set_err(DML_E_CAPACITY, "destination too small");
    if (int rc = begin_call(s)) return rc;
    HIPCHK(hipMemcpyAsync(host_dst, s->data, (size_t)need, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_store_write_dense(dml_store* s, const void* host_src, int64_t bytes) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    const int64_t need = s->rows * s->cols * s->V;
    if (!host_src || bytes != need) return set_err(DML_E_CAPACITY, "source size does not match the shard");
    if (int rc = begin_call(s)) return rc;
    HIPCHK(hipMemcpyAsync(s->data, host_src, (size_t)need, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_store_device_ptr(dml_store* s, void** dev_ptr) {
    if (int rc = check_store(s)) return rc;
    if (!dev_ptr) return set_err(DML_E_INVALID_ARG, "null out");
    *dev_ptr = s->data;
    return DML_OK;
}

int dml_store_read_adagrad(dml_store* s, float* alpha_dst, float* delta_dst, int64_t elems) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (!s->adagrad) return set_err(DML_E_UNSUPPORTED, "not an AdaGrad store");
    if (elems < s->rows * s->cols) return set_err(DML_E_CAPACITY, "destination too small");
    if (int rc = begin_call(s)) return rc;
    const size_t n = (size_t)(s->rows * s->cols) * 4;
    if (alpha_dst) HIPCHK(hipMemcpyAsync(alpha_dst, s->alpha, n, hipMemcpyDeviceToHost, s->stream));
    if (delta_dst) HIPCHK(hipMemcpyAsync(delta_dst, s->delta, n, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_store_read_rows(dml_store* s, int32_t which, int64_t row0, int64_t nrows, void* host_dst, int64_t bytes) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (which < 0 || which > 2 || row0 < 0 || nrows < 0 || row0 > s->rows || nrows > s->rows - row0)
        return set_err(DML_E_INVALID_ARG, "bad row range or array");
    if (which != 0 && !s->adagrad) return set_err(DML_E_UNSUPPORTED, "not an AdaGrad store");
    const int64_t esz = which == 0 ? s->V : 4;
    const int64_t need = nrows * s->cols * esz;
    if (need > 0 && (!host_dst || bytes < need)) return set_err(DML_E_CAPACITY, "destination too small");
    if (int rc = begin_call(s)) return rc;
    if (need == 0) return DML_OK;
    const uint8_t* src = (const uint8_t*)(which == 0 ? s->data : which == 1 ? (void*)s->alpha : (void*)s->delta);
    HIPCHK(hipMemcpyAsync(host_dst, src + row0 * s->cols * esz, (size_t)need, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_store_fill(dml_store* s, double v) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    HIPCHK(launch_fill(vtype_of(s->desc), s->data, s->rows * s->cols, v, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_store_set_alpha(dml_store* s, float initial_alpha, float min_alpha, float factor) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (!s->adagrad) return set_err(DML_E_UNSUPPORTED, "not an AdaGrad store");
    if (int rc = begin_call(s)) return rc;
    // setAlpha: setAlphaValue(initialAlpha) then the three fields (FloatMatrixStoreAdaGrad.java:77-82)
    HIPCHK(launch_fill_f32(s->alpha, s->rows * s->cols, initial_alpha, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    s->initial_alpha = initial_alpha;
    s->min_alpha = min_alpha;
    s->factor = factor;
    return DML_OK;
}

int dml_store_max_delta(dml_store* s, float* max_delta, int32_t* row, int32_t* col) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (!s->adagrad) return set_err(DML_E_UNSUPPORTED, "not an AdaGrad store");
    if (int rc = begin_call(s)) return rc;
    MaxDelta m;
    HIPCHK(hipMemcpyAsync(&m, s->md, sizeof m, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    if (max_delta) *max_delta = m.value;
    if (row) *row = m.row;
    if (col) *col = m.col;
    return DML_OK;
}

// keys == nullptr: the keys are key_lo .. key_lo + nkeys - 1 (a KeyRange already
// clipped to the shard), encoded without a key array.
static int fetch_impl(dml_store* s, const int64_t* keys, int64_t nkeys, int64_t key_lo, uint8_t* out, int64_t cap,
                      int64_t* out_len) {
    if (nkeys < 0 || !out_len) return set_err(DML_E_INVALID_ARG, "bad fetch arguments");
    // record layout of handleFetch (dense column)
    int64_t rec;
    int value_slot;
    if (s->is_matrix) {
        value_slot = s->adagrad ? 8 : s->V;
        rec = s->K + (int64_t)s->cols * value_slot;
    } else {
        value_slot = (s->desc.value_type == DML_ELEMENT_TYPE_FLOAT) ? 8 : s->V;  // FloatArrayStore VALUE_SIZE 8
        rec = s->K + value_slot;
    }
    *out_len = nkeys * rec;
    if (!out || cap < *out_len) return set_err(DML_E_CAPACITY, "fetch output buffer too small");
    if (keys) {
        for (int64_t j = 0; j < nkeys; ++j) {
            const int32_t idx = (int32_t)(uint32_t)((uint64_t)keys[j] - (uint64_t)s->first);
            if (idx < 0 || idx >= s->rows) return record_error(s, DML_E_KEY_OUT_OF_SHARD, keys[j], -1);
        }
    }
    if (nkeys == 0) return DML_OK;
    const size_t kbytes = keys ? ((size_t)nkeys * 8 + 255) & ~(size_t)255 : 0;
    if (int rc = ensure_scratch(s, kbytes + (size_t)*out_len)) return rc;
    const int64_t* dkeys = keys ? (const int64_t*)s->dscr : nullptr;
    if (keys) HIPCHK(hipMemcpyAsync(s->dscr, keys, (size_t)nkeys * 8, hipMemcpyHostToDevice, s->stream));
    uint8_t* dout = s->dscr + kbytes;
    HIPCHK(launch_fetch(vtype_of(s->desc), s->data, s->adagrad ? s->alpha : nullptr, s->cols, dkeys, key_lo, nkeys,
                        s->first, dout, rec, s->K, value_slot, s->stream));
    return d2h(s, out, dout, (size_t)*out_len);
}

int dml_store_fetch(dml_store* s, const int64_t* keys, int64_t nkeys, uint8_t* out, int64_t cap, int64_t* out_len) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    if (nkeys > 0 && !keys) return set_err(DML_E_INVALID_ARG, "null keys");
    return fetch_impl(s, keys, nkeys, 0, out, cap, out_len);
}

int dml_store_fetch_range(dml_store* s, int64_t first_key, int64_t last_key, uint8_t* out, int64_t cap,
                          int64_t* out_len) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    // KeyRange.intersect (KeyRange.java:124-136): clip to the shard, ascending
    const int64_t lo = std::max(first_key, s->first), hi = std::min(last_key, s->last);
    if (!out_len) return set_err(DML_E_INVALID_ARG, "null out_len");
    return fetch_impl(s, nullptr, lo <= hi ? hi - lo + 1 : 0, lo, out, cap, out_len);
}

// Rows [lo, hi] (local indices), big-endian, row-major: DataOutputStream.write{Float,Int,Double}.
static int write_rows_be(dml_store* s, int64_t lo, int64_t hi, uint8_t* out) {
    if (hi < lo) return DML_OK;
    const int64_t n = (hi - lo + 1) * s->cols;
    const size_t bytes = (size_t)n * (size_t)s->V;
    if (int rc = ensure_scratch(s, bytes)) return rc;
    HIPCHK(launch_bswap(s->V, (const uint8_t*)s->data + (size_t)lo * s->cols * s->V, s->dscr, n, s->stream));
    return d2h(s, out, s->dscr, bytes);
}

// The first `nelem` elements from row lo on, from big-endian bytes (DataInputStream.read*).
static int read_elems_be(dml_store* s, int64_t lo, int64_t nelem, const uint8_t* in) {
    if (nelem <= 0) return DML_OK;
    const size_t bytes = (size_t)nelem * (size_t)s->V;
    if (int rc = ensure_scratch(s, bytes)) return rc;
    if (int rc = h2d(s, s->dscr, in, bytes)) return rc;
    HIPCHK(launch_bswap(s->V, s->dscr, (uint8_t*)s->data + (size_t)lo * s->cols * s->V, nelem, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_store_write_all(dml_store* s, uint8_t* out_be, int64_t cap, int64_t* out_len) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    const int64_t bytes = s->rows * s->cols * s->V;
    if (out_len) *out_len = bytes;
    if (!out_be || cap < bytes) return set_err(DML_E_CAPACITY, "writeAll buffer too small");
    return write_rows_be(s, 0, s->rows - 1, out_be);
}

int dml_store_read_all(dml_store* s, const uint8_t* in_be, int64_t len) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    const int64_t n = s->rows * s->cols;
    if (len < 0 || (len > 0 && !in_be)) return set_err(DML_E_INVALID_ARG, "bad readAll arguments");
    // readFloat past the end throws EOFException after the elements before it were assigned
    const int64_t avail = std::min(n, len / s->V);
    if (int rc = read_elems_be(s, 0, avail, in_be)) return rc;
    if (avail < n) return set_err(DML_E_TRUNCATED, "readAll: stream shorter than the shard");
    return DML_OK;
}

int dml_store_sync_to(dml_store* s, int32_t from_row, int32_t to_row, uint8_t* out_be, int64_t cap,
                      int64_t* out_len) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    if (!out_len) return set_err(DML_E_INVALID_ARG, "null out_len");
    *out_len = 0;
    if (to_row < from_row) return DML_OK;  // the loop body never runs
    // localData[i] for i = from..to: a negative row throws before any write, a row
    // past the shard after the rows before it were written (ArrayIndexOutOfBounds)
    if (from_row < 0) return set_err(DML_E_KEY_OUT_OF_SHARD, "syncTo: negative row");
    const int64_t hi = std::min<int64_t>(to_row, s->rows - 1);
    const int64_t bytes = hi >= from_row ? (hi - from_row + 1) * s->cols * s->V : 0;
    if (!out_be || cap < bytes) {
        *out_len = bytes;
        return set_err(DML_E_CAPACITY, "syncTo buffer too small");
    }
    if (int rc = write_rows_be(s, from_row, hi, out_be)) return rc;
    *out_len = bytes;
    if (to_row >= s->rows) return set_err(DML_E_KEY_OUT_OF_SHARD, "syncTo: row past the shard");
    return DML_OK;
}

int dml_store_sync_from(dml_store* s, int32_t from_row, int32_t to_row, const uint8_t* in_be, int64_t len) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    if (len < 0 || (len > 0 && !in_be)) return set_err(DML_E_INVALID_ARG, "bad syncFrom arguments");
    if (to_row < from_row) return DML_OK;
    if (from_row < 0) return set_err(DML_E_KEY_OUT_OF_SHARD, "syncFrom: negative row");
    // elements assigned in order until the stream ends (EOF) or a row falls past the shard
    const int64_t hi = std::min<int64_t>(to_row, s->rows - 1);
    const int64_t want = hi >= from_row ? (hi - from_row + 1) * s->cols : 0;
    const int64_t avail = std::min(want, len / s->V);
    if (int rc = read_elems_be(s, from_row, avail, in_be)) return rc;
    if (avail < want) return set_err(DML_E_TRUNCATED, "syncFrom: stream shorter than the rows");
    if (to_row >= s->rows) return set_err(DML_E_KEY_OUT_OF_SHARD, "syncFrom: row past the shard");
    return DML_OK;
}

int dml_host_alloc(int64_t bytes, void** host_ptr) {
    if (bytes < 0 || !host_ptr) return set_err(DML_E_INVALID_ARG, "bad host alloc arguments");
    *host_ptr = nullptr;
    HIPCHK(hipHostMalloc(host_ptr, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault));
    return DML_OK;
}

void dml_host_free(void* host_ptr) {
    if (host_ptr) (void)hipHostFree(host_ptr);
}

int dml_store_stream(dml_store* s, void** stream) {
    if (int rc = check_store(s)) return rc;
    if (!stream) return set_err(DML_E_INVALID_ARG, "null out");
    *stream = (void*)s->stream;
    return DML_OK;
}

int dml_store_set_timing(dml_store* s, int32_t enable) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    s->timing = enable != 0;
    s->timing_every = enable > 1 ? enable : 1;
    s->timing_k = 0;
    return DML_OK;
}

// DML_KNOB_INDEX_CUS: the index stream (the next chunk's key index / sparse partition)
// on k of the device's CUs and the apply stream on the others (k = 0: both streams on
// every CU, the default). pattern 0 spreads the k CUs evenly over the CU numbering,
// 1 takes the first k. Caller holds s->mu.
static int set_cu_split(dml_store* s, int k, int pattern) {
    DeviceGuard g(s->device);
    int ncu = 0;
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s->device));
    if (k < 0 || k >= ncu || pattern < 0 || pattern > 1) return set_err(DML_E_INVALID_ARG, "bad CU split");
    if (int rc = begin_call(s)) return rc;
    HIPCHK(hipStreamSynchronize(s->stream));
    HIPCHK(hipStreamSynchronize(s->istream));
    const int words = (ncu + 31) / 32;
    std::vector<uint32_t> mi((size_t)words, 0u), ma((size_t)words, 0u);
    for (int c = 0; c < ncu; ++c) {
        const bool idx = k > 0 && (pattern == 1 ? c < k : (int64_t)c * k % ncu < k);
        (idx ? mi : ma)[(size_t)(c / 32)] |= 1u << (c % 32);
    }
    hipStream_t ns = nullptr, ni = nullptr;
    if (k == 0) {
        HIPCHK(hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&ni, hipStreamNonBlocking));
    } else {
        HIPCHK(hipExtStreamCreateWithCUMask(&ns, (uint32_t)words, ma.data()));
        HIPCHK(hipExtStreamCreateWithCUMask(&ni, (uint32_t)words, mi.data()));
    }
    (void)hipStreamDestroy(s->stream);
    (void)hipStreamDestroy(s->istream);
    s->stream = ns;
    s->istream = ni;
    return DML_OK;
}

int dml_diag_store_knob(dml_store* s, int32_t knob, int64_t value) {
    if (int rc = check_store(s)) return rc;
    if (value < 0) return set_err(DML_E_INVALID_ARG, "negative knob value");
    std::lock_guard<std::mutex> lk(s->mu);
    switch (knob) {
        case DML_KNOB_IDENT_FULL_MIN_BYTES: s->ident_full_min = value; return DML_OK;
        case DML_KNOB_INDEX_CUS: return set_cu_split(s, (int)(value & 0xFFFF), (int)(value >> 16));
        default: return set_err(DML_E_INVALID_ARG, "unknown knob");
    }
}

int dml_store_kernel_name(dml_store* s, char* out, int32_t cap) {
    if (int rc = check_store(s)) return rc;
    if (!out || cap <= 0) return set_err(DML_E_INVALID_ARG, "bad name buffer");
    std::lock_guard<std::mutex> lk(s->mu);
    const char* n = s->kname ? s->kname : "";
    std::snprintf(out, (size_t)cap, "%s", n);
    return (int32_t)std::strlen(n) < cap ? DML_OK : set_err(DML_E_CAPACITY, "name buffer too small");
}

int dml_store_kernel_time(dml_store* s, double* total_ms, int64_t* launches, int32_t reset) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    HIPCHK(hipStreamSynchronize(s->stream));
    ev_collect(s);
    if (total_ms) *total_ms = s->timed_ms;
    if (launches) *launches = s->timed_n;
    if (reset) {
        s->timed_ms = 0.0;
        s->timed_n = 0;
    }
    return DML_OK;
}

int dml_store_apply_dense_device(dml_store* s, const void* dev_src, int64_t elems) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    // pushes before it are retired (an error there stops the store like the
    // reference); the previous owner apply's check is read only if it has finished:
    // blocking on it would serialize the sharded int32 pipeline
    if (int rc = retire_all(s)) return rc;
    if (int rc = collect_apply_check(s, false)) return rc;
    if (s->err) return set_err(s->err, "store is in a failed state (see dml_store_error_state)");
    if (!dev_src || elems != s->rows * s->cols) return set_err(DML_E_INVALID_ARG, "apply size mismatch");
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (s->timing) {
        ev = ev_pair(s);
        HIPCHK(hipEventRecord(ev.first, s->stream));
    }
    if (vtype_of(s->desc) == kI32) {
        // IntMatrixStore: check the final counters (IntMatrixStore.java:174-176); the
        // kernel skips itself once an earlier apply left a negative (sticky neg_dev)
        if (!s->neg_dev) {
            HIPCHK(hipMalloc((void**)&s->neg_dev, sizeof(unsigned long long)));
            HIPCHK(hipMemsetAsync(s->neg_dev, 0xFF, sizeof(unsigned long long), s->stream));
            HIPCHK(hipHostMalloc((void**)&s->neg_host, sizeof(unsigned long long), hipHostMallocDefault));
            HIPCHK(hipEventCreateWithFlags(&s->neg_ev, hipEventDisableTiming));
        }
        HIPCHK(launch_apply_dense_i32chk((int32_t*)s->data, (const int32_t*)dev_src, elems, s->neg_dev, s->stream));
        HIPCHK(hipMemcpyAsync(s->neg_host, s->neg_dev, sizeof(unsigned long long), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipEventRecord(s->neg_ev, s->stream));
        s->neg_pending = true;
    } else {
        HIPCHK(launch_apply_dense(vtype_of(s->desc), s->data, dev_src, elems, s->stream));
    }
    if (s->timing) {
        HIPCHK(hipEventRecord(ev.second, s->stream));
        s->ev_used.push_back(ev);
    }
    return DML_OK;
}

int dml_store_apply_adagrad_moments_device(dml_store* s, const void* dev_src, int64_t rows) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (!s->adagrad) return set_err(DML_E_UNSUPPORTED, "not an AdaGrad store");
    if (!dev_src || rows != s->rows) return set_err(DML_E_INVALID_ARG, "moments size mismatch");
    if (s->cols % 4) return set_err(DML_E_UNSUPPORTED, "two-moment apply: rows of whole 16-B vectors");
    if (int rc = retire_all(s)) return rc;
    if (s->err) return set_err(s->err, "store is in a failed state (see dml_store_error_state)");
    if (s->cand_n < kMomentBlocks) {  // one candidate per apply block
        HIPCHK(hipStreamSynchronize(s->stream));
        HIPCHK(hipFree(s->cand));
        s->cand = nullptr;
        HIPCHK(hipMalloc((void**)&s->cand, sizeof(DeltaCand) * (size_t)(kMomentBlocks + kMdParts)));
        s->cand_n = kMomentBlocks;
    }
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (s->timing) ev = ev_pair(s);
    HIPCHK(launch_ada_moments((float*)s->data, (const float*)dev_src, s->rows, s->cols, ada_args(s), s->md, s->first,
                              s->stream, LaunchEv{ev.first, ev.second}));
    if (s->timing) s->ev_used.push_back(ev);
    s->kname = g_kernel_name;
    return DML_OK;
}

}  // extern "C"

// Per-device pool of pre-reduce workspaces (Ctrl + slot table + rowflags).
// hipMalloc/hipFree per step cost ~0.2 ms of host time (hipFree synchronizes
// the device); leases are taken and returned instead, one per in-flight call.
struct WsLease {
    uint8_t* ptr = nullptr;
    size_t bytes = 0;
    bool clean = false;     // slot table all -1 and rowflags 0 (left so by a clearing pre-reduce)
    Ctrl* hctrl = nullptr;  // pinned host copy of the Ctrl (read without touching a stream)
};
static std::mutex g_ws_mu;
static std::unordered_map<int, std::vector<WsLease>> g_ws_free;

static int ws_acquire(int dev, size_t bytes, WsLease* out) {
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        auto& v = g_ws_free[dev];
        for (size_t i = 0; i < v.size(); ++i)
            if (v[i].bytes >= bytes) {
                *out = v[i];
                v.erase(v.begin() + (ptrdiff_t)i);
                return DML_OK;
            }
    }
    WsLease l;
    hipError_t e = hipMalloc((void**)&l.ptr, bytes);
    if (e == hipSuccess) e = hipHostMalloc((void**)&l.hctrl, sizeof(Ctrl), hipHostMallocDefault);
    if (e != hipSuccess) {
        if (l.ptr) (void)hipFree(l.ptr);
        return set_err(DML_E_HIP, hipGetErrorString(e));
    }
    l.bytes = bytes;
    *out = l;
    return DML_OK;
}

static void ws_release(int dev, const WsLease& l) {
    if (!l.ptr) return;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    g_ws_free[dev].push_back(l);
}

extern "C" {

// Stand-alone ordered pre-reduce (multi-GPU): per-device scratch for Ctrl+slots.
int dml_reduce_buckets_dense(const dml_desc* desc, int64_t first_key, int64_t rows, int32_t cols,
                             const void* const* dev_bufs, const int64_t* lens, int32_t n, void* dev_out, void* stream) {
    if (!desc || !dev_out || rows <= 0 || cols <= 0 || n < 0 || (n > 0 && (!dev_bufs || !lens)))
        return set_err(DML_E_INVALID_ARG, "bad reduce arguments");
    if (desc->data_type != 1 || !desc->dense_column || desc->ada_grad)
        return set_err(DML_E_UNSUPPORTED, "pre-reduce supports dense-column plain matrices");
    const int vt = desc->value_type;
    if (vt != 0 && vt != 1 && vt != 3) return set_err(DML_E_BAD_DESC, "bad value type");
    const int K = desc->key_type == 0 ? 4 : 8, V = vt == 3 ? 8 : 4;
    const int64_t stride = K + (int64_t)V * cols;
    hipStream_t st = (hipStream_t)stream;
    const size_t sb = (size_t)rows * kMaxW * sizeof(int32_t);
    const size_t wsb = sizeof(Ctrl) + sb + (size_t)rows * sizeof(uint32_t);
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    WsLease lease;
    if (int rc = ws_acquire(dev, wsb, &lease)) return rc;
    uint8_t* ws = lease.ptr;
    Ctrl* ctrl = (Ctrl*)ws;
    int32_t* slot = (int32_t*)(ws + sizeof(Ctrl));
    uint32_t* rflag = (uint32_t*)(ws + sizeof(Ctrl) + sb);
    AdaArgs none{};
    int rc = DML_OK;
    for (int c0 = 0; c0 < std::max(n, 1) && rc == DML_OK; c0 += kMaxW) {
        Batch bt{};
        const int nb = std::max(0, std::min(kMaxW, n - c0));
        int64_t max_nrec = 0;
        for (int j = 0; j < nb; ++j) {
            bt.base[j] = (const uint8_t*)dev_bufs[c0 + j];
            bt.len[j] = lens[c0 + j];
            bt.nrec[j] = lens[c0 + j] / stride;
            bt.bidx[j] = c0 + j;
            if (lens[c0 + j] % stride) rc = set_err(DML_E_TRUNCATED, "ragged full-range bucket");
            max_nrec = std::max(max_nrec, bt.nrec[j]);
        }
        if (rc) break;
        hipError_t e = hipMemsetAsync(ws, 0xFF, sizeof(Ctrl) + sb, st);
        if (e == hipSuccess) e = hipMemsetAsync(rflag, 0, (size_t)rows * sizeof(uint32_t), st);
        if (e == hipSuccess) e = launch_index(bt, nb, max_nrec, stride, K, first_key, rows, slot, rflag, ctrl, kNoPos, st);
        if (e == hipSuccess)
            e = launch_reduce(vt, c0 == 0 ? kPreReduce : kAdd, dev_out, rows, cols, bt, nb, stride, K, slot, nullptr,
                              ctrl, kNoPos, none, st, nullptr);
        Ctrl h;
        if (e == hipSuccess) e = hipMemcpyAsync(&h, ctrl, sizeof h, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = set_err(DML_E_HIP, hipGetErrorString(e));
        else if (h.cutoff != kNoPos) rc = set_err(DML_E_KEY_OUT_OF_SHARD, "pre-reduce: key outside the matrix");
        else if (h.no_dup == 0u) rc = set_err(DML_E_UNSUPPORTED, "pre-reduce: a bucket repeats a row");
        if (n == 0) break;
    }
    lease.clean = false;  // this path memsets per chunk and does not track cleanliness
    ws_release(dev, lease);
    return rc;
}

// ---- piecewise pre-reduce (multi-GPU pipelining) ----------------------------
}  // extern "C"

struct dml_prereduce {
    dml_desc desc{};
    int64_t first = 0, rows = 0;
    int32_t cols = 0;
    int K = 4, V = 4;
    int64_t stride = 0;
    Batch bt{};
    int nb = 0;
    uint8_t* ws = nullptr;
    size_t ws_bytes = 0;
    Ctrl* ctrl = nullptr;
    int32_t* slot = nullptr;
    uint32_t* rowflag = nullptr;
    hipStream_t stream = nullptr;
    int device = 0;
    int64_t rows_done = 0;  // model rows the pieces reduced (all of them: the slot table is clean again)
    Ctrl* hctrl = nullptr;  // the lease's pinned Ctrl copy, DMA'd right behind the index
    hipEvent_t idx_ev = nullptr;   // begin stream: key index built
    hipEvent_t last_ev = nullptr;  // piece stream: last piece enqueued so far
    hipStream_t last_st = nullptr;
    bool idx_waited = false;
    bool timed = false;
    hipEvent_t done_ev = nullptr;  // completion of the last piece: last_ev, or its timing stop event
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;  // per-piece start/stop of a timed call
    // speculative calls of a pre-reduce context (dml_prereduce_begin_ctx)
    dml_prectx* ctx = nullptr;
    int wi = -1;            // the context's workspace
    bool spec = false;      // identity / kept-column speculation, verified by the pieces
    bool verified = false;  // dml_prereduce_verify ran (the partial is exact)
    int64_t max_nrec = 0;
    struct PieceRec {
        int64_t block, stride, off, ntask;
        void* out;
    };
    std::vector<PieceRec> prec;  // the pieces as launched (a failed verification re-runs them)
    hipEvent_t rerun_ev = nullptr;
    const Ctrl* hidx = nullptr;  // the workspace's Ctrl as the index left it (speculative calls of the flat shape)
};

// Pre-reduce context (dml_prectx_*): the sharded path's pre-reduce with the
// store's speculation. Three workspaces in a ring, like a store's;
// a verified call keeps its slot table, whose permutations the call three later
// may reuse. The partial is reduce-scattered only after dml_prereduce_verify has
// read the pieces' verdict (and re-run them exactly if it failed).
struct PreWs {
    uint8_t* base = nullptr;
    Ctrl* ctrl = nullptr;
    int32_t* slot = nullptr;
    uint32_t* rowflag = nullptr;
    Ctrl* hctrl = nullptr;          // pinned Ctrl, copied after the pieces (or their re-run)
    Ctrl* hidx = nullptr;           // pinned Ctrl, copied right after the index (k_flat_ident's choice)
    hipEvent_t ctrl_ev = nullptr;   // that copy done
    hipEvent_t free_ev = nullptr;   // the workspace's last call ended (pieces / re-run done)
    bool used = false, clean = false, kept = false;
    bool busy = false;              // a call holds it: begun, not yet ended
    int kept_nb = 0;
    uint64_t perm = 0;              // kept columns holding verified permutations (see Workspace)
};
struct dml_prectx {
    std::mutex mu;
    dml_desc desc{};
    int64_t first = 0, rows = 0;
    int32_t cols = 0;
    int K = 4, V = 4;
    int64_t stride = 0;
    int device = 0;
    size_t slot_bytes = 0;
    PreWs ws[kRing];
    int next = 0;
    hipStream_t xstream = nullptr;  // Ctrl read-back and re-runs
    dml_store_counters st{};
};

// Pre-reduce kernel timing (dml_prereduce_timing(every)): one call in `every`
// gets start/stop events in its pieces' dispatch packets (events in every packet
// cost ~10 us per launch: at config 2's 0.4 ms calls, 4 pieces per call would
// move the step time itself, so bench.py samples 1 in 16 there and every call of
// config 4's 40 ms calls); _end adds their elapsed time to the totals. Events
// come from a pool.
static std::atomic<int32_t> g_pre_timing{0};  // sample one call in g_pre_timing (0 = off)
static std::atomic<int64_t> g_pre_calls{0};
static std::mutex g_pre_mu;
static double g_pre_ms = 0.0;
static int64_t g_pre_launches = 0;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_pre_pool;

static void prereduce_free(dml_prereduce* p) {
    if (p->idx_ev) (void)hipEventDestroy(p->idx_ev);
    if (p->last_ev) (void)hipEventDestroy(p->last_ev);
    if (p->rerun_ev) (void)hipEventDestroy(p->rerun_ev);
    delete p;
}

// Read a context call's verdict once its pieces are done; if speculation failed,
// re-run the call exactly on the context's stream: a fresh slot table, the full
// key index (repeated rows detected), every recorded piece without speculation.
static int prereduce_verify(dml_prereduce* p, int32_t* rerun) {
    if (rerun) *rerun = 0;
    if (!p->ctx || p->verified) return DML_OK;
    dml_prectx* x = p->ctx;
    PreWs& W = x->ws[p->wi];
    HIPCHK(hipStreamWaitEvent(x->xstream, p->done_ev ? p->done_ev : p->idx_ev, 0));
    HIPCHK(hipMemcpyAsync(W.hctrl, W.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, x->xstream));
    HIPCHK(hipEventRecord(W.ctrl_ev, x->xstream));
    HIPCHK(hipEventSynchronize(W.ctrl_ev));
    const Ctrl h = *W.hctrl;
    x->st.chunks += 1;
    if (p->spec && h.spec_ok != 0u) {
        x->st.spec_chunks += 1;
        uint64_t perm = 0;
        for (int b = 0; b < p->nb; ++b) {
            if (ctrl_identity(&h, h.ident, b)) {
                x->st.identity_pushes += 1;
                continue;
            }
            if ((h.ident >> b) & 1ull) x->st.reused_pushes += 1;
            else x->st.indexed_pushes += 1;
            perm |= 1ull << ctrl_col(&h, b);
        }
        // every row verified: the table's columns are the pushes' permutations
        if (p->rows_done == p->rows) {
            W.kept = true;
            W.kept_nb = p->nb;
            W.perm = perm;
        }
    } else if (p->spec) {
        x->st.spec_chunks += 1;
        x->st.spec_reruns += 1;
        x->st.indexed_pushes += p->nb;
        Batch bt = p->bt;
        bt.spec = 0;
        bt.keeps = 0;
        bt.kept_cols = 0;
        bt.ident_ok = 0;
        bt.prev = nullptr;
        hipStream_t xs = x->xstream;
        HIPCHK(hipMemsetAsync(W.base, 0xFF, sizeof(Ctrl) + x->slot_bytes, xs));
        HIPCHK(hipMemsetAsync(W.rowflag, 0, (size_t)x->rows * sizeof(uint32_t), xs));
        HIPCHK(launch_index(bt, p->nb, p->max_nrec, p->stride, p->K, p->first, p->rows, W.slot, W.rowflag, W.ctrl,
                            kNoPos, xs));
        AdaArgs none{};
        for (const auto& pr : p->prec) {
            RowMap rm;
            rm.block = pr.block;
            rm.stride = pr.stride;
            rm.off = pr.off;
            rm.rows_total = p->rows;
            rm.out = pr.out;
            HIPCHK(launch_reduce(p->desc.value_type, kPreReduce, pr.out, pr.ntask, p->cols, bt, p->nb, p->stride,
                                 p->K, W.slot, nullptr, W.ctrl, kNoPos, none, xs, nullptr, LaunchEv{}, rm));
        }
        if (!p->rerun_ev) HIPCHK(hipEventCreateWithFlags(&p->rerun_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(p->rerun_ev, xs));
        p->done_ev = p->rerun_ev;  // consumers of the partial (dml_prereduce_stream_wait) wait for the re-run
        HIPCHK(hipMemcpyAsync(W.hctrl, W.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, xs));
        HIPCHK(hipEventRecord(W.ctrl_ev, xs));
        p->bt = bt;
        p->spec = false;
        if (rerun) *rerun = 1;
    } else {
        for (int b = 0; b < p->nb; ++b) {
            if (p->bt.ident_ok && ((h.ident >> b) & 1ull)) x->st.identity_pushes += 1;
            else x->st.indexed_pushes += 1;
        }
    }
    p->verified = true;
    return DML_OK;
}

extern "C" {

int dml_prereduce_begin(const dml_desc* desc, int64_t first_key, int64_t rows, int32_t cols, const void* const* dev_bufs,
                        const int64_t* lens, int32_t n, void* stream, dml_prereduce** out) {
    if (!desc || !out || rows <= 0 || cols <= 0 || n < 0 || n > kMaxW || (n > 0 && (!dev_bufs || !lens)))
        return set_err(DML_E_INVALID_ARG, "bad pre-reduce arguments (n must be <= 64)");
    // AdaGrad matrices: only the two-moment pieces (dml_prereduce_moments_piece)
    if (desc->data_type != 1 || !desc->dense_column || (desc->ada_grad && desc->value_type != DML_ELEMENT_TYPE_FLOAT))
        return set_err(DML_E_UNSUPPORTED, "pre-reduce supports dense-column matrices");
    if (desc->value_type != 0 && desc->value_type != 1 && desc->value_type != 3)
        return set_err(DML_E_BAD_DESC, "bad value type");
    auto* p = new (std::nothrow) dml_prereduce();
    if (!p) return set_err(DML_E_NOMEM, "out of host memory");
    p->desc = *desc;
    p->first = first_key;
    p->rows = rows;
    p->cols = cols;
    p->K = desc->key_type == 0 ? 4 : 8;
    p->V = desc->value_type == 3 ? 8 : 4;
    p->stride = p->K + (int64_t)p->V * cols;
    p->stream = (hipStream_t)stream;
    HIPCHK(hipGetDevice(&p->device));
    int64_t max_nrec = 0;
    for (int j = 0; j < n; ++j) {
        if (lens[j] % p->stride) {
            delete p;
            return set_err(DML_E_TRUNCATED, "ragged full-range push");
        }
        p->bt.base[j] = (const uint8_t*)dev_bufs[j];
        p->bt.len[j] = lens[j];
        p->bt.nrec[j] = lens[j] / p->stride;
        p->bt.bidx[j] = j;
        max_nrec = std::max(max_nrec, p->bt.nrec[j]);
    }
    p->nb = n;
    const size_t sb = (size_t)rows * kMaxW * sizeof(int32_t);
    WsLease lease;
    if (int rc = ws_acquire(p->device, sizeof(Ctrl) + sb + (size_t)rows * sizeof(uint32_t), &lease)) {
        delete p;
        return rc;
    }
    p->ws = lease.ptr;
    p->ws_bytes = lease.bytes;
    p->hctrl = lease.hctrl;
    const bool clean = lease.clean;
    p->ctrl = (Ctrl*)p->ws;
    p->slot = (int32_t*)(p->ws + sizeof(Ctrl));
    p->rowflag = (uint32_t*)(p->ws + sizeof(Ctrl) + sb);
    // a clean lease needs only its Ctrl reset (see launch_chunk)
    hipError_t e = hipMemsetAsync(p->ws, 0xFF, sizeof(Ctrl) + (clean ? 0 : sb), p->stream);
    if (e == hipSuccess && !clean) e = hipMemsetAsync(p->rowflag, 0, (size_t)rows * sizeof(uint32_t), p->stream);
    // Full-range pushes whose records are rows in order (Java HashMap<Integer> order)
    // skip the key index: every key is checked (k_ident_full) before the pieces,
    // which take slot = row for them. Complete rather than speculative: the
    // reduce-scatter reads the partial as soon as a piece is done. Only for slot
    // tables beyond the caches, where the index's slot atomics go to DRAM (config
    // 4 at N > 1: 160 M records, a 640 MB table; world-1 group path 40.8 -> 36.7
    // ms/call): for config 2's 2 MB table the complete check reads as many key
    // lines as the index and lengthens the index stream's chain, which must end
    // before the running pre-reduce does (0.450 -> 0.490 ms/call, measured).
    bool full = n > 0 && (int64_t)rows * slot_stride(n) * 4 > ((int64_t)64 << 20);
    for (int j = 0; j < n && full; ++j) full = p->bt.nrec[j] == rows;
    p->bt.first = first_key;
    if (e == hipSuccess && full) {
        e = launch_ident_full(p->bt, n, max_nrec, p->stride, p->K, first_key, rows, p->ctrl, p->stream);
        p->bt.ident_ok = 1;
    }
    if (e == hipSuccess)
        e = launch_index(p->bt, n, max_nrec, p->stride, p->K, first_key, rows, p->slot, p->rowflag, p->ctrl, kNoPos,
                         p->stream);
    // the index alone writes the Ctrl: copy it out now, so _end reads it without
    // queueing anything behind the caller's later work
    if (e == hipSuccess) e = hipMemcpyAsync(p->hctrl, p->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->idx_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(p->idx_ev, p->stream);
    if (e != hipSuccess) {
        // the stream may still reference the workspace: drain it before reuse
        (void)hipStreamSynchronize(p->stream);
        ws_release(p->device, WsLease{p->ws, p->ws_bytes, false, p->hctrl});
        prereduce_free(p);
        return set_err(DML_E_HIP, hipGetErrorString(e));
    }
    const int32_t every = g_pre_timing.load(std::memory_order_relaxed);
    p->timed = every > 0 && g_pre_calls.fetch_add(1, std::memory_order_relaxed) % every == 0;
    *out = p;
    return DML_OK;
}

int dml_prereduce_moments_piece(dml_prereduce* p, int64_t row_block, int64_t row_stride, int64_t row_off,
                                int64_t ntask_rows, void* dev_out, void* stream) {
    if (!p || !dev_out || row_block <= 0 || ntask_rows < 0) return set_err(DML_E_INVALID_ARG, "bad piece arguments");
    if (p->ctx || p->desc.value_type != DML_ELEMENT_TYPE_FLOAT || p->cols % 4 || p->cols * 4 >= 4096)
        return set_err(DML_E_UNSUPPORTED, "two-moment pieces: f32 rows of whole 16-B vectors under 4 KiB");
    hipStream_t st = (hipStream_t)stream;
    if (st != p->stream && !p->idx_waited) {
        HIPCHK(hipEventSynchronize(p->idx_ev));
        p->idx_waited = true;
    }
    RowMap rm;
    rm.block = row_block;
    rm.stride = row_stride;
    rm.off = row_off;
    rm.rows_total = p->rows;
    rm.out = dev_out;
    if (!p->last_ev) HIPCHK(hipEventCreateWithFlags(&p->last_ev, hipEventDisableTiming));
    HIPCHK(launch_moments(ntask_rows, p->cols, p->bt, p->nb, p->stride, p->K, p->slot, p->ctrl, rm, st,
                          LaunchEv{nullptr, p->last_ev}));
    p->done_ev = p->last_ev;
    for (int64_t t0 = 0; t0 < ntask_rows; t0 += row_block) {
        const int64_t lo = (t0 / row_block) * row_stride + row_off;
        const int64_t hi = std::min(lo + std::min(row_block, ntask_rows - t0), p->rows);
        if (hi > lo) p->rows_done += hi - lo;
    }
    p->last_st = st;
    return DML_OK;
}

int dml_prereduce_piece(dml_prereduce* p, int64_t row_block, int64_t row_stride, int64_t row_off, int64_t ntask_rows,
                        void* dev_out, void* stream) {
    if (!p || !dev_out || row_block <= 0 || ntask_rows < 0) return set_err(DML_E_INVALID_ARG, "bad piece arguments");
    if (p->desc.ada_grad) return set_err(DML_E_UNSUPPORTED, "AdaGrad pre-reduce: dml_prereduce_moments_piece");
    hipStream_t st = (hipStream_t)stream;  // as given: 0 is HIP's null stream
    if (st != p->stream && !p->idx_waited) {
        // pieces on another stream (the index ran on a side stream, overlapping the
        // caller's previous work): wait for the index on the host, then enqueue the
        // piece straight behind whatever that stream runs (no cross-queue barrier)
        HIPCHK(hipEventSynchronize(p->idx_ev));
        p->idx_waited = true;
    }
    RowMap rm;
    rm.block = row_block;
    rm.stride = row_stride;
    rm.off = row_off;
    rm.rows_total = p->rows;
    rm.out = dev_out;
    AdaArgs none{};
    if (!p->last_ev) HIPCHK(hipEventCreateWithFlags(&p->last_ev, hipEventDisableTiming));
    // the piece's completion event rides in its dispatch packet (no marker packet between pieces)
    LaunchEv ev{nullptr, p->last_ev};
    if (p->timed) {
        std::pair<hipEvent_t, hipEvent_t> t{nullptr, nullptr};
        {
            std::lock_guard<std::mutex> lk(g_pre_mu);
            if (!g_pre_pool.empty()) {
                t = g_pre_pool.back();
                g_pre_pool.pop_back();
            }
        }
        if (!t.first) {
            HIPCHK(hipEventCreate(&t.first));
            HIPCHK(hipEventCreate(&t.second));
        }
        p->tev.push_back(t);
        ev = LaunchEv{t.first, t.second};
    }
    // all-identity calls (seen in the index's Ctrl, once the host has waited for it):
    // the lean kernel, when no wave's rows straddle two row blocks of the map
    const int Rw = flat_ident_rows_per_wave(p->desc.value_type, p->cols);
    if (p->hidx && p->idx_waited && (row_block % Rw == 0 || ntask_rows <= row_block) &&
        flat_ident_ok(*p->hidx, p->bt, p->nb, p->rows, kNoPos)) {
        if (p->ctx) {
            std::lock_guard<std::mutex> lk(p->ctx->mu);
            p->ctx->st.ident_launches += 1;
        }
        HIPCHK(launch_flat_ident(p->desc.value_type, kPreReduce, dev_out, ntask_rows, p->cols, p->bt, p->nb, p->stride,
                                 p->K, p->ctrl, st, nullptr, ev, rm));
    } else
        HIPCHK(launch_reduce(p->desc.value_type, kPreReduce, dev_out, ntask_rows, p->cols, p->bt, p->nb, p->stride,
                             p->K, p->slot, nullptr, p->ctrl, kNoPos, none, st, nullptr, ev, rm));
    p->done_ev = ev.stop;
    p->prec.push_back({row_block, row_stride, row_off, ntask_rows, dev_out});
    // model rows this piece covered: blocks of row_block task rows at row_off + q*row_stride
    for (int64_t t0 = 0; t0 < ntask_rows; t0 += row_block) {
        const int64_t lo = (t0 / row_block) * row_stride + row_off;
        const int64_t hi = std::min(lo + std::min(row_block, ntask_rows - t0), p->rows);
        if (hi > lo) p->rows_done += hi - lo;
    }
    p->last_st = st;
    return DML_OK;
}

int dml_prereduce_timing(int32_t every) {
    g_pre_timing.store(every > 0 ? every : 0);
    g_pre_calls.store(0);
    return DML_OK;
}

int dml_prereduce_kernel_time(double* ms, int64_t* launches, int32_t reset) {
    if (!ms || !launches) return set_err(DML_E_INVALID_ARG, "null output");
    std::lock_guard<std::mutex> lk(g_pre_mu);
    *ms = g_pre_ms;
    *launches = g_pre_launches;
    if (reset) {
        g_pre_ms = 0.0;
        g_pre_launches = 0;
    }
    return DML_OK;
}

int dml_prereduce_stream_wait(dml_prereduce* p, void* stream) {
    if (!p || !p->done_ev) return set_err(DML_E_INVALID_ARG, "no piece enqueued yet");
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, p->done_ev, 0));
    return DML_OK;
}

int dml_prereduce_verify(dml_prereduce* p, int32_t* rerun) {
    if (!p) return set_err(DML_E_INVALID_ARG, "null pre-reduce");
    if (!p->ctx) {  // a call without a context does not speculate
        if (rerun) *rerun = 0;
        return DML_OK;
    }
    std::lock_guard<std::mutex> lk(p->ctx->mu);
    return prereduce_verify(p, rerun);
}

int dml_prereduce_end(dml_prereduce* p) {
    if (!p) return set_err(DML_E_INVALID_ARG, "null pre-reduce");
    if (p->ctx) {
        dml_prectx* x = p->ctx;
        std::lock_guard<std::mutex> lk(x->mu);
        PreWs& W = x->ws[p->wi];
        int rc = prereduce_verify(p, nullptr);
        hipError_t e = rc == DML_OK ? hipEventSynchronize(W.ctrl_ev) : hipErrorUnknown;  // pieces / re-run done
        const Ctrl h = *W.hctrl;
        if (!p->tev.empty()) {
            double ms = 0.0;
            for (auto& t : p->tev) {
                float v = 0.f;
                if (e == hipSuccess && hipEventElapsedTime(&v, t.first, t.second) == hipSuccess) ms += v;
            }
            std::lock_guard<std::mutex> lk2(g_pre_mu);
            if (e == hipSuccess) {
                g_pre_ms += ms;
                g_pre_launches += (int64_t)p->tev.size();
            }
            g_pre_pool.insert(g_pre_pool.end(), p->tev.begin(), p->tev.end());
            p->tev.clear();
        }
        if (rc == DML_OK && e != hipSuccess) rc = set_err(DML_E_HIP, hipGetErrorString(e));
        else if (rc == DML_OK && h.cutoff != kNoPos) rc = set_err(DML_E_KEY_OUT_OF_SHARD, "pre-reduce: key outside the matrix");
        else if (rc == DML_OK && h.no_dup == 0u) rc = set_err(DML_E_UNSUPPORTED, "pre-reduce: a push repeats a row");
        // a kept table stays (not clean); a non-speculative call whose pieces covered every
        // row through the clearing kernel left it clean; anything else is memset next time
        W.clean = !W.kept && !p->spec && rc == DML_OK && p->rows_done == p->rows &&
                  reduce_clears_slots(p->desc.value_type, kPreReduce, p->cols);
        if (rc != DML_OK) W.kept = false;
        (void)hipEventRecord(W.free_ev, x->xstream);
        W.busy = false;
        prereduce_free(p);
        return rc;
    }
    hipError_t e = hipEventSynchronize(p->idx_ev);  // index done, Ctrl copied out
    const Ctrl h = *p->hctrl;
    // the workspace is free once the last piece ran
    if (e == hipSuccess && p->done_ev) e = hipEventSynchronize(p->done_ev);
    if (!p->tev.empty()) {
        double ms = 0.0;
        for (auto& t : p->tev) {
            float x = 0.f;
            if (e == hipSuccess && hipEventElapsedTime(&x, t.first, t.second) == hipSuccess) ms += x;
        }
        std::lock_guard<std::mutex> lk(g_pre_mu);
        if (e == hipSuccess) {
            g_pre_ms += ms;
            g_pre_launches += (int64_t)p->tev.size();
        }
        g_pre_pool.insert(g_pre_pool.end(), p->tev.begin(), p->tev.end());
        p->tev.clear();
    }
    int rc = DML_OK;
    if (e != hipSuccess) rc = set_err(DML_E_HIP, hipGetErrorString(e));
    else if (h.cutoff != kNoPos) rc = set_err(DML_E_KEY_OUT_OF_SHARD, "pre-reduce: key outside the matrix");
    else if (h.no_dup == 0u) rc = set_err(DML_E_UNSUPPORTED, "pre-reduce: a push repeats a row");
    // after a failed sync the device state is unknown: drop the lease. A normal chunk
    // whose pieces reduced every row through the clearing kernel left the table clean.
    const bool clean = rc == DML_OK && p->rows_done == p->rows &&
                       reduce_clears_slots(p->desc.value_type, kPreReduce, p->cols);
    if (e == hipSuccess) ws_release(p->device, WsLease{p->ws, p->ws_bytes, clean, p->hctrl});
    prereduce_free(p);
    return rc;
}

int dml_prectx_create(const dml_desc* desc, int64_t first_key, int64_t rows, int32_t cols, int32_t device,
                      dml_prectx** out) {
    if (!desc || !out || rows <= 0 || cols <= 0) return set_err(DML_E_INVALID_ARG, "bad pre-reduce context arguments");
    *out = nullptr;
    if (desc->data_type != 1 || !desc->dense_column || desc->ada_grad)
        return set_err(DML_E_UNSUPPORTED, "pre-reduce supports dense-column plain matrices");
    if (desc->value_type != 0 && desc->value_type != 1 && desc->value_type != 3)
        return set_err(DML_E_BAD_DESC, "bad value type");
    if (rows > INT32_MAX) return set_err(DML_E_INVALID_ARG, "matrix larger than a Java array");
    DeviceGuard g(device);
    auto* x = new (std::nothrow) dml_prectx();
    if (!x) return set_err(DML_E_NOMEM, "out of host memory");
    x->desc = *desc;
    x->first = first_key;
    x->rows = rows;
    x->cols = cols;
    x->K = desc->key_type == 0 ? 4 : 8;
    x->V = desc->value_type == 3 ? 8 : 4;
    x->stride = x->K + (int64_t)x->V * cols;
    x->device = device;
    x->slot_bytes = (size_t)rows * kMaxW * sizeof(int32_t);
    auto fail = [&](hipError_t e) {
        dml_prectx_destroy(x);
        return set_err(DML_E_HIP, std::string("pre-reduce context: ") + hipGetErrorString(e));
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&x->xstream, hipStreamNonBlocking)) != hipSuccess) return fail(e);
    for (PreWs& W : x->ws) {
        if ((e = hipMalloc((void**)&W.base, sizeof(Ctrl) + x->slot_bytes + (size_t)rows * sizeof(uint32_t))) !=
            hipSuccess)
            return fail(e);
        W.ctrl = (Ctrl*)W.base;
        W.slot = (int32_t*)(W.base + sizeof(Ctrl));
        W.rowflag = (uint32_t*)(W.base + sizeof(Ctrl) + x->slot_bytes);
        if ((e = hipHostMalloc((void**)&W.hctrl, sizeof(Ctrl), hipHostMallocDefault)) != hipSuccess) return fail(e);
        if ((e = hipEventCreateWithFlags(&W.ctrl_ev, hipEventDisableTiming)) != hipSuccess) return fail(e);
        if ((e = hipEventCreateWithFlags(&W.free_ev, hipEventDisableTiming)) != hipSuccess) return fail(e);
    }
    *out = x;
    return DML_OK;
}

void dml_prectx_destroy(dml_prectx* x) {
    if (!x) return;
    {
        std::lock_guard<std::mutex> lk(x->mu);
        DeviceGuard g(x->device);
        if (x->xstream) (void)hipStreamSynchronize(x->xstream);
        for (PreWs& W : x->ws) {
            if (W.free_ev) (void)hipEventSynchronize(W.free_ev);
            (void)hipFree(W.base);
            if (W.hidx) (void)hipHostFree(W.hidx);
            if (W.hctrl) (void)hipHostFree(W.hctrl);
            if (W.ctrl_ev) (void)hipEventDestroy(W.ctrl_ev);
            if (W.free_ev) (void)hipEventDestroy(W.free_ev);
        }
        if (x->xstream) (void)hipStreamDestroy(x->xstream);
    }
    delete x;
}

int dml_prectx_stats(dml_prectx* x, dml_store_counters* out, int32_t reset) {
    if (!x || !out) return set_err(DML_E_INVALID_ARG, "null argument");
    std::lock_guard<std::mutex> lk(x->mu);
    *out = x->st;
    if (reset) x->st = dml_store_counters{};
    return DML_OK;
}

int dml_prereduce_begin_ctx(dml_prectx* x, const void* const* dev_bufs, const int64_t* lens, int32_t n, void* stream,
                            dml_prereduce** out) {
    if (!x || !out || n < 0 || n > kMaxW || (n > 0 && (!dev_bufs || !lens)))
        return set_err(DML_E_INVALID_ARG, "bad pre-reduce arguments (n must be <= 64)");
    std::lock_guard<std::mutex> lk(x->mu);
    DeviceGuard g(x->device);
    // the ring's next workspace must have been ended: a call still holding it would
    // have its Ctrl and slot table rewritten under its pieces
    if (x->ws[x->next].busy)
        return set_err(DML_E_INVALID_ARG, "three calls of this pre-reduce context are outstanding: end one first");
    auto* p = new (std::nothrow) dml_prereduce();
    if (!p) return set_err(DML_E_NOMEM, "out of host memory");
    p->desc = x->desc;
    p->first = x->first;
    p->rows = x->rows;
    p->cols = x->cols;
    p->K = x->K;
    p->V = x->V;
    p->stride = x->stride;
    p->stream = (hipStream_t)stream;
    p->device = x->device;
    for (int j = 0; j < n; ++j) {
        if (lens[j] % p->stride) {
            delete p;
            return set_err(DML_E_TRUNCATED, "ragged full-range push");
        }
        p->bt.base[j] = (const uint8_t*)dev_bufs[j];
        p->bt.len[j] = lens[j];
        p->bt.nrec[j] = lens[j] / p->stride;
        p->bt.bidx[j] = j;
        p->max_nrec = std::max(p->max_nrec, p->bt.nrec[j]);
    }
    p->nb = n;
    p->bt.first = x->first;
    const int wi = x->next;
    x->next = (x->next + 1) % kRing;
    PreWs& W = x->ws[wi];
    p->ctx = x;
    p->wi = wi;
    p->ws = W.base;
    p->ctrl = W.ctrl;
    p->slot = W.slot;
    p->rowflag = W.rowflag;
    p->hctrl = W.hctrl;
    const int vt = x->desc.value_type;
    bool full = n > 0;
    for (int j = 0; j < n && full; ++j) full = p->bt.nrec[j] == x->rows;
    // full-range pushes of the speculation shapes: identity / kept-column pushes skip
    // the key index and the pieces verify every record (a failure re-runs the call)
    p->spec = full && spec_shape(vt, x->cols);
    p->bt.spec = p->bt.keeps = p->spec ? 1 : 0;
    p->bt.kept_cols = (p->spec && W.kept && slot_stride(W.kept_nb) == slot_stride(n)) ? W.perm : 0;
    hipStream_t st = p->stream;
    hipError_t e = hipSuccess;
    if (W.used) e = hipStreamWaitEvent(st, W.free_ev, 0);  // its last call's pieces / re-run
    const bool slots_ok = W.clean || (W.kept && p->spec);
    if (e == hipSuccess) e = hipMemsetAsync(W.base, 0xFF, sizeof(Ctrl) + (slots_ok ? 0 : x->slot_bytes), st);
    if (e == hipSuccess && !(W.clean || W.kept)) e = hipMemsetAsync(W.rowflag, 0, (size_t)x->rows * sizeof(uint32_t), st);
    W.clean = W.kept = false;
    W.used = true;
    W.busy = true;
    if (e == hipSuccess && p->spec) {
        e = launch_ident_check(p->bt, n, p->stride, p->K, x->first, x->rows, W.slot, W.ctrl, st);
        if (e == hipSuccess && p->bt.kept_cols) e = launch_assign_cols(W.ctrl, n, st);
    } else if (e == hipSuccess && full && (int64_t)x->rows * slot_stride(n) * 4 > ((int64_t)64 << 20)) {
        // other shapes: the complete identity check of dml_prereduce_begin
        e = launch_ident_full(p->bt, n, p->max_nrec, p->stride, p->K, x->first, x->rows, W.ctrl, st);
        p->bt.ident_ok = 1;
    }
    if (e == hipSuccess)
        e = launch_index(p->bt, n, p->max_nrec, p->stride, p->K, x->first, x->rows, W.slot, W.rowflag, W.ctrl, kNoPos,
                         st);
    // speculative calls of the flat shape: a pinned copy of the Ctrl the index left, so
    // that the pieces (after the host's wait for the index) can run k_flat_ident
    p->hidx = nullptr;
    if (e == hipSuccess && p->spec && use_flat(vt, kPreReduce, x->cols, p->bt, n, x->rows)) {
        if (!W.hidx) e = hipHostMalloc((void**)&W.hidx, sizeof(Ctrl), hipHostMallocDefault);
        if (e == hipSuccess) {
            W.hidx->cutoff = 0;  // not all-identity unless the copy lands
            e = hipMemcpyAsync(W.hidx, W.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, st);
            p->hidx = W.hidx;
        }
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->idx_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(p->idx_ev, st);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);
        (void)hipEventRecord(W.free_ev, st);
        W.busy = false;
        prereduce_free(p);
        return set_err(DML_E_HIP, hipGetErrorString(e));
    }
    const int32_t every = g_pre_timing.load(std::memory_order_relaxed);
    p->timed = every > 0 && g_pre_calls.fetch_add(1, std::memory_order_relaxed) % every == 0;
    *out = p;
    return DML_OK;
}

// ---- synthetic data --------------------------------------------------------
int dml_synth_dense_bucket(void* dev_out, const dml_desc* desc, int64_t first_key, int64_t shard_rows, int64_t nrec,
                           int32_t cols, uint64_t seed, uint64_t perm_a, uint64_t perm_c, void* stream) {
    if (!dev_out || !desc || shard_rows <= 0 || nrec < 0 || cols <= 0) return set_err(DML_E_INVALID_ARG, "bad synth args");
    if (perm_a >= (1ull << 32) || (uint64_t)nrec >= (1ull << 32)) return set_err(DML_E_INVALID_ARG, "perm_a/nrec must be < 2^32");
    const int K = desc->key_type == 0 ? 4 : 8;
    HIPCHK(launch_synth_dense((uint8_t*)dev_out, K, desc->value_type, first_key, shard_rows, nrec, cols,
                              splitmix64(seed), perm_a % (uint64_t)shard_rows, perm_c % (uint64_t)shard_rows,
                              (hipStream_t)stream));
    return DML_OK;
}

int dml_synth_sparse_bucket(void* dev_out, const dml_desc* desc, int64_t first_key, int64_t key_space, int64_t nrec,
                            uint64_t seed, uint64_t perm_a, uint64_t perm_c, void* stream) {
    if (!dev_out || !desc || key_space <= 0 || nrec < 0) return set_err(DML_E_INVALID_ARG, "bad synth args");
    if (perm_a >= (1ull << 32) || (uint64_t)nrec >= (1ull << 32)) return set_err(DML_E_INVALID_ARG, "perm_a/nrec must be < 2^32");
    const int K = desc->key_type == 0 ? 4 : 8;
    const int V = desc->value_type == DML_ELEMENT_TYPE_DOUBLE ? 8 : 4;
    HIPCHK(launch_synth_sparse((uint8_t*)dev_out, K, desc->value_type, V, first_key, key_space, nrec, splitmix64(seed),
                               perm_a % (uint64_t)key_space, perm_c % (uint64_t)key_space, (hipStream_t)stream));
    return DML_OK;
}

int dml_diag_stream(int32_t copy, void* dev_dst, const void* dev_src, int64_t bytes, void* stream, float* ms) {
    if (!dev_dst || !dev_src || bytes < 0 || bytes % 16 || ((uintptr_t)dev_dst | (uintptr_t)dev_src) % 16)
        return set_err(DML_E_INVALID_ARG, "stream copy needs 16-B aligned buffers and a multiple of 16 bytes");
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHK(hipEventCreate(&e0));
    hipError_t e = hipEventCreate(&e1);
    if (e == hipSuccess) e = launch_stream(copy != 0, dev_dst, dev_src, bytes / 16, st, LaunchEv{e0, e1});
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e != hipSuccess) return set_err(DML_E_HIP, hipGetErrorString(e));
    if (ms) *ms = t;
    return DML_OK;
}

int dml_diag_ring_rs(int32_t value_type, const void* dev_partial, void* dev_recv, void* dev_landing,
                     int64_t chunk_bytes, int32_t world, int32_t rank, int32_t channels, void* stream) {
    if (!dev_partial || !dev_recv || !dev_landing || chunk_bytes < 0 || chunk_bytes % 16 || world < 1 || rank < 0 ||
        rank >= world || channels < 1)
        return set_err(DML_E_INVALID_ARG, "bad ring reduce-scatter arguments");
    HIPCHK(launch_ring_rs(value_type, dev_partial, dev_recv, dev_landing, chunk_bytes, world, rank, channels,
                          (hipStream_t)stream));
    return DML_OK;
}

int dml_diag_rmw_floor(float* dev_array, const uint32_t* dev_index, const float* dev_values, int64_t n, void* stream,
                       float* ms) {
    if (!dev_array || n < 0 || (n > 0 && (!dev_index || !dev_values)))
        return set_err(DML_E_INVALID_ARG, "bad rmw floor arguments");
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHK(hipEventCreate(&e0));
    hipError_t e = hipEventCreate(&e1);
    if (e == hipSuccess) e = launch_rmw_floor(dev_array, dev_index, dev_values, n, st, LaunchEv{e0, e1});
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e != hipSuccess) return set_err(DML_E_HIP, hipGetErrorString(e));
    if (ms) *ms = t;
    return DML_OK;
}

int dml_diag_dense_floor(dml_store* s, const void* const* dev_bufs, const int64_t* lens, int32_t n, void* stream,
                         float* ms, int32_t* out_of_place) {
    if (int rc = check_store(s)) return rc;
    if (!s->is_matrix || s->V != 4 || vtype_of(s->desc) != kF32 || s->cols % 4 || n < 1 || n > kMaxW || !dev_bufs ||
        !lens)
        return set_err(DML_E_INVALID_ARG, "dense floor: an f32 matrix store of whole 16-B vectors, 1..64 pushes");
    for (int b = 0; b < n; ++b)
        if (!dev_bufs[b] || lens[b] != s->rows * s->stride)
            return set_err(DML_E_INVALID_ARG, "dense floor: every push lists every row once (full range)");
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    Batch bt{};
    for (int b = 0; b < n; ++b) bt.base[b] = (const uint8_t*)dev_bufs[b];
    // out of place into the speculative second buffer where the store has one (k_flat_ident's
    // layout); AdaGrad stores apply in place (k_ada_ident)
    float* out = (float*)(s->data_alt && !s->adagrad ? s->data_alt : s->data);
    if (out_of_place) *out_of_place = out != s->data ? 1 : 0;
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHK(hipEventCreate(&e0));
    hipError_t e = hipEventCreate(&e1);
    if (e == hipSuccess)
        e = launch_dense_floor((const float*)s->data, out, s->adagrad ? s->delta : nullptr, bt, n, s->stride, s->K,
                               s->cols, s->rows * s->cols, st, LaunchEv{e0, e1});
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e != hipSuccess) return set_err(DML_E_HIP, hipGetErrorString(e));
    if (ms) *ms = t;
    return DML_OK;
}

int dml_diag_gather_floor(int32_t* dev_shard, int32_t cols, const int32_t* dev_rows, const int32_t* dev_ptr,
                          const uint64_t* dev_addr, int64_t ntouched, void* stream, float* ms) {
    if (!dev_shard || cols <= 0 || cols % 4 || cols > 1024 || ntouched < 0 ||
        (ntouched > 0 && (!dev_rows || !dev_ptr || !dev_addr)) || (uintptr_t)dev_shard % 16)
        return set_err(DML_E_INVALID_ARG, "bad gather floor arguments (cols a multiple of 4, at most 1024)");
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHK(hipEventCreate(&e0));
    hipError_t e = hipEventCreate(&e1);
    if (e == hipSuccess) e = launch_gather_floor(dev_shard, cols, dev_rows, dev_ptr, dev_addr, ntouched, st, LaunchEv{e0, e1});
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e != hipSuccess) return set_err(DML_E_HIP, hipGetErrorString(e));
    if (ms) *ms = t;
    return DML_OK;
}

int dml_store_rand(dml_store* s, uint64_t seed) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    const int vt = vtype_of(s->desc);
    if (!s->is_matrix || vt == kI32) return DML_OK;  // DataStore.rand(): no-op (DataStore.java:22)
    if (vt == kF64) {
        // DoubleMatrixStore.rand() seeds Random(1L) on every shard: reproduced exactly,
        // on the host (init, not the push path), a block of rows at a time
        const int64_t cols = s->cols, rb = std::max<int64_t>(1, (int64_t(1) << 21) / cols);
        JavaRandom jr(1);
        std::vector<double> blk((size_t)(std::min(rb, s->rows) * cols));
        for (int64_t r0 = 0; r0 < s->rows; r0 += rb) {
            const int64_t nr = std::min(rb, s->rows - r0);
            for (int64_t i = 0; i < nr; ++i) java_unit_abs_gaussian_row(jr, blk.data() + i * cols, cols);
            HIPCHK(hipMemcpyAsync((double*)s->data + r0 * cols, blk.data(), (size_t)(nr * cols) * 8,
                                  hipMemcpyHostToDevice, s->stream));
            HIPCHK(hipStreamSynchronize(s->stream));
        }
        return DML_OK;
    }
    HIPCHK(launch_rand(vt, s->data, s->rows, s->cols, splitmix64(seed ^ 0x5241'4e44ull), s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

int dml_synth_fill_store(dml_store* s, uint64_t seed) {
    if (int rc = check_store(s)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    DeviceGuard g(s->device);
    if (int rc = begin_call(s)) return rc;
    HIPCHK(launch_synth_fill(vtype_of(s->desc), s->data, s->rows * s->cols, splitmix64(seed), s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return DML_OK;
}

}  // extern "C"
