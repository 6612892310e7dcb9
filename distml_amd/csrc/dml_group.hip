// dml_group.hip — native multi-GPU shard group over RCCL (C-ABI dml_group_*).
//
// The JNI deployment has no torch.distributed: one PS process per GPU owns
// shard `rank` of KeyRange.linearSplit(world) (KeyRange.java:68-80,
// DMatrix.partition DMatrix.java:53-64) and reduces device-resident full-range
// pushes with the same three steps as distml_amd/group.py:
//   1. ordered pre-reduce of the rank's pushes into a partial of the whole
//      matrix (dml_prereduce_*, k_reduce_rows in pre-reduce mode), in P row
//      slices laid out [rank][row];
//   2. ncclReduceScatter(sum) of the slices on a communication stream, once the
//      call's speculation is verified: full-range pushes whose records are rows in
//      order, or the permutations a call three before listed, skip the key index
//      and the pieces verify every record (dml_prectx); the next call reads the
//      verdict (a failure re-runs the pieces exactly) and then launches this
//      call's reduce-scatter, so it runs on xGMI under the next call's pre-reduce;
//   3. owner apply shard += received on the store's stream.
// Calls are asynchronous and overlap exactly as in group.py: the next call's key
// index runs on a high-priority side stream, two partial / receive buffer sets
// alternate, and a call's key / repeated-row errors surface at the next call or
// at dml_group_flush. The communicator comes from ncclCommInitRankConfig (the
// channel count pinned, kRsChannels) with a unique id the caller distributes (the
// JVM's control plane).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "distml_ps.h"
#include "dml_internal.h"

using namespace dml;

#define GHIP(x)                                                                                        \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) return set_error(DML_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define GNCCL(x)                                                                                       \
    do {                                                                                               \
        ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) return set_error(DML_E_HIP, std::string(#x) + ": " + ncclGetErrorString(r_)); \
    } while (0)
#define GRC(x)                     \
    do {                           \
        int rc_ = (x);             \
        if (rc_ != DML_OK) return rc_; \
    } while (0)

struct dml_group {
    int rank = 0, world = 1, device = 0, pieces = 4;
    dml_desc desc{};
    int64_t total_rows = 0, step_rows = 0, shard_first = 0, shard_rows = 0;
    int32_t cols = 0;
    size_t vbytes = 4;
    ncclComm_t comm = nullptr;
    ncclDataType_t dtype = ncclFloat32;
    hipStream_t cstream = nullptr;  // pre-reduce pieces
    hipStream_t istream = nullptr;  // key index of the next call (high priority: its own queue)
    hipStream_t rstream = nullptr;  // reduce-scatter
    dml_store* store = nullptr;
    hipStream_t sstream = nullptr;  // the store's stream (owner apply)
    void* partial[2] = {nullptr, nullptr};
    void* recv[2] = {nullptr, nullptr};
    hipEvent_t rs_done[2] = {nullptr, nullptr};
    hipEvent_t applied[2] = {nullptr, nullptr};
    dml_prectx* pctx = nullptr;  // speculative pre-reduce (workspace ring with kept slot tables)
    // calls whose pieces are enqueued but whose partial is not yet reduce-scattered:
    // the reduce-scatter waits for the call's verdict (dml_prereduce_verify)
    struct Call {
        dml_prereduce* h;  // null when the call failed before its pieces were recorded
        int set;           // partial / recv buffer set
        int rc;            // a local failure of the call's pre-reduce (DML_OK otherwise)
    };
    int fail_verify_at = 0;  // fault injection (dml_group_debug_fail_verify): the n-th next verdict fails
    std::deque<Call> pending;
    int k = 0;
    bool plain = true;  // plain-sum dense matrix: the full-range pre-reduce path applies
    // exchange path (dml_group_push_exchange), two buffer sets alternating by call:
    // split output (read by that call's all-to-all), receive buffer (read by the
    // store when the NEXT call hands it over), count buffers
    void* xsend[2] = {nullptr, nullptr};
    void* xrecv[2] = {nullptr, nullptr};
    int64_t xsend_cap[2] = {0, 0}, xrecv_cap[2] = {0, 0};
    hipEvent_t xsent[2] = {nullptr, nullptr};      // rstream: the set's all-to-all finished
    hipEvent_t xconsumed[2] = {nullptr, nullptr};  // store stream: the store's reduce of the set's slices ran
    // store push-call number of the set's slices (dml_store_push_seq): before the
    // set's receive buffer is overwritten, the store retires that call
    // (dml_store_retire), since a retiring chunk may read its pushes again (exact
    // replay of repeated rows, int32 rollback, re-run of a failed speculation)
    uint64_t xseq[2] = {0, 0};
    int64_t* xcnt = nullptr;  // device [2][world * kMaxW]: counts sent / received
    int xk = 0;
    // received slices of the last call, handed to the store by the next call or the flush
    bool xheld = false;
    int xheld_set = 0;
    std::vector<const void*> xptrs;
    std::vector<int64_t> xlens;
    // two-moment AdaGrad path (dml_group_push_moments), two buffer sets by call:
    // [rank][row][Σu | Σu²] partials and the shard's received moments
    void* mpart[2] = {nullptr, nullptr};
    void* mrecv[2] = {nullptr, nullptr};
    hipEvent_t mrs_done[2] = {nullptr, nullptr};
    hipEvent_t mapplied[2] = {nullptr, nullptr};
    std::deque<dml_prereduce*> mpending;  // calls whose index errors are not yet collected
    int mk = 0;
};

namespace {

constexpr int kRsChannels = 128;  // RCCL CTAs (channels) per collective of the group


// The oldest pending call: read its verdict (a failed speculation re-runs its
// pieces exactly), then reduce-scatter its partial on the communication stream
// and apply the received rows on the store's stream; its errors are returned.
//
// Every rank issues the same collectives in the same order whatever happens
// locally: a rank whose call failed here (its verdict, its re-run, a
// HIP error before the pieces) still enters the reduce-scatter, with a zeroed
// partial, and skips only its own apply; the error is returned to its caller.
// The other ranks' shards then hold every rank's sums except that rank's call.
int finish_front(dml_group* g) {
    dml_group::Call c = g->pending.front();
    g->pending.pop_front();
    int rc = c.rc;
    if (rc == DML_OK) {
        rc = dml_prereduce_verify(c.h, nullptr);
        if (rc == DML_OK && g->fail_verify_at > 0 && --g->fail_verify_at == 0)
            rc = set_error(DML_E_HIP, "injected verify failure (dml_group_debug_fail_verify)");
    }
    if (rc == DML_OK) rc = dml_prereduce_stream_wait(c.h, g->rstream);
    const int64_t S = g->step_rows, P = g->pieces, blk = S / P, W = g->world, C = g->cols;
    uint8_t* part = (uint8_t*)g->partial[c.set];
    // one rank: the [rank][row] slices are the shard's rows in order, the
    // reduce-scatter would be a copy; the owner apply reads the partial itself
    uint8_t* rcv = W == 1 ? part : (uint8_t*)g->recv[c.set];
    const int local = rc;
    if (local != DML_OK && W > 1) {
        // contribute zeros: the pieces (or their re-run) are done with the partial first,
        // and the apply of the call two back (store stream) with this set's recv — a call
        // that failed in _begin_ctx skipped the host wait for it
        (void)hipStreamSynchronize(g->cstream);
        if (c.h) (void)dml_prereduce_stream_wait(c.h, g->rstream);
        (void)hipStreamWaitEvent(g->rstream, g->applied[c.set], 0);
        (void)hipMemsetAsync(part, 0, (size_t)(W * S * C) * g->vbytes, g->rstream);
    }
    int crc = DML_OK;  // the collective's own status
    for (int64_t j = 0; j < P && W > 1; ++j) {
        const ncclResult_t r = ncclReduceScatter(part + (size_t)(j * W * blk * C) * g->vbytes,
                                                 rcv + (size_t)(j * blk * C) * g->vbytes, (size_t)(blk * C), g->dtype,
                                                 ncclSum, g->comm, g->rstream);
        if (r != ncclSuccess && crc == DML_OK)
            crc = set_error(DML_E_HIP, std::string("ncclReduceScatter: ") + ncclGetErrorString(r));
    }
    if (local != DML_OK) {
        // the set stays busy until the zero-contribution reduce-scatter has read the
        // partial and written recv: its next use (two calls on) waits on applied[set],
        // which for this call is the scatter itself (there is no apply)
        if (W > 1) {
            (void)hipEventRecord(g->rs_done[c.set], g->rstream);
            (void)hipEventRecord(g->applied[c.set], g->rstream);
        }
        if (c.h) (void)dml_prereduce_end(c.h);
        return local;
    }
    if (crc != DML_OK) {  // no apply: the set is free once the stream is past the scatter
        (void)hipEventRecord(g->applied[c.set], g->rstream);
        (void)dml_prereduce_end(c.h);
        return crc;
    }
    if (rc == DML_OK && hipEventRecord(g->rs_done[c.set], g->rstream) != hipSuccess) rc = set_error(DML_E_HIP, "event");
    if (rc == DML_OK && hipStreamWaitEvent(g->sstream, g->rs_done[c.set], 0) != hipSuccess)
        rc = set_error(DML_E_HIP, "stream wait");
    if (rc == DML_OK) rc = dml_store_apply_dense_device(g->store, rcv, g->shard_rows * C);
    if (rc == DML_OK && hipEventRecord(g->applied[c.set], g->sstream) != hipSuccess) rc = set_error(DML_E_HIP, "event");
    const int r2 = dml_prereduce_end(c.h);  // the call's key / repeated-row errors
    return rc != DML_OK ? rc : r2;
}

int end_pending(dml_group* g, size_t keep) {
    int rc = DML_OK;
    while (g->pending.size() > keep) {
        const int r = finish_front(g);
        if (rc == DML_OK) rc = r;
    }
    return rc;
}

int end_moments(dml_group* g, size_t keep) {
    int rc = DML_OK;
    while (g->mpending.size() > keep) {
        dml_prereduce* p = g->mpending.front();
        g->mpending.pop_front();
        const int r = dml_prereduce_end(p);
        if (rc == DML_OK) rc = r;
    }
    return rc;
}

void group_free(dml_group* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    (void)end_pending(g, 0);
    (void)end_moments(g, 0);
    if (g->pctx) dml_prectx_destroy(g->pctx);
    for (int i = 0; i < 2; ++i) {
        if (g->mpart[i]) (void)hipFree(g->mpart[i]);
        if (g->mrecv[i]) (void)hipFree(g->mrecv[i]);
        if (g->mrs_done[i]) (void)hipEventDestroy(g->mrs_done[i]);
        if (g->mapplied[i]) (void)hipEventDestroy(g->mapplied[i]);
    }
    if (g->xcnt) (void)hipFree(g->xcnt);
    for (int i = 0; i < 2; ++i) {
        if (g->xsend[i]) (void)hipFree(g->xsend[i]);
        if (g->xrecv[i]) (void)hipFree(g->xrecv[i]);
        if (g->xsent[i]) (void)hipEventDestroy(g->xsent[i]);
        if (g->xconsumed[i]) (void)hipEventDestroy(g->xconsumed[i]);
        if (g->partial[i]) (void)hipFree(g->partial[i]);
        if (g->recv[i]) (void)hipFree(g->recv[i]);
        if (g->rs_done[i]) (void)hipEventDestroy(g->rs_done[i]);
        if (g->applied[i]) (void)hipEventDestroy(g->applied[i]);
    }
    if (g->comm) (void)ncclCommDestroy(g->comm);
    if (g->store) dml_store_destroy(g->store);
    for (hipStream_t s : {g->cstream, g->istream, g->rstream})
        if (s) (void)hipStreamDestroy(s);
    delete g;
}

int group_init(dml_group* g, const uint8_t* unique_id) {
    GHIP(hipSetDevice(g->device));
    int lo = 0, hi = 0;
    GHIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    GHIP(hipStreamCreateWithFlags(&g->cstream, hipStreamNonBlocking));
    GHIP(hipStreamCreateWithPriority(&g->istream, hipStreamNonBlocking, hi));
    // RCCL's stream is high-priority too: a reduce-scatter's blocks are dispatched
    // ahead of the next call's pre-reduce blocks when both wait for CUs
    GHIP(hipStreamCreateWithPriority(&g->rstream, hipStreamNonBlocking, hi));
    // linearSplit(world): every rank's slice of the partial is step_rows long
    std::vector<int64_t> f((size_t)g->world), l((size_t)g->world);
    GRC(dml_linear_split(0, g->total_rows - 1, g->world, f.data(), l.data()));
    g->step_rows = l[0] - f[0] + 1;
    g->shard_first = f[(size_t)g->rank];
    g->shard_rows = l[(size_t)g->rank] - f[(size_t)g->rank] + 1;
    if (g->shard_rows <= 0) return set_error(DML_E_UNSUPPORTED, "empty shard (world > rows)");
    GRC(dml_store_create_range(&g->desc, g->shard_first, l[(size_t)g->rank], g->cols, g->device, 0, &g->store));
    void* ss = nullptr;
    GRC(dml_store_stream(g->store, &ss));
    g->sstream = (hipStream_t)ss;
    for (int i = 0; i < 2; ++i) {
        GHIP(hipEventCreateWithFlags(&g->rs_done[i], hipEventDisableTiming));
        GHIP(hipEventCreateWithFlags(&g->applied[i], hipEventDisableTiming));
        GHIP(hipEventCreateWithFlags(&g->xsent[i], hipEventDisableTiming));
        GHIP(hipEventCreateWithFlags(&g->xconsumed[i], hipEventDisableTiming));
    }
    GHIP(hipMalloc((void**)&g->xcnt, sizeof(int64_t) * 4 * (size_t)g->world * kMaxW));
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof id);
    // The reduce-scatter's channel count is pinned instead of left to RCCL's tuning: one
    // rank's ring footprint emulated on one GPU beside the real pre-reduce (DESIGN.md §6,
    // bench.py --emulate-rs) runs N = 4 / 8 at 2.6x / 5.3x the one-GPU store with 32
    // blocks, 3.0x / 6.1x with 64 and 3.4x / 6.7x with 128
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.minCTAs = kRsChannels;
    cfg.maxCTAs = kRsChannels;
    GNCCL(ncclCommInitRankConfig(&g->comm, g->world, id, g->rank, &cfg));
    return DML_OK;
}

// Full-range buffers on first use (an exchange-only group never allocates them).
int ensure_partials(dml_group* g) {
    if (g->partial[0]) return DML_OK;
    const size_t part = (size_t)g->world * (size_t)g->step_rows * (size_t)g->cols * g->vbytes;
    const size_t rcv = (size_t)g->step_rows * (size_t)g->cols * g->vbytes;
    for (int i = 0; i < 2; ++i) {
        GHIP(hipMalloc(&g->partial[i], part));
        if (g->world > 1) GHIP(hipMalloc(&g->recv[i], rcv));  // one rank applies the partial itself
    }
    GRC(dml_prectx_create(&g->desc, 0, g->total_rows, g->cols, g->device, &g->pctx));
    return DML_OK;
}

// Hand the last exchange call's received slices to the store, in rank-major push
// order. Its all-to-all must be complete (the caller synchronized rstream).
int hand_over(dml_group* g) {
    if (!g->xheld) return DML_OK;
    g->xheld = false;
    if (g->xptrs.empty()) return DML_OK;
    const int rc = dml_store_push_batch_device(g->store, g->xptrs.data(), g->xlens.data(), (int32_t)g->xptrs.size());
    // the store's device reads of the set are queued on its stream by now (index
    // host-waited, reduce enqueued); its host-side retire may read them once more
    GHIP(hipEventRecord(g->xconsumed[g->xheld_set], g->sstream));
    GRC(dml_store_push_seq(g->store, &g->xseq[g->xheld_set]));
    return rc;
}

int grow(void** p, int64_t* cap, int64_t need) {
    if (*cap >= need) return DML_OK;
    if (*p) GHIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    const int64_t n = std::max<int64_t>(need, 1) + (need >> 3);  // 12.5 % headroom for the next call
    GHIP(hipMalloc(p, (size_t)n));
    *cap = n;
    return DML_OK;
}

}  // namespace

extern "C" {

int dml_group_unique_id(uint8_t* out, int32_t cap) {
    if (!out || cap < NCCL_UNIQUE_ID_BYTES) return set_error(DML_E_INVALID_ARG, "need 128 bytes for the unique id");
    ncclUniqueId id;
    GNCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof id);
    return DML_OK;
}

int dml_group_create(const uint8_t* unique_id, int32_t world, int32_t rank, int32_t device, const dml_desc* desc,
                     int64_t total_rows, int32_t cols, int32_t pieces, dml_group** out) {
    if (!unique_id || !desc || !out || world <= 0 || rank < 0 || rank >= world || total_rows <= 0 || cols <= 0 ||
        pieces <= 0)
        return set_error(DML_E_INVALID_ARG, "bad group arguments");
    if (desc->data_type == DML_DATA_TYPE_MATRIX && !desc->dense_column)
        return set_error(DML_E_UNSUPPORTED, "sparse-column matrices are not supported");
    auto* g = new (std::nothrow) dml_group();
    if (!g) return set_error(DML_E_NOMEM, "out of host memory");
    g->world = world;
    g->rank = rank;
    g->device = device;
    g->desc = *desc;
    g->total_rows = total_rows;
    g->cols = cols;
    g->pieces = pieces;
    g->plain = desc->data_type == DML_DATA_TYPE_MATRIX && !desc->ada_grad;
    if (desc->data_type != DML_DATA_TYPE_MATRIX) g->cols = 1;
    switch (desc->value_type) {
        case DML_ELEMENT_TYPE_FLOAT: g->dtype = ncclFloat32; g->vbytes = 4; break;
        case DML_ELEMENT_TYPE_INT: g->dtype = ncclInt32; g->vbytes = 4; break;  // exact: mod 2^32 like the JVM int
        case DML_ELEMENT_TYPE_DOUBLE: g->dtype = ncclFloat64; g->vbytes = 8; break;
        default: delete g; return set_error(DML_E_BAD_DESC, "bad value type");
    }
    if (int rc = group_init(g, unique_id)) {
        group_free(g);
        return rc;
    }
    *out = g;
    return DML_OK;
}

int dml_group_prereduce_stats(dml_group* g, dml_store_counters* out, int32_t reset) {
    if (!g || !out) return set_error(DML_E_INVALID_ARG, "null argument");
    if (!g->pctx) {
        *out = dml_store_counters{};
        return DML_OK;
    }
    return dml_prectx_stats(g->pctx, out, reset);
}

int dml_group_store(dml_group* g, dml_store** store) {
    if (!g || !store) return set_error(DML_E_INVALID_ARG, "null group");
    *store = g->store;
    return DML_OK;
}

int dml_group_push_full_range(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n) {
    if (!g || n < 0 || n > kMaxW || (n > 0 && (!dev_bufs || !lens)))
        return set_error(DML_E_INVALID_ARG, "bad push arguments (n must be <= 64)");
    if (!g->plain)
        return set_error(DML_E_UNSUPPORTED, "the full-range pre-reduce path needs a plain-sum matrix (use dml_group_push_exchange)");
    GHIP(hipSetDevice(g->device));
    if (g->xheld) {  // an exchange call's slices come first: the store applies calls in order
        GHIP(hipStreamSynchronize(g->rstream));
        GRC(hand_over(g));
    }
    GRC(ensure_partials(g));
    const int64_t S = g->step_rows, P = g->pieces;
    if (S % P) return set_error(DML_E_INVALID_ARG, "pieces must divide the linearSplit step");
    const int64_t blk = S / P, W = g->world, C = g->cols;
    const int k = g->k;
    g->k ^= 1;
    dml_prereduce* h = nullptr;
    int rc = dml_prereduce_begin_ctx(g->pctx, dev_bufs, lens, n, g->istream, &h);
    // buffer set k was used two calls ago: its apply (behind its reduce-scatter) is done
    if (rc == DML_OK && hipEventSynchronize(g->applied[k]) != hipSuccess) rc = set_error(DML_E_HIP, "applied wait");
    uint8_t* part = (uint8_t*)g->partial[k];
    for (int64_t j = 0; j < P && rc == DML_OK; ++j)
        rc = dml_prereduce_piece(h, blk, S, j * blk, W * blk, part + (size_t)(j * W * blk * C) * g->vbytes,
                                 g->cstream);
    if (rc != DML_OK && h) {
        (void)dml_prereduce_end(h);
        h = nullptr;
    }
    // a call that failed here still takes its place in the collective sequence
    // (finish_front contributes zeros for it and reports rc)
    g->pending.push_back({h, k, rc});
    // the previous call: verdict, reduce-scatter (under this call's pieces), apply, errors
    const int r1 = end_pending(g, 1);
    if (rc != DML_OK) {
        const int r2 = end_pending(g, 0);  // this call's failure, reported now
        return r1 != DML_OK ? r1 : r2;
    }
    return r1;
}

int dml_group_push_exchange(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n) {
    if (!g || n < 0 || n > kMaxW || (n > 0 && (!dev_bufs || !lens)))
        return set_error(DML_E_INVALID_ARG, "bad push arguments (n must be <= 64)");
    GHIP(hipSetDevice(g->device));
    // full-range calls still waiting for their reduce-scatter come first: the store
    // applies calls in order
    GRC(end_pending(g, 0));
    const int W = g->world;
    const int64_t K = g->desc.key_type == 0 ? 4 : 8;
    const int64_t stride = g->desc.data_type == DML_DATA_TYPE_MATRIX ? K + (int64_t)g->vbytes * g->cols
                                                                      : K + (int64_t)g->vbytes;
    if (W == 1 && n > 0) {
        // one owner and every key inside the matrix: the split would copy each push whole
        // and nothing crosses a link, so the store takes the pushes themselves (they stay
        // valid until dml_group_flush, the group's contract)
        std::vector<int64_t> cnt((size_t)n);
        GRC(dml_shard_split(&g->desc, g->cols, g->total_rows, 1, dev_bufs, lens, n, nullptr, 0, cnt.data(),
                            g->cstream));
        bool whole = true;
        for (int b = 0; b < n; ++b) whole = whole && cnt[(size_t)b] * stride == lens[b];
        if (whole) {
            if (g->xheld) {  // the previous exchange call's slices come first
                GHIP(hipStreamSynchronize(g->rstream));
                GRC(hand_over(g));
            }
            return dml_store_push_batch_device(g->store, dev_bufs, lens, n);
        }
    }
    // Pipelined over calls (two buffer sets): this call's split runs while the
    // previous call's all-to-all moves its slices; the previous slices reach the
    // store once this call's count exchange (queued behind that all-to-all on the
    // same stream) has completed, and the store applies them while this call's
    // all-to-all runs. The only host waits: the split's counts and the count exchange.
    const int i = g->xk;
    g->xk ^= 1;
    int64_t total = 0;
    for (int b = 0; b < n; ++b) total += lens[b];
    GHIP(hipEventSynchronize(g->xsent[i]));  // the set's last all-to-all (two calls ago) read xsend[i]
    std::vector<int64_t> cnt((size_t)n * W, 0);  // [push][dest]
    // a local failure (a push that is not whole records, a HIP error) still takes part
    // in both exchanges, sending nothing, so that no peer waits for this rank; the
    // error is returned after them
    int local = grow(&g->xsend[i], &g->xsend_cap[i], total);
    if (local == DML_OK)
        local = dml_shard_split(&g->desc, g->cols, g->total_rows, W, dev_bufs, lens, n, g->xsend[i],
                                g->xsend_cap[i], cnt.data(), g->cstream);
    if (local != DML_OK) std::fill(cnt.begin(), cnt.end(), 0);
    // counts per destination, then per source: mine[d][b] out, theirs[q][b] in (n per peer)
    std::vector<int64_t> mine((size_t)W * n), theirs((size_t)W * n);
    for (int d = 0; d < W; ++d)
        for (int b = 0; b < n; ++b) mine[(size_t)d * n + b] = cnt[(size_t)b * W + d];
    int64_t* dmine = g->xcnt + (size_t)i * 2 * W * kMaxW;
    int64_t* dtheirs = dmine + (size_t)W * kMaxW;
    GHIP(hipMemcpyAsync(dmine, mine.data(), sizeof(int64_t) * mine.size(), hipMemcpyHostToDevice, g->rstream));
    GNCCL(ncclGroupStart());
    for (int q = 0; q < W; ++q) {
        GNCCL(ncclSend(dmine + (size_t)q * n, (size_t)n, ncclInt64, q, g->comm, g->rstream));
        GNCCL(ncclRecv(dtheirs + (size_t)q * n, (size_t)n, ncclInt64, q, g->comm, g->rstream));
    }
    GNCCL(ncclGroupEnd());
    GHIP(hipMemcpyAsync(theirs.data(), dtheirs, sizeof(int64_t) * theirs.size(), hipMemcpyDeviceToHost, g->rstream));
    GHIP(hipStreamSynchronize(g->rstream));  // also completes the previous call's all-to-all
    GRC(hand_over(g));
    std::vector<int64_t> soff((size_t)W + 1, 0), roff((size_t)W + 1, 0);
    for (int q = 0; q < W; ++q) {
        int64_t sb = 0, rb = 0;
        for (int b = 0; b < n; ++b) {
            sb += mine[(size_t)q * n + b] * stride;
            rb += theirs[(size_t)q * n + b] * stride;
        }
        soff[(size_t)q + 1] = soff[(size_t)q] + sb;
        roff[(size_t)q + 1] = roff[(size_t)q] + rb;
    }
    // xrecv[i] was last read by the store for the call two back: its chunks retire
    // (host side) before the buffer is rewritten or freed, its reduce ran before
    // this call's all-to-all writes it (device side)
    GRC(dml_store_retire(g->store, g->xseq[i]));
    if (g->xrecv_cap[i] < roff[(size_t)W]) GHIP(hipEventSynchronize(g->xconsumed[i]));
    GRC(grow(&g->xrecv[i], &g->xrecv_cap[i], roff[(size_t)W]));
    GHIP(hipStreamWaitEvent(g->rstream, g->xconsumed[i], 0));
    uint8_t* sp = (uint8_t*)g->xsend[i];
    uint8_t* rp = (uint8_t*)g->xrecv[i];
    GNCCL(ncclGroupStart());
    for (int q = 0; q < W; ++q) {
        GNCCL(ncclSend(sp + soff[(size_t)q], (size_t)(soff[(size_t)q + 1] - soff[(size_t)q]), ncclUint8, q, g->comm,
                       g->rstream));
        GNCCL(ncclRecv(rp + roff[(size_t)q], (size_t)(roff[(size_t)q + 1] - roff[(size_t)q]), ncclUint8, q, g->comm,
                       g->rstream));
    }
    GNCCL(ncclGroupEnd());
    GHIP(hipEventRecord(g->xsent[i], g->rstream));
    // the owner's pushes, rank-major: rank 0's pushes in order, then rank 1's, ...
    g->xptrs.clear();
    g->xlens.clear();
    int64_t off = 0;
    for (int q = 0; q < W; ++q)
        for (int b = 0; b < n; ++b) {
            const int64_t ln = theirs[(size_t)q * n + b] * stride;
            if (ln > 0) {
                g->xptrs.push_back(rp + off);
                g->xlens.push_back(ln);
            }
            off += ln;
        }
    g->xheld = true;
    g->xheld_set = i;
    return local;
}

int dml_group_push_moments(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n) {
    if (!g || n < 0 || n > kMaxW || (n > 0 && (!dev_bufs || !lens)))
        return set_error(DML_E_INVALID_ARG, "bad push arguments (n must be <= 64)");
    if (!g->desc.ada_grad || g->desc.value_type != DML_ELEMENT_TYPE_FLOAT)
        return set_error(DML_E_UNSUPPORTED, "the two-moment path is for AdaGrad (float) matrices");
    GHIP(hipSetDevice(g->device));
    if (g->xheld) {  // earlier calls' slices first: the store applies calls in order
        GHIP(hipStreamSynchronize(g->rstream));
        GRC(hand_over(g));
    }
    GRC(end_pending(g, 0));
    const int64_t S = g->step_rows, W = g->world, C = g->cols;
    if (!g->mpart[0]) {
        for (int i = 0; i < 2; ++i) {
            GHIP(hipMalloc(&g->mpart[i], (size_t)(W * S * 2 * C) * sizeof(float)));
            GHIP(hipMalloc(&g->mrecv[i], (size_t)(S * 2 * C) * sizeof(float)));
            GHIP(hipEventCreateWithFlags(&g->mrs_done[i], hipEventDisableTiming));
            GHIP(hipEventCreateWithFlags(&g->mapplied[i], hipEventDisableTiming));
        }
    }
    const int k = g->mk;
    g->mk ^= 1;
    dml_prereduce* h = nullptr;
    int rc = dml_prereduce_begin(&g->desc, 0, g->total_rows, g->cols, dev_bufs, lens, n, g->istream, &h);
    // buffer set k was used two calls ago: its apply (behind its reduce-scatter) is done
    if (rc == DML_OK && hipEventSynchronize(g->mapplied[k]) != hipSuccess) rc = set_error(DML_E_HIP, "applied wait");
    if (rc == DML_OK) rc = dml_prereduce_moments_piece(h, S, S, 0, W * S, g->mpart[k], g->cstream);
    if (rc == DML_OK) rc = dml_prereduce_stream_wait(h, g->rstream);
    const int local = rc;
    if (local != DML_OK) {
        // the same collective on every rank: zeros from this one, no apply here
        (void)hipStreamSynchronize(g->cstream);
        (void)hipEventSynchronize(g->mapplied[k]);
        (void)hipMemsetAsync(g->mpart[k], 0, (size_t)(W * S * 2 * C) * sizeof(float), g->rstream);
    }
    const ncclResult_t r = ncclReduceScatter(g->mpart[k], g->mrecv[k], (size_t)(S * 2 * C), ncclFloat32, ncclSum,
                                             g->comm, g->rstream);
    if (local != DML_OK || r != ncclSuccess) {
        // no apply: the set's next use (two calls on) waits for the scatter instead
        (void)hipEventRecord(g->mapplied[k], g->rstream);
    }
    if (local != DML_OK) {
        if (h) (void)dml_prereduce_end(h);
        return local;
    }
    if (r != ncclSuccess) {
        (void)dml_prereduce_end(h);
        return set_error(DML_E_HIP, std::string("ncclReduceScatter: ") + ncclGetErrorString(r));
    }
    GHIP(hipEventRecord(g->mrs_done[k], g->rstream));
    GHIP(hipStreamWaitEvent(g->sstream, g->mrs_done[k], 0));
    GRC(dml_store_apply_adagrad_moments_device(g->store, g->mrecv[k], g->shard_rows));
    GHIP(hipEventRecord(g->mapplied[k], g->sstream));
    g->mpending.push_back(h);
    return end_moments(g, 1);  // the previous call's errors
}

// Pushes already split to this shard (the reference client's per-partition split,
// SparseMatrix.java:46-60): the store's exact ordered push, after every earlier
// group call, so the store applies calls in the order they were made.
int dml_group_push_local(dml_group* g, const void* const* dev_bufs, const int64_t* lens, int32_t n) {
    if (!g || n < 0 || n > kMaxW || (n > 0 && (!dev_bufs || !lens)))
        return set_error(DML_E_INVALID_ARG, "bad push arguments (n must be <= 64)");
    GHIP(hipSetDevice(g->device));
    if (g->xheld) {  // the last exchange call's slices
        GHIP(hipStreamSynchronize(g->rstream));
        GRC(hand_over(g));
    }
    GRC(end_pending(g, 0));  // full-range calls waiting for their reduce-scatter and apply
    return dml_store_push_batch_device(g->store, dev_bufs, lens, n);
}

int dml_group_debug_fail_verify(dml_group* g, int32_t nth) {
    if (!g || nth < 0) return set_error(DML_E_INVALID_ARG, "bad fault-injection arguments");
    g->fail_verify_at = nth;
    return DML_OK;
}

int dml_group_flush(dml_group* g) {
    if (!g) return set_error(DML_E_INVALID_ARG, "null group");
    GHIP(hipSetDevice(g->device));
    int rc = DML_OK;
    if (g->xheld) {  // the last exchange call's slices
        rc = hipStreamSynchronize(g->rstream) == hipSuccess ? DML_OK : set_error(DML_E_HIP, "exchange sync");
        if (rc == DML_OK) rc = hand_over(g);
    }
    const int r1 = end_pending(g, 0);
    if (rc == DML_OK) rc = r1;
    const int rm = end_moments(g, 0);
    if (rc == DML_OK) rc = rm;
    for (hipStream_t s : {g->cstream, g->rstream})
        if (hipStreamSynchronize(s) != hipSuccess && rc == DML_OK) rc = set_error(DML_E_HIP, "group stream sync");
    for (hipEvent_t e : g->applied)
        if (hipEventSynchronize(e) != hipSuccess && rc == DML_OK) rc = set_error(DML_E_HIP, "apply sync");
    const int r2 = dml_store_flush(g->store);
    return rc != DML_OK ? rc : r2;
}

void dml_group_destroy(dml_group* g) { group_free(g); }

}  // extern "C"
