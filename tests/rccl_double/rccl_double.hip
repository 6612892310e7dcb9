// rccl_double.hip — TEST-ONLY stand-in for the RCCL entry points libdistml_ps.so
// calls (ncclGetUniqueId, ncclCommInitRank(Config), ncclReduceScatter, ncclSend/ncclRecv
// in ncclGroupStart/End, ncclCommDestroy, ncclGetErrorString), so that the native
// group's N > 1 schedule (distml_amd/csrc/dml_group.hip) runs with several ranks
// on ONE GPU: RCCL itself refuses two ranks per device.
//
// Ranks are processes that share a POSIX shared-memory segment named by the
// unique id. Collectives are ASYNCHRONOUS, with RCCL's stream semantics: a call
// records an event on the caller's stream, enqueues a wait kernel behind it (it
// polls a host-mapped completion counter) and returns. A helper thread per
// communicator runs the collectives in call order: it waits for the event (the
// send data is ready), optionally sleeps DML_RCCL_DOUBLE_DELAY_US, moves the data
// device -> shared memory -> device on its own stream, sums on the host in rank
// order, and then releases the counter. Work enqueued on the caller's stream after
// the call therefore runs after the collective, while work on OTHER streams races
// with it unless the library orders it (events / stream waits) — a missing
// dependency shows up as wrong sums, above all with a delay. The product library
// is unchanged: tests/native_group_worker.py dlopens this library RTLD_GLOBAL
// before libdistml_ps.so, whose undefined nccl* symbols then resolve here (the
// global scope is searched before the library's own librccl).
//
// The wait kernel is bounded (about a minute): a collective that never completes
// ends it with an error mark instead of holding the GPU (the helper then reports
// the failure and the sums are wrong).
//
// Built by tests/rccl_double/Makefile; never linked into the product.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace {

constexpr int kMaxRanks = 16;
constexpr char kMagic[] = "dml-rccl-double:";

struct Header {
    std::atomic<uint32_t> arrive;
    std::atomic<uint32_t> gen;
    int64_t sizes[kMaxRanks][kMaxRanks];  // group send/recv: bytes src -> dst of the current group
};

int64_t slot_bytes() {
    const char* e = getenv("DML_RCCL_DOUBLE_SLOT_MB");
    const int64_t mb = e ? atoll(e) : 32;
    return (mb > 0 ? mb : 32) << 20;
}

int64_t delay_us() {
    const char* e = getenv("DML_RCCL_DOUBLE_DELAY_US");
    return e ? atoll(e) : 0;
}

std::atomic<int64_t> g_calls{0};

// Blocks the stream until the helper thread marks collective `seq` done
// (done[0] >= seq), or about a minute passed (then done[1] = seq: the stand-in's
// error mark). One wave; every path reaches the end.
__global__ void k_wait_done(volatile uint64_t* done, uint64_t seq) {
    if (threadIdx.x != 0) return;
    for (uint64_t i = 0; i < (1ull << 24); ++i) {  // ~16.7 M polls of >= 3 us each
        if (__hip_atomic_load((uint64_t*)done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >= seq) return;
        __builtin_amdgcn_s_sleep(127);
    }
    __hip_atomic_store((uint64_t*)done + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

bool ok(hipError_t e) {
    if (e == hipSuccess) return true;
    fprintf(stderr, "rccl_double: %s\n", hipGetErrorString(e));
    return false;
}

struct P2P {
    bool send;
    void* buf;
    int64_t bytes;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};

// One queued collective: a reduce-scatter or a group of sends / receives.
struct Op {
    bool rs = false;
    const void* sendbuff = nullptr;
    void* recvbuff = nullptr;
    size_t count = 0;
    ncclDataType_t dt = ncclFloat32;
    std::vector<P2P> p2p;
    std::vector<hipEvent_t> ready;  // the send data is ready when these complete
    uint64_t seq = 0;
};

}  // namespace

struct ncclComm {
    int rank = 0, world = 1;
    char name[128] = {};
    Header* hdr = nullptr;
    uint8_t* slots = nullptr;  // world x slot
    int64_t slot = 0;
    size_t map_bytes = 0;
    int device = 0;
    // asynchronous execution
    uint64_t* done = nullptr;  // host-mapped: [0] last completed seq, [1] wait-kernel timeout mark
    uint64_t next_seq = 0;
    hipStream_t hstream = nullptr;  // the helper's copies
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Op*> q;
    bool stop = false;
    std::atomic<int> failed{0};
    std::thread helper;

    uint8_t* slot_of(int r) const { return slots + (size_t)r * (size_t)slot; }
    void barrier() const {
        const uint32_t g = hdr->gen.load(std::memory_order_acquire);
        if (hdr->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)world) {
            hdr->arrive.store(0, std::memory_order_relaxed);
            hdr->gen.fetch_add(1, std::memory_order_acq_rel);
            return;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (int spin = 0; hdr->gen.load(std::memory_order_acquire) == g; ++spin) {
            if (spin > 1000) std::this_thread::sleep_for(std::chrono::microseconds(50));
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
                fprintf(stderr, "rccl_double: rank %d stuck in a collective for 120 s (a rank skipped it)\n", rank);
                abort();
            }
        }
    }
    bool d2h(void* dst, const void* src, size_t n) {
        return ok(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, hstream)) && ok(hipStreamSynchronize(hstream));
    }
    bool h2d(void* dst, const void* src, size_t n) {
        return ok(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, hstream)) && ok(hipStreamSynchronize(hstream));
    }
};

namespace {

thread_local int g_depth = 0;
thread_local std::vector<P2P> g_ops;

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

template <typename T>
void add_into(void* acc, const void* x, int64_t n) {
    T* a = (T*)acc;
    const T* b = (const T*)x;
    for (int64_t i = 0; i < n; ++i) a[i] = (T)(a[i] + b[i]);
}

bool sum_into(ncclDataType_t t, void* acc, const void* x, int64_t n) {
    switch (t) {
        case ncclFloat32: add_into<float>(acc, x, n); return true;
        case ncclFloat64: add_into<double>(acc, x, n); return true;
        case ncclInt32: case ncclUint32: add_into<uint32_t>(acc, x, n); return true;  // wraps mod 2^32
        case ncclInt64: case ncclUint64: add_into<uint64_t>(acc, x, n); return true;
        default: return false;
    }
}

// ---- the collectives, run by the helper thread once their inputs are ready ----
bool run_group(ncclComm_t c, const std::vector<P2P>& ops) {
    const int W = c->world, me = c->rank;
    std::vector<const P2P*> to(W, nullptr), from(W, nullptr);
    for (auto& o : ops) (o.send ? to : from)[o.peer] = &o;
    for (int p = 0; p < W; ++p) c->hdr->sizes[me][p] = to[p] ? to[p]->bytes : -1;
    c->barrier();
    const int64_t chunk = c->slot / W;
    int64_t rounds = 0;
    for (int s = 0; s < W; ++s)
        for (int d = 0; d < W; ++d) rounds = std::max<int64_t>(rounds, (c->hdr->sizes[s][d] + chunk - 1) / chunk);
    bool good = true;
    for (int p = 0; p < W; ++p)  // the sender's size must be what the receiver expects
        if (from[p] && c->hdr->sizes[p][me] != from[p]->bytes) {
            fprintf(stderr, "rccl_double: rank %d expects %ld B from %d, which sends %ld B\n", me,
                    (long)from[p]->bytes, p, (long)c->hdr->sizes[p][me]);
            good = false;
        }
    c->barrier();  // every rank checked the sizes table (or none proceeds)
    if (!good) return false;
    for (int64_t r = 0; r < rounds; ++r) {
        const int64_t off = r * chunk;
        for (int p = 0; p < W; ++p)
            if (to[p] && to[p]->bytes > off && good)
                good = c->d2h(c->slot_of(me) + p * chunk, (uint8_t*)to[p]->buf + off,
                              (size_t)std::min(chunk, to[p]->bytes - off));
        c->barrier();
        for (int p = 0; p < W; ++p)
            if (from[p] && from[p]->bytes > off && good)
                good = c->h2d((uint8_t*)from[p]->buf + off, c->slot_of(p) + me * chunk,
                              (size_t)std::min(chunk, from[p]->bytes - off));
        c->barrier();
    }
    c->barrier();  // the sizes table is read by everyone before the next group rewrites it
    return good;
}

bool run_rs(ncclComm_t c, const Op& o) {
    const size_t eb = type_bytes(o.dt);
    const int W = c->world, me = c->rank;
    const int64_t per = std::max<int64_t>(1, c->slot / W / (int64_t)eb);  // elements per destination per round
    std::vector<uint8_t> acc((size_t)std::min<int64_t>(per, (int64_t)o.count) * eb + 1);
    bool good = true;
    for (int64_t e = 0; e < (int64_t)o.count; e += per) {
        const int64_t n = std::min<int64_t>(per, (int64_t)o.count - e);
        for (int d = 0; d < W && good; ++d)
            good = c->d2h(c->slot_of(me) + (size_t)d * per * eb,
                          (const uint8_t*)o.sendbuff + ((size_t)d * o.count + (size_t)e) * eb, (size_t)n * eb);
        c->barrier();
        memcpy(acc.data(), c->slot_of(0) + (size_t)me * per * eb, (size_t)n * eb);
        for (int q = 1; q < W; ++q)
            if (!sum_into(o.dt, acc.data(), c->slot_of(q) + (size_t)me * per * eb, n)) good = false;
        if (good) good = c->h2d((uint8_t*)o.recvbuff + (size_t)e * eb, acc.data(), (size_t)n * eb);
        c->barrier();
    }
    return good;
}

void helper_main(ncclComm_t c) {
    (void)hipSetDevice(c->device);
    const int64_t delay = delay_us();
    for (;;) {
        Op* o = nullptr;
        {
            std::unique_lock<std::mutex> lk(c->mu);
            c->cv.wait(lk, [&] { return c->stop || !c->q.empty(); });
            if (c->q.empty()) return;  // stop requested and drained
            o = c->q.front();
            c->q.pop_front();
        }
        bool good = true;
        for (hipEvent_t e : o->ready) good = ok(hipEventSynchronize(e)) && good;
        if (delay > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay));
        good = (o->rs ? run_rs(c, *o) : run_group(c, o->p2p)) && good;
        if (!good) c->failed.store(1);
        for (hipEvent_t e : o->ready) (void)hipEventDestroy(e);
        __atomic_store_n(&c->done[0], o->seq, __ATOMIC_RELEASE);  // releases the wait kernels
        if (__atomic_load_n(&c->done[1], __ATOMIC_ACQUIRE) != 0) {
            fprintf(stderr, "rccl_double: rank %d: a wait kernel timed out\n", c->rank);
            c->failed.store(1);
        }
        delete o;
        g_calls.fetch_add(1);
    }
}

// Record the ready events, block the streams behind the collective, queue it.
ncclResult_t enqueue(ncclComm_t c, Op* o, const std::vector<hipStream_t>& streams) {
    if (c->failed.load()) {
        delete o;
        return ncclUnhandledCudaError;  // an earlier collective failed (RCCL's async error)
    }
    o->seq = ++c->next_seq;
    for (hipStream_t s : streams) {
        hipEvent_t e;
        if (!ok(hipEventCreateWithFlags(&e, hipEventDisableTiming)) || !ok(hipEventRecord(e, s))) {
            delete o;
            return ncclUnhandledCudaError;
        }
        o->ready.push_back(e);
        hipLaunchKernelGGL(k_wait_done, dim3(1), dim3(64), 0, s, (volatile uint64_t*)c->done, o->seq);
        if (!ok(hipGetLastError())) {
            delete o;
            return ncclUnhandledCudaError;
        }
    }
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->q.push_back(o);
    }
    c->cv.notify_one();
    return ncclSuccess;
}

ncclResult_t submit_group(std::vector<P2P>& ops) {
    if (ops.empty()) return ncclSuccess;
    ncclComm_t c = ops[0].comm;
    std::vector<const P2P*> to(kMaxRanks, nullptr), from(kMaxRanks, nullptr);
    std::vector<hipStream_t> streams;
    for (auto& o : ops) {
        if (o.comm != c || o.peer < 0 || o.peer >= c->world) return ncclInvalidArgument;
        auto& v = o.send ? to : from;
        if (v[o.peer]) return ncclInvalidUsage;  // one send and one receive per peer and group
        v[o.peer] = &o;
        if (std::find(streams.begin(), streams.end(), o.stream) == streams.end()) streams.push_back(o.stream);
    }
    Op* op = new Op();
    op->p2p = ops;
    return enqueue(c, op, streams);
}

void drain(ncclComm_t c) {
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->stop = true;
    }
    c->cv.notify_one();
    if (c->helper.joinable()) c->helper.join();
}

}  // namespace

extern "C" {

// Collectives this process ran through the double (tests assert it was used).
int64_t rccl_double_calls(void) { return g_calls.load(); }
// minCTAs / maxCTAs of the last ncclCommInitRankConfig (-1: none, or left undefined):
// tests assert the library pins the reduce-scatter's channel count
static int g_min_ctas = -1, g_max_ctas = -1;
int32_t rccl_double_ctas(int32_t which) { return which ? g_max_ctas : g_min_ctas; }

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (rccl_double)";
        case ncclInvalidArgument: return "invalid argument (rccl_double)";
        case ncclInvalidUsage: return "invalid usage (rccl_double)";
        case ncclUnhandledCudaError: return "HIP error (rccl_double)";
        default: return "error (rccl_double)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof *id);
    uint8_t rnd[12] = {};
    FILE* f = fopen("/dev/urandom", "rb");
    if (!f || fread(rnd, 1, sizeof rnd, f) != sizeof rnd) {
        if (f) fclose(f);
        return ncclSystemError;
    }
    fclose(f);
    char* p = id->internal + snprintf(id->internal, 64, "%s/dmlrccl_", kMagic);
    for (uint8_t b : rnd) p += snprintf(p, 3, "%02x", b);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks <= 0 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    if (strncmp(id.internal, kMagic, sizeof kMagic - 1) != 0) return ncclInvalidArgument;
    auto* c = new ncclComm();
    c->rank = rank;
    c->world = nranks;
    snprintf(c->name, sizeof c->name, "%s", id.internal + sizeof kMagic - 1);
    c->slot = slot_bytes();
    c->map_bytes = 4096 + (size_t)nranks * (size_t)c->slot;
    if (!ok(hipGetDevice(&c->device)) || !ok(hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking)) ||
        !ok(hipHostMalloc((void**)&c->done, 2 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent))) {
        delete c;
        return ncclUnhandledCudaError;
    }
    c->done[0] = c->done[1] = 0;
    const int fd = shm_open(c->name, O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)c->map_bytes) != 0) {
        if (fd >= 0) close(fd);
        delete c;
        return ncclSystemError;
    }
    void* m = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        delete c;
        return ncclSystemError;
    }
    c->hdr = (Header*)m;
    c->slots = (uint8_t*)m + 4096;
    c->barrier();
    c->helper = std::thread(helper_main, c);
    *out = c;
    return ncclSuccess;
}

// RCCL's config variant: checks the initializer's size / magic as RCCL does, records the
// CTA bounds, then the same communicator (the double has no channels to size)
ncclResult_t ncclCommInitRankConfig(ncclComm_t* out, int nranks, ncclUniqueId id, int rank, ncclConfig_t* config) {
    if (config && (config->size != sizeof(ncclConfig_t) || config->magic != 0xcafebeef)) return ncclInvalidArgument;
    if (config) {
        g_min_ctas = config->minCTAs == NCCL_CONFIG_UNDEF_INT ? -1 : config->minCTAs;
        g_max_ctas = config->maxCTAs == NCCL_CONFIG_UNDEF_INT ? -1 : config->maxCTAs;
    }
    return ncclCommInitRank(out, nranks, id, rank);
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclSuccess;
    drain(c);  // every queued collective ran (the helper's barriers before this one)
    c->barrier();
    if (c->rank == 0) shm_unlink(c->name);
    munmap(c->hdr, c->map_bytes);
    (void)hipHostFree(c->done);
    (void)hipStreamDestroy(c->hstream);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) {
    if (!c) return ncclSuccess;
    drain(c);
    munmap(c->hdr, c->map_bytes);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount, ncclDataType_t dt,
                               ncclRedOp_t op, ncclComm_t c, hipStream_t stream) {
    if (!c || !type_bytes(dt) || op != ncclSum) return ncclInvalidArgument;
    Op* o = new Op();
    o->rs = true;
    o->sendbuff = sendbuff;
    o->recvbuff = recvbuff;
    o->count = recvcount;
    o->dt = dt;
    return enqueue(c, o, {stream});
}

ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth > 0) return ncclSuccess;
    std::vector<P2P> ops;
    ops.swap(g_ops);
    return submit_group(ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t stream) {
    g_ops.push_back({true, const_cast<void*>(buf), (int64_t)(count * type_bytes(dt)), peer, c, stream});
    if (g_depth > 0) return ncclSuccess;
    std::vector<P2P> ops;
    ops.swap(g_ops);
    return submit_group(ops);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t stream) {
    g_ops.push_back({false, buf, (int64_t)(count * type_bytes(dt)), peer, c, stream});
    if (g_depth > 0) return ncclSuccess;
    std::vector<P2P> ops;
    ops.swap(g_ops);
    return submit_group(ops);
}

}  // extern "C"
