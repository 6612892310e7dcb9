// rccl_double.cc — TEST-ONLY stand-in for the RCCL entry points libdistml_ps.so
// calls (ncclGetUniqueId, ncclCommInitRank, ncclReduceScatter, ncclSend/ncclRecv
// in ncclGroupStart/End, ncclCommDestroy, ncclGetErrorString), so that the native
// group's N > 1 schedule (distml_amd/csrc/dml_group.hip) runs with several ranks
// on ONE GPU: RCCL itself refuses two ranks per device.
//
// Ranks are processes that share a POSIX shared-memory segment named by the
// unique id. Every collective is executed synchronously at the call: the stream
// is synchronized (everything enqueued before the call has run), the data moves
// device -> shared memory -> device with hipMemcpy, sums are formed on the host in
// rank order, and the call returns after the result is in the receive buffer —
// so work enqueued on the stream after the call sees it, as with RCCL. The
// product library is unchanged: tests/native_group_worker.py dlopens this
// library RTLD_GLOBAL before libdistml_ps.so, whose undefined nccl* symbols then
// resolve here (the global scope is searched before the library's own librccl).
//
// Built by tests/rccl_double/Makefile; never linked into the product.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

std::atomic<int64_t> g_calls{0};

}  // namespace

struct ncclComm {
    int rank = 0, world = 1;
    char name[128] = {};
    Header* hdr = nullptr;
    uint8_t* slots = nullptr;  // world x slot
    int64_t slot = 0;
    size_t map_bytes = 0;
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
};

namespace {

struct P2P {
    bool send;
    void* buf;
    int64_t bytes;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};
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

bool ok(hipError_t e) {
    if (e == hipSuccess) return true;
    fprintf(stderr, "rccl_double: %s\n", hipGetErrorString(e));
    return false;
}

ncclResult_t run_group(std::vector<P2P>& ops) {
    if (ops.empty()) return ncclSuccess;
    ncclComm_t c = ops[0].comm;
    for (auto& o : ops)
        if (o.comm != c || o.peer < 0 || o.peer >= c->world) return ncclInvalidArgument;
    for (auto& o : ops)
        if (!ok(hipStreamSynchronize(o.stream))) return ncclUnhandledCudaError;
    const int W = c->world, me = c->rank;
    std::vector<const P2P*> to(W, nullptr), from(W, nullptr);
    for (auto& o : ops) {
        auto& v = o.send ? to : from;
        if (v[o.peer]) return ncclInvalidUsage;  // one send and one receive per peer and group
        v[o.peer] = &o;
    }
    for (int p = 0; p < W; ++p) c->hdr->sizes[me][p] = to[p] ? to[p]->bytes : -1;
    c->barrier();
    const int64_t chunk = c->slot / W;
    int64_t rounds = 0;
    for (int s = 0; s < W; ++s)
        for (int d = 0; d < W; ++d) rounds = std::max<int64_t>(rounds, (c->hdr->sizes[s][d] + chunk - 1) / chunk);
    for (int p = 0; p < W; ++p)  // the sender's size must be what the receiver expects
        if (from[p] && c->hdr->sizes[p][me] != from[p]->bytes) {
            fprintf(stderr, "rccl_double: rank %d expects %ld B from %d, which sends %ld B\n", me,
                    (long)from[p]->bytes, p, (long)c->hdr->sizes[p][me]);
            c->barrier();
            return ncclInvalidUsage;
        }
    ncclResult_t rc = ncclSuccess;
    for (int64_t r = 0; r < rounds; ++r) {
        const int64_t off = r * chunk;
        for (int p = 0; p < W; ++p)
            if (to[p] && to[p]->bytes > off && rc == ncclSuccess &&
                !ok(hipMemcpy(c->slot_of(me) + p * chunk, (uint8_t*)to[p]->buf + off,
                              (size_t)std::min(chunk, to[p]->bytes - off), hipMemcpyDeviceToHost)))
                rc = ncclUnhandledCudaError;
        c->barrier();
        for (int p = 0; p < W; ++p)
            if (from[p] && from[p]->bytes > off && rc == ncclSuccess &&
                !ok(hipMemcpy((uint8_t*)from[p]->buf + off, c->slot_of(p) + me * chunk,
                              (size_t)std::min(chunk, from[p]->bytes - off), hipMemcpyHostToDevice)))
                rc = ncclUnhandledCudaError;
        c->barrier();
    }
    c->barrier();  // the sizes table is read by everyone before the next group rewrites it
    g_calls.fetch_add(1);
    return rc;
}

}  // namespace

extern "C" {

// Collectives this process ran through the double (tests assert it was used).
int64_t rccl_double_calls(void) { return g_calls.load(); }

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
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclSuccess;
    c->barrier();
    if (c->rank == 0) shm_unlink(c->name);
    munmap(c->hdr, c->map_bytes);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) {
    if (!c) return ncclSuccess;
    munmap(c->hdr, c->map_bytes);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount, ncclDataType_t dt,
                               ncclRedOp_t op, ncclComm_t c, hipStream_t stream) {
    const size_t eb = type_bytes(dt);
    if (!c || !eb || op != ncclSum) return ncclInvalidArgument;
    if (!ok(hipStreamSynchronize(stream))) return ncclUnhandledCudaError;
    const int W = c->world, me = c->rank;
    const int64_t per = std::max<int64_t>(1, c->slot / W / (int64_t)eb);  // elements per destination per round
    std::vector<uint8_t> acc((size_t)std::min<int64_t>(per, (int64_t)recvcount) * eb + 1);
    ncclResult_t rc = ncclSuccess;
    for (int64_t e = 0; e < (int64_t)recvcount; e += per) {
        const int64_t n = std::min<int64_t>(per, (int64_t)recvcount - e);
        for (int d = 0; d < W && rc == ncclSuccess; ++d)
            if (!ok(hipMemcpy(c->slot_of(me) + (size_t)d * per * eb,
                              (const uint8_t*)sendbuff + ((size_t)d * recvcount + (size_t)e) * eb, (size_t)n * eb,
                              hipMemcpyDeviceToHost)))
                rc = ncclUnhandledCudaError;
        c->barrier();
        memcpy(acc.data(), c->slot_of(0) + (size_t)me * per * eb, (size_t)n * eb);
        for (int q = 1; q < W; ++q)
            if (!sum_into(dt, acc.data(), c->slot_of(q) + (size_t)me * per * eb, n)) rc = ncclInvalidArgument;
        if (rc == ncclSuccess &&
            !ok(hipMemcpy((uint8_t*)recvbuff + (size_t)e * eb, acc.data(), (size_t)n * eb, hipMemcpyHostToDevice)))
            rc = ncclUnhandledCudaError;
        c->barrier();
    }
    g_calls.fetch_add(1);
    return rc;
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
    return run_group(ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t stream) {
    g_ops.push_back({true, const_cast<void*>(buf), (int64_t)(count * type_bytes(dt)), peer, c, stream});
    if (g_depth > 0) return ncclSuccess;
    std::vector<P2P> ops;
    ops.swap(g_ops);
    return run_group(ops);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t c, hipStream_t stream) {
    g_ops.push_back({false, buf, (int64_t)(count * type_bytes(dt)), peer, c, stream});
    if (g_depth > 0) return ncclSuccess;
    std::vector<P2P> ops;
    ops.swap(g_ops);
    return run_group(ops);
}

}  // extern "C"
