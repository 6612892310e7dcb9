// dml_jni.cc — JNI shim: com.intel.distml.util.store.GpuDataStore -> include/distml_ps.h.
// Build (where a JDK provides jni.h):
//   g++ -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include
//       dml_jni.cc -L../../distml_amd -ldistml_ps -Wl,-rpath,'$ORIGIN' -o libdistml_jni.so
// Status codes become the exceptions the reference throws (DataStore.java:91,
// IntMatrixStore.java:175, array bounds): see include/distml_ps.h.
#include <jni.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>

#include <vector>

#include "distml_ps.h"

static void throw_for(JNIEnv* env, int rc) {
    const char* cls = "java/lang/RuntimeException";
    switch (rc) {
        case DML_E_BAD_DESC: cls = "java/lang/IllegalArgumentException"; break;
        case DML_E_KEY_OUT_OF_SHARD:
        case DML_E_TRUNCATED: cls = "java/lang/ArrayIndexOutOfBoundsException"; break;
        case DML_E_NEGATIVE_COUNTER: cls = "java/lang/IllegalStateException"; break;
        default: break;
    }
    env->ThrowNew(env->FindClass(cls), dml_last_error());
}

#define FN(name) Java_com_intel_distml_util_store_GpuDataStore_##name
static dml_store* H(jlong h) { return reinterpret_cast<dml_store*>(h); }

extern "C" {

JNIEXPORT jlong JNICALL FN(nativeCreate)(JNIEnv* env, jclass, jint dt, jint kt, jint vt, jint dr, jint dc, jint ada,
                                         jlong first, jlong last, jint cols, jint device, jint flags) {
    dml_desc d{dt, kt, vt, dr, dc, ada};
    dml_store* s = nullptr;
    int rc = dml_store_create_range(&d, first, last, cols, device, (uint32_t)flags, &s);
    if (rc) throw_for(env, rc);
    return reinterpret_cast<jlong>(s);
}

// Per-thread pinned staging for JVM-heap byte[]s: GetByteArrayRegion copies the
// array into it (no GC-blocking critical section across the GPU work), and the
// library DMAs pinned memory without a further staging copy. The push is
// synchronous, so the buffer is free again when dml_store_push returns.
namespace {
struct PinnedStage {
    void* p = nullptr;
    int64_t cap = 0;
    ~PinnedStage() { if (p) dml_host_free(p); }
    uint8_t* get(int64_t n) {
        if (n > cap) {
            if (p) dml_host_free(p);
            p = nullptr;
            cap = 0;
            const int64_t want = n < (1 << 20) ? (1 << 20) : n;
            if (dml_host_alloc(want, &p) != DML_OK) return nullptr;
            cap = want;
        }
        return static_cast<uint8_t*>(p);
    }
};
thread_local PinnedStage t_stage;

// Copy a byte[] into the thread's pinned stage; nullptr (exception pending) on failure.
const uint8_t* stage_array(JNIEnv* env, jbyteArray a, jsize* n_out) {
    const jsize n = env->GetArrayLength(a);
    uint8_t* p = t_stage.get(n);
    if (!p) {
        throw_for(env, DML_E_NOMEM);
        return nullptr;
    }
    env->GetByteArrayRegion(a, 0, n, reinterpret_cast<jbyte*>(p));
    *n_out = n;
    return p;
}
}  // namespace

// The byte[] is borrowed for the call only (PSAgent.java:278-281): its bytes are
// copied into pinned staging first; nothing retains the array after return.
JNIEXPORT void JNICALL FN(nativePush)(JNIEnv* env, jclass, jlong h, jbyteArray a) {
    jsize n = 0;
    const uint8_t* p = stage_array(env, a, &n);
    if (!p) return;
    if (int rc = dml_store_push(H(h), p, n)) throw_for(env, rc);
}

// DataStore.rand() (PSActor OP_RAND): the reference's distributions (dml_store_rand).
JNIEXPORT void JNICALL FN(nativeRand)(JNIEnv* env, jclass, jlong h, jlong seed) {
    if (int rc = dml_store_rand(H(h), (uint64_t)seed)) throw_for(env, rc);
}

// Largest Java array (the JVM's limit on `new byte[n]`): a larger result cannot be
// returned as one byte[]; the JVM itself would throw OutOfMemoryError.
constexpr int64_t kMaxJavaArray = 0x7FFFFFF7;

static jbyteArray fetch_common(JNIEnv* env, dml_store* s, const int64_t* keys, int64_t n, bool range, int64_t f,
                               int64_t l) {
    int64_t rows = 0;
    int32_t cols = 0;
    dml_store_shape(s, &rows, &cols);
    const int64_t cap = (range ? (l - f + 1) : n) * (8 + 16 * (int64_t)cols);
    if (cap > kMaxJavaArray) {
        env->ThrowNew(env->FindClass("java/lang/OutOfMemoryError"), "fetch result exceeds the maximum Java array size");
        return nullptr;
    }
    // the library DMAs straight into the thread's pinned stage (no bounce buffer);
    // SetByteArrayRegion is the one host copy into the Java heap
    uint8_t* out = t_stage.get(cap > 0 ? cap : 1);
    if (!out) {
        throw_for(env, DML_E_NOMEM);
        return nullptr;
    }
    int64_t len = 0;
    int rc = range ? dml_store_fetch_range(s, f, l, out, cap, &len) : dml_store_fetch(s, keys, n, out, cap, &len);
    if (rc) { throw_for(env, rc); return nullptr; }
    jbyteArray r = env->NewByteArray((jsize)len);
    if (!r) return nullptr;  // OutOfMemoryError pending
    env->SetByteArrayRegion(r, 0, (jsize)len, reinterpret_cast<const jbyte*>(out));
    return r;
}

JNIEXPORT jbyteArray JNICALL FN(nativeFetch)(JNIEnv* env, jclass, jlong h, jlongArray ks) {
    const jsize n = env->GetArrayLength(ks);
    std::vector<int64_t> keys((size_t)n);
    env->GetLongArrayRegion(ks, 0, n, reinterpret_cast<jlong*>(keys.data()));
    return fetch_common(env, H(h), keys.data(), n, false, 0, 0);
}

JNIEXPORT jbyteArray JNICALL FN(nativeFetchRange)(JNIEnv* env, jclass, jlong h, jlong f, jlong l) {
    return fetch_common(env, H(h), nullptr, 0, true, f, l);
}

JNIEXPORT jlong JNICALL FN(nativeShardBytes)(JNIEnv*, jclass, jlong h) {
    int64_t len = 0;
    dml_store_write_all(H(h), nullptr, 0, &len);  // size query (returns DML_E_CAPACITY)
    return len;
}

JNIEXPORT jbyteArray JNICALL FN(nativeWriteAll)(JNIEnv* env, jclass, jlong h) {
    int64_t len = 0;
    dml_store_write_all(H(h), nullptr, 0, &len);
    if (len > kMaxJavaArray) {
        env->ThrowNew(env->FindClass("java/lang/OutOfMemoryError"), "shard exceeds the maximum Java array size");
        return nullptr;
    }
    uint8_t* out = t_stage.get(len > 0 ? len : 1);
    if (!out) { throw_for(env, DML_E_NOMEM); return nullptr; }
    int rc = dml_store_write_all(H(h), out, len, &len);
    if (rc) { throw_for(env, rc); return nullptr; }
    jbyteArray r = env->NewByteArray((jsize)len);
    if (!r) return nullptr;
    env->SetByteArrayRegion(r, 0, (jsize)len, reinterpret_cast<const jbyte*>(out));
    return r;
}

JNIEXPORT void JNICALL FN(nativeReadAll)(JNIEnv* env, jclass, jlong h, jbyteArray a) {
    jsize n = 0;
    const uint8_t* p = stage_array(env, a, &n);
    if (!p) return;
    if (int rc = dml_store_read_all(H(h), p, n)) throw_for(env, rc);
}

// syncTo / syncFrom (PSSync.java:131,160): local rows from..to, big-endian.
JNIEXPORT jbyteArray JNICALL FN(nativeSyncTo)(JNIEnv* env, jclass, jlong h, jint from, jint to) {
    int64_t rows = 0;
    int32_t cols = 0;
    dml_store_shape(H(h), &rows, &cols);
    int64_t len = 0;
    // size query: the rows that exist in [from, to]
    const int64_t hi = to < rows ? to : rows - 1;
    const int64_t cap = (from >= 0 && hi >= from) ? (hi - from + 1) * (int64_t)cols * 8 : 0;
    if (cap > kMaxJavaArray) {
        env->ThrowNew(env->FindClass("java/lang/OutOfMemoryError"), "rows exceed the maximum Java array size");
        return nullptr;
    }
    uint8_t* out = t_stage.get(cap > 0 ? cap : 1);
    if (!out) { throw_for(env, DML_E_NOMEM); return nullptr; }
    const int rc = dml_store_sync_to(H(h), from, to, out, cap, &len);
    jbyteArray r = env->NewByteArray((jsize)len);
    if (!r) return nullptr;
    env->SetByteArrayRegion(r, 0, (jsize)len, reinterpret_cast<const jbyte*>(out));
    if (rc) { throw_for(env, rc); return nullptr; }  // the caller writes the rows before rethrowing
    return r;
}

JNIEXPORT void JNICALL FN(nativeSyncFrom)(JNIEnv* env, jclass, jlong h, jint from, jint to, jbyteArray a) {
    jsize n = 0;
    const uint8_t* p = stage_array(env, a, &n);
    if (!p) return;
    if (int rc = dml_store_sync_from(H(h), from, to, p, n)) throw_for(env, rc);
}

// Pinned host memory as a DirectByteBuffer: PSAgent's NIO channel reads a
// PushRequest straight into it (PSAgent.java:27-62) and nativePushDirect hands
// the record bytes to the DMA without a staging copy.
JNIEXPORT jobject JNICALL FN(nativeHostAlloc)(JNIEnv* env, jclass, jlong bytes) {
    void* p = nullptr;
    if (int rc = dml_host_alloc(bytes, &p)) { throw_for(env, rc); return nullptr; }
    return env->NewDirectByteBuffer(p, bytes);
}

JNIEXPORT void JNICALL FN(nativeHostFree)(JNIEnv* env, jclass, jobject buf) {
    dml_host_free(env->GetDirectBufferAddress(buf));
}

JNIEXPORT void JNICALL FN(nativePushDirect)(JNIEnv* env, jclass, jlong h, jobject buf, jint offset, jint len) {
    auto* p = static_cast<const uint8_t*>(env->GetDirectBufferAddress(buf));
    if (!p) { throw_for(env, DML_E_INVALID_ARG); return; }
    if (int rc = dml_store_push(H(h), p + offset, len)) throw_for(env, rc);
}

JNIEXPORT void JNICALL FN(nativeFill)(JNIEnv* env, jclass, jlong h, jdouble v) {
    if (int rc = dml_store_fill(H(h), v)) throw_for(env, rc);
}

JNIEXPORT void JNICALL FN(nativeSetAlpha)(JNIEnv* env, jclass, jlong h, jfloat a, jfloat m, jfloat f) {
    if (int rc = dml_store_set_alpha(H(h), a, m, f)) throw_for(env, rc);
}

// Iter snapshot (GpuXStore.iter()): the shard's values (which 0) or
// AdaGrad's alpha (1) / delta (2) copied into the Java heap arrays the reference's
// Iter reads — dims 2: a T[rows][cols] (FloatMatrixStore.localData, ...), dims 1: a
// T[rows] (DoubleArrayStore.localData, ...); elem = the DataDesc element type of the
// array (INT 0, FLOAT 1, DOUBLE 3). Bounded chunks of rows through the thread's
// pinned stage (dml_store_read_rows), then Set<T>ArrayRegion per row.
JNIEXPORT void JNICALL FN(nativeSnapshot)(JNIEnv* env, jclass, jlong h, jint which, jint elem, jint dims,
                                          jobject dst) {
    int64_t rows = 0;
    int32_t cols = 0;
    if (int rc = dml_store_shape(H(h), &rows, &cols)) { throw_for(env, rc); return; }
    // the array must hold the store's own element type (alpha / delta: float), or the
    // rows would be reinterpreted
    int32_t vt = -1, ada = 0;
    if (int rc = dml_store_value_type(H(h), &vt, &ada)) { throw_for(env, rc); return; }
    if ((which == 0 && elem != vt) || ((which == 1 || which == 2) && (elem != DML_ELEMENT_TYPE_FLOAT || !ada))) {
        env->ThrowNew(env->FindClass("java/lang/IllegalArgumentException"),
                      "snapshot element type does not match the store");
        return;
    }
    const int64_t esz = elem == DML_ELEMENT_TYPE_DOUBLE ? 8 : 4;
    const int64_t per_row = dims == 2 ? cols : 1;  // elements per local row
    if ((dims != 1 && dims != 2) || (elem != DML_ELEMENT_TYPE_INT && elem != DML_ELEMENT_TYPE_FLOAT &&
                                     elem != DML_ELEMENT_TYPE_DOUBLE) || !dst ||
        env->GetArrayLength(static_cast<jarray>(dst)) != rows) {
        env->ThrowNew(env->FindClass("java/lang/IllegalArgumentException"), "snapshot array does not match the shard");
        return;
    }
    const int64_t row_bytes = per_row * esz;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(16 << 20) / std::max<int64_t>(row_bytes, 1));
    for (int64_t r0 = 0; r0 < rows; r0 += chunk) {
        const int64_t n = std::min(chunk, rows - r0);
        uint8_t* buf = t_stage.get(std::max<int64_t>(n * row_bytes, 1));
        if (!buf) { throw_for(env, DML_E_NOMEM); return; }
        if (int rc = dml_store_read_rows(H(h), which, r0, n, buf, n * row_bytes)) { throw_for(env, rc); return; }
        for (int64_t i = 0; i < (dims == 2 ? n : 1); ++i) {
            jobject a = dims == 2 ? env->GetObjectArrayElement(static_cast<jobjectArray>(dst), (jsize)(r0 + i)) : dst;
            if (!a) {
                if (!env->ExceptionCheck())
                    env->ThrowNew(env->FindClass("java/lang/NullPointerException"), "snapshot row is null");
                return;
            }
            const jsize at = dims == 2 ? 0 : (jsize)r0, len = (jsize)(dims == 2 ? per_row : n);
            const uint8_t* src = buf + (dims == 2 ? i * row_bytes : 0);
            if (dims == 2 && env->GetArrayLength(static_cast<jarray>(a)) != per_row) {
                env->ThrowNew(env->FindClass("java/lang/IllegalArgumentException"), "snapshot row length != rowSize");
                return;
            }
            if (elem == DML_ELEMENT_TYPE_FLOAT)
                env->SetFloatArrayRegion(static_cast<jfloatArray>(a), at, len, reinterpret_cast<const jfloat*>(src));
            else if (elem == DML_ELEMENT_TYPE_INT)
                env->SetIntArrayRegion(static_cast<jintArray>(a), at, len, reinterpret_cast<const jint*>(src));
            else
                env->SetDoubleArrayRegion(static_cast<jdoubleArray>(a), at, len, reinterpret_cast<const jdouble*>(src));
            if (dims == 2) env->DeleteLocalRef(a);
            if (env->ExceptionCheck()) return;
        }
    }
}

// FloatMatrixStoreAdaGrad's maxDelta / maxDeltaRow / maxDeltaCol (:27-29, :273-277):
// returns maxDelta, rowCol[0] = maxDeltaRow (the key, as the reference's (int)key),
// rowCol[1] = maxDeltaCol.
JNIEXPORT jfloat JNICALL FN(nativeMaxDelta)(JNIEnv* env, jclass, jlong h, jintArray row_col) {
    float v = 0.f;
    int32_t rc2[2] = {0, 0};
    if (int rc = dml_store_max_delta(H(h), &v, &rc2[0], &rc2[1])) { throw_for(env, rc); return 0.f; }
    env->SetIntArrayRegion(row_col, 0, 2, reinterpret_cast<const jint*>(rc2));
    return v;
}

JNIEXPORT void JNICALL FN(nativeDestroy)(JNIEnv*, jclass, jlong h) { dml_store_destroy(H(h)); }

}  // extern "C"

// ---- com.intel.distml.util.store.GpuShardGroup -> dml_group_* -------------
#define GFN(name) Java_com_intel_distml_util_store_GpuShardGroup_##name
static dml_group* G(jlong h) { return reinterpret_cast<dml_group*>(h); }

extern "C" {

JNIEXPORT jbyteArray JNICALL GFN(nativeUniqueId)(JNIEnv* env, jclass) {
    uint8_t id[128];
    if (int rc = dml_group_unique_id(id, 128)) {
        throw_for(env, rc);
        return nullptr;
    }
    jbyteArray out = env->NewByteArray(128);
    env->SetByteArrayRegion(out, 0, 128, reinterpret_cast<const jbyte*>(id));
    return out;
}

JNIEXPORT jlong JNICALL GFN(nativeGroupCreate)(JNIEnv* env, jclass, jbyteArray id, jint world, jint rank,
                                               jint device, jint dt, jint kt, jint vt, jint dr, jint dc, jint ada,
                                               jlong total_rows, jint cols, jint pieces) {
    uint8_t buf[128] = {0};
    if (env->GetArrayLength(id) != 128) {
        env->ThrowNew(env->FindClass("java/lang/IllegalArgumentException"), "unique id must be 128 bytes");
        return 0;
    }
    env->GetByteArrayRegion(id, 0, 128, reinterpret_cast<jbyte*>(buf));
    dml_desc d{dt, kt, vt, dr, dc, ada};
    dml_group* g = nullptr;
    if (int rc = dml_group_create(buf, world, rank, device, &d, total_rows, cols, pieces, &g)) throw_for(env, rc);
    return reinterpret_cast<jlong>(g);
}

// mode: 0 full-range pre-reduce, 1 exact exchange, 2 two-moment AdaGrad, 3 local (already split)
JNIEXPORT void JNICALL GFN(nativeGroupPush)(JNIEnv* env, jclass, jlong g, jlongArray ptrs, jlongArray lens,
                                             jint mode) {
    const jsize n = env->GetArrayLength(ptrs);
    std::vector<jlong> p((size_t)n), l((size_t)n);
    env->GetLongArrayRegion(ptrs, 0, n, p.data());
    env->GetLongArrayRegion(lens, 0, n, l.data());
    std::vector<const void*> dp((size_t)n);
    std::vector<int64_t> dl((size_t)n);
    for (jsize i = 0; i < n; ++i) {
        dp[(size_t)i] = reinterpret_cast<const void*>(p[(size_t)i]);
        dl[(size_t)i] = l[(size_t)i];
    }
    int rc = DML_E_INVALID_ARG;
    switch (mode) {
        case 0: rc = dml_group_push_full_range(G(g), dp.data(), dl.data(), (int32_t)n); break;
        case 1: rc = dml_group_push_exchange(G(g), dp.data(), dl.data(), (int32_t)n); break;
        case 2: rc = dml_group_push_moments(G(g), dp.data(), dl.data(), (int32_t)n); break;
        case 3: rc = dml_group_push_local(G(g), dp.data(), dl.data(), (int32_t)n); break;
        default: break;
    }
    if (rc) throw_for(env, rc);
}

JNIEXPORT void JNICALL GFN(nativeGroupFlush)(JNIEnv* env, jclass, jlong g) {
    if (int rc = dml_group_flush(G(g))) throw_for(env, rc);
}

JNIEXPORT jlong JNICALL GFN(nativeGroupStore)(JNIEnv* env, jclass, jlong g) {
    dml_store* s = nullptr;
    if (int rc = dml_group_store(G(g), &s)) throw_for(env, rc);
    return reinterpret_cast<jlong>(s);
}

JNIEXPORT void JNICALL GFN(nativeGroupDestroy)(JNIEnv*, jclass, jlong g) { dml_group_destroy(G(g)); }

}  // extern "C"
