// mock_jvm.cc — test infrastructure: a minimal in-process JNIEnv so that the JNI
// shim (integration/jni/dml_jni.cc) can be linked and RUN without a JVM (the image
// has no JDK). It implements exactly the JNIEnv members declared in
// tests/jni_stub/jni.h, with the JNI specification's semantics for them: Java
// byte[] / long[] objects, direct ByteBuffers, FindClass / ThrowNew recording the
// pending exception. tests/test_jni_shim.py drives the shim's Java_* entry points
// through ctypes with these objects, exactly as the JVM would call them from
// GpuDataStore.java / GpuShardGroup.java.
//   g++ -std=c++17 -fPIC -shared -I tests/jni_stub -I include integration/jni/dml_jni.cc
//       tests/jni_mock/mock_jvm.cc -L distml_amd -ldistml_ps -o tests/jni_mock/libdml_jni_mock.so
#include <jni.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {
enum Kind { kClass, kBytes, kLongs, kDirect, kObjs, kFloats, kInts, kDoubles };
struct Obj : _jobject {
    Kind kind;
    std::string name;            // kClass
    std::vector<jbyte> bytes;    // kBytes; kFloats / kInts / kDoubles: the elements' bytes
    std::vector<jlong> longs;    // kLongs
    std::vector<Obj*> elems;     // kObjs (an Object[]: e.g. float[][])
    void* addr = nullptr;        // kDirect
    jlong cap = 0;
    explicit Obj(Kind k) : kind(k) {}
    size_t esize() const { return kind == kDoubles ? 8 : (kind == kFloats || kind == kInts) ? 4 : 1; }
    jsize length() const {
        switch (kind) {
            case kLongs: return (jsize)longs.size();
            case kObjs: return (jsize)elems.size();
            default: return (jsize)(bytes.size() / esize());
        }
    }
};
Obj* O(jobject o) { return static_cast<Obj*>(o); }
JNIEnv g_env;
bool g_pending = false;
std::string g_exc_class, g_exc_msg;
int g_calls = 0;  // JNIEnv calls made (the tests check the shim went through them)
}  // namespace

// ---- the JNIEnv members the shim uses (JNI specification semantics) ----------
jclass JNIEnv::FindClass(const char* name) {
    ++g_calls;
    Obj* c = new Obj(kClass);
    c->name = name;
    return c;
}
jint JNIEnv::ThrowNew(jclass clazz, const char* msg) {
    ++g_calls;
    g_pending = true;
    g_exc_class = O(clazz)->name;
    g_exc_msg = msg ? msg : "";
    delete O(clazz);
    return 0;
}
jsize JNIEnv::GetArrayLength(jarray a) {
    ++g_calls;
    return O(a)->length();
}
void JNIEnv::GetByteArrayRegion(jbyteArray a, jsize start, jsize len, jbyte* buf) {
    ++g_calls;
    if (start < 0 || len < 0 || (size_t)start + (size_t)len > O(a)->bytes.size()) {
        g_pending = true;
        g_exc_class = "java/lang/ArrayIndexOutOfBoundsException";
        return;
    }
    std::memcpy(buf, O(a)->bytes.data() + start, (size_t)len);
}
void JNIEnv::SetByteArrayRegion(jbyteArray a, jsize start, jsize len, const jbyte* buf) {
    ++g_calls;
    if (start < 0 || len < 0 || (size_t)start + (size_t)len > O(a)->bytes.size()) {
        g_pending = true;
        g_exc_class = "java/lang/ArrayIndexOutOfBoundsException";
        return;
    }
    std::memcpy(O(a)->bytes.data() + start, buf, (size_t)len);
}
void JNIEnv::GetLongArrayRegion(jlongArray a, jsize start, jsize len, jlong* buf) {
    ++g_calls;
    std::memcpy(buf, O(a)->longs.data() + start, sizeof(jlong) * (size_t)len);
}
jbyteArray JNIEnv::NewByteArray(jsize len) {
    ++g_calls;
    Obj* a = new Obj(kBytes);
    a->bytes.assign((size_t)len, 0);
    return a;
}
namespace {
// Set<T>ArrayRegion on a primitive array of kind k (ArrayIndexOutOfBoundsException /
// ArrayStoreException semantics of the JNI specification)
void set_region(jobject a, Kind k, jsize start, jsize len, const void* buf) {
    Obj* o = O(a);
    if (o->kind != k) {
        g_pending = true;
        g_exc_class = "java/lang/ArrayStoreException";
        return;
    }
    if (start < 0 || len < 0 || start + len > o->length()) {
        g_pending = true;
        g_exc_class = "java/lang/ArrayIndexOutOfBoundsException";
        return;
    }
    std::memcpy(o->bytes.data() + (size_t)start * o->esize(), buf, (size_t)len * o->esize());
}
}  // namespace
jobject JNIEnv::GetObjectArrayElement(jobjectArray a, jsize i) {
    ++g_calls;
    if (O(a)->kind != kObjs || i < 0 || i >= O(a)->length()) {
        g_pending = true;
        g_exc_class = "java/lang/ArrayIndexOutOfBoundsException";
        return nullptr;
    }
    return O(a)->elems[(size_t)i];  // a "local reference" to the element (DeleteLocalRef drops it)
}
void JNIEnv::SetFloatArrayRegion(jfloatArray a, jsize start, jsize len, const jfloat* buf) {
    ++g_calls;
    set_region(a, kFloats, start, len, buf);
}
void JNIEnv::SetIntArrayRegion(jintArray a, jsize start, jsize len, const jint* buf) {
    ++g_calls;
    set_region(a, kInts, start, len, buf);
}
void JNIEnv::SetDoubleArrayRegion(jdoubleArray a, jsize start, jsize len, const jdouble* buf) {
    ++g_calls;
    set_region(a, kDoubles, start, len, buf);
}
void JNIEnv::DeleteLocalRef(jobject) { ++g_calls; }
jboolean JNIEnv::ExceptionCheck() { return g_pending ? 1 : 0; }
jobject JNIEnv::NewDirectByteBuffer(void* address, jlong capacity) {
    ++g_calls;
    Obj* b = new Obj(kDirect);
    b->addr = address;
    b->cap = capacity;
    return b;
}
void* JNIEnv::GetDirectBufferAddress(jobject buf) {
    ++g_calls;
    return buf && O(buf)->kind == kDirect ? O(buf)->addr : nullptr;
}

// ---- the test side (ctypes) -----------------------------------------------------
extern "C" {
JNIEnv* mock_env() { return &g_env; }
jobject mock_byte_array(const void* data, int32_t len) {
    Obj* a = new Obj(kBytes);
    a->bytes.resize((size_t)len);
    if (len) std::memcpy(a->bytes.data(), data, (size_t)len);
    return a;
}
jobject mock_long_array(const int64_t* data, int32_t n) {
    Obj* a = new Obj(kLongs);
    a->longs.assign(data, data + n);
    return a;
}
int32_t mock_array_length(jobject a) { return a ? (int32_t)O(a)->length() : -1; }
// a Java float[] / int[] / double[] (kind 'F', 'I', 'D') of n zero elements
jobject mock_prim_array(char kind, int32_t n) {
    Obj* a = new Obj(kind == 'F' ? kFloats : kind == 'I' ? kInts : kDoubles);
    a->bytes.assign((size_t)n * a->esize(), 0);
    return a;
}
// an Object[] (e.g. float[][]) holding n given elements (owned by the array)
jobject mock_object_array(jobject* elems, int32_t n) {
    Obj* a = new Obj(kObjs);
    for (int32_t i = 0; i < n; ++i) a->elems.push_back(O(elems[i]));
    return a;
}
jobject mock_object_element(jobject a, int32_t i) { return O(a)->elems[(size_t)i]; }
const void* mock_array_data(jobject a) { return a ? O(a)->bytes.data() : nullptr; }
void* mock_direct_address(jobject b) { return b ? O(b)->addr : nullptr; }
int64_t mock_direct_capacity(jobject b) { return b ? O(b)->cap : -1; }
void mock_free(jobject o) {
    for (Obj* e : O(o)->elems) delete e;
    delete O(o);
}
int mock_calls() { return g_calls; }
// 1 and the exception's class / message if one is pending (then cleared), else 0
int mock_take_exception(char* cls, int32_t ccap, char* msg, int32_t mcap) {
    if (!g_pending) return 0;
    std::snprintf(cls, (size_t)ccap, "%s", g_exc_class.c_str());
    std::snprintf(msg, (size_t)mcap, "%s", g_exc_msg.c_str());
    g_pending = false;
    return 1;
}
}
