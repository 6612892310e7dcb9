/* Minimal stand-in for the JDK's jni.h, for checks of integration/jni/dml_jni.cc in
 * an image without a JDK (tests/test_jni_shim.py): a -fsyntax-only compile, and a
 * build linked with tests/jni_mock/mock_jvm.cc (an in-process JNIEnv implementing
 * exactly these members) whose Java_* entry points the tests call. It declares only
 * the JNI types and JNIEnv members the shim uses, with the JNI specification's
 * signatures. A real build uses $JAVA_HOME/include/jni.h (see dml_jni.cc). */
#ifndef DML_TEST_JNI_STUB_H
#define DML_TEST_JNI_STUB_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;
class _jobject {};
typedef _jobject* jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jobject jbyteArray;
typedef jobject jlongArray;
typedef jobject jobjectArray;
typedef jobject jfloatArray;
typedef jobject jintArray;
typedef jobject jdoubleArray;
typedef jobject jthrowable;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
struct JNIEnv {
    jclass FindClass(const char* name);
    jint ThrowNew(jclass clazz, const char* msg);
    jsize GetArrayLength(jarray array);
    void GetByteArrayRegion(jbyteArray array, jsize start, jsize len, jbyte* buf);
    void SetByteArrayRegion(jbyteArray array, jsize start, jsize len, const jbyte* buf);
    void GetLongArrayRegion(jlongArray array, jsize start, jsize len, jlong* buf);
    jbyteArray NewByteArray(jsize len);
    jobject NewDirectByteBuffer(void* address, jlong capacity);
    void* GetDirectBufferAddress(jobject buf);
    jobject GetObjectArrayElement(jobjectArray array, jsize index);
    void SetFloatArrayRegion(jfloatArray array, jsize start, jsize len, const jfloat* buf);
    void SetIntArrayRegion(jintArray array, jsize start, jsize len, const jint* buf);
    void SetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, const jdouble* buf);
    void DeleteLocalRef(jobject obj);
    jboolean ExceptionCheck();
};
#endif
