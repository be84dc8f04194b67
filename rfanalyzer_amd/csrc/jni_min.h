/*
 * jni_min.h -- minimal JNI types for the librfa JNI shim.
 *
 * This image has no JDK, so instead of <jni.h> the shim uses this restatement
 * of the JNI specification's primitive types and of the JNINativeInterface
 * function table LAYOUT: the slots the shim calls sit at their specified
 * indices (GetArrayLength 171, GetByteArrayRegion 200, GetIntArrayRegion 203,
 * GetFloatArrayRegion 205, SetIntArrayRegion 211, SetFloatArrayRegion 213,
 * ExceptionCheck 228); every other slot is opaque.
 * JNIEnv* points at a pointer to that table, which is binary-identical to both
 * the C and the C++ flavour of <jni.h>.
 */
#ifndef RFA_JNI_MIN_H
#define RFA_JNI_MIN_H

#include <stddef.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef float jfloat;
typedef jint jsize;
typedef void *jobject;
typedef jobject jarray;
typedef jarray jfloatArray;
typedef jarray jbyteArray;
typedef jarray jintArray;

#define JNI_FALSE 0
#define JNI_TRUE 1

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
    void *reserved_0_170[171];
    jsize(JNICALL *GetArrayLength)(JNIEnv *env, jarray array); /* 171 */
    void *reserved_172_199[28];
    void(JNICALL *GetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, jbyte *buf); /* 200 */
    void *reserved_201_202[2];
    void(JNICALL *GetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, jint *buf); /* 203 */
    void *reserved_204;
    void(JNICALL *GetFloatArrayRegion)(JNIEnv *env, jfloatArray array, jsize start, jsize len, jfloat *buf); /* 205 */
    void *reserved_206_210[5];
    void(JNICALL *SetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, const jint *buf); /* 211 */
    void *reserved_212;
    void(JNICALL *SetFloatArrayRegion)(JNIEnv *env, jfloatArray array, jsize start, jsize len,
                                       const jfloat *buf); /* 213 */
    void *reserved_214_227[14];
    jboolean(JNICALL *ExceptionCheck)(JNIEnv *env); /* 228 */
    void *reserved_229_232[4];
};

#define RFA_JNI_TABLE_SLOTS 233

#ifdef __cplusplus
}
static_assert(offsetof(JNINativeInterface_, GetArrayLength) == 171 * sizeof(void *), "JNI slot 171");
static_assert(offsetof(JNINativeInterface_, GetByteArrayRegion) == 200 * sizeof(void *), "JNI slot 200");
static_assert(offsetof(JNINativeInterface_, GetIntArrayRegion) == 203 * sizeof(void *), "JNI slot 203");
static_assert(offsetof(JNINativeInterface_, GetFloatArrayRegion) == 205 * sizeof(void *), "JNI slot 205");
static_assert(offsetof(JNINativeInterface_, SetIntArrayRegion) == 211 * sizeof(void *), "JNI slot 211");
static_assert(offsetof(JNINativeInterface_, SetFloatArrayRegion) == 213 * sizeof(void *), "JNI slot 213");
static_assert(offsetof(JNINativeInterface_, ExceptionCheck) == 228 * sizeof(void *), "JNI slot 228");
static_assert(sizeof(JNINativeInterface_) == RFA_JNI_TABLE_SLOTS * sizeof(void *), "JNI table size");
#endif

#endif /* RFA_JNI_MIN_H */
