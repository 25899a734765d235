/* jni.h (test-only mock) -- just enough of the JNI C interface for jni/jwave_hip_jni.c to compile
 * and run without a JDK (the image has none).  Types and JNINativeInterface_ members have the
 * JNI specification's names and C signatures, so the glue compiles unchanged against this file
 * and against a real $JAVA_HOME/include/jni.h; only the members the glue calls exist here.
 * The implementation (tests/c/jni_mock/mock_env.c) models Java objects with C memory: double[],
 * Object[] (including double[][] and double[][][]), direct NIO buffers, classes (by name) and
 * strings, plus one pending exception (class name + message) per environment. */
#ifndef JWAVE_TEST_MOCK_JNI_H
#define JWAVE_TEST_MOCK_JNI_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;

#define JNI_FALSE 0
#define JNI_TRUE 1

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass(JNICALL* FindClass)(JNIEnv* env, const char* name);
  jint(JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jboolean(JNICALL* ExceptionCheck)(JNIEnv* env);
  void(JNICALL* DeleteLocalRef)(JNIEnv* env, jobject obj);
  jsize(JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
  jobjectArray(JNICALL* NewObjectArray)(JNIEnv* env, jsize len, jclass clazz, jobject init);
  jobject(JNICALL* GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
  void(JNICALL* SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
  jdoubleArray(JNICALL* NewDoubleArray)(JNIEnv* env, jsize len);
  void(JNICALL* GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len,
                                      jdouble* buf);
  void(JNICALL* SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len,
                                      const jdouble* buf);
  jstring(JNICALL* NewStringUTF)(JNIEnv* env, const char* utf);
  void*(JNICALL* GetDirectBufferAddress)(JNIEnv* env, jobject buf);
  jlong(JNICALL* GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
};

#endif
