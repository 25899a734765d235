/* mock_env.c (test-only) -- a JNIEnv for jni/jwave_hip_jni.c without a JVM.
 *
 * Built together with the glue into tests/c/libjni_harness.so (tests/c/Makefile); the GPU test
 * tests/test_jni_glue_gpu.py builds Java objects through the mock_* functions below (ctypes),
 * calls the glue's Java_jwave_hip_* entry points exactly as a JVM would (env, class, arguments)
 * and reads the results and any pending exception back.
 *
 * Java semantics kept where the glue could get them wrong:
 *  - Get/SetDoubleArrayRegion outside the array raise ArrayIndexOutOfBoundsException;
 *  - Object[] element stores check the element's class against the array's ("[D" in "[[D");
 *  - calling anything but ExceptionCheck / DeleteLocalRef with an exception pending, or passing
 *    a null array, counts as a JNI violation (mock_violations()), which the tests require to
 *    stay 0 -- a real JVM would abort or behave undefined there. */
#define _POSIX_C_SOURCE 200809L /* strdup */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_DARRAY = 1, K_OARRAY, K_DIRECT, K_CLASS, K_STRING };

struct _jobject {
  int kind;
  jsize len;        /* arrays */
  double* d;        /* double[] */
  jobject* elems;   /* Object[] */
  char* name;       /* class name; element class of an Object[] (its own class is "[" + name);
                       string text */
  void* addr;       /* direct buffer */
  jlong cap;        /* direct buffer capacity in bytes */
  struct _jobject* next_alloc;
};

typedef struct {
  const struct JNINativeInterface_* fns; /* JNIEnv* points here: (*env)->Fn */
  int pending;
  char exc_cls[128];
  char exc_msg[512];
} MockEnv;

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static struct _jobject* g_objs;
static int g_violations;
static long g_local_deletes;

static jobject new_obj(int kind) {
  struct _jobject* o = calloc(1, sizeof *o);
  if (!o) return NULL;
  o->kind = kind;
  pthread_mutex_lock(&g_mu);
  o->next_alloc = g_objs;
  g_objs = o;
  pthread_mutex_unlock(&g_mu);
  return o;
}

static void violation(void) {
  pthread_mutex_lock(&g_mu);
  g_violations++;
  pthread_mutex_unlock(&g_mu);
}

static MockEnv* menv(JNIEnv* env) { return (MockEnv*)env; }

/* every call but ExceptionCheck / DeleteLocalRef must see no pending exception */
static void entry(JNIEnv* env) {
  if (menv(env)->pending) violation();
}

static void throw_(JNIEnv* env, const char* cls, const char* msg) {
  MockEnv* m = menv(env);
  if (m->pending) return; /* keep the first */
  m->pending = 1;
  strncpy(m->exc_cls, cls, sizeof m->exc_cls - 1);
  m->exc_cls[sizeof m->exc_cls - 1] = 0;
  strncpy(m->exc_msg, msg ? msg : "", sizeof m->exc_msg - 1);
  m->exc_msg[sizeof m->exc_msg - 1] = 0;
}

static jclass JNICALL FindClass(JNIEnv* env, const char* name) {
  entry(env);
  jobject c = new_obj(K_CLASS);
  if (c) c->name = strdup(name);
  return c;
}

static jint JNICALL ThrowNew(JNIEnv* env, jclass clazz, const char* msg) {
  entry(env);
  if (!clazz || clazz->kind != K_CLASS) {
    violation();
    return -1;
  }
  throw_(env, clazz->name, msg);
  return 0;
}

static jboolean JNICALL ExceptionCheck(JNIEnv* env) { return menv(env)->pending ? JNI_TRUE : JNI_FALSE; }

static void JNICALL DeleteLocalRef(JNIEnv* env, jobject obj) {
  (void)env, (void)obj;
  pthread_mutex_lock(&g_mu);
  g_local_deletes++;
  pthread_mutex_unlock(&g_mu);
}

static jsize JNICALL GetArrayLength(JNIEnv* env, jarray a) {
  entry(env);
  if (!a || (a->kind != K_DARRAY && a->kind != K_OARRAY)) {
    violation();
    return 0;
  }
  return a->len;
}

static jobjectArray JNICALL NewObjectArray(JNIEnv* env, jsize len, jclass clazz, jobject init) {
  entry(env);
  if (len < 0 || !clazz || clazz->kind != K_CLASS) {
    violation();
    return NULL;
  }
  jobject a = new_obj(K_OARRAY);
  if (!a) return NULL;
  a->len = len;
  a->elems = calloc((size_t)(len ? len : 1), sizeof(jobject));
  a->name = strdup(clazz->name);
  for (jsize i = 0; i < len; ++i) a->elems[i] = init;
  return a;
}

static jobject JNICALL GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) {
  entry(env);
  if (!a || a->kind != K_OARRAY) {
    violation();
    return NULL;
  }
  if (i < 0 || i >= a->len) {
    throw_(env, "java/lang/ArrayIndexOutOfBoundsException", "GetObjectArrayElement");
    return NULL;
  }
  return a->elems[i];
}

/* the class an element of this kind has, as a JVM descriptor */
static const char* class_of(jobject o) {
  if (!o) return NULL;
  if (o->kind == K_DARRAY) return "[D";
  if (o->kind == K_OARRAY) return NULL; /* "[" + element class, compared below */
  return "";
}

static void JNICALL SetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i, jobject v) {
  entry(env);
  if (!a || a->kind != K_OARRAY) {
    violation();
    return;
  }
  if (i < 0 || i >= a->len) {
    throw_(env, "java/lang/ArrayIndexOutOfBoundsException", "SetObjectArrayElement");
    return;
  }
  if (v) { /* ArrayStoreException unless the element's class is the array's element class */
    int ok;
    if (v->kind == K_OARRAY) {
      ok = a->name[0] == '[' && strcmp(a->name + 1, v->name) == 0;
    } else {
      const char* c = class_of(v);
      ok = c && strcmp(a->name, c) == 0;
    }
    if (!ok) {
      throw_(env, "java/lang/ArrayStoreException", a->name);
      return;
    }
  }
  a->elems[i] = v;
}

static jdoubleArray JNICALL NewDoubleArray(JNIEnv* env, jsize len) {
  entry(env);
  if (len < 0) {
    throw_(env, "java/lang/NegativeArraySizeException", "NewDoubleArray");
    return NULL;
  }
  jobject a = new_obj(K_DARRAY);
  if (!a) return NULL;
  a->len = len;
  a->d = calloc((size_t)(len ? len : 1), sizeof(double));
  return a;
}

static int region_ok(JNIEnv* env, jdoubleArray a, jsize start, jsize len) {
  if (!a || a->kind != K_DARRAY) {
    violation();
    return 0;
  }
  if (start < 0 || len < 0 || start > a->len - len) {
    throw_(env, "java/lang/ArrayIndexOutOfBoundsException", "double array region");
    return 0;
  }
  return 1;
}

static void JNICALL GetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len,
                                         jdouble* buf) {
  entry(env);
  if (region_ok(env, a, start, len) && len) memcpy(buf, a->d + start, sizeof(double) * (size_t)len);
}

static void JNICALL SetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len,
                                         const jdouble* buf) {
  entry(env);
  if (region_ok(env, a, start, len) && len) memcpy(a->d + start, buf, sizeof(double) * (size_t)len);
}

static jstring JNICALL NewStringUTF(JNIEnv* env, const char* utf) {
  entry(env);
  jobject s = new_obj(K_STRING);
  if (s) s->name = strdup(utf ? utf : "");
  return s;
}

static void* JNICALL GetDirectBufferAddress(JNIEnv* env, jobject buf) {
  entry(env);
  return buf && buf->kind == K_DIRECT ? buf->addr : NULL; /* NULL: not a direct buffer (JNI) */
}

static jlong JNICALL GetDirectBufferCapacity(JNIEnv* env, jobject buf) {
  entry(env);
  return buf && buf->kind == K_DIRECT ? buf->cap : -1;
}

static const struct JNINativeInterface_ kFns = {
    FindClass,      ThrowNew,       ExceptionCheck, DeleteLocalRef,         GetArrayLength,
    NewObjectArray, GetObjectArrayElement, SetObjectArrayElement, NewDoubleArray,
    GetDoubleArrayRegion, SetDoubleArrayRegion, NewStringUTF, GetDirectBufferAddress,
    GetDirectBufferCapacity,
};

/* ------------------------------------------------------------ harness API (ctypes) */
JNIEXPORT JNIEnv* mock_env_new(void) {
  MockEnv* m = calloc(1, sizeof *m);
  if (!m) return NULL;
  m->fns = &kFns;
  return (JNIEnv*)m;
}

JNIEXPORT void mock_env_free(JNIEnv* env) { free(env); }

/* frees every object made so far (by the glue or the test) */
JNIEXPORT void mock_reset(void) {
  pthread_mutex_lock(&g_mu);
  struct _jobject* o = g_objs;
  g_objs = NULL;
  g_violations = 0;
  pthread_mutex_unlock(&g_mu);
  while (o) {
    struct _jobject* nx = o->next_alloc;
    free(o->d), free(o->elems), free(o->name), free(o);
    o = nx;
  }
}

JNIEXPORT int mock_violations(void) { return g_violations; }

JNIEXPORT jobject mock_darray(const double* data, jsize n) {
  jobject a = new_obj(K_DARRAY);
  if (!a) return NULL;
  a->len = n;
  a->d = calloc((size_t)(n ? n : 1), sizeof(double));
  if (data && n) memcpy(a->d, data, sizeof(double) * (size_t)n);
  return a;
}

/* Object[] of element class elem ("[D" for double[][], "[[D" for double[][][]) */
JNIEXPORT jobject mock_oarray(jsize n, const char* elem) {
  jobject a = new_obj(K_OARRAY);
  if (!a) return NULL;
  a->len = n;
  a->elems = calloc((size_t)(n ? n : 1), sizeof(jobject));
  a->name = strdup(elem); /* an Object[]'s name is its element class, as NewObjectArray's */
  return a;
}

JNIEXPORT void mock_oset(jobject a, jsize i, jobject e) { a->elems[i] = e; }
JNIEXPORT jobject mock_oget(jobject a, jsize i) { return a && i < a->len ? a->elems[i] : NULL; }

JNIEXPORT jobject mock_direct(void* addr, jlong cap) {
  jobject b = new_obj(K_DIRECT);
  if (!b) return NULL;
  b->addr = addr;
  b->cap = cap;
  return b;
}

/* -1 for null, else the array length */
JNIEXPORT jsize mock_length(jobject a) { return a ? a->len : -1; }
JNIEXPORT int mock_kind(jobject o) { return o ? o->kind : 0; }
JNIEXPORT const char* mock_text(jobject o) { return o && o->name ? o->name : ""; }

JNIEXPORT int mock_darray_read(jobject a, double* out) {
  if (!a || a->kind != K_DARRAY) return -1;
  if (a->len) memcpy(out, a->d, sizeof(double) * (size_t)a->len);
  return 0;
}

/* 1 and the class / message when an exception is pending (and clears it), else 0 */
JNIEXPORT int mock_exception(JNIEnv* env, char* cls, int ncls, char* msg, int nmsg) {
  MockEnv* m = menv(env);
  if (!m->pending) return 0;
  strncpy(cls, m->exc_cls, (size_t)ncls - 1);
  cls[ncls - 1] = 0;
  strncpy(msg, m->exc_msg, (size_t)nmsg - 1);
  msg[nmsg - 1] = 0;
  m->pending = 0;
  return 1;
}
