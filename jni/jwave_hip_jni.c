/* jwave_hip_jni.c -- JNI glue binding the C-ABI of libjwave_hip.so (include/jwave_hip.h) as the
 * native methods of the drop-in subclasses in java/jwave/hip/ (INTEGRATION.md).
 *
 * Build (needs a JDK; none exists in this image, so it is not compiled here):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       jni/jwave_hip_jni.c -Ljwave-pro_amd -ljwave_hip -Wl,-rpath,'$ORIGIN' \
 *       -o libjwave_hip_jni.so
 *
 * Rules the glue keeps:
 *  * no JVM array is pinned across a HIP call: Java arrays are copied into / out of C buffers
 *    with Get/Set<Type>ArrayRegion (a GC may run while the GPU works); batched callers pass
 *    direct NIO buffers, whose addresses go to the engine as they are (JW_HOST staging);
 *  * every status maps to the exception class the reference throws, with
 *    jw_last_error()'s text, which is the reference's message where one exists;
 *  * plans are immutable and shared by all threads of a transform object; the Java side frees
 *    them only after in-flight calls finish (a reference count, see HipMODWTTransform). */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "jwave_hip.h"

static void jw_throw(JNIEnv* env, int st) {
  const char* cls = st == JW_ERR_ILLEGAL_ARGUMENT ? "java/lang/IllegalArgumentException"
                    : st == JW_ERR_FAILURE        ? "jwave/exceptions/JWaveFailure"
                    : st == JW_ERR_NO_MEMORY      ? "java/lang/OutOfMemoryError"
                    : st == JW_ERR_UNSUPPORTED    ? "java/lang/UnsupportedOperationException"
                                                  : "jwave/exceptions/JWaveError";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, jw_last_error());
}

static void oom(JNIEnv* env) {
  jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
  if (c) (*env)->ThrowNew(env, c, "jwave_hip_jni: host buffer");
}

/* double[] -> malloc'd copy (NULL + pending exception on failure) */
static double* copy_in(JNIEnv* env, jdoubleArray a, jsize* n_out) {
  const jsize n = a ? (*env)->GetArrayLength(env, a) : 0;
  double* p = malloc(sizeof(double) * (size_t)(n ? n : 1));
  if (!p) {
    oom(env);
    return NULL;
  }
  if (n) (*env)->GetDoubleArrayRegion(env, a, 0, n, p);
  if (n_out) *n_out = n;
  return p;
}

/* rows x n doubles -> double[rows][n] */
static jobjectArray rows_out(JNIEnv* env, const double* c, jsize rows, jsize n) {
  jclass dcls = (*env)->FindClass(env, "[D");
  jobjectArray out = (*env)->NewObjectArray(env, rows, dcls, NULL);
  if (!out) return NULL;
  for (jsize r = 0; r < rows; ++r) {
    jdoubleArray row = (*env)->NewDoubleArray(env, n);
    if (!row) return NULL;
    (*env)->SetDoubleArrayRegion(env, row, 0, n, c + (size_t)r * n);
    (*env)->SetObjectArrayElement(env, out, r, row);
    (*env)->DeleteLocalRef(env, row);
  }
  return out;
}

static void iae(JNIEnv* env, const char* msg) {
  jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (c) (*env)->ThrowNew(env, c, msg);
}

/* double[rows][n] -> rows x n doubles; every row must have length n.  An empty outer array
 * gives rows = n = 0 and a 1-element buffer (the engine treats n == 0 as a no-op). */
static double* rows_in(JNIEnv* env, jobjectArray a, jsize* rows_out_, jsize* n_out) {
  const jsize R = a ? (*env)->GetArrayLength(env, a) : 0;
  jsize n = 0;
  if (R > 0) {
    jdoubleArray r0 = (jdoubleArray)(*env)->GetObjectArrayElement(env, a, 0);
    if ((*env)->ExceptionCheck(env)) return NULL;
    n = r0 ? (*env)->GetArrayLength(env, r0) : 0;
    if (r0) (*env)->DeleteLocalRef(env, r0);
  }
  double* c = malloc(sizeof(double) * (size_t)(R ? R : 1) * (n ? n : 1));
  if (!c) {
    oom(env);
    return NULL;
  }
  for (jsize r = 0; r < R; ++r) {
    jdoubleArray row = (jdoubleArray)(*env)->GetObjectArrayElement(env, a, r);
    if (!row || (*env)->GetArrayLength(env, row) != n) {
      free(c);
      jclass e = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
      if (e) (*env)->ThrowNew(env, e, "Coefficient rows must all have the same length");
      return NULL;
    }
    (*env)->GetDoubleArrayRegion(env, row, 0, n, c + (size_t)r * n);
    (*env)->DeleteLocalRef(env, row);
  }
  *rows_out_ = R;
  *n_out = n;
  return c;
}

/* Direct NIO buffer of at least `doubles` doubles (capacity in bytes), or NULL with an
 * IllegalArgumentException pending.  The buffer's position is ignored (the engine reads from
 * its base address) and its contents must be in native byte order: HipMODWTTransform checks
 * both on the Java side. */
static void* direct_buffer(JNIEnv* env, jobject buf, long long doubles, const char* what) {
  void* p = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
  if (!p) {
    iae(env, "direct ByteBuffers required");
    return NULL;
  }
  const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
  if (cap < 0 || (long long)cap / (long long)sizeof(double) < doubles) {
    char msg[160];
    snprintf(msg, sizeof msg, "%s buffer holds %lld bytes, %lld doubles needed", what,
             (long long)cap, doubles);
    iae(env, msg);
    return NULL;
  }
  return p;
}

/* ---------------------------------------------------------------- device selection */
JNIEXPORT jstring JNICALL Java_jwave_hip_HipEngine_nVersion(JNIEnv* env, jclass cls) {
  (void)cls;
  return (*env)->NewStringUTF(env, jw_version());
}

/* jw_set_device for the calling thread (every transform with a device ordinal calls it before
 * its native call, on the same thread) */
JNIEXPORT void JNICALL Java_jwave_hip_HipEngine_nSetDevice(JNIEnv* env, jclass cls, jint ordinal) {
  (void)cls;
  const int st = jw_set_device(ordinal);
  if (st != JW_OK) jw_throw(env, st);
}

JNIEXPORT jint JNICALL Java_jwave_hip_HipEngine_nDeviceCount(JNIEnv* env, jclass cls) {
  (void)env, (void)cls;
  int n = 0;
  (void)jw_device_count(&n);
  return n;
}

/* MODWTTransform.clearFilterCache's device side: every cached table (jw_release_caches) */
JNIEXPORT jlong JNICALL Java_jwave_hip_HipEngine_nReleaseCaches(JNIEnv* env, jclass cls) {
  (void)env, (void)cls;
  return (jlong)jw_release_caches();
}

/* ---------------------------------------------------------------- MODWT */
JNIEXPORT jlong JNICALL Java_jwave_hip_HipMODWTTransform_nPlanCreate(JNIEnv* env, jclass cls,
                                                                     jdoubleArray sD,
                                                                     jdoubleArray wD, jint thr,
                                                                     jint arith) {
  (void)cls;
  jsize L = 0, L2 = 0;
  double* s = copy_in(env, sD, &L);
  if (!s) return 0;
  double* w = copy_in(env, wD, &L2);
  if (!w) {
    free(s);
    return 0;
  }
  jw_modwt_plan* p = NULL;
  const int st = L == L2 ? jw_modwt_plan_create(&p, s, w, (int)L, thr, arith)
                         : jw_modwt_plan_create(&p, s, w, -1, thr, arith); /* -> message */
  free(s);
  free(w);
  if (st != JW_OK) {
    jw_throw(env, st);
    return 0;
  }
  return (jlong)(intptr_t)p;
}

JNIEXPORT void JNICALL Java_jwave_hip_HipMODWTTransform_nPlanDestroy(JNIEnv* env, jclass cls,
                                                                     jlong plan) {
  (void)env, (void)cls;
  jw_modwt_plan_destroy((jw_modwt_plan*)(intptr_t)plan);
}

/* forwardMODWT(double[] data, int maxLevel) -> double[maxLevel+1][n] (MODWTTransform.java:256) */
JNIEXPORT jobjectArray JNICALL Java_jwave_hip_HipMODWTTransform_nForward(
    JNIEnv* env, jclass cls, jlong plan, jdoubleArray x, jint J, jint method) {
  (void)cls;
  jsize n = 0;
  double* xs = copy_in(env, x, &n);
  if (!xs) return NULL;
  double* c = malloc(sizeof(double) * (size_t)(J > 0 ? J + 1 : 1) * (n ? n : 1));
  if (!c) {
    free(xs);
    oom(env);
    return NULL;
  }
  const int st = jw_modwt_forward((const jw_modwt_plan*)(intptr_t)plan, xs, c, (long)n, J, 1,
                                  method, JW_HOST, NULL);
  free(xs);
  jobjectArray out = st == JW_OK ? rows_out(env, c, J + 1, n) : NULL;
  free(c);
  if (st != JW_OK) jw_throw(env, st);
  return out;
}

/* inverseMODWT(double[][] coefficients) -> double[n] (MODWTTransform.java:337) */
JNIEXPORT jdoubleArray JNICALL Java_jwave_hip_HipMODWTTransform_nInverse(JNIEnv* env,
                                                                         jclass cls, jlong plan,
                                                                         jobjectArray coeffs,
                                                                         jint method) {
  (void)cls;
  /* null, no rows or one row (no level): new double[0], as MODWTTransform.java:338-346 */
  if (!coeffs || (*env)->GetArrayLength(env, coeffs) <= 1) return (*env)->NewDoubleArray(env, 0);
  jsize R = 0, n = 0;
  double* c = rows_in(env, coeffs, &R, &n);
  if (!c) return NULL;
  double* x = malloc(sizeof(double) * (size_t)(n ? n : 1));
  if (!x) {
    free(c);
    oom(env);
    return NULL;
  }
  const int st = jw_modwt_inverse((const jw_modwt_plan*)(intptr_t)plan, c, x, (long)n, R - 1, 1,
                                  method, JW_HOST, NULL);
  free(c);
  jdoubleArray out = NULL;
  if (st == JW_OK && (out = (*env)->NewDoubleArray(env, n)) != NULL)
    (*env)->SetDoubleArrayRegion(env, out, 0, n, x);
  free(x);
  if (st != JW_OK) jw_throw(env, st);
  return out;
}

/* Batched forward/inverse over direct NIO buffers (no copies on the JVM side):
 * x: batch*n doubles, coeffs: batch*(J+1)*n doubles, native byte order, position ignored.
 * Sizes are checked against the buffers' capacities before the engine touches them. */
static int direct_sizes_ok(JNIEnv* env, jlong n, jint J, jint batch) {
  if (n < 0 || J < 0 || batch < 0) {
    iae(env, "n, levels and batch must not be negative");
    return 0;
  }
  return 1;
}

JNIEXPORT void JNICALL Java_jwave_hip_HipMODWTTransform_nForwardDirect(
    JNIEnv* env, jclass cls, jlong plan, jobject xbuf, jobject cbuf, jlong n, jint J, jint batch,
    jint method) {
  (void)cls;
  if (!direct_sizes_ok(env, n, J, batch)) return;
  const double* x = (const double*)direct_buffer(env, xbuf, (long long)batch * n, "signal");
  if (!x) return;
  double* c = (double*)direct_buffer(env, cbuf, (long long)batch * (J + 1) * n, "coefficient");
  if (!c) return;
  const int st = jw_modwt_forward((const jw_modwt_plan*)(intptr_t)plan, x, c, (long)n, J, batch,
                                  method, JW_HOST, NULL);
  if (st != JW_OK) jw_throw(env, st);
}

JNIEXPORT void JNICALL Java_jwave_hip_HipMODWTTransform_nInverseDirect(
    JNIEnv* env, jclass cls, jlong plan, jobject cbuf, jobject xbuf, jlong n, jint J, jint batch,
    jint method) {
  (void)cls;
  if (!direct_sizes_ok(env, n, J, batch)) return;
  const double* c =
      (const double*)direct_buffer(env, cbuf, (long long)batch * (J + 1) * n, "coefficient");
  if (!c) return;
  double* x = (double*)direct_buffer(env, xbuf, (long long)batch * n, "signal");
  if (!x) return;
  const int st = jw_modwt_inverse((const jw_modwt_plan*)(intptr_t)plan, c, x, (long)n, J, batch,
                                  method, JW_HOST, NULL);
  if (st != JW_OK) jw_throw(env, st);
}

/* ---------------------------------------------------------------- FWT / WPT */
JNIEXPORT jlong JNICALL Java_jwave_hip_HipFastWaveletTransform_nPlanCreate(
    JNIEnv* env, jclass cls, jdoubleArray sD, jdoubleArray wD, jdoubleArray sR, jdoubleArray wR,
    jint motherWavelength, jint transformWavelength, jint kind, jint arith) {
  (void)cls;
  double *a = copy_in(env, sD, NULL), *b = a ? copy_in(env, wD, NULL) : NULL;
  double *c = b ? copy_in(env, sR, NULL) : NULL, *d = c ? copy_in(env, wR, NULL) : NULL;
  jw_fwt_plan* p = NULL;
  int st = JW_OK;
  if (d)
    st = jw_fwt_plan_create(&p, a, b, c, d, motherWavelength, transformWavelength, kind, arith);
  free(a), free(b), free(c), free(d);
  if (!d) return 0; /* exception pending */
  if (st != JW_OK) {
    jw_throw(env, st);
    return 0;
  }
  return (jlong)(intptr_t)p;
}

JNIEXPORT void JNICALL Java_jwave_hip_HipFastWaveletTransform_nPlanDestroy(JNIEnv* env, jclass cls,
                                                                           jlong plan) {
  (void)env, (void)cls;
  jw_fwt_plan_destroy((jw_fwt_plan*)(intptr_t)plan);
}

/* op: 0 fwt forward, 1 fwt reverse, 2 wpt forward, 3 wpt reverse (double[] arrTime, level) */
JNIEXPORT jdoubleArray JNICALL Java_jwave_hip_HipFastWaveletTransform_nLine(
    JNIEnv* env, jclass cls, jlong plan, jint op, jdoubleArray in, jint level) {
  (void)cls;
  jsize n = 0;
  double* x = copy_in(env, in, &n);
  if (!x) return NULL;
  double* y = malloc(sizeof(double) * (size_t)(n ? n : 1));
  if (!y) {
    free(x);
    oom(env);
    return NULL;
  }
  const jw_fwt_plan* p = (const jw_fwt_plan*)(intptr_t)plan;
  int st;
  switch (op) {
    case 0: st = jw_fwt_forward(p, x, y, (long)n, level, 1, JW_HOST, NULL); break;
    case 1: st = jw_fwt_reverse(p, x, y, (long)n, level, 1, JW_HOST, NULL); break;
    case 2: st = jw_wpt_forward(p, x, y, (long)n, level, 1, JW_HOST, NULL); break;
    default: st = jw_wpt_reverse(p, x, y, (long)n, level, 1, JW_HOST, NULL); break;
  }
  free(x);
  jdoubleArray out = NULL;
  if (st == JW_OK && (out = (*env)->NewDoubleArray(env, n)) != NULL)
    (*env)->SetDoubleArrayRegion(env, out, 0, n, y);
  free(y);
  if (st != JW_OK) jw_throw(env, st);
  return out;
}

/* 2-D: op 0 forward, 1 reverse (double[][] matTime, lvlM, lvlN), BasicTransform.java:361/:436 */
JNIEXPORT jobjectArray JNICALL Java_jwave_hip_HipFastWaveletTransform_nMatrix(
    JNIEnv* env, jclass cls, jlong plan, jint op, jobjectArray in, jint lvlM, jint lvlN) {
  (void)cls;
  jsize rows = 0, cols = 0;
  double* x = rows_in(env, in, &rows, &cols);
  if (!x) return NULL;
  double* y = malloc(sizeof(double) * (size_t)rows * (cols ? cols : 1));
  if (!y) {
    free(x);
    oom(env);
    return NULL;
  }
  const jw_fwt_plan* p = (const jw_fwt_plan*)(intptr_t)plan;
  const int st = op == 0 ? jw_fwt2d_forward(p, x, y, rows, cols, lvlM, lvlN, 1, JW_HOST, NULL)
                         : jw_fwt2d_reverse(p, x, y, rows, cols, lvlM, lvlN, 1, JW_HOST, NULL);
  free(x);
  jobjectArray out = st == JW_OK ? rows_out(env, y, rows, cols) : NULL;
  free(y);
  if (st != JW_OK) jw_throw(env, st);
  return out;
}

/* The exceptions the reference's own array indexing throws (the JVM's messages). */
static void npe(JNIEnv* env) {
  jclass c = (*env)->FindClass(env, "java/lang/NullPointerException");
  if (c) (*env)->ThrowNew(env, c, NULL);
}
static void aioobe(JNIEnv* env, jsize index, jsize length) {
  char msg[96];
  snprintf(msg, sizeof msg, "Index %d out of bounds for length %d", (int)index, (int)length);
  jclass c = (*env)->FindClass(env, "java/lang/ArrayIndexOutOfBoundsException");
  if (c) (*env)->ThrowNew(env, c, msg);
}

/* Box [0, d2) x [0, d3) of one slab into dst, read the way BasicTransform.java:518-528 reads
 * spcTime[i][j][k]: a null slab or row throws NullPointerException, one shorter than the box
 * ArrayIndexOutOfBoundsException, and anything past the box is ignored.  0 = exception pending. */
static int slab_in(JNIEnv* env, jobjectArray m, jsize d2, jsize d3, double* dst) {
  if (d2 == 0 || d3 == 0) return 1;  /* the copy loops never index spcTime[i]: nothing to read */
  if (!m) {
    npe(env);
    return 0;
  }
  const jsize r = (*env)->GetArrayLength(env, m);
  for (jsize j = 0; j < d2 && d3 > 0; ++j) {
    if (j >= r) {
      aioobe(env, j, r);
      return 0;
    }
    jdoubleArray row = (jdoubleArray)(*env)->GetObjectArrayElement(env, m, j);
    if ((*env)->ExceptionCheck(env)) return 0;
    if (!row) {
      npe(env);
      return 0;
    }
    const jsize c = (*env)->GetArrayLength(env, row);
    if (c < d3) aioobe(env, c, c);
    else (*env)->GetDoubleArrayRegion(env, row, 0, d3, dst + (size_t)j * d3);
    (*env)->DeleteLocalRef(env, row);
    if (c < d3) return 0;
  }
  return 1;
}

/* 3-D: op 0 forward, 1 reverse (double[][][] spc, lvlP, lvlQ, lvlR), BasicTransform.java:509/:602.
 * The shape is slab 0's (noOfRows = spc.length, noOfCols = spc[0].length, noOfHigh =
 * spc[0][0].length, :512-514 / :605-607), every slab is read over that box (slab_in). */
JNIEXPORT jobjectArray JNICALL Java_jwave_hip_HipFastWaveletTransform_nSpace(
    JNIEnv* env, jclass cls, jlong plan, jint op, jobjectArray in, jint lvlP, jint lvlQ,
    jint lvlR) {
  (void)cls;
  if (!in) {  // spcTime.length
    npe(env);
    return NULL;
  }
  const jsize d1 = (*env)->GetArrayLength(env, in);
  if (d1 == 0) {  // spcTime[0]
    aioobe(env, 0, 0);
    return NULL;
  }
  jobjectArray m0 = (jobjectArray)(*env)->GetObjectArrayElement(env, in, 0);
  if ((*env)->ExceptionCheck(env)) return NULL;
  if (!m0) {  // spcTime[0].length
    npe(env);
    return NULL;
  }
  const jsize d2 = (*env)->GetArrayLength(env, m0);
  if (d2 == 0) {  // spcTime[0][0]
    (*env)->DeleteLocalRef(env, m0);
    aioobe(env, 0, 0);
    return NULL;
  }
  jdoubleArray r00 = (jdoubleArray)(*env)->GetObjectArrayElement(env, m0, 0);
  (*env)->DeleteLocalRef(env, m0);
  if ((*env)->ExceptionCheck(env)) return NULL;
  if (!r00) {  // spcTime[0][0].length
    npe(env);
    return NULL;
  }
  const jsize d3 = (*env)->GetArrayLength(env, r00);
  (*env)->DeleteLocalRef(env, r00);
  const size_t slab = (size_t)d2 * d3;
  double* x = malloc(sizeof(double) * (size_t)d1 * (slab ? slab : 1));
  if (!x) {
    oom(env);
    return NULL;
  }
  for (jsize i = 0; i < d1; ++i) {
    jobjectArray m = (jobjectArray)(*env)->GetObjectArrayElement(env, in, i);
    if ((*env)->ExceptionCheck(env)) {
      free(x);
      return NULL;
    }
    const int ok = slab_in(env, m, d2, d3, x + (size_t)i * slab);
    if (m) (*env)->DeleteLocalRef(env, m);
    if (!ok) {
      free(x);
      return NULL;
    }
    if (i == 0) {
      /* the reference runs slab 0's 2-D transform (:530 / :623), which checks lvlP and lvlQ,
       * before it reads slab 1: a level error wins over a malformed later slab.  batch 0 =
       * the 2-D entry's checks only, in its order (the 3-D entry's for those two levels). */
      const jw_fwt_plan* p0 = (const jw_fwt_plan*)(intptr_t)plan;
      const int lv = op == 0
                         ? jw_fwt2d_forward(p0, NULL, NULL, d2, d3, lvlP, lvlQ, 0, JW_HOST, NULL)
                         : jw_fwt2d_reverse(p0, NULL, NULL, d2, d3, lvlP, lvlQ, 0, JW_HOST, NULL);
      if (lv != JW_OK) {
        free(x);
        jw_throw(env, lv);
        return NULL;
      }
    }
  }
  double* y = malloc(sizeof(double) * (size_t)d1 * (slab ? slab : 1));
  if (!y) {
    free(x);
    oom(env);
    return NULL;
  }
  const jw_fwt_plan* p = (const jw_fwt_plan*)(intptr_t)plan;
  const int st = op == 0 ? jw_fwt3d_forward(p, x, y, d1, d2, d3, lvlP, lvlQ, lvlR, 1, JW_HOST, NULL)
                         : jw_fwt3d_reverse(p, x, y, d1, d2, d3, lvlP, lvlQ, lvlR, 1, JW_HOST, NULL);
  free(x);
  jobjectArray out = NULL;
  if (st == JW_OK) {
    jclass mcls = (*env)->FindClass(env, "[[D");
    out = mcls ? (*env)->NewObjectArray(env, d1, mcls, NULL) : NULL;
    for (jsize i = 0; out && i < d1; ++i) {
      jobjectArray m = rows_out(env, y + (size_t)i * slab, d2, d3);
      if (!m) {
        out = NULL;
        break;
      }
      (*env)->SetObjectArrayElement(env, out, i, m);
      (*env)->DeleteLocalRef(env, m);
    }
  }
  free(y);
  if (st != JW_OK) jw_throw(env, st);
  return out;
}

/* ---------------------------------------------------------------- CWT */
/* kind: JW_CWT_*; params: the wavelet's parameter block; padding: PaddingType.ordinal().
 * Returns double[ns][2n] rows of interleaved (re, im); the Java side builds Complex[][]. */
JNIEXPORT jobjectArray JNICALL Java_jwave_hip_HipContinuousWaveletTransform_nTransformFFT(
    JNIEnv* env, jclass cls, jint kind, jdoubleArray params, jdoubleArray x, jdoubleArray scales,
    jdouble fs, jint padding) {
  (void)cls;
  jsize n = 0, ns = 0;
  double* pr = copy_in(env, params, NULL);
  double* xs = pr ? copy_in(env, x, &n) : NULL;
  double* sc = xs ? copy_in(env, scales, &ns) : NULL;
  double* out = sc ? malloc(sizeof(double) * 2 * (size_t)(ns ? ns : 1) * (n ? n : 1)) : NULL;
  if (!out) {
    if (sc) oom(env);
    free(pr), free(xs), free(sc);
    return NULL;
  }
  const int st = jw_cwt_fft(kind, pr, xs, (long)n, sc, ns, fs, padding, out, 1, JW_HOST, NULL);
  free(pr), free(xs), free(sc);
  jobjectArray rows = st == JW_OK ? rows_out(env, out, ns, 2 * n) : NULL;
  free(out);
  if (st != JW_OK) jw_throw(env, st);
  return rows;
}

/* transformFFT(...).getScalogram() without the coefficients crossing PCIe: double[ns] */
JNIEXPORT jdoubleArray JNICALL Java_jwave_hip_HipContinuousWaveletTransform_nScalogramFFT(
    JNIEnv* env, jclass cls, jint kind, jdoubleArray params, jdoubleArray x, jdoubleArray scales,
    jdouble fs, jint padding) {
  (void)cls;
  jsize n = 0, ns = 0;
  double* pr = copy_in(env, params, NULL);
  double* xs = pr ? copy_in(env, x, &n) : NULL;
  double* sc = xs ? copy_in(env, scales, &ns) : NULL;
  double* e = sc ? malloc(sizeof(double) * (size_t)(ns ? ns : 1)) : NULL;
  if (!e) {
    if (sc) oom(env);
    free(pr), free(xs), free(sc);
    return NULL;
  }
  const int st =
      jw_cwt_fft_scalogram(kind, pr, xs, (long)n, sc, ns, fs, padding, e, 1, JW_HOST, NULL);
  free(pr), free(xs), free(sc);
  jdoubleArray out = NULL;
  if (st == JW_OK) {
    out = (*env)->NewDoubleArray(env, ns);
    if (out) (*env)->SetDoubleArrayRegion(env, out, 0, ns, e);
  }
  free(e);
  if (st != JW_OK) jw_throw(env, st);
  return out;
}

/* the direct (time-domain) CWT, same shapes; arith: JW_ARITH_* */
JNIEXPORT jobjectArray JNICALL Java_jwave_hip_HipContinuousWaveletTransform_nTransformDirect(
    JNIEnv* env, jclass cls, jint kind, jdoubleArray params, jdoubleArray x, jdoubleArray scales,
    jdouble fs, jint arith) {
  (void)cls;
  jsize n = 0, ns = 0;
  double* pr = copy_in(env, params, NULL);
  double* xs = pr ? copy_in(env, x, &n) : NULL;
  double* sc = xs ? copy_in(env, scales, &ns) : NULL;
  double* out = sc ? malloc(sizeof(double) * 2 * (size_t)(ns ? ns : 1) * (n ? n : 1)) : NULL;
  if (!out) {
    if (sc) oom(env);
    free(pr), free(xs), free(sc);
    return NULL;
  }
  const int st = jw_cwt_direct(kind, pr, xs, (long)n, sc, ns, fs, arith, out, 1, JW_HOST, NULL);
  free(pr), free(xs), free(sc);
  jobjectArray rows = st == JW_OK ? rows_out(env, out, ns, 2 * n) : NULL;
  free(out);
  if (st != JW_OK) jw_throw(env, st);
  return rows;
}

/* ---------------------------------------------------------------- FFT */
/* FastFourierTransform.forward/reverse(Complex[]) on interleaved (re, im) doubles:
 * dir 0 forward, 1 reverse (with the reference's 1/n); arith JW_ARITH_STRICT runs the
 * reference's own algorithm (bit-identical for power-of-two lengths). */
JNIEXPORT jdoubleArray JNICALL Java_jwave_hip_HipFastFourierTransform_nFFT(JNIEnv* env,
                                                                           jclass cls,
                                                                           jdoubleArray reim,
                                                                           jint dir, jint arith) {
  (void)cls;
  jsize m = 0;
  double* in = copy_in(env, reim, &m);
  if (!in) return NULL;
  double* out = malloc(sizeof(double) * (size_t)(m ? m : 1));
  if (!out) {
    free(in);
    oom(env);
    return NULL;
  }
  const long n = (long)m / 2;
  const int st = dir == 0 ? jw_fft_forward_ex(in, out, n, 1, arith, JW_HOST, NULL)
                          : jw_fft_reverse_ex(in, out, n, 1, arith, JW_HOST, NULL);
  free(in);
  jdoubleArray res = NULL;
  if (st == JW_OK && (res = (*env)->NewDoubleArray(env, m)) != NULL)
    (*env)->SetDoubleArrayRegion(env, res, 0, m, out);
  free(out);
  if (st != JW_OK) jw_throw(env, st);
  return res;
}
