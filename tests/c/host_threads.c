/* host_threads.c -- the JW_HOST path as a JVM drives it: 8 threads at once, one shared plan
 * (MODWTThreadSafetyTest.java:23-104 pattern: concurrent forwardMODWT / inverseMODWT on one
 * MODWTTransform), each thread with its own signals and lengths, host arrays in and out.
 * Every result is checked bit for bit against the oracle (JW_ARITH_STRICT), so staging-buffer
 * reuse across threads, stream ordering and the pinned pool are all exercised.
 * Built by tests/c/Makefile; run by tests/test_host_threads_gpu.py on the GPU box.
 * Exit status 0 = every comparison exact. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jwave_hip.h"
#include "jwave_oracle.h"

#define THREADS 8
#define ITERS 10

/* Daubechies-2-like 8-tap scaling filter and its quadrature mirror (any filter pair serves:
 * the check is engine vs oracle with the same taps). */
static const double kScal[8] = {0.2303778133088964, 0.7148465705529154, 0.6308807679298587,
                                -0.0279837694168599, -0.1870348117190931, 0.0308413818355607,
                                0.0328830116668852, -0.0105974017850690};
static double kWav[8];

static const jw_modwt_plan* g_plan;
static double g_g[8], g_h[8];
static int g_device = -1; /* argv[1]: every thread jw_set_device()s it first */

typedef struct {
  int id;
  int failures;
  char msg[256];
} job;

static int same_bits(const double* a, const double* b, size_t n) {
  return memcmp(a, b, n * sizeof(double)) == 0;
}

/* Every 5th call runs ConvolutionMethod.AUTO (JWave's default; power-of-two n, so the FFT
 * levels run the reference's own FFT and stay bit-exact against the oracle's AUTO path), and
 * thread 0 calls jw_release_caches() every 10th iteration while the others run -- the
 * MODWTThreadSafetyTest pattern with clearFilterCache() (MODWTThreadSafetyTest.java:53-54). */
static void* worker(void* arg) {
  job* jb = (job*)arg;
  if (g_device >= 0 && jw_set_device(g_device) != JW_OK) {
    jb->failures++;
    snprintf(jb->msg, sizeof jb->msg, "thread %d: jw_set_device(%d): %s", jb->id, g_device,
             jw_last_error());
    return NULL;
  }
  for (int it = 0; it < ITERS; ++it) {
    const int autom = it % 5 == 4;
    const long n = autom ? 4096L << (it % 3) : 4096 + 1000L * jb->id + 37L * it; /* distinct sizes */
    const int J = 3 + (jb->id + it) % 6;
    const int B = 1 + (it % 3);
    const int method = autom ? JW_CONV_AUTO : JW_CONV_DIRECT;
    if (jb->id == 0 && it % 10 == 9 && jw_release_caches() < 0) {
      jb->failures++;
      snprintf(jb->msg, sizeof jb->msg, "jw_release_caches failed: %s", jw_last_error());
    }
    double* x = malloc(sizeof(double) * n * B);
    double* c = malloc(sizeof(double) * n * (J + 1) * B);
    double* xr = malloc(sizeof(double) * n * B);
    double* cref = malloc(sizeof(double) * n * (J + 1));
    double* xref = malloc(sizeof(double) * n);
    for (int b = 0; b < B; ++b) jwo_fill_uniform(x + (size_t)b * n, n, 1000L * jb->id + 10L * it + b);
    int st = jw_modwt_forward(g_plan, x, c, n, J, B, method, JW_HOST, NULL);
    if (st == JW_OK) st = jw_modwt_inverse(g_plan, c, xr, n, J, B, method, JW_HOST, NULL);
    if (st != JW_OK) {
      jb->failures++;
      snprintf(jb->msg, sizeof jb->msg, "thread %d iter %d: status %d (%s)", jb->id, it, st,
               jw_last_error());
    } else {
      for (int b = 0; b < B; ++b) {
        if (autom) {
          jwo_modwt_forward_auto(x + (size_t)b * n, n, J, g_g, g_h, 8, 4096, cref);
          jwo_modwt_inverse_auto(c + (size_t)b * n * (J + 1), n, J, g_g, g_h, 8, 4096, xref);
        } else {
          jwo_modwt_forward_direct_nz(x + (size_t)b * n, n, J, g_g, g_h, 8, cref);
          jwo_modwt_inverse_direct_nz(cref, n, J, g_g, g_h, 8, xref);
        }
        if (!same_bits(c + (size_t)b * n * (J + 1), cref, (size_t)n * (J + 1)) ||
            !same_bits(xr + (size_t)b * n, xref, (size_t)n)) {
          jb->failures++;
          snprintf(jb->msg, sizeof jb->msg, "thread %d iter %d signal %d: mismatch (n=%ld J=%d)",
                   jb->id, it, b, n, J);
        }
      }
    }
    free(x), free(c), free(xr), free(cref), free(xref);
  }
  return NULL;
}

int main(int argc, char** argv) {
  if (argc > 1) g_device = atoi(argv[1]);
  for (int k = 0; k < 8; ++k) kWav[k] = (k & 1 ? -1.0 : 1.0) * kScal[7 - k];
  jw_modwt_plan* p = NULL;
  if (jw_modwt_plan_create(&p, kScal, kWav, 8, 4096, JW_ARITH_STRICT) != JW_OK) {
    fprintf(stderr, "plan: %s\n", jw_last_error());
    return 2;
  }
  g_plan = p;
  jw_modwt_plan_filters(p, g_g, g_h);
  double og[8], oh[8];
  jwo_modwt_filters(kScal, kWav, 8, og, oh);
  if (!same_bits(og, g_g, 8) || !same_bits(oh, g_h, 8)) {
    fprintf(stderr, "plan filters differ from the oracle's normalisation\n");
    return 1;
  }
  pthread_t th[THREADS];
  job jobs[THREADS];
  for (int i = 0; i < THREADS; ++i) {
    jobs[i].id = i;
    jobs[i].failures = 0;
    jobs[i].msg[0] = 0;
    pthread_create(&th[i], NULL, worker, &jobs[i]);
  }
  int fails = 0;
  for (int i = 0; i < THREADS; ++i) {
    pthread_join(th[i], NULL);
    fails += jobs[i].failures;
    if (jobs[i].failures) fprintf(stderr, "%s\n", jobs[i].msg);
  }
  jw_modwt_plan_destroy(p);
  printf("host_threads: %d threads x %d calls (device %d), %d failures\n", THREADS, ITERS,
         g_device, fails);
  return fails ? 1 : 0;
}
