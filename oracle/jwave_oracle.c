#define _GNU_SOURCE
/*
 * jwave_oracle.c -- TEST INFRASTRUCTURE ONLY (see jwave_oracle.h).
 *
 * Operation-for-operation restatement of JWave-Pro's hot path.  Compile with
 * -O2 -ffp-contract=off (oracle/Makefile): no FMA contraction, left-to-right
 * evaluation exactly as the Java expressions are written.  Every function cites
 * the reference lines it follows (paths relative to src/main/java/jwave/).
 *
 * JVM parity of the FFT paths (radix-2 twiddles, Bluestein chirps) rests on one assumption:
 * Math.sin / Math.cos return the correctly rounded value at every angle those paths take.  Java
 * specifies them to within 1 ulp only, so a JVM whose intrinsic misrounds an angle would differ
 * from this oracle (and from the engine, which takes the same correctly rounded values) in that
 * table entry.  The tests check engine against oracle, which share the assumption; no JVM exists
 * in this image to generate fixtures that would pin it, so for non-power-of-two lengths (up to
 * 2^23 chirp angles) "bit-identical to the JVM" means "under correctly rounded sin/cos".
 */
#include "jwave_oracle.h"

#include <math.h>
#include <quadmath.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define JAVA_PI 3.141592653589793 /* Math.PI */

/* ------------------------------------------------------------------------ */
/* java.util.Random (JDK 21 java/util/Random.java: constructor, next, nextDouble) */
/* ------------------------------------------------------------------------ */
#define LCG_A 0x5DEECE66DULL
#define LCG_C 0xBULL
#define LCG_MASK ((1ULL << 48) - 1)

void jwo_random_init(jwo_random* r, int64_t seed) {
  r->seed = ((uint64_t)seed ^ LCG_A) & LCG_MASK;
}

int32_t jwo_random_next(jwo_random* r, int bits) {
  r->seed = (r->seed * LCG_A + LCG_C) & LCG_MASK;
  return (int32_t)(r->seed >> (48 - bits));
}

double jwo_random_next_double(jwo_random* r) {
  int64_t hi = (int64_t)jwo_random_next(r, 26);
  int64_t lo = (int64_t)jwo_random_next(r, 27);
  return (double)((hi << 27) + lo) * 0x1.0p-53;
}

void jwo_fill_uniform(double* out, long n, int64_t seed) {
  jwo_random r;
  jwo_random_init(&r, seed);
  for (long i = 0; i < n; i++) out[i] = jwo_random_next_double(&r) * 2.0 - 1.0;
}

/* k-step LCG jump: s_k = A^k s + C_k (mod 2^48) by squaring the affine map. */
static uint64_t lcg_skip(uint64_t s, uint64_t k) {
  uint64_t a = LCG_A, c = LCG_C, acc_a = 1, acc_c = 0;
  while (k) {
    if (k & 1) { acc_a = (acc_a * a) & LCG_MASK; acc_c = (acc_c * a + c) & LCG_MASK; }
    c = (c * (a + 1)) & LCG_MASK;
    a = (a * a) & LCG_MASK;
    k >>= 1;
  }
  return (acc_a * s + acc_c) & LCG_MASK;
}

void jwo_fill_uniform_range(double* out, long start, long count, int64_t seed) {
  jwo_random r;
  jwo_random_init(&r, seed);
  r.seed = lcg_skip(r.seed, 2ULL * (uint64_t)start);
  for (long i = 0; i < count; i++) out[i] = jwo_random_next_double(&r) * 2.0 - 1.0;
}

/* ------------------------------------------------------------------------ */
/* MODWT filters: MODWTTransform.initializeFilterCache :452-484, normalize :599-606 */
/* ------------------------------------------------------------------------ */
static void java_normalize(double* f, int L) {
  double energy = 0.0;
  for (int i = 0; i < L; i++) energy += f[i] * f[i];
  double norm = sqrt(energy);
  if (norm > 1e-12)
    for (int i = 0; i < L; i++) f[i] /= norm;
}

void jwo_modwt_filters(const double* scal_dec, const double* wav_dec, int L, double* g, double* h) {
  double* gd = (double*)malloc(sizeof(double) * L);
  double* hd = (double*)malloc(sizeof(double) * L);
  memcpy(gd, scal_dec, sizeof(double) * L);
  memcpy(hd, wav_dec, sizeof(double) * L);
  java_normalize(gd, L);
  java_normalize(hd, L);
  double scale = sqrt(2.0);
  for (int i = 0; i < L; i++) {
    g[i] = gd[i] / scale;
    h[i] = hd[i] / scale;
  }
  free(gd);
  free(hd);
}

/* upsample :618-630 -- gap = 2^(level-1)-1 zeros between taps. */
long jwo_modwt_upsample(const double* base, int L, int level, double* out) {
  if (level <= 1) {
    memcpy(out, base, sizeof(double) * L);
    return L;
  }
  long gap = (1L << (level - 1)) - 1;
  long M = L + (long)(L - 1) * gap;
  memset(out, 0, sizeof(double) * M);
  for (int i = 0; i < L; i++) out[i * (gap + 1)] = base[i];
  return M;
}

static long floor_mod(long a, long n) { /* Math.floorMod */
  long r = a % n;
  return (r != 0 && ((r < 0) != (n < 0))) ? r + n : r;
}

/* circularConvolve :677-690 (all M taps, zeros included, floorMod). */
static void circ_conv(const double* s, long N, const double* f, long M, int L, double* out) {
  (void)L;
  for (long n = 0; n < N; n++) {
    double sum = 0.0;
    for (long m = 0; m < M; m++) sum += s[floor_mod(n - m, N)] * f[m];
    out[n] = sum;
  }
}

/* circularConvolveAdjoint :703-716. */
static void circ_conv_adj(const double* s, long N, const double* f, long M, int L,
                          double* out) {
  (void)L;
  for (long n = 0; n < N; n++) {
    double sum = 0.0;
    for (long m = 0; m < M; m++) sum += s[floor_mod(n + m, N)] * f[m];
    out[n] = sum;
  }
}

int jwo_modwt_auto_uses_fft(long N, long M, int threshold) {
  int32_t prod = (int32_t)((uint32_t)N * (uint32_t)M); /* Java int multiply wraps */
  return prod > threshold;
}

typedef void (*conv_fn)(const double*, long, const double*, long, int, double*);

static void modwt_forward(const double* x, long N, int J, const double* g, const double* h, int L,
                          double* coeffs, conv_fn conv) {
  long Mmax = (long)(L - 1) * (1L << (J - 1)) + 1;
  double* gu = (double*)malloc(sizeof(double) * Mmax);
  double* hu = (double*)malloc(sizeof(double) * Mmax);
  double* v = (double*)malloc(sizeof(double) * N);
  memcpy(v, x, sizeof(double) * N); /* vCurrent = copyOf(data) :288 */
  for (int j = 1; j <= J; j++) {    /* :290-304 */
    long M = jwo_modwt_upsample(g, L, j, gu);
    jwo_modwt_upsample(h, L, j, hu);
    conv(v, N, hu, M, L, coeffs + (long)(j - 1) * N); /* W_j */
    conv(v, N, gu, M, L, coeffs + (long)J * N);       /* V_j */
    memcpy(v, coeffs + (long)J * N, sizeof(double) * N);
  }
  free(gu); free(hu); free(v);
}

static void modwt_inverse(const double* coeffs, long N, int J, const double* g, const double* h,
                          int L, double* x, conv_fn conv_adj) {
  long Mmax = (long)(L - 1) * (1L << (J - 1)) + 1;
  double* gu = (double*)malloc(sizeof(double) * Mmax);
  double* hu = (double*)malloc(sizeof(double) * Mmax);
  double* va = (double*)malloc(sizeof(double) * N);
  double* vd = (double*)malloc(sizeof(double) * N);
  memcpy(x, coeffs + (long)J * N, sizeof(double) * N); /* :353 */
  for (int j = J; j >= 1; j--) {                        /* :355-372 */
    long M = jwo_modwt_upsample(g, L, j, gu);
    jwo_modwt_upsample(h, L, j, hu);
    conv_adj(x, N, gu, M, L, va);
    conv_adj(coeffs + (long)(j - 1) * N, N, hu, M, L, vd);
    for (long i = 0; i < N; i++) x[i] = va[i] + vd[i];
  }
  free(gu); free(hu); free(va); free(vd);
}

/* Same sums with the up-sampled zero taps skipped (x*0 = +-0 added to a running sum that is
 * never -0.0 leaves it bit-identical for finite x); tests pin it to the faithful version. */
static void circ_conv_nz_impl(const double* s, long N, const double* f, long M, int L,
                              double* out, int adj) {
  const long d = L > 1 ? (M - 1) / (L - 1) : 1; /* M = (L-1)*2^(j-1) + 1 */
  for (long n = 0; n < N; n++) {
    double sum = 0.0;
    for (int k = 0; k < L; k++) {
      long m = (long)k * d;
      sum += s[floor_mod(adj ? n + m : n - m, N)] * f[m];
    }
    out[n] = sum;
  }
}
static void circ_conv_nz(const double* s, long N, const double* f, long M, int L, double* out) {
  circ_conv_nz_impl(s, N, f, M, L, out, 0);
}
static void circ_conv_adj_nz(const double* s, long N, const double* f, long M, int L,
                             double* out) {
  circ_conv_nz_impl(s, N, f, M, L, out, 1);
}

void jwo_modwt_forward_direct_nz(const double* x, long N, int J, const double* g,
                                 const double* h, int L, double* coeffs) {
  modwt_forward(x, N, J, g, h, L, coeffs, circ_conv_nz);
}

void jwo_modwt_inverse_direct_nz(const double* coeffs, long N, int J, const double* g,
                                 const double* h, int L, double* x) {
  modwt_inverse(coeffs, N, J, g, h, L, x, circ_conv_adj_nz);
}

void jwo_modwt_forward_direct(const double* x, long N, int J, const double* g, const double* h,
                              int L, double* coeffs) {
  modwt_forward(x, N, J, g, h, L, coeffs, circ_conv);
}

void jwo_modwt_inverse_direct(const double* coeffs, long N, int J, const double* g,
                              const double* h, int L, double* x) {
  modwt_inverse(coeffs, N, J, g, h, L, x, circ_conv_adj);
}

/* ------------------------------------------------------------------------ */
/* FFT: FastFourierTransform.java forward/reverse :112-164, fftCooleyTukey :172-212,   */
/* fftCooleyTukeyInternal (no 1/n), fftBluestein :259-324.  Complex.mul :286-288.      */
/* ------------------------------------------------------------------------ */
/* Test switch: 1 = correctly rounded twiddles (cosl/sinl per butterfly index) instead of the
 * reference's recurrence wn = wn * w.  The GPU engine uses exact tables; comparing it with
 * both variants separates engine error from the reference's own twiddle drift. */
static int g_exact_twiddles = 0;
void jwo_set_exact_twiddles(int on) { g_exact_twiddles = on; }

/* Math.cos / Math.sin (:189-190, :269-271) restated as the correctly rounded values: Java
 * specifies them to 1 ulp and its implementations round correctly for all but a vanishing
 * fraction of arguments, while glibc's sin / cos / sincos each misround some (e.g. the chirp
 * of n = 2049).  Long double first; the quad-precision value where that cannot decide. */
static double cr_round(long double v, __float128 (*slow)(__float128), double x) {
  double d = (double)v;
  if (v == 0.0L || !isfinite(d)) return d;
  long double err = ldexpl(1.0L, ilogbl(v) - 63 + 4);
  long double ld = d;
  long double hi = (ld + (long double)nextafter(d, INFINITY)) / 2;
  long double lo = (ld + (long double)nextafter(d, -INFINITY)) / 2;
  if (fabsl(v - hi) > err && fabsl(v - lo) > err) return d;
  return (double)slow((__float128)x);
}
static void java_sincos(double x, double* s, double* c) {
  *s = cr_round(sinl((long double)x), sinq, x);
  *c = cr_round(cosl((long double)x), cosq, x);
}

static void fft_ct(double* x, long n, int inverse, int normalize) {
  int p = 0;
  while ((1L << p) < n) p++;
  for (long k = 0; k < n; k++) { /* bit reversal :176-184 */
    long j = 0;
    for (int b = 0; b < p; b++) j |= ((k >> b) & 1L) << (p - 1 - b);
    if (j > k) {
      double tr = x[2 * j], ti = x[2 * j + 1];
      x[2 * j] = x[2 * k]; x[2 * j + 1] = x[2 * k + 1];
      x[2 * k] = tr; x[2 * k + 1] = ti;
    }
  }
  for (long size = 2; size <= n; size *= 2) { /* :188-202 */
    double angle = 2 * JAVA_PI / (double)size * (inverse ? 1 : -1);
    double wr, wi;
    java_sincos(angle, &wi, &wr);
    long half = size / 2;
    double* tw = NULL; /* exact twiddles of this size, computed once (not per block) */
    if (g_exact_twiddles) {
      tw = (double*)malloc(sizeof(double) * 2 * half);
      for (long k = 0; k < half; k++) {
        const long double a = (long double)2 * 3.141592653589793238462643383279503L *
                              (long double)k / (long double)size * (inverse ? 1 : -1);
        tw[2 * k] = (double)cosl(a);
        tw[2 * k + 1] = (double)sinl(a);
      }
    }
    for (long start = 0; start < n; start += size) {
      double nr = 1, ni = 0; /* wn = (1,0) */
      for (long k = 0; k < half; k++) {
        if (tw) {
          nr = tw[2 * k];
          ni = tw[2 * k + 1];
        }
        double* u = x + 2 * (start + k);
        double* v = x + 2 * (start + k + half);
        double ur = u[0], ui = u[1];
        double tr = nr * v[0] - ni * v[1]; /* t = wn.mul(x[..]) */
        double ti = nr * v[1] + ni * v[0];
        u[0] = ur + tr; u[1] = ui + ti;
        v[0] = ur - tr; v[1] = ui - ti;
        double nnr = nr * wr - ni * wi; /* wn = wn.mul(w) */
        double nni = nr * wi + ni * wr;
        nr = nnr; ni = nni;
      }
    }
    free(tw);
  }
  if (inverse && normalize) { /* :207-211  x[i].mul(1.0/n) */
    double s = 1.0 / (double)n;
    for (long i = 0; i < n; i++) { x[2 * i] *= s; x[2 * i + 1] *= s; }
  }
}

static void fft_bluestein(double* x, long n, int inverse) {
  long m = 1;
  while (m < 2 * n - 1) m *= 2;
  double* chirp = (double*)malloc(sizeof(double) * 2 * n);
  double* a = (double*)calloc(2 * m, sizeof(double));
  double* b = (double*)calloc(2 * m, sizeof(double));
  /* one independent angle per index (:268-272); threads only share the work out */
#pragma omp parallel for schedule(static) if (n >= (1L << 16))
  for (long i = 0; i < n; i++) {
    double angle = JAVA_PI * (double)i * (double)i / (double)n * (inverse ? 1 : -1);
    java_sincos(angle, &chirp[2 * i + 1], &chirp[2 * i]);
  }
  for (long i = 0; i < n; i++) { /* a[i] = x[i].mul(chirp[i]) */
    double xr = x[2 * i], xi = x[2 * i + 1], cr = chirp[2 * i], ci = chirp[2 * i + 1];
    a[2 * i] = xr * cr - xi * ci;
    a[2 * i + 1] = xr * ci + xi * cr;
  }
  b[0] = chirp[0]; b[1] = -chirp[1];
  for (long i = 1; i < n; i++) {
    b[2 * i] = chirp[2 * i]; b[2 * i + 1] = -chirp[2 * i + 1];
    b[2 * (m - i)] = chirp[2 * i]; b[2 * (m - i) + 1] = -chirp[2 * i + 1];
  }
  fft_ct(a, m, 0, 0);
  fft_ct(b, m, 0, 0);
  for (long i = 0; i < m; i++) {
    double ar = a[2 * i], ai = a[2 * i + 1], br = b[2 * i], bi = b[2 * i + 1];
    a[2 * i] = ar * br - ai * bi;
    a[2 * i + 1] = ar * bi + ai * br;
  }
  fft_ct(a, m, 1, 0);
  double sm = 1.0 / (double)m;
  for (long i = 0; i < m; i++) { a[2 * i] *= sm; a[2 * i + 1] *= sm; }
  double sn = 1.0 / (double)n;
  for (long i = 0; i < n; i++) {
    double ar = a[2 * i], ai = a[2 * i + 1], cr = chirp[2 * i], ci = chirp[2 * i + 1];
    double rr = ar * cr - ai * ci, ri = ar * ci + ai * cr;
    if (inverse) { rr *= sn; ri *= sn; }
    x[2 * i] = rr; x[2 * i + 1] = ri;
  }
  free(chirp); free(a); free(b);
}

/* The twiddles one stage of fftCooleyTukey uses (:188-201): wn_k, k < size / 2, by the
 * recurrence wn = wn.mul(w) from (1, 0) -- the same in every block of the stage, and the same
 * whatever n (the angle is 2 pi / size).  Test helper: the last stage of an n-point transform
 * combines the n/2-point transforms of the even and odd samples with these. */
void jwo_fft_stage_twiddles(long size, int inverse, double* out) {
  double angle = 2 * JAVA_PI / (double)size * (inverse ? 1 : -1);
  double wr, wi;
  java_sincos(angle, &wi, &wr);
  double nr = 1, ni = 0;
  for (long k = 0; k < size / 2; k++) {
    out[2 * k] = nr;
    out[2 * k + 1] = ni;
    double nnr = nr * wr - ni * wi, nni = nr * wi + ni * wr;
    nr = nnr; ni = nni;
  }
}

void jwo_fft(double* reim, long n, int inverse) {
  if (n <= 1) return;
  if ((n & (n - 1)) == 0) fft_ct(reim, n, inverse, 1);
  else fft_bluestein(reim, n, inverse);
}

/* wrapFilterToSignalLength :729-741 */
static void wrap_filter(const double* f, long M, long N, double* p) {
  memset(p, 0, sizeof(double) * N);
  for (long i = 0; i < M; i++) p[i % N] += f[i];
}

/* circularConvolveFFT :752-786 and circularConvolveFFTAdjoint :798-837 */
static void fft_conv_impl(const double* s, long N, const double* f, long M, double* out, int adj) {
  double* sc = (double*)malloc(sizeof(double) * 2 * N);
  double* fc = (double*)malloc(sizeof(double) * 2 * N);
  double* p = (double*)malloc(sizeof(double) * N);
  wrap_filter(f, M, N, p);
  for (long i = 0; i < N; i++) {
    sc[2 * i] = s[i]; sc[2 * i + 1] = 0;
    fc[2 * i] = p[i]; fc[2 * i + 1] = 0;
  }
  jwo_fft(sc, N, 0);
  jwo_fft(fc, N, 0);
  for (long i = 0; i < N; i++) {
    double sr = sc[2 * i], si = sc[2 * i + 1], fr = fc[2 * i], fi = fc[2 * i + 1];
    if (adj) fi = -fi; /* filterFFT[i].conjugate() */
    sc[2 * i] = sr * fr - si * fi;
    sc[2 * i + 1] = sr * fi + si * fr;
  }
  jwo_fft(sc, N, 1);
  for (long i = 0; i < N; i++) out[i] = sc[2 * i];
  free(sc); free(fc); free(p);
}
static void fft_conv(const double* s, long N, const double* f, long M, int L, double* out) {
  (void)L;
  fft_conv_impl(s, N, f, M, out, 0);
}
static void fft_conv_adj(const double* s, long N, const double* f, long M, int L, double* out) {
  (void)L;
  fft_conv_impl(s, N, f, M, out, 1);
}

void jwo_modwt_forward_fft(const double* x, long N, int J, const double* g, const double* h,
                           int L, double* coeffs) {
  modwt_forward(x, N, J, g, h, L, coeffs, fft_conv);
}

void jwo_modwt_inverse_fft(const double* coeffs, long N, int J, const double* g,
                           const double* h, int L, double* x) {
  modwt_inverse(coeffs, N, J, g, h, L, x, fft_conv_adj);
}

/* performConvolution with ConvolutionMethod.AUTO (:640-664): per call, FFT when the int32
 * product signal.length * filter.length exceeds fftConvolutionThreshold, else DIRECT: the
 * faithful every-tap circularConvolve{,Adjoint}, so non-finite samples meet the zero taps as
 * in the reference (0 * Inf = NaN). */
static __thread int g_auto_threshold = 4096;
static void auto_conv(const double* s, long N, const double* f, long M, int L, double* out) {
  if (jwo_modwt_auto_uses_fft(N, M, g_auto_threshold)) fft_conv(s, N, f, M, L, out);
  else circ_conv(s, N, f, M, L, out);
}
static void auto_conv_adj(const double* s, long N, const double* f, long M, int L, double* out) {
  if (jwo_modwt_auto_uses_fft(N, M, g_auto_threshold)) fft_conv_adj(s, N, f, M, L, out);
  else circ_conv_adj(s, N, f, M, L, out);
}
void jwo_modwt_forward_auto(const double* x, long N, int J, const double* g, const double* h,
                            int L, int threshold, double* coeffs) {
  g_auto_threshold = threshold;
  modwt_forward(x, N, J, g, h, L, coeffs, auto_conv);
}
void jwo_modwt_inverse_auto(const double* coeffs, long N, int J, const double* g,
                            const double* h, int L, int threshold, double* x) {
  g_auto_threshold = threshold;
  modwt_inverse(coeffs, N, J, g, h, L, x, auto_conv_adj);
}

/* ------------------------------------------------------------------------ */
/* FWT: Wavelet.forward :236-260, Wavelet.reverse :277-303,                           */
/* Haar1Orthogonal.reverse :175-207 (x0.5), FastWaveletTransform.forward/reverse :71-153 */
/* ------------------------------------------------------------------------ */
void jwo_wavelet_forward(const double* in, int len, const double* sD, const double* wD, int M,
                         double* out) {
  int h = len >> 1;
  for (int i = 0; i < h; i++) {
    out[i] = out[i + h] = 0.;
    for (int j = 0; j < M; j++) {
      int k = (i << 1) + j;
      while (k >= len) k -= len;
      out[i] += in[k] * sD[j];
      out[i + h] += in[k] * wD[j];
    }
  }
}

void jwo_wavelet_reverse(const double* in, int len, const double* sR, const double* wR, int M,
                         int kind, double* out) {
  for (int i = 0; i < len; i++) out[i] = 0.;
  int h = len >> 1;
  for (int i = 0; i < h; i++) {
    for (int j = 0; j < M; j++) {
      int k = (i << 1) + j;
      while (k >= len) k -= len;
      if (kind == 1)
        out[k] += .5 * ((in[i] * sR[j]) + (in[i + h] * wR[j]));
      else
        out[k] += (in[i] * sR[j]) + (in[i + h] * wR[j]);
    }
  }
}

static int java_get_exponent(double f) { /* MathToolKit.getExponent :202-206 */
  return (int)(log(f) / log(2.));
}

void jwo_fwt_forward(const double* x, long n, int level, const double* sD, const double* wD,
                     int M, int tw, double* y) {
  double* tmp = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  memcpy(y, x, sizeof(double) * n);
  int l = 0;
  long h = n;
  while (h >= tw && l < level) {
    jwo_wavelet_forward(y, (int)h, sD, wD, M, tmp);
    memcpy(y, tmp, sizeof(double) * h);
    h = h >> 1;
    l++;
  }
  free(tmp);
}

void jwo_fwt_reverse(const double* y, long n, int level, const double* sR, const double* wR,
                     int M, int tw, int kind, double* x) {
  double* tmp = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  memcpy(x, y, sizeof(double) * n);
  long h = tw;
  int steps = java_get_exponent((double)n);
  for (int l = level; l < steps; l++) h = h << 1;
  while (h <= n && h >= tw) {
    jwo_wavelet_reverse(x, (int)h, sR, wR, M, kind, tmp);
    memcpy(x, tmp, sizeof(double) * h);
    h = h << 1;
  }
  free(tmp);
}

/* WaveletPacketTransform.forward :60-117 / reverse :119-191: every packet of the level */
void jwo_wpt_forward(const double* x, long n, int level, const double* sD, const double* wD,
                     int M, int tw, double* y) {
  double* tmp = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  memcpy(y, x, sizeof(double) * n);
  long k = n, h = n;
  int l = 0;
  while (h >= tw && l < level) {
    long g = k / h;
    for (long p = 0; p < g; p++) {
      jwo_wavelet_forward(y + p * h, (int)h, sD, wD, M, tmp);
      memcpy(y + p * h, tmp, sizeof(double) * h);
    }
    h = h >> 1;
    l++;
  }
  free(tmp);
}

void jwo_wpt_reverse(const double* y, long n, int level, const double* sR, const double* wR,
                     int M, int tw, int kind, double* x) {
  double* tmp = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  memcpy(x, y, sizeof(double) * n);
  long k = n, h = tw;
  int steps = java_get_exponent((double)n);
  for (int l = level; l < steps; l++) h = h << 1;
  while (h <= n && h >= tw) {
    long g = k / h;
    for (long p = 0; p < g; p++) {
      jwo_wavelet_reverse(x + p * h, (int)h, sR, wR, M, kind, tmp);
      memcpy(x + p * h, tmp, sizeof(double) * h);
    }
    h = h << 1;
  }
  free(tmp);
}

void jwo_fwt2d_forward(const double* x, int rows, int cols, int lvlM, int lvlN, const double* sD,
                       const double* wD, int M, int tw, double* y) {
  int mx = rows > cols ? rows : cols;
  double* a = (double*)malloc(sizeof(double) * mx);
  double* b = (double*)malloc(sizeof(double) * mx);
  for (int i = 0; i < rows; i++) jwo_fwt_forward(x + (long)i * cols, cols, lvlN, sD, wD, M, tw,
                                                  y + (long)i * cols);
  for (int j = 0; j < cols; j++) {
    for (int i = 0; i < rows; i++) a[i] = y[(long)i * cols + j];
    jwo_fwt_forward(a, rows, lvlM, sD, wD, M, tw, b);
    for (int i = 0; i < rows; i++) y[(long)i * cols + j] = b[i];
  }
  free(a); free(b);
}

void jwo_fwt2d_reverse(const double* y, int rows, int cols, int lvlM, int lvlN, const double* sR,
                       const double* wR, int M, int tw, int kind, double* x) {
  int mx = rows > cols ? rows : cols;
  double* a = (double*)malloc(sizeof(double) * mx);
  double* b = (double*)malloc(sizeof(double) * mx);
  for (int j = 0; j < cols; j++) {
    for (int i = 0; i < rows; i++) a[i] = y[(long)i * cols + j];
    jwo_fwt_reverse(a, rows, lvlM, sR, wR, M, tw, kind, b);
    for (int i = 0; i < rows; i++) x[(long)i * cols + j] = b[i];
  }
  for (int i = 0; i < rows; i++) {
    memcpy(a, x + (long)i * cols, sizeof(double) * cols);
    jwo_fwt_reverse(a, cols, lvlN, sR, wR, M, tw, kind, x + (long)i * cols);
  }
  free(a); free(b);
}

/* 3-D: BasicTransform.forward(double[][][], lvlP, lvlQ, lvlR) :509-565 -- the 2-D forward
 * of every slab i ([d2][d3]) with (lvlP, lvlQ), then the 1-D forward along i with lvlR;
 * reverse :602-659 -- the 2-D reverse of every slab, then the 1-D reverse along i. */
void jwo_fwt3d_forward(const double* x, int d1, int d2, int d3, int lvlP, int lvlQ, int lvlR,
                       const double* sD, const double* wD, int M, int tw, double* y) {
  const long slab = (long)d2 * d3;
  double* a = (double*)malloc(sizeof(double) * d1);
  double* b = (double*)malloc(sizeof(double) * d1);
  for (int i = 0; i < d1; i++)
    jwo_fwt2d_forward(x + i * slab, d2, d3, lvlP, lvlQ, sD, wD, M, tw, y + i * slab);
  for (long jk = 0; jk < slab; jk++) {
    for (int i = 0; i < d1; i++) a[i] = y[i * slab + jk];
    jwo_fwt_forward(a, d1, lvlR, sD, wD, M, tw, b);
    for (int i = 0; i < d1; i++) y[i * slab + jk] = b[i];
  }
  free(a); free(b);
}

void jwo_fwt3d_reverse(const double* y, int d1, int d2, int d3, int lvlP, int lvlQ, int lvlR,
                       const double* sR, const double* wR, int M, int tw, int kind, double* x) {
  const long slab = (long)d2 * d3;
  double* a = (double*)malloc(sizeof(double) * d1);
  double* b = (double*)malloc(sizeof(double) * d1);
  for (int i = 0; i < d1; i++)
    jwo_fwt2d_reverse(y + i * slab, d2, d3, lvlP, lvlQ, sR, wR, M, tw, kind, x + i * slab);
  for (long jk = 0; jk < slab; jk++) {
    for (int i = 0; i < d1; i++) a[i] = x[i * slab + jk];
    jwo_fwt_reverse(a, d1, lvlR, sR, wR, M, tw, kind, b);
    for (int i = 0; i < d1; i++) x[i * slab + jk] = b[i];
  }
  free(a); free(b);
}

/* ------------------------------------------------------------------------ */
/* CWT FFT path: ContinuousWaveletTransform.transformFFT :183-229, padSignal :269-306, */
/* createFrequencyAxis :450-459, ContinuousWavelet.fourierTransform :122-141,          */
/* MorletWavelet.fourierTransform :114-124, MexicanHatWavelet :65-119, Paul / DOG / Meyer. */
/* ------------------------------------------------------------------------ */
static double meyer_nu(double x) { /* MeyerWavelet.transitionFunction :279-295 */
  if (x <= 0) return 0.0;
  if (x >= 1) return 1.0;
  double x2 = x * x, x3 = x2 * x, x4 = x3 * x;
  return x4 * (35.0 + -84.0 * x + 70.0 * x2 + -20.0 * x3);
}

/* F[psi_{a,0}](omega) as (re, im).  Kinds: 0 Morlet {fb, fc}, 1 Mexican Hat {sigma},
 * 2 Paul {m} (PaulWavelet.java:76-99, override :152-164), 3 DOG {n, sigma}
 * (DOGWavelet.java:129-220, 357-382), 4 Meyer {} (MeyerWavelet.java:223-295). */
void jwo_cwt_wavelet_ft_c(int wavelet, const double* params, double omega, double scale,
                          double* re_out, double* im_out) {
  double w = scale * omega; /* fourierTransform(scale * omega) */
  double re = 0.0, im = 0.0;
  if (wavelet == 0) {
    double fb = params[0], fc = params[1];
    double f = w / (2.0 * JAVA_PI);
    double norm = sqrt(2.0 * JAVA_PI * fb);
    double exponent = -2.0 * JAVA_PI * JAVA_PI * fb * (f - fc) * (f - fc);
    re = norm * exp(exponent);
  } else if (wavelet == 1) {
    double sigma = params[0];
    double nc = 2.0 / (sqrt(3.0 * sigma) * pow(JAVA_PI, 0.25));
    double ftNorm = nc * sigma * sqrt(2.0 * JAVA_PI);
    double omega2 = w * w;
    re = ftNorm * omega2 * exp(-0.5 * sigma * sigma * omega2);
  } else if (wavelet == 2) { /* the override returns without a further sqrt(scale) */
    int m = (int)params[0];
    *re_out = omega <= 0 ? 0.0 : sqrt(scale) * sqrt(2.0 * JAVA_PI) * pow(w, m) * exp(-w);
    *im_out = 0.0;
    return;
  } else if (wavelet == 3) {
    int n = (int)params[0];
    double sigma = params[1];
    double df = 1.0;
    for (int i = 2 * n - 1; i > 0; i -= 2) df *= i;
    double nc = sqrt(df / (pow(2, n) * sqrt(JAVA_PI) * pow(sigma, 2 * n + 1)));
    double mag = sqrt(2.0 * JAVA_PI) * pow(sigma, n + 1) * pow(fabs(w), n) *
                 exp(-0.5 * sigma * sigma * w * w);
    mag *= nc;
    double sg = w > 0 ? 1.0 : (w < 0 ? -1.0 : w); /* Math.signum */
    switch (n % 4) {
      case 0: re = mag; break;
      case 1: im = mag * sg; break;
      case 2: re = -mag; break;
      default: im = -mag * sg; break;
    }
  } else {
    double a = fabs(w), v = 0.0;
    if (a >= 2.0 * JAVA_PI / 3.0 && a <= 8.0 * JAVA_PI / 3.0) {
      if (a <= 4.0 * JAVA_PI / 3.0) {
        v = sin(JAVA_PI / 2.0 * meyer_nu(3.0 * a / (2.0 * JAVA_PI) - 1.0));
      } else {
        v = cos(JAVA_PI / 2.0 * meyer_nu(3.0 * a / (4.0 * JAVA_PI) - 1.0));
      }
      v *= sqrt(2.0 * JAVA_PI);
      re = v * cos(w / 2.0);
      im = v * sin(w / 2.0);
    }
  }
  *re_out = re * sqrt(scale); /* ft.mul(Math.sqrt(scale)) */
  *im_out = im * sqrt(scale);
}

double jwo_cwt_wavelet_ft(int wavelet, const double* params, double omega, double scale) {
  double re, im;
  jwo_cwt_wavelet_ft_c(wavelet, params, omega, scale, &re, &im);
  return re;
}

void jwo_cwt_fft(int wavelet, const double* params, const double* x, long n,
                 const double* scales, int ns, double fs, int padding, double* out_reim) {
  long np = 1;
  if (n > 1) { np = 1; while (np < n) np <<= 1; } /* MathUtils.nextPowerOfTwo */
  double* X = (double*)calloc(2 * np, sizeof(double));
  for (long i = 0; i < n; i++) X[2 * i] = x[i];
  for (long i = n; i < np; i++) {
    double v = 0.0;
    if (padding == 1) {
      long mi = 2 * n - i - 2;
      if (mi >= 0 && mi < n) v = x[mi];
    } else if (padding == 2) {
      v = x[i % n];
    } else if (padding == 3) {
      v = x[n - 1];
    }
    X[2 * i] = v;
  }
  jwo_fft(X, np, 0);
  double* omega = (double*)malloc(sizeof(double) * np);
  for (long i = 0; i < np; i++) {
    omega[i] = 2.0 * JAVA_PI * (double)i * fs / (double)np;
    if (i > np / 2) omega[i] -= 2.0 * JAVA_PI * fs;
  }
  double* P = (double*)malloc(sizeof(double) * 2 * np);
  for (int s = 0; s < ns; s++) {
    double scale = scales[s];
    for (long i = 0; i < np; i++) {
      double wr, wi;
      jwo_cwt_wavelet_ft_c(wavelet, params, omega[i], scale, &wr, &wi);
      wi = -wi; /* conjugate() */
      double sr = X[2 * i], si = X[2 * i + 1];
      P[2 * i] = sr * wr - si * wi;
      P[2 * i + 1] = sr * wi + si * wr;
    }
    jwo_fft(P, np, 1);
    memcpy(out_reim + (long)s * n * 2, P, sizeof(double) * 2 * n);
  }
  free(X); free(omega); free(P);
}

/* ------------------------------------------------------------------------ */
/* CPU baselines: the reference's ForkJoin patterns restated with OpenMP tasks.      */
/* RecursiveAction halving (ParallelTransform.java:222-335: split [lo, hi) in two    */
/* while hi - lo > THRESHOLD, invokeAll, leaves run serially).                       */
/* ------------------------------------------------------------------------ */
typedef void (*jwo_range_fn)(long lo, long hi, void* ctx);

static void fj_invoke(long lo, long hi, long leaf, jwo_range_fn fn, void* ctx) {
  if (hi - lo <= leaf) {
    fn(lo, hi, ctx);
    return;
  }
  long mid = lo + (hi - lo) / 2;
#pragma omp task firstprivate(lo, mid, leaf, fn, ctx)
  fj_invoke(lo, mid, leaf, fn, ctx);
  fj_invoke(mid, hi, leaf, fn, ctx);
#pragma omp taskwait
}

/* ForkJoinPool.invoke: one pool of `threads` workers runs the whole task tree. */
static void fj_pool(long n, long leaf, int threads, jwo_range_fn fn, void* ctx) {
  if (leaf < 1) leaf = 1;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#pragma omp single
#endif
  fj_invoke(0, n, leaf, fn, ctx);
}

/* leaf size: the reference's THRESHOLD of 16, lowered when the bounded sample has fewer
 * than 16 items per worker so every worker gets a leaf */
static long fj_leaf(long n, int threads) {
  long per = threads > 0 ? n / threads : n;
  return per < 1 ? 1 : (per < 16 ? per : 16);
}

typedef struct {
  const double *x, *g, *h;
  long N;
  int J, L, use_fft;
  double *coeffs, *xr;
} modwt_batch_ctx;

static void modwt_batch_leaf(long lo, long hi, void* p) {
  modwt_batch_ctx* c = (modwt_batch_ctx*)p;
  for (long b = lo; b < hi; b++) {
    double* cf = c->coeffs + b * (c->J + 1) * c->N;
    if (c->use_fft) {
      jwo_modwt_forward_fft(c->x + b * c->N, c->N, c->J, c->g, c->h, c->L, cf);
      jwo_modwt_inverse_fft(cf, c->N, c->J, c->g, c->h, c->L, c->xr + b * c->N);
    } else {
      jwo_modwt_forward_direct(c->x + b * c->N, c->N, c->J, c->g, c->h, c->L, cf);
      jwo_modwt_inverse_direct(cf, c->N, c->J, c->g, c->h, c->L, c->xr + b * c->N);
    }
  }
}

/* MODWT over a batch of independent signals: forwardMODWT + inverseMODWT per signal
 * (MODWTTransform.java:256-375), signals split by ForkJoin halving. */
void jwo_modwt_fwdinv_batch(const double* x, long N, int J, const double* g, const double* h,
                            int L, int B, int use_fft, int threads, double* coeffs, double* xr) {
  modwt_batch_ctx c = {x, g, h, N, J, L, use_fft, coeffs, xr};
  fj_pool(B, fj_leaf(B, threads), threads, modwt_batch_leaf, &c);
}

/* ParallelTransform 2-D (ParallelTransform.java:70-126): per matrix, pool.invoke(RowTransformTask)
 * then pool.invoke(ColumnTransformTask) for the forward, columns then rows for the reverse;
 * leaves of <= 16 rows / columns (THRESHOLD :28) run FastWaveletTransform 1-D per line. */
typedef struct {
  const double* src;
  double* dst;
  int rows, cols, lvl, fwd, M, tw, kind;
  const double *f0, *f1;
} fwt2d_ctx;

static void fwt2d_rows_leaf(long lo, long hi, void* p) {
  fwt2d_ctx* c = (fwt2d_ctx*)p;
  for (long i = lo; i < hi; i++) {
    if (c->fwd)
      jwo_fwt_forward(c->src + i * c->cols, c->cols, c->lvl, c->f0, c->f1, c->M, c->tw,
                      c->dst + i * c->cols);
    else
      jwo_fwt_reverse(c->src + i * c->cols, c->cols, c->lvl, c->f0, c->f1, c->M, c->tw, c->kind,
                      c->dst + i * c->cols);
  }
}

static void fwt2d_cols_leaf(long lo, long hi, void* p) {
  fwt2d_ctx* c = (fwt2d_ctx*)p;
  double* a = (double*)malloc(sizeof(double) * c->rows);
  double* b = (double*)malloc(sizeof(double) * c->rows);
  for (long j = lo; j < hi; j++) {
    for (int i = 0; i < c->rows; i++) a[i] = c->src[(long)i * c->cols + j];
    if (c->fwd)
      jwo_fwt_forward(a, c->rows, c->lvl, c->f0, c->f1, c->M, c->tw, b);
    else
      jwo_fwt_reverse(a, c->rows, c->lvl, c->f0, c->f1, c->M, c->tw, c->kind, b);
    for (int i = 0; i < c->rows; i++) c->dst[(long)i * c->cols + j] = b[i];
  }
  free(a);
  free(b);
}

/* forward + reverse of B matrices (rows x cols): y = forward(x), xr = reverse(y) */
void jwo_fwt2d_fwdrev_parallel(const double* x, int B, int rows, int cols, int lvlM, int lvlN,
                               const double* sD, const double* wD, const double* sR,
                               const double* wR, int M, int tw, int kind, int threads,
                               double* y, double* xr) {
  const long img = (long)rows * cols;
  for (int b = 0; b < B; b++) {
    fwt2d_ctx r = {x + b * img, y + b * img, rows, cols, lvlN, 1, M, tw, kind, sD, wD};
    fj_pool(rows, 16, threads, fwt2d_rows_leaf, &r);
    fwt2d_ctx c = {y + b * img, y + b * img, rows, cols, lvlM, 1, M, tw, kind, sD, wD};
    fj_pool(cols, 16, threads, fwt2d_cols_leaf, &c);
    fwt2d_ctx rc = {y + b * img, xr + b * img, rows, cols, lvlM, 0, M, tw, kind, sR, wR};
    fj_pool(cols, 16, threads, fwt2d_cols_leaf, &rc);
    fwt2d_ctx rr = {xr + b * img, xr + b * img, rows, cols, lvlN, 0, M, tw, kind, sR, wR};
    fj_pool(rows, 16, threads, fwt2d_rows_leaf, &rr);
  }
}

/* transformFFTParallel (ContinuousWaveletTransform.java:511-565) over a batch of signals:
 * signals in the outer pool, per signal one FFT then the scales in parallel, each scale
 * psi_hat conj x X -> IFFT -> first n samples.  Recurrence twiddles (the reference's FFT). */
typedef struct {
  int wavelet;
  const double* params;
  const double* x;
  long n, np;
  const double* scales;
  int ns;
  double fs;
  int padding;
  double* out;
  /* per-signal state, set by the signal task */
  const double* X;
  const double* omega;
  long sig;
} cwt_ctx;

static void cwt_scale_leaf(long lo, long hi, void* p) {
  cwt_ctx* c = (cwt_ctx*)p;
  double* P = (double*)malloc(sizeof(double) * 2 * c->np);
  for (long s = lo; s < hi; s++) {
    for (long i = 0; i < c->np; i++) {
      double wr, wi;
      jwo_cwt_wavelet_ft_c(c->wavelet, c->params, c->omega[i], c->scales[s], &wr, &wi);
      wi = -wi;
      double sr = c->X[2 * i], si = c->X[2 * i + 1];
      P[2 * i] = sr * wr - si * wi;
      P[2 * i + 1] = sr * wi + si * wr;
    }
    jwo_fft(P, c->np, 1);
    memcpy(c->out + (c->sig * c->ns + s) * c->n * 2, P, sizeof(double) * 2 * c->n);
  }
  free(P);
}

static void cwt_signal_leaf(long lo, long hi, void* p) {
  const cwt_ctx* c0 = (const cwt_ctx*)p;
  for (long b = lo; b < hi; b++) {
    const long n = c0->n, np = c0->np;
    const double* x = c0->x + b * n;
    double* X = (double*)calloc(2 * np, sizeof(double));
    for (long i = 0; i < n; i++) X[2 * i] = x[i];
    for (long i = n; i < np; i++) { /* padSignal :269-306 */
      double v = 0.0;
      if (c0->padding == 1) {
        long mi = 2 * n - i - 2;
        if (mi >= 0 && mi < n) v = x[mi];
      } else if (c0->padding == 2) {
        v = x[i % n];
      } else if (c0->padding == 3) {
        v = x[n - 1];
      }
      X[2 * i] = v;
    }
    jwo_fft(X, np, 0);
    double* omega = (double*)malloc(sizeof(double) * np);
    for (long i = 0; i < np; i++) {
      omega[i] = 2.0 * JAVA_PI * (double)i * c0->fs / (double)np;
      if (i > np / 2) omega[i] -= 2.0 * JAVA_PI * c0->fs;
    }
    cwt_ctx c = *c0;
    c.X = X;
    c.omega = omega;
    c.sig = b;
    fj_invoke(0, c.ns, 1, cwt_scale_leaf, &c); /* IntStream.range(0, nScales).parallel() */
    free(omega);
    free(X);
  }
}

void jwo_cwt_fft_parallel_batch(int wavelet, const double* params, const double* x, long n,
                                const double* scales, int ns, double fs, int padding, int B,
                                int threads, double* out_reim) {
  long np = 1;
  while (np < n) np <<= 1;
  cwt_ctx c = {wavelet, params, x, n, np, scales, ns, fs, padding, out_reim, NULL, NULL, 0};
  fj_pool(B, 1, threads, cwt_signal_leaf, &c);
}

/* ------------------------------------------------------------------------ */
/* CWT direct path: ContinuousWaveletTransform.transform(signal, scales, fs) :153-172,      */
/* computeCoefficient :240-260, ContinuousWavelet.wavelet(t, a, b) :90-102, and each       */
/* class's wavelet(double t) and getEffectiveSupport().  Test infrastructure only.          */
/* ------------------------------------------------------------------------ */
static int jwo_java_d2i(double v) { /* Java (int) cast */
  if (v != v) return 0;
  if (v >= 2147483647.0) return 2147483647;
  if (v <= -2147483648.0) return -2147483647 - 1;
  return (int)v;
}

/* psi(t) of MorletWavelet.java:85-100, MexicanHatWavelet.java:85-95, PaulWavelet.java:142-150
 * (+ complexPower :262-271), DOGWavelet.java:166-180 (+ Hermite :289-335, norm :357-366),
 * MeyerWavelet.wavelet(double t) (+ sinc); support[] = getEffectiveSupport(). */
void jwo_cwt_wavelet_t(int wavelet, const double* params, double t, double* re, double* im,
                       double* support) {
  const double PI = 3.14159265358979323846;
  *re = 0.0; *im = 0.0;
  if (wavelet == 0) { /* Morlet(fb, fc) */
    double fb = params[0], fc = params[1];
    double norm = 1.0 / sqrt(2.0 * PI * fb);
    double envelope = exp(-t * t / (2.0 * fb));
    double phase = 2.0 * PI * fc * t, sn, cs;
    sincos(phase, &sn, &cs); /* one libm routine for both (the library does the same) */
    *re = norm * envelope * cs;
    *im = norm * envelope * sn;
    support[0] = -(4.0 * sqrt(fb)); support[1] = 4.0 * sqrt(fb);
  } else if (wavelet == 1) { /* Mexican hat(sigma) */
    double sigma = params[0];
    double nc = 2.0 / (sqrt(3.0 * sigma) * pow(PI, 0.25));
    double tNorm = t / sigma, tNorm2 = tNorm * tNorm;
    *re = nc * (1.0 - tNorm2) * exp(-0.5 * tNorm2);
    support[0] = -5.0 * sigma; support[1] = 5.0 * sigma;
  } else if (wavelet == 2) { /* Paul(m) */
    int m = (int)params[0];
    double fm = 1.0, f2m = 1.0;
    for (int i = 2; i <= m; i++) fm *= i;
    for (int i = 2; i <= 2 * m; i++) f2m *= i;
    double nc = pow(2, m) * fm / sqrt(PI * f2m);
    static const double ipr[4] = {1, 0, -1, 0}, ipi[4] = {0, 1, 0, -1};
    double zr = 1.0, zi = -t; /* new Complex(1.0, -t) */
    double mag = sqrt(zr * zr + zi * zi), arg = atan2(zi, zr);
    double p = -(m + 1);
    double newMag = pow(mag, p), newArg = p * arg;
    double sn, cs;
    sincos(newArg, &sn, &cs);
    double pr = newMag * cs, pi = newMag * sn;
    double ar = ipr[m % 4] * nc, ai = ipi[m % 4] * nc; /* _iPowerM.mul(_normConstant) */
    *re = ar * pr - ai * pi;                             /* .mul(power) */
    *im = ar * pi + ai * pr;
    support[0] = -1.0; support[1] = 2.0 * (m + 1);
  } else if (wavelet == 3) { /* DOG(n, sigma) */
    int n = (int)params[0];
    double sigma = params[1];
    double c[12][12];
    memset(c, 0, sizeof(c));
    c[0][0] = 1.0;
    if (n > 0) { c[1][0] = 0.0; c[1][1] = 2.0; }
    for (int k = 2; k <= n; k++) {
      for (int i = 1; i <= k; i++) if (i - 1 < k) c[k][i] += 2.0 * c[k - 1][i - 1];
      for (int i = 0; i <= k - 2; i++) c[k][i] -= 2.0 * (k - 1) * c[k - 2][i];
    }
    double sign = ((n + 1) % 2 == 0) ? 1.0 : -1.0;
    double df = 1.0;
    for (int i = 2 * n - 1; i > 0; i -= 2) df *= i;
    double nc = sqrt(df / (pow(2, n) * sqrt(PI) * pow(sigma, 2 * n + 1)));
    double x = t / sigma;
    double gaussian = exp(-0.5 * x * x);
    double h = 0.0;
    for (int i = n; i >= 0; i--) h = h * x + c[n][i] * sign;
    *re = nc * h * gaussian;
    double r = (3.0 + n / 2.0) * sigma;
    support[0] = -r; support[1] = r;
  } else { /* Meyer */
    support[0] = -15.0; support[1] = 15.0;
    if (fabs(t) > 15.0) return;
    double envelope = exp(-0.5 * t * t / 25.0);
    double om[3] = {0.7, 1.4 * 0.7, 0.5 * 0.7}, amp[3] = {1.0, 0.2, -0.1};
    double value = 0.0;
    for (int q = 0; q < 3; q++) {
      double xx = om[q] * t, s;
      if (fabs(xx) < 1e-10) { double x2 = xx * xx; s = 1.0 - x2 / 6.0 + x2 * x2 / 120.0; }
      else s = sin(xx) / xx;
      double term = q == 0 ? om[q] * s * envelope : amp[q] * om[q] * s * envelope;
      value = q == 0 ? term : value + term;
    }
    value *= sqrt(2.0 / PI);
    *re = value;
  }
}

/* out[s][t] = (re, im) for one signal; returns 0, or -1 if a scale <= 0 meets a non-empty
 * window (ContinuousWavelet.wavelet throws IllegalArgumentException there). */
int jwo_cwt_direct(int wavelet, const double* params, const double* x, long n,
                   const double* scales, int ns, double fs, double* out) {
  double dt = 1.0 / fs;
  for (int s = 0; s < ns; s++) {
    double scale = scales[s], sup[2], wr, wi;
    jwo_cwt_wavelet_t(wavelet, params, 0.0, &wr, &wi, sup);
    for (long ti = 0; ti < n; ti++) {
      long minIdx = ti + jwo_java_d2i(sup[0] * scale * fs);
      long maxIdx = ti + jwo_java_d2i(sup[1] * scale * fs);
      if (minIdx < 0) minIdx = 0;
      if (maxIdx > n - 1) maxIdx = n - 1;
      double sr = 0.0, si = 0.0;
      for (long i = minIdx; i <= maxIdx; i++) {
        if (scale <= 0) return -1;
        double t = (double)(i - ti) * dt;
        double vr, vi;
        jwo_cwt_wavelet_t(wavelet, params, (t - 0.0) / scale, &vr, &vi, sup);
        double nf = 1.0 / sqrt(scale);
        vr = vr * nf; vi = -(vi * nf);           /* .mul(normFactor).conjugate() */
        sr = sr + vr * x[i]; si = si + vi * x[i]; /* sum.add(waveletValue.mul(signal[i])) */
      }
      out[2 * ((long)s * n + ti)] = sr * dt;      /* sum.mul(dt) */
      out[2 * ((long)s * n + ti) + 1] = si * dt;
    }
  }
  return 0;
}
