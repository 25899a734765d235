/*
 * jwave_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, operation-for-operation CPU restatement of JWave-Pro's hot path
 * (reference: Prophetizo/JWave-Pro @ 2025-07-18, Java 21).  It is the parity
 * checker for the HIP engine and the "port" CPU baseline in bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product library (libjwave_hip.so) never links or calls it.
 *
 * Built with -O2 -ffp-contract=off: Java never contracts a*b+c into an FMA, so
 * every FWT / MODWT-DIRECT result here is the bit-identical IEEE sequence the
 * JVM executes (no JVM exists in this image; see DESIGN.md "Oracle").
 * Parity pin: tests/test_oracle_golden.py checks this file against every
 * known-answer test and fixture the reference's own test suite holds for the path.
 *
 * All file:line citations are relative to /root/reference/src/main/java/jwave/.
 */
#ifndef JWAVE_ORACLE_H
#define JWAVE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- java.util.Random restated (seed scramble, 48-bit LCG, nextDouble) ---- */
typedef struct { uint64_t seed; } jwo_random;
void     jwo_random_init(jwo_random* r, int64_t seed);
int32_t  jwo_random_next(jwo_random* r, int bits);
double   jwo_random_next_double(jwo_random* r);
/* out[i] = nextDouble()*2 - 1 for a fresh Random(seed): the synthetic signal generator. */
void     jwo_fill_uniform(double* out, long n, int64_t seed);
/* Same values as jwo_fill_uniform but for elements [start, start+count) of the stream
 * (LCG jump-ahead); lets a GPU-generated batch be spot-checked without replaying it. */
void     jwo_fill_uniform_range(double* out, long start, long count, int64_t seed);

/* ---- MODWT (transforms/MODWTTransform.java) ---- */
/* initializeFilterCache + normalize (:452-484, :599-606): g,h base taps. */
void jwo_modwt_filters(const double* scal_dec, const double* wav_dec, int L, double* g, double* h);
/* upsample (:618-630): returns M_j; writes M_j taps (zeros included) into out (cap >= M_j). */
long jwo_modwt_upsample(const double* base, int L, int level, double* out);
/* forwardMODWT with convolutionMethod DIRECT (:256-306, circularConvolve :677-690).
 * Faithful: iterates every up-sampled tap, zeros included, Math.floorMod indexing.
 * coeffs: (J+1) x N row-major = [W_1 .. W_J, V_J]. */
void jwo_modwt_forward_direct(const double* x, long N, int J, const double* g, const double* h,
                              int L, double* coeffs);
/* inverseMODWT with DIRECT (:337-375, circularConvolveAdjoint :703-716). */
void jwo_modwt_inverse_direct(const double* coeffs, long N, int J, const double* g,
                              const double* h, int L, double* x);
/* The same two functions evaluating only the L non-zero taps per level (bit-identical for
 * finite inputs; used where the faithful loop would take minutes, e.g. N = 2^20). */
void jwo_modwt_forward_direct_nz(const double* x, long N, int J, const double* g,
                                 const double* h, int L, double* coeffs);
void jwo_modwt_inverse_direct_nz(const double* coeffs, long N, int J, const double* g,
                                 const double* h, int L, double* x);
/* FFT convolution path (:752-837) with the reference FFT (FastFourierTransform.java). */
void jwo_modwt_forward_fft(const double* x, long N, int J, const double* g, const double* h,
                           int L, double* coeffs);
void jwo_modwt_inverse_fft(const double* coeffs, long N, int J, const double* g,
                           const double* h, int L, double* x);
/* forward/inverse with ConvolutionMethod.AUTO: each convolution DIRECT or FFT by the rule below
 * (MODWTTransform.java:640-664), as a default-constructed MODWTTransform runs them. */
void jwo_modwt_forward_auto(const double* x, long N, int J, const double* g, const double* h,
                            int L, int threshold, double* coeffs);
void jwo_modwt_inverse_auto(const double* coeffs, long N, int J, const double* g,
                            const double* h, int L, int threshold, double* x);
/* performConvolution AUTO rule (:650-654): (int32)(N*M) > threshold, int32 wrap included. */
int  jwo_modwt_auto_uses_fft(long N, long M, int threshold);

/* ---- FFT (transforms/FastFourierTransform.java:112-324) ---- */
/* In-place on interleaved (re,im) of length n.  Power of 2 -> Cooley-Tukey with
 * recurrence twiddles; otherwise Bluestein.  inverse scales by 1/n. */
void jwo_fft(double* reim, long n, int inverse);
void jwo_fft_stage_twiddles(long size, int inverse, double* out);
void jwo_set_exact_twiddles(int on); /* test switch, see jwave_oracle.c */

/* ---- FWT (transforms/wavelets/Wavelet.java:236-303, FastWaveletTransform.java:71-153) ---- */
/* kind: 0 = generic Wavelet, 1 = Haar1Orthogonal (reverse x0.5, Haar1Orthogonal.java:175-207) */
void jwo_wavelet_forward(const double* in, int len, const double* sD, const double* wD, int M,
                         double* out);
void jwo_wavelet_reverse(const double* in, int len, const double* sR, const double* wR, int M,
                         int kind, double* out);
void jwo_fwt_forward(const double* x, long n, int level, const double* sD, const double* wD,
                     int M, int tw, double* y);
void jwo_fwt_reverse(const double* y, long n, int level, const double* sR, const double* wR,
                     int M, int tw, int kind, double* x);
/* BasicTransform.forward/reverse(double[][], lvlM, lvlN) (BasicTransform.java:361-474). */
void jwo_wpt_forward(const double* x, long n, int level, const double* sD, const double* wD,
                     int M, int tw, double* y);
void jwo_wpt_reverse(const double* y, long n, int level, const double* sR, const double* wR,
                     int M, int tw, int kind, double* x);
void jwo_fwt2d_forward(const double* x, int rows, int cols, int lvlM, int lvlN, const double* sD,
                       const double* wD, int M, int tw, double* y);
void jwo_fwt2d_reverse(const double* y, int rows, int cols, int lvlM, int lvlN, const double* sR,
                       const double* wR, int M, int tw, int kind, double* x);
void jwo_fwt3d_forward(const double* x, int d1, int d2, int d3, int lvlP, int lvlQ, int lvlR,
                       const double* sD, const double* wD, int M, int tw, double* y);
void jwo_fwt3d_reverse(const double* y, int d1, int d2, int d3, int lvlP, int lvlQ, int lvlR,
                       const double* sR, const double* wR, int M, int tw, int kind, double* x);

/* ---- CWT FFT path (transforms/ContinuousWaveletTransform.java:183-229) ---- */
/* wavelet: 0 = Morlet(params[0]=fb, params[1]=fc), 1 = MexicanHat(params[0]=sigma),
 * 2 = Paul(params[0]=m), 3 = DOG(params[0]=n, params[1]=sigma), 4 = Meyer()
 * padding: 0 ZERO, 1 SYMMETRIC, 2 PERIODIC, 3 CONSTANT.  out: ns x n x 2 (re,im). */
void jwo_cwt_fft(int wavelet, const double* params, const double* x, long n,
                 const double* scales, int ns, double fs, int padding, double* out_reim);
/* ContinuousWavelet.fourierTransform(omega, scale, 0) (ContinuousWavelet.java:122-141). */
double jwo_cwt_wavelet_ft(int wavelet, const double* params, double omega, double scale);
void jwo_cwt_wavelet_ft_c(int wavelet, const double* params, double omega, double scale,
                          double* re, double* im);
void jwo_cwt_wavelet_t(int wavelet, const double* params, double t, double* re, double* im,
                       double* support);
int jwo_cwt_direct(int wavelet, const double* params, const double* x, long n,
                   const double* scales, int ns, double fs, double* out);

/* ---- CPU baselines: the reference's ForkJoin patterns (OpenMP tasks, recursive halving) ---- */
void jwo_modwt_fwdinv_batch(const double* x, long N, int J, const double* g, const double* h,
                            int L, int B, int use_fft, int threads, double* coeffs, double* xr);
/* ParallelTransform 2-D forward (rows task, then columns task) + reverse (columns, rows) */
void jwo_fwt2d_fwdrev_parallel(const double* x, int B, int rows, int cols, int lvlM, int lvlN,
                               const double* sD, const double* wD, const double* sR,
                               const double* wR, int M, int tw, int kind, int threads,
                               double* y, double* xr);
/* transformFFTParallel per signal, signals in the outer pool */
void jwo_cwt_fft_parallel_batch(int wavelet, const double* params, const double* x, long n,
                                const double* scales, int ns, double fs, int padding, int B,
                                int threads, double* out_reim);

#ifdef __cplusplus
}
#endif
#endif
