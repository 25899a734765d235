/*
 * jwave_hip.h -- C-ABI of the MI355X (gfx950) JWave-Pro hot-path engine.
 *
 * This is the drop-in boundary: a JNI shim binds exactly these entry
 * points from Java subclasses of JWave-Pro's own transforms.  Plain pointers and sizes
 * only; all buffers are caller-owned, row-major, batch-major.  Citations are relative to
 * the reference's src/main/java/jwave/.
 *
 * Status codes mirror the reference's exception classes so the glue can rethrow the
 * exact Java type with jw_last_error()'s message:
 *   JW_ERR_ILLEGAL_ARGUMENT -> java.lang.IllegalArgumentException (unchecked)
 *   JW_ERR_FAILURE          -> jwave.exceptions.JWaveFailure      (checked)
 *
 * Threading: plans are immutable after creation and may be shared by any number of host
 * threads (the reference's MODWTThreadSafetyTest pattern).  Every call is reentrant.
 * Process-wide state, all internally synchronised:
 *   - a thread-local error message (jw_last_error) and the calling thread's current device
 *     (jw_set_device; HIP's own per-thread device);
 *   - per-device caches of tables that depend on sizes / filters only (FFT twiddles, chirp-z
 *     tables, MODWT filter spectra and pair tables), each within a byte budget (a call past
 *     the budget builds its own), built once per key (the first call for a key synchronises
 *     its stream once) and freed by jw_release_caches();
 *   - one private stream-ordered memory pool per device for workspaces (the device's default
 *     pool is never touched); it keeps freed memory for reuse, gives it back when an
 *     allocation would fail, and on jw_release_caches();
 *   - per host thread and device, three non-blocking streams and a ring of three 32 MiB pinned
 *     bounce buffers per direction (192 MiB) for JW_HOST staging, freed when the thread exits
 *     (JW_PIN_RING / JW_PIN_MB / JW_COPY_THREADS tune them);
 *   - per host thread and device, one more non-blocking stream and two events on which
 *     jw_cwt_fft runs its one-pass (band) scales beside the two-pass ones, forked from and
 *     joined back into the caller's stream by events (stream order for the caller is
 *     unchanged; JW_CWT_OVERLAP=0 keeps the whole call on the caller's stream).
 */
#ifndef JWAVE_HIP_H
#define JWAVE_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define JW_OK 0
#define JW_ERR_ILLEGAL_ARGUMENT (-1) /* IllegalArgumentException */
#define JW_ERR_FAILURE (-2)          /* JWaveFailure */
#define JW_ERR_DEVICE (-3)           /* HIP runtime / kernel launch error */
#define JW_ERR_NO_MEMORY (-4)
#define JW_ERR_UNSUPPORTED (-5)      /* UnsupportedOperationException: a length or mode this
                                        engine does not run (the message names the limit) */

/* ---- where the caller's buffers live ---- */
#define JW_HOST 0   /* host memory: the call stages through HBM and synchronises */
#define JW_DEVICE 1 /* HBM pointers; work is enqueued on `stream` (hipStream_t), async */

/* ---- MODWTTransform.ConvolutionMethod (MODWTTransform.java:149-153) ---- */
#define JW_CONV_AUTO 0
#define JW_CONV_DIRECT 1
#define JW_CONV_FFT 2

/* ---- arithmetic contract ---- */
#define JW_ARITH_STRICT 0 /* Java operation order, no FMA contraction: bit-identical to the JVM */
#define JW_ARITH_FMA 1    /* same tap order, fused multiply-add: <= 1e-15 normwise from STRICT */

/* Thread-local text of the last error on this thread (exact reference message where the
 * reference defines one).  Never NULL. */
const char* jw_last_error(void);

/* Library version string and the gfx target it was built for. */
const char* jw_version(void);

/* ---- devices (one process may drive several GPUs, e.g. a JVM whose ForkJoin workers fan out
 * as ParallelTransform.java:83-86 / ContinuousWaveletTransform.java:511-565 do) ---- */
/* Number of visible HIP devices (0 when none; never an error). */
int jw_device_count(int* count);
/* Make `ordinal` the calling thread's device: every later call of this thread runs there, its
 * JW_DEVICE pointers must live there, and the caches are kept per device.  Invalid ordinals ->
 * JW_ERR_ILLEGAL_ARGUMENT ("device ordinal must be >= 0", "... out of range: k HIP device(s)
 * visible"). */
int jw_set_device(int ordinal);
int jw_get_device(int* ordinal);
/* MODWTTransform.clearFilterCache (:556) for the device side: frees every cached table (FFT
 * twiddles, chirp-z tables, MODWT filter spectra / pair tables) on every device the library has
 * run on and returns the memory pools' unused workspace memory to the driver.  Waits for calls
 * in flight (and the kernels they queued) before freeing; later calls rebuild what they need.
 * Returns the bytes of tables freed (>= 0). */
long jw_release_caches(void);
/* Engine settings for same-box A/B runs and tests (not part of the reference interface): the
 * JW_* names the engine consults (JW_CWT_INTERP, JW_FWT_GENERIC, JW_INV_KERNEL, ...; DESIGN.md
 * §9).  Each is read from the environment once, on first use; jw_set_knob(name, value)
 * replaces that value for later calls (value NULL = unset), so a test changes a setting without
 * setenv racing the engine's threads.  name must start with "JW_" (else
 * JW_ERR_ILLEGAL_ARGUMENT).  JW_PIN_MB, JW_PIN_RING and JW_COPY_THREADS size process-wide
 * host staging on first use and are environment-only: jw_set_knob refuses them
 * (JW_ERR_ILLEGAL_ARGUMENT).  jw_get_knob returns the value in effect, or NULL when unset; the
 * string stays valid for the life of the process. */
int jw_set_knob(const char* name, const char* value);
const char* jw_get_knob(const char* name);

/* ======================================================================
 * MODWT  (replaces MODWTTransform.forwardMODWT :256 / inverseMODWT :337)
 * ====================================================================== */
typedef struct jw_modwt_plan jw_modwt_plan;

/* new MODWTTransform(wavelet[, fftThreshold]) (MODWTTransform.java:180-195) followed by
 * initializeFilterCache (:452-484): normalises the wavelet's scaling/wavelet
 * decomposition filters (Wavelet.getScalingDeComposition/getWaveletDeComposition) to unit
 * energy and divides by sqrt(2).  L in [1, 64].  arith: JW_ARITH_*. */
int jw_modwt_plan_create(jw_modwt_plan** plan, const double* scaling_dec,
                         const double* wavelet_dec, int L, int fft_threshold, int arith);
void jw_modwt_plan_destroy(jw_modwt_plan* plan);
/* The cached base filters g (scaling) and h (wavelet), L each. */
int jw_modwt_plan_filters(const jw_modwt_plan* plan, double* g, double* h);

/* forwardMODWT(data, levels) for `batch` independent signals of length n.
 * x: batch x n.  coeffs: batch x (levels+1) x n = [W_1..W_J, V_J] per signal.
 * Validation order and messages follow MODWTTransform.java:257-282; n == 0 is a no-op.
 * method: JW_CONV_* (the Java object's setConvolutionMethod state, passed per call).
 * With a JW_ARITH_STRICT plan (the JVM's arithmetic) every level takes the convolution the
 * reference's performConvolution takes (:640-664): FFT always, DIRECT never, AUTO when the
 * int32 product n * M_j > fftConvolutionThreshold (M_j = (L-1) 2^(j-1) + 1, wrap included).
 * DIRECT levels are bit-identical to circularConvolve (:677-690), non-finite data included:
 * like the reference, which multiplies the up-sampled zero taps too (upsample :618-630), an
 * output whose window holds a +-Inf or NaN sample on a zero tap is NaN (0 * Inf = NaN); the
 * engine flags signals with non-finite values on the device and re-runs only those through a
 * zero-tap pass on the same stream (JW_DEVICE stays asynchronous; FMA plans get the same NaN
 * pattern).  FFT levels run the
 * reference's circularConvolveFFT (:752-786) with its own FFT: radix 2 with recurrence
 * twiddles for powers of two (FastFourierTransform.java:172-212) and its Bluestein transform for
 * other lengths (:259-324), both bit-identical to the JVM over the reference's own domain:
 * power-of-two n <= 2^30 and other n <= 2^29 (Bluestein's m <= 2^30; past that the reference's
 * int arithmetic overflows), the longest transforms in three column passes (the levels from 2^25,
 * jw_fft_*_ex from 2^23: the split changes access shapes, not one operation) -- given that the
 * JVM's Math.sin/Math.cos are correctly rounded at the twiddle and chirp angles (Java specifies
 * them to 1 ulp; the engine and the oracle both take the correctly rounded value).
 * With a JW_ARITH_FMA plan (the fast contract) FFT runs the exact-twiddle frequency-domain
 * pyramid for 2 <= n <= 2^23 (within 1e-10 of DIRECT); AUTO and DIRECT run the direct kernels
 * (faster and more accurate than any FFT path on this engine).
 * A call with an FFT level (FFT, or AUTO's rule) past its contract's range (STRICT: the limits
 * above; FMA: n > 2^23) returns JW_ERR_UNSUPPORTED naming the limit (never DIRECT values in its
 * place); DIRECT runs any n. */
int jw_modwt_forward(const jw_modwt_plan* plan, const double* x, double* coeffs, long n,
                     int levels, int batch, int method, int where, void* stream);
/* inverseMODWT(coefficients) (:337-375): coeffs batch x (levels+1) x n -> x batch x n.
 * Method and arithmetic as jw_modwt_forward (circularConvolveAdjoint :703-716,
 * circularConvolveFFTAdjoint :798-837). */
int jw_modwt_inverse(const jw_modwt_plan* plan, const double* coeffs, double* x, long n,
                     int levels, int batch, int method, int where, void* stream);

/* ======================================================================
 * FFT  (replaces FastFourierTransform.forward/reverse(Complex[]) :112-164)
 * ====================================================================== */
/* batch independent lines of n complex values, interleaved (re, im), batch-major.
 * forward: X_k = sum_t x_t e^{-2 pi i t k / n};  reverse: x_t = (1/n) sum_k X_k e^{+2 pi i t k / n}
 * (the reference's 1/n, :207-211).  n = 0: nothing; n = 1: a copy; powers of two run the
 * four-step engine, other n <= 2^23 a chirp-z (Bluestein, :259-324) transform over it.
 * Twiddles are correctly rounded (the reference builds them by recurrence, :188-201), so
 * results agree with the reference's to its own rounding drift.  in == out is allowed. */
int jw_fft_forward(const double* in_reim, double* out_reim, long n, int batch, int where,
                   void* stream);
int jw_fft_reverse(const double* in_reim, double* out_reim, long n, int batch, int where,
                   void* stream);
/* The same transforms under an arithmetic contract.  JW_ARITH_STRICT runs the reference's own
 * algorithm operation for operation -- bit reversal, radix-2 decimation in time with the
 * recurrence twiddles wn = wn.mul(w) of every stage (:172-212), Complex.mul's (ac - bd, ad + bc),
 * Bluestein for other n (:259-324) -- so results are the JVM's bit for bit for power-of-two
 * n <= 2^30 and other n <= 2^29, the reference's own domain (a Java array holds at most 2^30 as a
 * power of two; its Bluestein `int m` doubling overflows past n = 2^29, :261-265), correctly
 * rounded Math.sin/cos assumed, as above; longer STRICT lines return JW_ERR_UNSUPPORTED.  Host
 * tables past 2^26 take seconds to build (cached while they fit, jw_release_caches drops them).
 * JW_ARITH_FMA is jw_fft_forward / jw_fft_reverse (correctly rounded twiddle tables). */
int jw_fft_forward_ex(const double* in_reim, double* out_reim, long n, int batch, int arith,
                      int where, void* stream);
int jw_fft_reverse_ex(const double* in_reim, double* out_reim, long n, int batch, int arith,
                      int where, void* stream);

/* ======================================================================
 * FWT  (replaces FastWaveletTransform.forward/reverse(double[], level) :71/:119,
 *       the 1-D kernel Wavelet.forward/reverse :236/:277, and the 2-D
 *       BasicTransform.forward/reverse(double[][], lvlM, lvlN) :361/:436)
 * ====================================================================== */
typedef struct jw_fwt_plan jw_fwt_plan;

#define JW_WAVELET_GENERIC 0   /* Wavelet.reverse as written (Wavelet.java:277-303) */
#define JW_WAVELET_HAAR_ORTH 1 /* Haar1Orthogonal.reverse: contribution x 0.5 (:175-207) */

/* Filters as the Wavelet object holds them (_scalingDeCom, _waveletDeCom, _scalingReCon,
 * _waveletReCon), motherWavelength M in [1, 64], transformWavelength tw >= 1. */
int jw_fwt_plan_create(jw_fwt_plan** plan, const double* scaling_dec, const double* wavelet_dec,
                       const double* scaling_rec, const double* wavelet_rec, int M,
                       int transform_wavelength, int kind, int arith);
void jw_fwt_plan_destroy(jw_fwt_plan* plan);
/* y = forward(x, level) for batch signals of length n (n must be 2^p). */
int jw_fwt_forward(const jw_fwt_plan* plan, const double* x, double* y, long n, int level,
                   int batch, int where, void* stream);
int jw_fwt_reverse(const jw_fwt_plan* plan, const double* y, double* x, long n, int level,
                   int batch, int where, void* stream);
/* WaveletPacketTransform.forward/reverse(double[], level) (WaveletPacketTransform.java:60-191):
 * every level transforms all n/h packets.  Same plan and arithmetic as the FWT. */
int jw_wpt_forward(const jw_fwt_plan* plan, const double* x, double* y, long n, int level,
                   int batch, int where, void* stream);
int jw_wpt_reverse(const jw_fwt_plan* plan, const double* y, double* x, long n, int level,
                   int batch, int where, void* stream);
/* 2-D: rows with lvlN then columns with lvlM (reverse: columns, then rows). */
int jw_fwt2d_forward(const jw_fwt_plan* plan, const double* x, double* y, int rows, int cols,
                     int lvlM, int lvlN, int batch, int where, void* stream);
int jw_fwt2d_reverse(const jw_fwt_plan* plan, const double* y, double* x, int rows, int cols,
                     int lvlM, int lvlN, int batch, int where, void* stream);
/* 3-D, space [d1][d2][d3] = Java's spc[i][j][k] (BasicTransform.java:509-565, :602-659):
 * forward = the 2-D forward of every slab i with (lvlP, lvlQ) (rows of d3 samples with lvlQ,
 * columns of d2 samples with lvlP), then the 1-D forward of every line along i with lvlR;
 * reverse = the 2-D reverse of every slab, then the 1-D reverse along i (the reference's
 * order).  BasicTransform.forward(double[][][]) passes lvlP = log2 d1, lvlQ = log2 d2,
 * lvlR = log2 d3 (:487-495): callers that mirror it pass those. */
int jw_fwt3d_forward(const jw_fwt_plan* plan, const double* x, double* y, int d1, int d2, int d3,
                     int lvlP, int lvlQ, int lvlR, int batch, int where, void* stream);
int jw_fwt3d_reverse(const jw_fwt_plan* plan, const double* y, double* x, int d1, int d2, int d3,
                     int lvlP, int lvlQ, int lvlR, int batch, int where, void* stream);

/* ======================================================================
 * CWT  (replaces ContinuousWaveletTransform.transformFFT :183-229 and
 *       transformFFTParallel :511-565, which compute the same values)
 * ====================================================================== */
#define JW_CWT_MORLET 0 /* MorletWavelet(fb, fc): params = {fb, fc} (MorletWavelet.java:66-124) */
#define JW_CWT_MEXHAT 1 /* MexicanHatWavelet(sigma): params = {sigma} (MexicanHatWavelet.java) */
#define JW_CWT_PAUL 2   /* PaulWavelet(m): params = {m}, integer 1..20 (PaulWavelet.java:76-99) */
#define JW_CWT_DOG 3    /* DOGWavelet(n, sigma): params = {n, sigma}, n integer 1..10
                           (DOGWavelet.java:129-157) */
#define JW_CWT_MEYER 4  /* MeyerWavelet(): no parameters (MeyerWavelet.java:164-169) */
/* ContinuousWaveletTransform.PaddingType (ContinuousWaveletTransform.java:74-79) */
#define JW_PAD_ZERO 0
#define JW_PAD_SYMMETRIC 1
#define JW_PAD_PERIODIC 2
#define JW_PAD_CONSTANT 3

/* coeffs[b][s][t] = IFFT(FFT(pad(x_b)) * conj(psi_hat(omega, scales[s], 0)))[t], t < n,
 * for batch signals x (batch x n); out_reim: batch x ns x n complex, interleaved (re, im).
 * scales: host array of ns positive scales (read at call time).  The padded length is
 * nextPowerOfTwo(n) <= 2^28 (past 2^26 in three passes; longer is JW_ERR_UNSUPPORTED).  Parameter checks follow the Java constructors:
 * fb, fc, sigma > 0 ("Bandwidth parameter must be positive", ...), Paul m and DOG n in range
 * ("Order parameter m must be a positive integer", ...), scales > 0 ("Scale must be positive";
 * not for Paul, whose fourierTransform(omega, scale, b) override :152-164 does not check).
 * psi_hat is complex for DOG with odd n and for Meyer; the product is X * conj(psi_hat). */
int jw_cwt_fft(int wavelet, const double* params, const double* x, long n, const double* scales,
               int ns, double sampling_rate, int padding, double* out_reim, int batch, int where,
               void* stream);
/* How jw_cwt_fft splits a call's scales (no device work, no data): *two_pass scales through
 * the two-pass FFT, *band through the one-pass band kernel, *coarse_grid through the coarse
 * grid + Kaiser-Bessel interpolation, under the engine's current settings
 * (jw_set_knob JW_CWT_BAND / JW_CWT_INTERP).  For measurement tools and tests; the counts
 * sum to ns.  Argument checks as jw_cwt_fft. */
int jw_cwt_fft_paths(int wavelet, const double* params, long n, const double* scales, int ns,
                     double sampling_rate, int* two_pass, int* band, int* coarse_grid);
/* ContinuousWaveletTransform.transform(signal, scales, fs) -- the direct time-domain CWT
 * (:153-172, computeCoefficient :240-260; transformParallel :470-500 and
 * transformParallelCustom :577-680 give the same values).  Same wavelet kinds and parameter
 * blocks as jw_cwt_fft; out_reim is B x ns x n interleaved (re, im).  JW_ARITH_STRICT is
 * bit-identical to the reference's sum order; JW_ARITH_FMA fuses each product into the sum.
 * O(n x support x scale) work: the reference's path for short signals. */
int jw_cwt_direct(int wavelet, const double* params, const double* x, long n,
                  const double* scales, int ns, double sampling_rate, int arith, double* out_reim,
                  int batch, int where, void* stream);

/* CWTResult accessors over coefficient arrays (device-resident for JW_DEVICE), so a scalogram
 * or magnitude map needs no copy of the complex coefficients to the host:
 *   jw_cwt_magnitude: out[i] = |c_i| = sqrt(re^2 + im^2)  -- CWTResult.getMagnitude
 *     (CWTResult.java:94-106, Complex.getMag :202-204), bit-identical to Java;
 *   jw_cwt_phase: Complex.getPhi's quadrant rules in radians -- CWTResult.getPhase (:113-126);
 *   jw_cwt_scalogram: energy[r] = sum_t |c[r][t]|^2 over rows of n coefficients --
 *     CWTResult.getScalogram (:272-287), tree-summed (within 1e-15 relative of Java's loop).
 * coef_reim: count (or rows x n) interleaved (re, im) values. */
int jw_cwt_magnitude(const double* coef_reim, long count, double* out, int where, void* stream);
int jw_cwt_phase(const double* coef_reim, long count, double* out, int where, void* stream);
int jw_cwt_scalogram(const double* coef_reim, long rows, long n, double* energy, int where,
                     void* stream);
/* ContinuousWaveletTransform.transformFFT(x_b, scales, fs).getScalogram() for batch signals
 * (ContinuousWaveletTransform.java:183-229 then CWTResult.java:272-287) with the coefficients
 * kept on the GPU (signals in chunks of <= ~2 GiB of coefficients): energy is batch x ns.
 * Argument checks and messages as jw_cwt_fft. */
int jw_cwt_fft_scalogram(int wavelet, const double* params, const double* x, long n,
                         const double* scales, int ns, double sampling_rate, int padding,
                         double* energy, int batch, int where, void* stream);

/* ======================================================================
 * Synthetic input (bench / tests): java.util.Random(seed0 + b).nextDouble()*2-1 for
 * signal b, generated in HBM with LCG jump-ahead.  Identical to the oracle's stream.
 * ====================================================================== */
int jw_synth_uniform(double* x_dev, long n, int batch, long seed0, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* JWAVE_HIP_H */
