// jw_internal.hpp -- shared internals of libjwave_hip.so (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "jwave_hip.h"

namespace jw {

constexpr int kMaxTaps = 64;      // longest filter a plan accepts (Daubechies20 / Symlet20 = 40)
constexpr int kMaxModwtLevel = 13;  // MODWTTransform.MAX_DECOMPOSITION_LEVEL (MODWTTransform.java:111)

// Thread-local error text, returned by jw_last_error().
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void clear_error();

#define JW_HIP_TRY(expr)                                                                   \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return ::jw::fail(JW_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                               \
  } while (0)

// The device's default memory pool keeps what the workspaces free instead of returning it to
// the driver at every synchronisation (the default release threshold is 0): without this a
// call whose workspace is several GB (the 2-D FWT of cfg4: 6.4 GB) re-maps it every time,
// ~200 ms per call on some boxes.  Set once per device, on first use.
void keep_pool_memory();

// Stream-ordered device allocations of one call, released on every exit path (the early
// returns of JW_HIP_TRY included): hipFreeAsync on the call's stream, so the memory is
// reused only after the work queued on that stream has consumed it.
class StreamAllocs {
 public:
  explicit StreamAllocs(hipStream_t s) : s_(s) {}
  StreamAllocs(const StreamAllocs&) = delete;
  StreamAllocs& operator=(const StreamAllocs&) = delete;
  ~StreamAllocs() {
    for (int i = n_ - 1; i >= 0; --i) (void)hipFreeAsync(p_[i], s_);
  }
  template <class T>
  hipError_t alloc(T** out, size_t bytes) {
    *out = nullptr;
    if (n_ == kMax) return hipErrorOutOfMemory;
    keep_pool_memory();
    void* p = nullptr;
    const hipError_t e = hipMallocAsync(&p, bytes, s_);
    if (e == hipSuccess) {
      p_[n_++] = p;
      *out = (T*)p;
    }
    return e;
  }

 private:
  static constexpr int kMax = 16;
  hipStream_t s_;
  void* p_[kMax] = {};
  int n_ = 0;
};

// Host -> device copy that stays asynchronous: the bytes are copied into a heap buffer that
// a host callback on the stream frees once the transfer has been reached (the caller's
// buffer may go away as soon as this returns).
hipError_t upload_async(void* dst, const void* src, size_t bytes, hipStream_t s);

// Filter taps passed to kernels by value (lands in SGPRs: wave-uniform).
struct Taps {
  double a[kMaxTaps];
  double b[kMaxTaps];
};

// MODWT plan = an initialised MODWTTransform (filters cached, MODWTTransform.java:452-484).
struct ModwtPlan {
  int L;
  int fft_threshold;
  int arith;
  double g[kMaxTaps];  // g_modwt_base
  double h[kMaxTaps];  // h_modwt_base
};

struct FwtPlan {
  int M;
  int tw;
  int kind;
  int arith;
  double sD[kMaxTaps], wD[kMaxTaps], sR[kMaxTaps], wR[kMaxTaps];
};

// ---- launchers (return JW_OK or a JW_ERR_* with the error text set) ----
int modwt_forward_device(const ModwtPlan& p, const double* x, double* coeffs, long n, int J,
                         int batch, hipStream_t s);
int modwt_inverse_device(const ModwtPlan& p, const double* coeffs, double* x, long n, int J,
                         int batch, hipStream_t s);
bool modwt_fft_supported(long n);
int modwt_forward_fft_device(const ModwtPlan& p, const double* x, double* coeffs, long n, int J,
                             int batch, hipStream_t s);
int modwt_inverse_fft_device(const ModwtPlan& p, const double* coeffs, double* x, long n, int J,
                             int batch, hipStream_t s);
// JW_ARITH_STRICT FFT paths (jw_jfft.hip): the reference's own FFT, bit for bit.
// MODWT with fft_level[j] (j = 1..J) choosing each level's convolution like
// performConvolution (MODWTTransform.java:640-664); DIRECT levels run modwt_level_*_device.
bool modwt_strict_fft_supported(long n);
int modwt_forward_strict_device(const ModwtPlan& p, const double* x, double* coeffs, long n,
                                int J, int batch, const bool* fft_level, hipStream_t s);
int modwt_inverse_strict_device(const ModwtPlan& p, const double* coeffs, double* x, long n,
                                int J, int batch, const bool* fft_level, hipStream_t s);
int fft_strict_device(int S, const double* in, double* out, long n, long batch, hipStream_t s);
// Frees the cached twiddle / filter-spectrum / chirp tables of every FFT path (bytes freed).
size_t release_strict_caches();
size_t release_fft_caches();
// One direct MODWT level (circularConvolve{,Adjoint}, :677-716) on batch rows with strides:
// forward W_j, V_j <- V_{j-1}; inverse out = g_j^T V_j + h_j^T W_j.
int modwt_level_forward_device(const ModwtPlan& p, int j, const double* v, long vs, double* w,
                               long ws, double* vn, long vns, long N, int batch, hipStream_t s);
int modwt_level_inverse_device(const ModwtPlan& p, int j, const double* v, long vs,
                               const double* w, long ws, double* out, long os, long N, int batch,
                               hipStream_t s);
// FastFourierTransform.forward (S = -1) / reverse (S = +1, scaled by 1/n) of batch lines of n
// interleaved complex values in HBM; in == out allowed.
int fft_device(int S, const double* in, double* out, long n, long batch, hipStream_t s);
int cwt_fft_device(int wavelet, const double* params, const double* x, long n,
                   const double* scales_host, int ns, double fs, int padding, double* out,
                   int batch, hipStream_t s);
int cwt_magnitude_device(const double* c, long count, double* out, hipStream_t s);
int cwt_phase_device(const double* c, long count, double* out, hipStream_t s);
int cwt_scalogram_device(const double* c, long rows, long n, double* energy, hipStream_t s);
int cwt_direct_device(int wavelet, const double* params, const double* x, long n,
                      const double* scales, int ns, double fs, int arith, double* out, int batch,
                      hipStream_t s);
// Direct CWT window of one scale: (int)(support[0] a fs), (int)(support[1] a fs) as doubles.
void cwt_direct_support(int wavelet, const double* params, double a, double fs, double* lo,
                        double* hi);
bool cwt_direct_window_nonempty(double lo, double hi, long n);
int wpt_forward_device(const FwtPlan& p, const double* x, double* y, long n, int level, int batch,
                       hipStream_t s);
int wpt_reverse_device(const FwtPlan& p, const double* y, double* x, long n, int level, int batch,
                       hipStream_t s);
int fwt_forward_device(const FwtPlan& p, const double* x, double* y, long n, int level, int batch,
                       hipStream_t s);
int fwt_reverse_device(const FwtPlan& p, const double* y, double* x, long n, int level, int batch,
                       hipStream_t s);
int fwt2d_forward_device(const FwtPlan& p, const double* x, double* y, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s);
int fwt2d_reverse_device(const FwtPlan& p, const double* y, double* x, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s);
int fwt3d_forward_device(const FwtPlan& p, const double* x, double* y, int R, int C, int H,
                         int lvlP, int lvlQ, int lvlR, int batch, hipStream_t s);
int fwt3d_reverse_device(const FwtPlan& p, const double* y, double* x, int R, int C, int H,
                         int lvlP, int lvlQ, int lvlR, int batch, hipStream_t s);
int synth_uniform_device(double* x, long n, int batch, long seed0, hipStream_t s);

}  // namespace jw
