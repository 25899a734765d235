// jw_internal.hpp -- shared internals of libjwave_hip.so (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <utility>
#include <vector>

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

// Workspaces come from a private stream-ordered memory pool per device (never the device's
// default pool, which PyTorch or a JVM's other libraries may tune).  The pool keeps what the
// workspaces free, so a call whose workspace is several GB (the 2-D FWT of cfg4: 6.4 GB) does
// not re-map it every time (~200 ms per call on some boxes when released at every sync); an
// allocation that fails trims the pool and retries once; jw_release_caches() trims it.
hipMemPool_t device_pool();  // the calling thread's current device's pool (created lazily)
void trim_pools();

// Stream-ordered device allocations of one call, released on every exit path (the early
// returns of JW_HIP_TRY included): hipFreeAsync on the call's stream, so the memory is
// reused only after the work queued on that stream has consumed it.
class StreamAllocs {
 public:
  explicit StreamAllocs(hipStream_t s) : s_(s) {}
  StreamAllocs(const StreamAllocs&) = delete;
  StreamAllocs& operator=(const StreamAllocs&) = delete;
  ~StreamAllocs() {
    for (size_t i = p_.size(); i-- > 0;) (void)hipFreeAsync(p_[i], s_);
  }
  template <class T>
  hipError_t alloc(T** out, size_t bytes) {
    *out = nullptr;
    hipMemPool_t pool = device_pool();
    if (!pool) return hipErrorOutOfMemory;
    void* p = nullptr;
    hipError_t e = hipMallocFromPoolAsync(&p, bytes, pool, s_);
    if (e == hipErrorOutOfMemory) {  // give back what the pool holds unused, then retry once
      (void)hipGetLastError();
      (void)hipStreamSynchronize(s_);
      (void)hipMemPoolTrimTo(pool, 0);
      e = hipMallocFromPoolAsync(&p, bytes, pool, s_);
    }
    if (e == hipSuccess) {
      p_.push_back(p);
      *out = (T*)p;
    }
    return e;
  }

 private:
  hipStream_t s_;
  std::vector<void*> p_;
};

// Calls in flight hold this shared; jw_release_caches() takes it exclusively, so no call is
// between looking up a cached table and launching the kernels that read it while it frees.
// A/B and test settings (JW_*): the environment read once per name, jw_set_knob overrides.
// The returned string is never freed (nullptr = unset).
const char* knob(const char* name);

std::shared_mutex& api_mutex();
void note_device_used(int dev);

// ---- library-owned device tables (twiddles, chirp-z, filter spectra, pair tables) ----
// Built on the caller's stream, synchronised once, then published; no lock is held across
// device work.  Each cache keeps at most `budget` bytes; beyond that a call builds a table of
// its own (stream-ordered, freed after the call).  jw_release_caches() clears them all.
class CacheBase {
 public:
  virtual ~CacheBase() = default;
  virtual size_t clear() = 0;
};
void register_cache(CacheBase* c);
size_t release_all_caches();  // bytes freed; the caller holds api_mutex() exclusively

template <class Key>
class DevCache : public CacheBase {
 public:
  explicit DevCache(size_t budget) : budget_(budget) { register_cache(this); }
  const void* find(const Key& k) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(k);
    return it == m_.end() ? nullptr : it->second.first;
  }
  bool fits(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    return bytes_ + bytes <= budget_;
  }
  // takes ownership of p (hipMalloc'd, complete); returns the entry to use -- another
  // thread's if it raced us, in which case p is freed
  const void* insert(const Key& k, void* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(k);
    if (it != m_.end()) {
      (void)hipFree(p);
      return it->second.first;
    }
    m_.emplace(k, std::make_pair(p, bytes));
    bytes_ += bytes;
    return p;
  }
  size_t clear() override {
    std::lock_guard<std::mutex> lk(mu_);
    const size_t b = bytes_;
    for (auto& e : m_) (void)hipFree(e.second.first);
    m_.clear();
    bytes_ = 0;
    return b;
  }

 private:
  std::mutex mu_;
  std::map<Key, std::pair<void*, size_t>> m_;
  size_t bytes_ = 0;
  size_t budget_;
};

// A cached table of `bytes` filled by fill(void* dst) on stream s (JW_OK or an error), or a
// per-call one past the budget.
template <class Key, class Fill>
int cached_table(DevCache<Key>& cache, const Key& key, size_t bytes, StreamAllocs& mem,
                 hipStream_t s, const void** out, Fill&& fill) {
  if ((*out = cache.find(key)) != nullptr) return JW_OK;
  // tests: a host allocation failure in a table build (the C-ABI's exception guard,
  // tests/test_jfft_limits_gpu.py)
  if (const char* t = knob("JW_TEST_THROW_BADALLOC"); t && t[0] == '1') throw std::bad_alloc();
  // A table is kept for the process only while it fits the cache's budget AND a quarter of the
  // device memory that is free right now, so a co-resident framework that holds most of HBM is
  // not starved by tables the engine would keep after the call.
  size_t free_b = 0, total_b = 0;
  const bool roomy = hipMemGetInfo(&free_b, &total_b) == hipSuccess && bytes <= free_b / 4;
  if (!roomy) (void)hipGetLastError();
  if (!roomy || !cache.fits(bytes)) {
    void* p = nullptr;
    JW_HIP_TRY(mem.alloc(&p, bytes));
    *out = p;
    return fill(p);
  }
  void* p = nullptr;
  JW_HIP_TRY(hipMalloc(&p, bytes));
  int st;
  try {
    st = fill(p);
  } catch (...) {  // reported by the C-ABI's guard (run_items); the table is not kept
    (void)hipStreamSynchronize(s);
    (void)hipFree(p);
    throw;
  }
  const hipError_t e = hipStreamSynchronize(s);  // complete before another thread may read it
  if (st != JW_OK || e != hipSuccess) {
    (void)hipFree(p);
    return st != JW_OK ? st : fail(JW_ERR_DEVICE, "table build: %s", hipGetErrorString(e));
  }
  *out = cache.insert(key, p, bytes);
  return JW_OK;
}

// Host -> device copy that stays asynchronous: the bytes are copied into a heap buffer that
// a host callback on the stream frees once the transfer has been reached (the caller's
// buffer may go away as soon as this returns).
hipError_t upload_async(void* dst, const void* src, size_t bytes, hipStream_t s);
// The same without the staging copy, for multi-GB tables: src comes from std::malloc and is
// owned by the stream from here on (freed by a host callback once the transfer is reached; on
// an error, after a stream synchronize).
hipError_t upload_owned(void* dst, void* src, size_t bytes, hipStream_t s);
// Host threads for table builds: OMP_NUM_THREADS when set, else the machine's, at most 16.
int host_threads();

// Correctly rounded sin and cos of x (jw_crmath.cc): the values of Math.sin / Math.cos the
// STRICT FFT tables use.
void cr_sincos(double x, double* s, double* c);

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
// FFT-path length ranges (inclusive, n >= 2).  The FMA pyramid (jw_modwt_fft.hip) takes
// n <= kPyramidFftMax; STRICT (JWave's own FFT, jw_jfft.hip) takes powers of two up to
// kStrictFftPow2Max and other n up to kStrictFftOtherMax (Bluestein, m <= 2^30).  Those are the
// reference's own limits: a Java int array length caps the powers of two at 2^30, and past
// n = 2^29 Bluestein's `int m` doubling loop (FastFourierTransform.java:261-265) overflows.  A
// STRICT level outside its range is JW_ERR_UNSUPPORTED, never the pyramid (not JWave's
// arithmetic): that is only sound while the STRICT range covers the pyramid's, which the
// assertion pins.
constexpr long kPyramidFftMax = 1L << 23;
constexpr long kStrictFftPow2Max = 1L << 30;
constexpr long kStrictFftOtherMax = kStrictFftPow2Max / 2;
static_assert(kPyramidFftMax <= kStrictFftOtherMax && kStrictFftOtherMax <= kStrictFftPow2Max,
              "the STRICT FFT range must contain the FMA pyramid's");
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
int cwt_fft_paths(int wavelet, const double* params, long n, const double* scales, int ns,
                  double fs, int* two_pass, int* band, int* coarse_grid);
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
