// jw_capi.cpp -- the extern "C" boundary (include/jwave_hip.h): argument validation with the
// reference's exception classes and messages, plan objects, host<->HBM staging.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <exception>
#include <thread>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "jw_internal.hpp"

namespace jw {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

void clear_error() { g_err[0] = '\0'; }

// ---- private memory pools (one per device), calls in flight, cache registry ----
namespace {
std::mutex g_pool_mu;
hipMemPool_t g_pools[64] = {};
std::atomic<uint64_t> g_used_devices{0};  // bit d: a call ran on device d
}  // namespace

hipMemPool_t device_pool() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (!g_pools[dev]) {
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) return nullptr;
    uint64_t keep = UINT64_MAX;  // keep freed workspaces for the next call
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    g_pools[dev] = pool;
  }
  return g_pools[dev];
}

void trim_pools() {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (hipMemPool_t p : g_pools)
    if (p) (void)hipMemPoolTrimTo(p, 0);
}

std::shared_mutex& api_mutex() {
  static std::shared_mutex m;
  return m;
}

namespace {
std::mutex g_knob_mu;
std::map<std::string, const std::string*>& knobs() {  // values are never freed: callers keep them
  static std::map<std::string, const std::string*> m;
  return m;
}
}  // namespace

const char* knob(const char* name) {
  std::lock_guard<std::mutex> lk(g_knob_mu);
  auto& m = knobs();
  auto it = m.find(name);
  if (it == m.end()) {
    const char* e = std::getenv(name);
    it = m.emplace(name, e ? new std::string(e) : nullptr).first;
  }
  return it->second ? it->second->c_str() : nullptr;
}

void note_device_used(int dev) {
  if (dev >= 0 && dev < 64) g_used_devices.fetch_or(1ULL << dev, std::memory_order_relaxed);
}

namespace {
std::vector<CacheBase*>& cache_registry() {
  static std::vector<CacheBase*> r;
  return r;
}
std::mutex& registry_mutex() {
  static std::mutex m;
  return m;
}
}  // namespace

void register_cache(CacheBase* c) {
  std::lock_guard<std::mutex> lk(registry_mutex());
  cache_registry().push_back(c);
}

size_t release_all_caches() {
  std::lock_guard<std::mutex> lk(registry_mutex());
  size_t b = 0;
  for (CacheBase* c : cache_registry()) b += c->clear();
  return b;
}

namespace {

// floor(log2 n) as the reference computes it for ints: 31 - numberOfLeadingZeros(N)
// (MODWTTransform.java:278).
int floor_log2(long n) {
  int e = -1;
  while (n > 0) {
    n >>= 1;
    ++e;
  }
  return e;
}

bool is_binary(long n) { return n > 0 && (n & (n - 1)) == 0; }  // MathToolKit.isBinary :185-188

// ---- JW_HOST staging (what a JNI crossing with double[] uses) ----
// Host copies between the caller's pageable arrays and the pinned bounce buffers run on a
// small pool of worker threads (one memcpy thread moves ~10 GB/s, PCIe 5 x16 ~50 GB/s per
// direction); the calling thread takes a share too.  Workers: JW_COPY_THREADS, else half of
// OMP_NUM_THREADS (the GPU box's per-GPU CPU share is 16) or of the hardware threads, <= 8.
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool();  // never destroyed: detached workers outlive main
    return *p;
  }
  void copy(void* dst, const void* src, size_t bytes) {
    const int parts = bytes >= (4u << 20) ? workers_ + 1 : 1;
    if (parts == 1) {
      std::memcpy(dst, src, bytes);
      return;
    }
    const size_t per = ((bytes + parts - 1) / parts + 4095) & ~(size_t)4095;
    std::atomic<int> left{0};
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (int i = 1; i < parts; ++i) {
        const size_t off = per * (size_t)i;
        if (off >= bytes) break;
        left.fetch_add(1, std::memory_order_relaxed);
        q_.push_back(Job{(char*)dst + off, (const char*)src + off, std::min(per, bytes - off),
                         &left});
      }
    }
    cv_.notify_all();
    std::memcpy(dst, src, std::min(per, bytes));
    while (left.load(std::memory_order_acquire) > 0) {  // help, then wait for our parts
      Job j;
      if (pop(&j)) {
        run(j);
      } else {
        std::this_thread::yield();
      }
    }
  }

 private:
  struct Job {
    char* d;
    const char* s;
    size_t n;
    std::atomic<int>* left;
  };
  CopyPool() {
    int t = 0;
    if (const char* e = knob("JW_COPY_THREADS")) {
      workers_ = std::max(0, std::atoi(e) - 1);
    } else {
      if (const char* o = std::getenv("OMP_NUM_THREADS")) t = std::atoi(o);
      if (t <= 0) t = (int)std::thread::hardware_concurrency();
      workers_ = std::min(7, std::max(0, t / 2 - 1));
    }
    for (int i = 0; i < workers_; ++i) std::thread([this] { loop(); }).detach();
  }
  bool pop(Job* j) {
    std::lock_guard<std::mutex> lk(mu_);
    if (q_.empty()) return false;
    *j = q_.front();
    q_.pop_front();
    return true;
  }
  static void run(const Job& j) {
    std::memcpy(j.d, j.s, j.n);
    j.left->fetch_sub(1, std::memory_order_release);
  }
  void loop() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !q_.empty(); });
        j = q_.front();
        q_.pop_front();
      }
      run(j);
    }
  }
  int workers_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
};

// Per host thread and device: a private non-blocking stream when the caller passes none
// (threads never meet on the null stream), one copy stream per direction, and two pinned
// bounce buffers per direction (memcpy of chunk k+1 beside the DMA of chunk k).  The HBM copies
// of the caller's arrays come from the library's memory pool per call.
// doubles per bounce buffer: 32 MiB (JW_PIN_MB for A/B runs)
size_t pin_doubles() {
  static const size_t v = [] {
    const char* e = knob("JW_PIN_MB");
    const long mb = e ? std::atol(e) : 32;
    return (size_t)std::max(1L, mb) << 17;
  }();
  return v;
}

// bounce buffers per direction: a ring of pin_ring() (JW_PIN_RING for A/B runs, 2..4)
constexpr int kMaxRing = 4;
int pin_ring() {
  static const int v = [] {
    const char* e = knob("JW_PIN_RING");
    const int r = e ? std::atoi(e) : 3;
    return std::max(2, std::min(kMaxRing, r));
  }();
  return v;
}

struct HostStage {
  int dev = -1;
  hipStream_t own = nullptr, h2d = nullptr, d2h = nullptr;
  double* pin_in[kMaxRing] = {};
  double* pin_out[kMaxRing] = {};
  hipEvent_t ev_in[kMaxRing] = {}, ev_out[kMaxRing] = {};  // bounce buffer reuse
  hipEvent_t loaded[2] = {}, done[2] = {}, drained[2] = {};  // sub-batch pipeline
  hipEvent_t allocated = nullptr;  // the workspaces' stream-ordered allocation, on the caller's stream

  ~HostStage() {
    if (dev < 0) return;
    (void)hipSetDevice(dev);
    for (hipStream_t s : {own, h2d, d2h})
      if (s) (void)hipStreamSynchronize(s);
    for (int i = 0; i < kMaxRing; ++i) {
      if (pin_in[i]) (void)hipHostFree(pin_in[i]);
      if (pin_out[i]) (void)hipHostFree(pin_out[i]);
      for (hipEvent_t e : {ev_in[i], ev_out[i]})
        if (e) (void)hipEventDestroy(e);
    }
    for (int i = 0; i < 2; ++i)
      for (hipEvent_t e : {loaded[i], done[i], drained[i]})
        if (e) (void)hipEventDestroy(e);
    if (allocated) (void)hipEventDestroy(allocated);
    for (hipStream_t s : {own, h2d, d2h})
      if (s) (void)hipStreamDestroy(s);
  }

  int init(int device) {
    dev = device;
    for (hipStream_t* s : {&own, &h2d, &d2h})
      JW_HIP_TRY(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
    for (int i = 0; i < pin_ring(); ++i) {
      JW_HIP_TRY(hipHostMalloc((void**)&pin_in[i], pin_doubles() * sizeof(double),
                               hipHostMallocDefault));
      JW_HIP_TRY(hipHostMalloc((void**)&pin_out[i], pin_doubles() * sizeof(double),
                               hipHostMallocDefault));
      for (hipEvent_t* e : {&ev_in[i], &ev_out[i]})
        JW_HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    for (int i = 0; i < 2; ++i)
      for (hipEvent_t* e : {&loaded[i], &done[i], &drained[i]})
        JW_HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    JW_HIP_TRY(hipEventCreateWithFlags(&allocated, hipEventDisableTiming));
    return JW_OK;
  }

  // host -> HBM through the bounce ring on stream cs; returns when the host buffer may be
  // reused (the last DMAs may still be in flight on cs)
  int put(double* dst, const double* src, size_t n, hipStream_t cs) {
    const int R = pin_ring();
    for (size_t off = 0, k = 0; off < n; off += pin_doubles(), ++k) {
      const size_t c = std::min(pin_doubles(), n - off);
      const int b = (int)(k % R);
      JW_HIP_TRY(hipEventSynchronize(ev_in[b]));  // this buffer's previous DMA has landed
      CopyPool::get().copy(pin_in[b], src + off, c * sizeof(double));
      JW_HIP_TRY(hipMemcpyAsync(dst + off, pin_in[b], c * sizeof(double), hipMemcpyHostToDevice, cs));
      JW_HIP_TRY(hipEventRecord(ev_in[b], cs));
    }
    return JW_OK;
  }

  // HBM -> host after the work queued on cs: up to R - 1 chunk DMAs in flight ahead of the
  // host copy of the oldest one
  int get(double* dst, const double* src, size_t n, hipStream_t cs) {
    const int R = pin_ring();
    const size_t P = pin_doubles();
    const size_t nch = (n + P - 1) / P;
    auto drain = [&](size_t k) -> int {  // chunk k's DMA has landed: copy it out
      const int b = (int)(k % R);
      const size_t off = k * P, c = std::min(P, n - off);
      JW_HIP_TRY(hipEventSynchronize(ev_out[b]));
      CopyPool::get().copy(dst + off, pin_out[b], c * sizeof(double));
      return JW_OK;
    };
    for (size_t k = 0; k < nch; ++k) {
      if (k >= (size_t)R) {  // buffer k % R is free once chunk k - R has been copied out
        const int r = drain(k - R);
        if (r != JW_OK) return r;
      }
      const int b = (int)(k % R);
      const size_t off = k * P, c = std::min(P, n - off);
      JW_HIP_TRY(hipMemcpyAsync(pin_out[b], src + off, c * sizeof(double), hipMemcpyDeviceToHost, cs));
      JW_HIP_TRY(hipEventRecord(ev_out[b], cs));
    }
    for (size_t k = nch > (size_t)R ? nch - R : 0; k < nch; ++k) {
      const int r = drain(k);
      if (r != JW_OK) return r;
    }
    return JW_OK;
  }
};

int host_stage(HostStage** out) {
  static thread_local std::vector<std::unique_ptr<HostStage>> stages;  // by device ordinal
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  if ((size_t)dev >= stages.size()) stages.resize(dev + 1);
  if (!stages[dev]) {
    auto st = std::make_unique<HostStage>();
    const int rc = st->init(dev);
    if (rc != JW_OK) return rc;
    stages[dev] = std::move(st);
  }
  *out = stages[dev].get();
  return JW_OK;
}

int check_where(int where) {
  if (where != JW_HOST && where != JW_DEVICE)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "where must be JW_HOST (0) or JW_DEVICE (1), got %d",
                where);
  return JW_OK;
}

// Runs f(din, dout, items, s) over `items` independent items (signals, images, lines) of
// in_per doubles in and out_per doubles out.  JW_DEVICE: the caller's HBM pointers, async on
// the caller's stream.  JW_HOST: staged through HBM in sub-batches of ~128 MiB, pipelined over
// three streams -- the host->HBM copy of sub-batch k+1 and the HBM->host copy of k-1 beside the
// compute of k -- and synchronised before returning.
constexpr size_t kSubDoubles = (size_t)16 << 20;  // 128 MiB of input + output per sub-batch

// f's work behind the C-ABI: a C++ exception (a multi-GB host table that cannot be allocated,
// a thread that cannot be started) becomes a status and an error text, never an unwind into
// the caller (a JVM through JNI, ctypes)
template <class F, class... A>
int guarded(F& f, A... a) {
  try {
    return f(a...);
  } catch (const std::bad_alloc&) {
    return fail(JW_ERR_NO_MEMORY, "host memory exhausted (std::bad_alloc)");
  } catch (const std::exception& e) {
    return fail(JW_ERR_FAILURE, "C++ exception: %s", e.what());
  } catch (...) {
    return fail(JW_ERR_FAILURE, "unknown C++ exception");
  }
}

template <class F>
int run_items(int where, void* stream, const double* in, size_t in_per, double* out,
              size_t out_per, long items, F&& f) {
  std::shared_lock<std::shared_mutex> in_flight(api_mutex());
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  note_device_used(dev);
  hipStream_t s = (hipStream_t)stream;
  if (where == JW_DEVICE) return guarded(f, in, out, items, s);
  HostStage* hs = nullptr;
  int st = host_stage(&hs);
  if (st != JW_OK) return st;
  if (!s) s = hs->own;
  const size_t per = std::max<size_t>(1, in_per + out_per);
  const long sub = std::max(1L, std::min<long>(items, (long)(kSubDoubles / per)));
  const long nsub = (items + sub - 1) / sub;
  hipError_t e1 = hipSuccess, e2 = hipSuccess, e3 = hipSuccess;
  {
    StreamAllocs mem(s);
    double *din[2] = {}, *dout[2] = {};
    for (int b = 0; b < (nsub > 1 ? 2 : 1); ++b) {
      JW_HIP_TRY(mem.alloc(&din[b], (size_t)sub * in_per * sizeof(double) + 8));
      JW_HIP_TRY(mem.alloc(&dout[b], (size_t)sub * out_per * sizeof(double) + 8));
    }
    // The pool may hand back blocks whose earlier hipFreeAsync (another call's workspace, or a
    // JW_DEVICE call queued on the same stream) is ordered only on s: the H2D stream must not
    // write into them before s reaches this point.
    JW_HIP_TRY(hipEventRecord(hs->allocated, s));
    JW_HIP_TRY(hipStreamWaitEvent(hs->h2d, hs->allocated, 0));
    auto count = [&](long k) { return std::min(sub, items - k * sub); };
    auto put = [&](long k) -> int {  // din[k&1] is free once f(k-2) has run
      const int b = (int)(k & 1);
      if (k >= 2) JW_HIP_TRY(hipStreamWaitEvent(hs->h2d, hs->done[b], 0));
      int r = hs->put(din[b], in + (size_t)k * sub * in_per, (size_t)count(k) * in_per, hs->h2d);
      if (r == JW_OK) JW_HIP_TRY(hipEventRecord(hs->loaded[b], hs->h2d));
      return r;
    };
    auto compute = [&](long k) -> int {  // dout[k&1] is free once sub-batch k-2 has drained
      const int b = (int)(k & 1);
      JW_HIP_TRY(hipStreamWaitEvent(s, hs->loaded[b], 0));
      if (k >= 2) JW_HIP_TRY(hipStreamWaitEvent(s, hs->drained[b], 0));
      int r = guarded(f, (const double*)din[b], dout[b], count(k), s);
      if (r == JW_OK) JW_HIP_TRY(hipEventRecord(hs->done[b], s));
      return r;
    };
    auto get = [&](long k) -> int {
      const int b = (int)(k & 1);
      JW_HIP_TRY(hipStreamWaitEvent(hs->d2h, hs->done[b], 0));
      int r = hs->get(out + (size_t)k * sub * out_per, dout[b], (size_t)count(k) * out_per, hs->d2h);
      if (r == JW_OK) JW_HIP_TRY(hipEventRecord(hs->drained[b], hs->d2h));
      return r;
    };
    st = put(0);
    if (st == JW_OK) st = compute(0);
    for (long k = 1; k < nsub && st == JW_OK; ++k) {
      st = put(k);
      if (st == JW_OK) st = compute(k);
      if (st == JW_OK) st = get(k - 1);
    }
    if (st == JW_OK) st = get(nsub - 1);
    // everything queued on the three streams has finished before the workspaces go back to
    // the pool (in s's order) and before the caller may reuse its arrays
    e1 = hipStreamSynchronize(hs->h2d);
    e2 = hipStreamSynchronize(s);
    e3 = hipStreamSynchronize(hs->d2h);
  }
  const hipError_t e4 = hipStreamSynchronize(s);
  if (st != JW_OK) return st;
  for (hipError_t e : {e1, e2, e3, e4})
    if (e != hipSuccess)
      return fail(JW_ERR_DEVICE, "hipStreamSynchronize failed: %s", hipGetErrorString(e));
  return JW_OK;
}

}  // namespace

hipError_t upload_async(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  void* tmp = std::malloc(bytes);
  if (!tmp) return hipErrorOutOfMemory;
  std::memcpy(tmp, src, bytes);
  hipError_t e = hipMemcpyAsync(dst, tmp, bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipLaunchHostFunc(s, [](void* p) { std::free(p); }, tmp);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(s);
    std::free(tmp);
  }
  return e;
}

hipError_t upload_owned(void* dst, void* src, size_t bytes, hipStream_t s) {
  hipError_t e = bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
  if (e == hipSuccess) e = hipLaunchHostFunc(s, [](void* p) { std::free(p); }, src);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(s);
    std::free(src);
  }
  return e;
}

int host_threads() {
  int t = 0;
  if (const char* o = std::getenv("OMP_NUM_THREADS")) t = std::atoi(o);
  if (t <= 0) t = (int)std::thread::hardware_concurrency();
  return std::min(16, std::max(1, t));
}
}  // namespace jw

using namespace jw;

struct jw_modwt_plan : ModwtPlan {};
struct jw_fwt_plan : FwtPlan {};

extern "C" {

const char* jw_last_error(void) { return g_err; }

const char* jw_version(void) { return "jwave-pro_amd 0.3.0 (gfx950)"; }

// ---------------------------------------------------------------------------------------- device
int jw_device_count(int* count) {
  clear_error();
  if (!count) return fail(JW_ERR_ILLEGAL_ARGUMENT, "count pointer is null");
  *count = 0;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return JW_OK;  // no HIP device visible
  }
  *count = n;
  return JW_OK;
}

int jw_set_device(int ordinal) {
  clear_error();
  if (ordinal < 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "device ordinal must be >= 0, got %d", ordinal);
  int n = 0;
  jw_device_count(&n);
  if (ordinal >= n)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "device ordinal %d out of range: %d HIP device(s) visible",
                ordinal, n);
  JW_HIP_TRY(hipSetDevice(ordinal));
  return JW_OK;
}

int jw_get_device(int* ordinal) {
  clear_error();
  if (!ordinal) return fail(JW_ERR_ILLEGAL_ARGUMENT, "ordinal pointer is null");
  JW_HIP_TRY(hipGetDevice(ordinal));
  return JW_OK;
}

// Frees every table the library caches (FFT twiddles, chirp-z tables, MODWT filter spectra and
// pair tables) on every device and returns the memory pools' unused workspace memory.  Calls
// in flight on other threads finish first (they hold the API lock shared); kernels they queued
// asynchronously (JW_DEVICE) are waited for before anything is freed.
long jw_release_caches(void) {
  clear_error();
  std::unique_lock<std::shared_mutex> lk(api_mutex());
  int cur = 0;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  const uint64_t used = g_used_devices.load();
  for (int d = 0; d < 64; ++d) {
    if (!(used >> d & 1)) continue;
    if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
  }
  if (have_cur) (void)hipSetDevice(cur);
  const size_t freed = release_all_caches();
  trim_pools();
  return (long)freed;
}

int jw_set_knob(const char* name, const char* value) {
  clear_error();
  if (!name || std::strncmp(name, "JW_", 3) != 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "setting name must start with JW_");
  // sized once per process (the pinned bounce buffers and the copy-thread pool are built on
  // first use): a later replacement could not take effect, so it is refused, not ignored
  for (const char* fixed : {"JW_PIN_MB", "JW_PIN_RING", "JW_COPY_THREADS"})
    if (std::strcmp(name, fixed) == 0)
      return fail(JW_ERR_ILLEGAL_ARGUMENT,
                  "%s is fixed at first use; set it in the environment before the first call",
                  name);
  (void)knob(name);  // the environment's value first, so it is not read later over this one
  std::lock_guard<std::mutex> lk(g_knob_mu);
  knobs()[name] = value ? new std::string(value) : nullptr;  // the old value stays allocated
  return JW_OK;
}

const char* jw_get_knob(const char* name) {
  clear_error();
  return name ? knob(name) : nullptr;
}

// ---------------------------------------------------------------- MODWT
int jw_modwt_plan_create(jw_modwt_plan** plan, const double* scaling_dec,
                         const double* wavelet_dec, int L, int fft_threshold, int arith) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan pointer is null");
  *plan = nullptr;
  if (!scaling_dec || !wavelet_dec) return fail(JW_ERR_ILLEGAL_ARGUMENT, "filter pointer is null");
  if (L < 1 || L > kMaxTaps)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "filter length must be in [1, %d], got %d", kMaxTaps, L);
  if (arith != JW_ARITH_STRICT && arith != JW_ARITH_FMA)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown arithmetic mode %d", arith);
  auto* p = new (std::nothrow) jw_modwt_plan();
  if (!p) return fail(JW_ERR_NO_MEMORY, "out of host memory");
  p->L = L;
  p->fft_threshold = fft_threshold;
  p->arith = arith;
  // initializeFilterCache (MODWTTransform.java:462-475) with normalize (:599-606); host code
  // is compiled with -ffp-contract=off, so this is the JVM's sequence.
  double gd[kMaxTaps], hd[kMaxTaps];
  for (int i = 0; i < L; ++i) {
    gd[i] = scaling_dec[i];
    hd[i] = wavelet_dec[i];
  }
  for (double* f : {gd, hd}) {
    double energy = 0.0;
    for (int i = 0; i < L; ++i) energy += f[i] * f[i];
    const double norm = std::sqrt(energy);
    if (norm > 1e-12)
      for (int i = 0; i < L; ++i) f[i] /= norm;
  }
  const double scale = std::sqrt(2.0);
  for (int i = 0; i < L; ++i) {
    p->g[i] = gd[i] / scale;
    p->h[i] = hd[i] / scale;
  }
  *plan = p;
  return JW_OK;
}

void jw_modwt_plan_destroy(jw_modwt_plan* plan) { delete plan; }

int jw_modwt_plan_filters(const jw_modwt_plan* plan, double* g, double* h) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  for (int i = 0; i < plan->L; ++i) {
    if (g) g[i] = plan->g[i];
    if (h) h[i] = plan->h[i];
  }
  return JW_OK;
}

static int modwt_method_check(int method) {
  if (method == JW_CONV_AUTO || method == JW_CONV_DIRECT || method == JW_CONV_FFT) return JW_OK;
  return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown convolution method %d", method);
}

// MODWTTransform.performConvolution AUTO (:640-664): a level's convolution takes the FFT path
// when signal.length * filter.length > fftConvolutionThreshold, a Java int multiply (it wraps
// for N*M >= 2^31, :653).  The up-sampled level-j filter has M_j = (L-1)*2^(j-1) + 1 taps.
static bool auto_level_fft(long n, int L, int j, int threshold) {
  const uint32_t m = (uint32_t)(L - 1) * (1u << (j - 1)) + 1u;
  const int32_t prod = (int32_t)((uint32_t)n * m);
  return prod > threshold;
}

// Which implementation runs a MODWT call.
//   JW_ARITH_STRICT (the JVM's arithmetic): every level takes the convolution the reference's
//     performConvolution takes (:640-664) -- FFT always, DIRECT never, AUTO by the int32
//     N*M_j > fftConvolutionThreshold rule -- and FFT levels run the reference's own FFT
//     (jw_jfft.hip), so results are the JVM's bit for bit.  A length outside that path's range
//     (kStrictFftPow2Max / kStrictFftOtherMax, jw_internal.hpp) is JW_ERR_UNSUPPORTED when any
//     level is FFT: the exact-twiddle pyramid is never a STRICT result.
//   JW_ARITH_FMA (fast contract): FFT runs the exact-twiddle frequency-domain pyramid; AUTO and
//     DIRECT run the direct kernels, which are faster and more accurate than any FFT path here.
//   A level the reference would run through its FFT at a length the FFT paths do not take
//     (STRICT: powers of two past 2^30, other n past 2^29; FMA's pyramid: n past 2^23) is
//     JW_ERR_UNSUPPORTED with the limit in the message -- never a silent switch to DIRECT, whose
//     values differ from the JVM's FFT path by up to ~1e-10.
enum class ModwtPath { kDirect, kStrictLevels, kPyramid, kUnsupported };

static ModwtPath modwt_path(const ModwtPlan& p, int method, long n, int levels, bool* fft) {
  bool any = false;
  for (int j = 1; j <= levels; ++j) {
    fft[j] = method == JW_CONV_FFT ||
             (method == JW_CONV_AUTO && auto_level_fft(n, p.L, j, p.fft_threshold));
    any = any || fft[j];
  }
  if (p.arith == JW_ARITH_FMA) {
    if (method != JW_CONV_FFT) return ModwtPath::kDirect;
    return modwt_fft_supported(n) ? ModwtPath::kPyramid : ModwtPath::kUnsupported;
  }
  if (!any) return ModwtPath::kDirect;
  return modwt_strict_fft_supported(n) ? ModwtPath::kStrictLevels : ModwtPath::kUnsupported;
}

static int modwt_unsupported(int arith, int method, long n, const bool* fft, int levels) {
  int j = 1;
  while (j < levels && !fft[j]) ++j;
  char lim[128];
  if (arith == JW_ARITH_STRICT)
    std::snprintf(lim, sizeof lim, "powers of two up to 2^%d (%ld) and other lengths up to 2^%d (%ld)",
                  floor_log2(kStrictFftPow2Max), kStrictFftPow2Max, floor_log2(kStrictFftOtherMax),
                  kStrictFftOtherMax);
  else
    std::snprintf(lim, sizeof lim, "2 <= N <= 2^%d (%ld)", floor_log2(kPyramidFftMax), kPyramidFftMax);
  return fail(JW_ERR_UNSUPPORTED,
              "MODWT FFT convolution (%s) at signal length %ld: level %d takes the FFT path "
              "(MODWTTransform.java:640-664) and this engine's %s FFT convolution supports %s; "
              "use ConvolutionMethod.DIRECT%s",
              method == JW_CONV_FFT ? "ConvolutionMethod.FFT" : "AUTO", n, j,
              arith == JW_ARITH_STRICT ? "STRICT" : "FMA", lim,
              method == JW_CONV_AUTO ? " or a larger fftConvolutionThreshold" : "");
}

int jw_modwt_forward(const jw_modwt_plan* plan, const double* x, double* coeffs, long n,
                     int levels, int batch, int method, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  // MODWTTransform.forwardMODWT validation order (:257-282).
  if (levels < 1)
    return fail(JW_ERR_ILLEGAL_ARGUMENT,
                "MODWTTransform#forwardMODWT - decomposition level must be at least 1, "
                "requested: %d",
                levels);
  if (levels > kMaxModwtLevel)
    return fail(JW_ERR_ILLEGAL_ARGUMENT,
                "MODWTTransform#forwardMODWT - maximum supported decomposition level is %d, "
                "requested: %d",
                kMaxModwtLevel, levels);
  if (n == 0 || batch == 0) return JW_OK;  // empty data -> levels+1 empty rows (:266-273)
  if (n < 0 || batch < 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative length %ld or batch %d", n, batch);
  const int theoretical = floor_log2(n);
  if (levels > theoretical)
    return fail(JW_ERR_ILLEGAL_ARGUMENT,
                "Decomposition level %d exceeds theoretical limit %d for signal length %ld",
                levels, theoretical, n);
  int st = modwt_method_check(method);
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (!x || !coeffs) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  bool fft[kMaxModwtLevel + 1] = {};
  const ModwtPath path = modwt_path(*plan, method, n, levels, fft);
  if (path == ModwtPath::kUnsupported) return modwt_unsupported(plan->arith, method, n, fft, levels);
  return run_items(where, stream, x, (size_t)n, coeffs, (size_t)n * (levels + 1), batch,
                   [&](const double* dx, double* dc, long nb, hipStream_t s) {
                     switch (path) {
                       case ModwtPath::kStrictLevels:
                         return modwt_forward_strict_device(*plan, dx, dc, n, levels, (int)nb, fft, s);
                       case ModwtPath::kPyramid:
                         return modwt_forward_fft_device(*plan, dx, dc, n, levels, (int)nb, s);
                       default:
                         return modwt_forward_device(*plan, dx, dc, n, levels, (int)nb, s);
                     }
                   });
}

int jw_modwt_inverse(const jw_modwt_plan* plan, const double* coeffs, double* x, long n,
                     int levels, int batch, int method, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  // inverseMODWT (:337-375): fewer than 2 rows -> empty result; upsample rejects j > 13 (:620).
  if (levels < 1 || n == 0 || batch == 0) return JW_OK;
  if (levels > kMaxModwtLevel)
    return fail(JW_ERR_ILLEGAL_ARGUMENT,
                "MODWTTransform#upsample - maximum supported decomposition level is %d, "
                "requested: %d",
                kMaxModwtLevel, levels);
  if (n < 0 || batch < 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative length %ld or batch %d", n, batch);
  int st = modwt_method_check(method);
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (!x || !coeffs) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  bool fft[kMaxModwtLevel + 1] = {};
  const ModwtPath path = modwt_path(*plan, method, n, levels, fft);
  if (path == ModwtPath::kUnsupported) return modwt_unsupported(plan->arith, method, n, fft, levels);
  return run_items(where, stream, coeffs, (size_t)n * (levels + 1), x, (size_t)n, batch,
                   [&](const double* dc, double* dx, long nb, hipStream_t s) {
                     switch (path) {
                       case ModwtPath::kStrictLevels:
                         return modwt_inverse_strict_device(*plan, dc, dx, n, levels, (int)nb, fft, s);
                       case ModwtPath::kPyramid:
                         return modwt_inverse_fft_device(*plan, dc, dx, n, levels, (int)nb, s);
                       default:
                         return modwt_inverse_device(*plan, dc, dx, n, levels, (int)nb, s);
                     }
                   });
}

// ---------------------------------------------------------------- FFT
// FastFourierTransform.forward / reverse(Complex[]) (FastFourierTransform.java:112-164):
// length 0 -> nothing, 1 -> a copy, powers of two -> Cooley-Tukey, others -> Bluestein.
static int fft_call(int S, int arith, const double* in, double* out, long n, int batch, int where,
                    void* stream) {
  clear_error();
  if (arith != JW_ARITH_STRICT && arith != JW_ARITH_FMA)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown arithmetic mode %d", arith);
  if (n < 0 || batch < 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative length %ld or batch %d", n, batch);
  int st = check_where(where);
  if (st != JW_OK) return st;
  if (n == 0 || batch == 0) return JW_OK;
  if (!in || !out) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  // STRICT: the reference's own FFT (jw_jfft.hip): radix 2 for powers of two, Bluestein for
  // other n, over the reference's own domain (jw_internal.hpp kStrictFft*)
  const bool pow2 = (n & (n - 1)) == 0;
  const bool strict = arith == JW_ARITH_STRICT;
  if (strict && n > (pow2 ? kStrictFftPow2Max : kStrictFftOtherMax))
    return fail(JW_ERR_UNSUPPORTED,
                "JW_ARITH_STRICT FFT (FastFourierTransform.java:112-324 operation for operation) "
                "at length %ld: supported up to 2^%d (%ld) for powers of two and 2^%d (%ld) "
                "otherwise (Bluestein's m <= 2^%d), the reference's own int limits",
                n, floor_log2(kStrictFftPow2Max), kStrictFftPow2Max, floor_log2(kStrictFftOtherMax),
                kStrictFftOtherMax, floor_log2(kStrictFftPow2Max));
  return run_items(where, stream, in, (size_t)2 * n, out, (size_t)2 * n, batch,
                   [&](const double* di, double* dout, long nb, hipStream_t s) {
                     return strict ? fft_strict_device(S, di, dout, n, nb, s)
                                   : fft_device(S, di, dout, n, nb, s);
                   });
}

int jw_fft_forward(const double* in_reim, double* out_reim, long n, int batch, int where,
                   void* stream) {
  return fft_call(-1, JW_ARITH_FMA, in_reim, out_reim, n, batch, where, stream);
}

int jw_fft_reverse(const double* in_reim, double* out_reim, long n, int batch, int where,
                   void* stream) {
  return fft_call(1, JW_ARITH_FMA, in_reim, out_reim, n, batch, where, stream);
}

int jw_fft_forward_ex(const double* in_reim, double* out_reim, long n, int batch, int arith,
                      int where, void* stream) {
  return fft_call(-1, arith, in_reim, out_reim, n, batch, where, stream);
}

int jw_fft_reverse_ex(const double* in_reim, double* out_reim, long n, int batch, int arith,
                      int where, void* stream) {
  return fft_call(1, arith, in_reim, out_reim, n, batch, where, stream);
}

// ---------------------------------------------------------------- FWT
int jw_fwt_plan_create(jw_fwt_plan** plan, const double* scaling_dec, const double* wavelet_dec,
                       const double* scaling_rec, const double* wavelet_rec, int M,
                       int transform_wavelength, int kind, int arith) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan pointer is null");
  *plan = nullptr;
  if (!scaling_dec || !wavelet_dec || !scaling_rec || !wavelet_rec)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "filter pointer is null");
  if (M < 1 || M > kMaxTaps)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "filter length must be in [1, %d], got %d", kMaxTaps, M);
  if (transform_wavelength < 1)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "transform wavelength must be >= 1, got %d",
                transform_wavelength);
  if (kind != JW_WAVELET_GENERIC && kind != JW_WAVELET_HAAR_ORTH)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown wavelet kind %d", kind);
  if (arith != JW_ARITH_STRICT && arith != JW_ARITH_FMA)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown arithmetic mode %d", arith);
  auto* p = new (std::nothrow) jw_fwt_plan();
  if (!p) return fail(JW_ERR_NO_MEMORY, "out of host memory");
  p->M = M;
  p->tw = transform_wavelength;
  p->kind = kind;
  p->arith = arith;
  for (int i = 0; i < M; ++i) {
    p->sD[i] = scaling_dec[i];
    p->wD[i] = wavelet_dec[i];
    p->sR[i] = scaling_rec[i];
    p->wR[i] = wavelet_rec[i];
  }
  *plan = p;
  return JW_OK;
}

void jw_fwt_plan_destroy(jw_fwt_plan* plan) { delete plan; }

// FastWaveletTransform.forward/reverse validation (FastWaveletTransform.java:74-83, :122-131).
static int fwt_check(long n, int level, const char* who) {
  if (!is_binary(n))
    return fail(JW_ERR_FAILURE,
                "FastWaveletTransform#%s - given array length is not 2^p | p E N ... = 1, 2, 4, "
                "8, 16, 32, .. please use the Ancient Egyptian Decomposition for any other array "
                "length!",
                who);
  const int levels = floor_log2(n);
  if (level < 0 || level > levels)
    return fail(JW_ERR_FAILURE,
                "FastWaveletTransform#%s - given level is out of range for given array", who);
  return JW_OK;
}

int jw_fwt_forward(const jw_fwt_plan* plan, const double* x, double* y, long n, int level,
                   int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  int st = fwt_check(n, level, "forward");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, x, (size_t)n, y, (size_t)n, batch,
                   [&](const double* dx, double* dy, long nb, hipStream_t s) {
                     return fwt_forward_device(*plan, dx, dy, n, level, (int)nb, s);
                   });
}

int jw_fwt_reverse(const jw_fwt_plan* plan, const double* y, double* x, long n, int level,
                   int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  int st = fwt_check(n, level, "reverse");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, y, (size_t)n, x, (size_t)n, batch,
                   [&](const double* dy, double* dx, long nb, hipStream_t s) {
                     return fwt_reverse_device(*plan, dy, dx, n, level, (int)nb, s);
                   });
}

// WaveletPacketTransform.forward/reverse validation (WaveletPacketTransform.java:63-72, :122-131).
static int wpt_check(long n, int level, const char* who) {
  if (!is_binary(n))
    return fail(JW_ERR_FAILURE,
                "given array length is not 2^p | p E N ... = 1, 2, 4, 8, 16, 32, .. please use "
                "the Ancient Egyptian Decomposition for any other array length!");
  if (level < 0 || level > floor_log2(n))
    return fail(JW_ERR_FAILURE,
                "WaveletPacketTransform#%s - given level is out of range for given array", who);
  return JW_OK;
}

int jw_wpt_forward(const jw_fwt_plan* plan, const double* x, double* y, long n, int level,
                   int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  int st = wpt_check(n, level, "forward");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, x, (size_t)n, y, (size_t)n, batch,
                   [&](const double* dx, double* dy, long nb, hipStream_t s) {
                     return wpt_forward_device(*plan, dx, dy, n, level, (int)nb, s);
                   });
}

int jw_wpt_reverse(const jw_fwt_plan* plan, const double* y, double* x, long n, int level,
                   int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  int st = wpt_check(n, level, "reverse");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, y, (size_t)n, x, (size_t)n, batch,
                   [&](const double* dy, double* dx, long nb, hipStream_t s) {
                     return wpt_reverse_device(*plan, dy, dx, n, level, (int)nb, s);
                   });
}

int jw_fwt2d_forward(const jw_fwt_plan* plan, const double* x, double* y, int rows, int cols,
                     int lvlM, int lvlN, int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  // rows are transformed first (with cols samples, lvlN), then columns (rows samples, lvlM)
  int st = fwt_check(cols, lvlN, "forward");
  if (st == JW_OK) st = fwt_check(rows, lvlM, "forward");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, x, (size_t)rows * cols, y, (size_t)rows * cols,
                   batch, [&](const double* dx, double* dy, long nb, hipStream_t s) {
                     return fwt2d_forward_device(*plan, dx, dy, rows, cols, lvlM, lvlN, (int)nb, s);
                   });
}

int jw_fwt2d_reverse(const jw_fwt_plan* plan, const double* y, double* x, int rows, int cols,
                     int lvlM, int lvlN, int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  // columns are transformed first (rows samples, lvlM), then rows (cols samples, lvlN)
  int st = fwt_check(rows, lvlM, "reverse");
  if (st == JW_OK) st = fwt_check(cols, lvlN, "reverse");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, y, (size_t)rows * cols, x, (size_t)rows * cols,
                   batch, [&](const double* dy, double* dx, long nb, hipStream_t s) {
                     return fwt2d_reverse_device(*plan, dy, dx, rows, cols, lvlM, lvlN, (int)nb, s);
                   });
}

// 3-D: BasicTransform.forward/reverse(double[][][], lvlP, lvlQ, lvlR) (:509-659).  The
// reference validates nothing itself; its first 1-D call fails first: forward -> slab 0's
// rows (H, lvlQ), its columns (C, lvlP), then the lines along dimension 1 (R, lvlR);
// reverse -> slab 0's columns (C, lvlP), rows (H, lvlQ), then (R, lvlR).
int jw_fwt3d_forward(const jw_fwt_plan* plan, const double* x, double* y, int d1, int d2, int d3,
                     int lvlP, int lvlQ, int lvlR, int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  int st = fwt_check(d3, lvlQ, "forward");
  if (st == JW_OK) st = fwt_check(d2, lvlP, "forward");
  if (st == JW_OK) st = fwt_check(d1, lvlR, "forward");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  const size_t elems = (size_t)d1 * d2 * d3;
  return run_items(where, stream, x, elems, y, elems, batch,
                   [&](const double* dx, double* dy, long nb, hipStream_t s) {
                     return fwt3d_forward_device(*plan, dx, dy, d1, d2, d3, lvlP, lvlQ, lvlR, (int)nb, s);
                   });
}
int jw_fwt3d_reverse(const jw_fwt_plan* plan, const double* y, double* x, int d1, int d2, int d3,
                     int lvlP, int lvlQ, int lvlR, int batch, int where, void* stream) {
  clear_error();
  if (!plan) return fail(JW_ERR_ILLEGAL_ARGUMENT, "plan is null");
  int st = fwt_check(d2, lvlP, "reverse");
  if (st == JW_OK) st = fwt_check(d3, lvlQ, "reverse");
  if (st == JW_OK) st = fwt_check(d1, lvlR, "reverse");
  if (st != JW_OK) return st;
  if (st = check_where(where); st != JW_OK) return st;
  if (batch <= 0) return batch == 0 ? JW_OK : fail(JW_ERR_ILLEGAL_ARGUMENT, "negative batch");
  if (!x || !y) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  const size_t elems = (size_t)d1 * d2 * d3;
  return run_items(where, stream, y, elems, x, elems, batch,
                   [&](const double* dy, double* dx, long nb, hipStream_t s) {
                     return fwt3d_reverse_device(*plan, dy, dx, d1, d2, d3, lvlP, lvlQ, lvlR, (int)nb, s);
                   });
}

// ---------------------------------------------------------------- synthetic input
// ---------------------------------------------------------------- CWT
// The wavelet constructors' validation (kind and parameter block), shared by both CWT paths.
static int cwt_wavelet_check(int wavelet, const double* params) {
  if (wavelet < JW_CWT_MORLET || wavelet > JW_CWT_MEYER)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown continuous wavelet kind %d", wavelet);
  if (!params && wavelet != JW_CWT_MEYER)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "wavelet parameters are null");
  // an integer order carried in a double (the Java constructors take int)
  auto order = [](double v, int hi, const char* lo_msg, const char* hi_msg) -> int {
    if (!(v >= 1) || v != std::floor(v)) return fail(JW_ERR_ILLEGAL_ARGUMENT, "%s", lo_msg);
    if (v > hi) return fail(JW_ERR_ILLEGAL_ARGUMENT, "%s", hi_msg);
    return JW_OK;
  };
  if (wavelet == JW_CWT_MORLET) {  // MorletWavelet.java:69-74
    if (!(params[0] > 0)) return fail(JW_ERR_ILLEGAL_ARGUMENT, "Bandwidth parameter must be positive");
    if (!(params[1] > 0)) return fail(JW_ERR_ILLEGAL_ARGUMENT, "Center frequency must be positive");
  } else if (wavelet == JW_CWT_MEXHAT) {  // MexicanHatWavelet.java:67-69
    if (!(params[0] > 0))
      return fail(JW_ERR_ILLEGAL_ARGUMENT, "Width parameter sigma must be positive");
  } else if (wavelet == JW_CWT_PAUL) {  // PaulWavelet.java:79-84
    const int st = order(params[0], 20, "Order parameter m must be a positive integer",
                         "Order parameter m > 20 may cause numerical issues");
    if (st != JW_OK) return st;
  } else if (wavelet == JW_CWT_DOG) {  // DOGWavelet.java:132-140
    const int st = order(params[0], 10, "Derivative order n must be a positive integer",
                         "Derivative order n > 10 may cause numerical issues");
    if (st != JW_OK) return st;
    if (!(params[1] > 0))
      return fail(JW_ERR_ILLEGAL_ARGUMENT, "Width parameter sigma must be positive");
  }
  return JW_OK;
}

// jw_cwt_fft's argument checks (shared with jw_cwt_fft_scalogram)
static int cwt_fft_check(int wavelet, const double* params, long n, const double* scales, int ns,
                         int padding, int batch, int where) {
  if (int st = cwt_wavelet_check(wavelet, params); st != JW_OK) return st;
  if (n < 0 || ns < 0 || batch < 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative size (n=%ld, ns=%d, batch=%d)", n, ns, batch);
  if (padding < JW_PAD_ZERO || padding > JW_PAD_CONSTANT)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown padding type %d", padding);
  if (n > 0 && ns > 0 && !scales) return fail(JW_ERR_ILLEGAL_ARGUMENT, "scales are null");
  // ContinuousWavelet.fourierTransform :123-125 (PaulWavelet's override :152-164 has no check)
  for (int i = 0; i < ns && n > 0 && wavelet != JW_CWT_PAUL; ++i)
    if (!(scales[i] > 0)) return fail(JW_ERR_ILLEGAL_ARGUMENT, "Scale must be positive");
  return check_where(where);
}

int jw_cwt_fft(int wavelet, const double* params, const double* x, long n, const double* scales,
               int ns, double sampling_rate, int padding, double* out_reim, int batch, int where,
               void* stream) {
  clear_error();
  int st = cwt_fft_check(wavelet, params, n, scales, ns, padding, batch, where);
  if (st != JW_OK) return st;
  if (n == 0 || ns == 0 || batch == 0) return JW_OK;
  return run_items(where, stream, x, (size_t)n, out_reim, (size_t)ns * n * 2, batch,
                   [&](const double* xi, double* o, long nb, hipStream_t s) {
                     return cwt_fft_device(wavelet, params, xi, n, scales, ns, sampling_rate,
                                           padding, o, (int)nb, s);
                   });
}

int jw_cwt_fft_paths(int wavelet, const double* params, long n, const double* scales, int ns,
                     double sampling_rate, int* two_pass, int* band, int* coarse_grid) {
  clear_error();
  int st = cwt_fft_check(wavelet, params, n, scales, ns, JW_PAD_ZERO, 0, JW_HOST);
  if (st != JW_OK) return st;
  if (!two_pass || !band || !coarse_grid)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "output pointer is null");
  return cwt_fft_paths(wavelet, params, n, scales, ns, sampling_rate, two_pass, band, coarse_grid);
}

// transformFFT(...).getScalogram() with the coefficients kept in a device workspace (signals
// in chunks of at most ~2 GiB of coefficients): only batch x ns energies leave the GPU.
int jw_cwt_fft_scalogram(int wavelet, const double* params, const double* x, long n,
                         const double* scales, int ns, double sampling_rate, int padding,
                         double* energy, int batch, int where, void* stream) {
  clear_error();
  int st = cwt_fft_check(wavelet, params, n, scales, ns, padding, batch, where);
  if (st != JW_OK) return st;
  if (ns == 0 || batch == 0) return JW_OK;
  return run_items(where, stream, x, (size_t)n, energy, (size_t)ns, batch,
             [&](const double* xi, double* o, long nbatch, hipStream_t s) {
               const int batch = (int)nbatch;
               const size_t nout = (size_t)batch * ns;
               if (n == 0) {  // no time points: zero energy (CWTResult.java:277-284)
                 JW_HIP_TRY(hipMemsetAsync(o, 0, nout * sizeof(double), s));
                 return (int)JW_OK;
               }
               const long per_sig = (long)ns * n * 2 * (long)sizeof(double);
               const long chunk = std::max(1L, std::min<long>(batch, (2L << 30) / per_sig));
               StreamAllocs mem(s);
               double* coef = nullptr;
               JW_HIP_TRY(mem.alloc(&coef, (size_t)chunk * per_sig));
               for (long b0 = 0; b0 < batch; b0 += chunk) {
                 const int nb = (int)std::min<long>(chunk, batch - b0);
                 int r = cwt_fft_device(wavelet, params, xi + b0 * n, n, scales, ns,
                                        sampling_rate, padding, coef, nb, s);
                 if (r == JW_OK) r = cwt_scalogram_device(coef, (long)nb * ns, n, o + b0 * ns, s);
                 if (r != JW_OK) return r;
               }
               return (int)JW_OK;
             });
}

// ContinuousWaveletTransform.transform(signal, scales, fs) (:153-172) and its parallel
// variants.  computeCoefficient (:240-260) evaluates wavelet(t, scale, 0) -- which throws
// "Scale must be positive" for scale <= 0 (ContinuousWavelet.java:91-93) -- only inside a
// non-empty window [max(0, t + lo), min(N - 1, t + hi)]: a negative scale turns the window
// around (zeros, no exception), a zero scale throws.  Scales are checked in the reference's
// loop order.
int jw_cwt_direct(int wavelet, const double* params, const double* x, long n,
                  const double* scales, int ns, double sampling_rate, int arith, double* out_reim,
                  int batch, int where, void* stream) {
  clear_error();
  if (int st = cwt_wavelet_check(wavelet, params); st != JW_OK) return st;
  if (n < 0 || ns < 0 || batch < 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative size (n=%ld, ns=%d, batch=%d)", n, ns, batch);
  if (arith != JW_ARITH_STRICT && arith != JW_ARITH_FMA)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "unknown arithmetic mode %d", arith);
  if (n > 0 && ns > 0 && !scales) return fail(JW_ERR_ILLEGAL_ARGUMENT, "scales are null");
  for (int i = 0; i < ns && n > 0; ++i) {
    double lo_f = 0, hi_f = 0;
    cwt_direct_support(wavelet, params, scales[i], sampling_rate, &lo_f, &hi_f);
    if (cwt_direct_window_nonempty(lo_f, hi_f, n) && scales[i] <= 0)
      return fail(JW_ERR_ILLEGAL_ARGUMENT, "Scale must be positive");
  }
  int st = check_where(where);
  if (st != JW_OK) return st;
  if (n == 0 || ns == 0 || batch == 0) return JW_OK;
  return run_items(where, stream, x, (size_t)n, out_reim, (size_t)ns * n * 2, batch,
                   [&](const double* xi, double* o, long nb, hipStream_t s) {
                     return cwt_direct_device(wavelet, params, xi, n, scales, ns, sampling_rate,
                                              arith, o, (int)nb, s);
                   });
}

// CWTResult.getMagnitude / getPhase / getScalogram (CWTResult.java:94-126, :272-287)
static int cwt_elementwise(const double* c, long count, double* out, int where, void* stream,
                           int (*dev)(const double*, long, double*, hipStream_t)) {
  clear_error();
  if (count < 0) return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative size (count=%ld)", count);
  int st = check_where(where);
  if (st != JW_OK) return st;
  if (count == 0) return JW_OK;
  if (!c || !out) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, c, 2, out, 1, count,
                   [&](const double* ci, double* o, long k, hipStream_t s) { return dev(ci, k, o, s); });
}

int jw_cwt_magnitude(const double* coef_reim, long count, double* out, int where, void* stream) {
  return cwt_elementwise(coef_reim, count, out, where, stream, cwt_magnitude_device);
}

int jw_cwt_phase(const double* coef_reim, long count, double* out, int where, void* stream) {
  return cwt_elementwise(coef_reim, count, out, where, stream, cwt_phase_device);
}

int jw_cwt_scalogram(const double* coef_reim, long rows, long n, double* energy, int where,
                     void* stream) {
  clear_error();
  if (rows < 0 || n < 0)
    return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative size (rows=%ld, n=%ld)", rows, n);
  int st = check_where(where);
  if (st != JW_OK) return st;
  if (rows == 0) return JW_OK;
  if (!coef_reim || !energy) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return run_items(where, stream, coef_reim, (size_t)n * 2, energy, 1, rows,
                   [&](const double* ci, double* o, long r, hipStream_t s) {
                     return cwt_scalogram_device(ci, r, n, o, s);
                   });
}

int jw_synth_uniform(double* x_dev, long n, int batch, long seed0, void* stream) {
  clear_error();
  if (n < 0 || batch < 0) return fail(JW_ERR_ILLEGAL_ARGUMENT, "negative size");
  if (n == 0 || batch == 0) return JW_OK;
  if (!x_dev) return fail(JW_ERR_ILLEGAL_ARGUMENT, "data pointer is null");
  return synth_uniform_device(x_dev, n, batch, seed0, (hipStream_t)stream);
}

}  // extern "C"
