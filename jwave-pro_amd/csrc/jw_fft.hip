// jw_fft.hip -- twiddle tables and the generic (any power-of-two) FFT passes.
#include <cmath>
#include <map>
#include <mutex>
#include <utility>

#include "jw_fft.hpp"

namespace jw {
namespace fft {

namespace {
std::mutex g_mu;
// per (device, N): device memory owned for the library's lifetime.  Keyed by the calling
// thread's current device, so one process driving several GPUs (a JVM with a thread per
// GPU) never hands one device's tables to another.
std::map<std::pair<int, long>, Tables> g_tables;

void fill(cplx* h, long n, long N, long stride) {
  const long double two_pi = 6.283185307179586476925286766559005768L;
  for (long j = 0; j < n; ++j) {
    const long double a = two_pi * (long double)((j * stride) % N) / (long double)N;
    h[j] = make_double2((double)cosl(a), (double)sinl(a));
  }
}
}  // namespace

int tables(long N, Tables* out) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  const std::pair<int, long> key(dev, N);
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_tables.find(key);
  if (it != g_tables.end()) {
    *out = it->second;
    return JW_OK;
  }
  int logN = 0;
  while ((1L << logN) < N) ++logN;
  const int logQ = (logN + 1) / 2;
  const long Q = 1L << logQ, NH = N >> logQ > 0 ? N >> logQ : 1;
  const long total = 512 + Q + NH;
  cplx* h = new cplx[total];
  fill(h, 512, 512, 1);
  fill(h + 512, Q, N, 1);
  fill(h + 512 + Q, NH, N, Q);
  cplx* d = nullptr;
  hipError_t e = hipMalloc((void**)&d, total * sizeof(cplx));
  if (e == hipSuccess) e = hipMemcpy(d, h, total * sizeof(cplx), hipMemcpyHostToDevice);
  delete[] h;
  if (e != hipSuccess) {
    if (d) (void)hipFree(d);
    return fail(JW_ERR_DEVICE, "FFT twiddle table for N=%ld: %s", N, hipGetErrorString(e));
  }
  Tables t;
  t.N = N;
  t.logQ = logQ;
  t.w512 = d;
  t.lo = d + 512;
  t.hi = d + 512 + Q;
  g_tables[key] = t;
  *out = t;
  return JW_OK;
}

}  // namespace fft
}  // namespace jw
