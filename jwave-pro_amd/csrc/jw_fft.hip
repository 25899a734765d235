// jw_fft.hip -- twiddle tables and the generic (any power-of-two) FFT passes.
#include <cmath>
#include <map>
#include <mutex>
#include <utility>

#include "jw_fft.hpp"

namespace jw {
namespace fft {

namespace {
// per (device, N): the calling thread's current device, so one process driving several GPUs (a
// JVM with a thread per GPU) never hands one device's tables to another.
DevCache<std::pair<int, long>> g_tables(1UL << 30);

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
  int logN = 0;
  while ((1L << logN) < N) ++logN;
  const int logQ = (logN + 1) / 2;
  const long Q = 1L << logQ, NH = N >> logQ > 0 ? N >> logQ : 1;
  const long total = 512 + Q + NH;
  const std::pair<int, long> key(dev, N);
  const cplx* d = (const cplx*)g_tables.find(key);
  if (!d) {  // small (512 + 2 sqrt(N) entries): built with a synchronous copy
    cplx* h = new cplx[total];
    fill(h, 512, 512, 1);
    fill(h + 512, Q, N, 1);
    fill(h + 512 + Q, NH, N, Q);
    cplx* p = nullptr;
    hipError_t e = hipMalloc((void**)&p, total * sizeof(cplx));
    if (e == hipSuccess) e = hipMemcpy(p, h, total * sizeof(cplx), hipMemcpyHostToDevice);
    delete[] h;
    if (e != hipSuccess) {
      if (p) (void)hipFree(p);
      return fail(JW_ERR_DEVICE, "FFT twiddle table for N=%ld: %s", N, hipGetErrorString(e));
    }
    d = (const cplx*)g_tables.insert(key, p, total * sizeof(cplx));
  }
  Tables t;
  t.N = N;
  t.logQ = logQ;
  t.w512 = d;
  t.lo = d + 512;
  t.hi = d + 512 + Q;
  *out = t;
  return JW_OK;
}

}  // namespace fft
}  // namespace jw
