// jw_synth.hip -- synthetic input in HBM: java.util.Random(seed0 + b).nextDouble()*2 - 1
// for signal b (BASELINE.md "Same inputs as the GPU").  Each thread jumps the 48-bit LCG
// ahead to its first element (affine-map squaring) and then steps it like the JDK does,
// so the values equal the oracle's jwo_fill_uniform bit for bit.
#include "jw_internal.hpp"

namespace jw {
namespace {

constexpr unsigned long long kA = 0x5DEECE66DULL;
constexpr unsigned long long kC = 0xBULL;
constexpr unsigned long long kMask = (1ULL << 48) - 1;
constexpr int kPerThread = 64;
constexpr int kNT = 256;

__device__ unsigned long long lcg_skip(unsigned long long s, unsigned long long k) {
  unsigned long long a = kA, c = kC, acc_a = 1, acc_c = 0;
  while (k) {
    if (k & 1) {
      acc_a = (acc_a * a) & kMask;
      acc_c = (acc_c * a + c) & kMask;
    }
    c = (c * (a + 1)) & kMask;
    a = (a * a) & kMask;
    k >>= 1;
  }
  return (acc_a * s + acc_c) & kMask;
}

__global__ __launch_bounds__(kNT) void synth_uniform_kernel(double* __restrict__ x, long n,
                                                            long seed0) {
  const long start = ((long)blockIdx.x * kNT + threadIdx.x) * kPerThread;
  if (start >= n) return;
  const long b = blockIdx.y;
  unsigned long long s = ((unsigned long long)(seed0 + b) ^ kA) & kMask;  // Random(seed)
  s = lcg_skip(s, 2ULL * (unsigned long long)start);
  double* out = x + b * n;
  const long end = start + kPerThread < n ? start + kPerThread : n;
  for (long i = start; i < end; ++i) {
    s = (s * kA + kC) & kMask;
    const long hi = (long)(s >> (48 - 26));  // next(26)
    s = (s * kA + kC) & kMask;
    const long lo = (long)(s >> (48 - 27));  // next(27)
    out[i] = (double)((hi << 27) + lo) * 0x1.0p-53 * 2.0 - 1.0;
  }
}

}  // namespace

int synth_uniform_device(double* x, long n, int batch, long seed0, hipStream_t s) {
  const long threads = (n + kPerThread - 1) / kPerThread;
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    dim3 grid((unsigned)((threads + kNT - 1) / kNT), (unsigned)nb);
    hipLaunchKernelGGL(synth_uniform_kernel, grid, dim3(kNT), 0, s, x + (long)b0 * n, n,
                       seed0 + b0);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace jw
