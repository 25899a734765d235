// Compute-only timing of the MODWT inverse step (jw_modwt_fast.hpp inv_step): the same
// LDS/VALU/barrier work per step as modwt_inv_fast, with the HBM fetch replaced by register
// arithmetic and every x-hat store range-dropped.  Compared with the real kernel's time it
// says how much of the inverse is compute (LDS + VALU + barriers) versus memory.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#ifdef NOSYNC  // -DNOSYNC: every barrier of the step removed (wrong results, timing only)
#define JW_INV_SYNC() do {} while (0)
#endif
#include "jw_modwt_fast.hpp"

namespace jw {
void set_error(const char*, ...) {}
int fail(int code, const char*, ...) { return code; }
void clear_error() {}
}  // namespace jw

using namespace jw;
using namespace jw::fast;

template <int L, int J, bool FMA, int C, int NT, int D, int MEM, int RF = J + 1>
__global__ __launch_bounds__(NT) void inv_nomem(const double* __restrict__ coeffs, double* x,
                                                long N, long steps, Taps taps) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = GeoI<L, J, C>;
  constexpr int R = C / NT;
  const int t = threadIdx.x;
  const rsrc_t rx = make_rsrc(x + (long)blockIdx.y * N, N);
  const double* cs = coeffs + (long)blockIdx.y * (long)(J + 1) * N;
  rsrc_t rc[J + 1];
#pragma unroll
  for (int j = 0; j <= J; ++j) rc[j] = make_rsrc(cs + (long)j * N, N);
  for (int i = t; i < G::inv_total; i += NT) lds[i] = 0.0;
  long lb = ((long)blockIdx.x * 131072) % N;
  double seed = (double)(blockIdx.x + t);
  auto fetch = [&](double (&dst)[R * (J + 1)]) {
    if constexpr (MEM) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        long p = lb + t + r * NT;
        p = p >= N ? p - N : p;
#pragma unroll
        for (int j = 0; j <= J; ++j) dst[(J + 1) * r + j] = bload(rc[j], (int)(p * 8));
      }
      lb -= C;
      if (lb < 0) lb += N;
    } else {
#pragma unroll
      for (int k = 0; k < R * (J + 1); ++k) dst[k] = seed + k;
      seed += 1.0;
    }
  };
  double S[D][R * (J + 1)];
#pragma unroll
  for (int q = 0; q < D; ++q) fetch(S[q]);
  int rb[J + 1] = {};
  double tv[R * 2 * L];
  auto no_taps = [] {};
  __syncthreads();
  long a = N - C;
  for (long k = 0; k < steps / D; ++k) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      // MEM 2: real x-hat stores (segment = whole row), else range-dropped
      const long P0 = MEM == 2 ? -(1L << 40) : (1L << 40);
      inv_step<L, J, FMA, C, NT, RF, false>((d2*)lds, S[q], fetch, a, P0, 1L << 41, rx, taps, rb, tv,
                                            no_taps);
      a -= C;
      if (a < 0) a += N;
    }
  }
}

int main() {
  const long N = 1L << 20;
  const int B = 1024;
  double *c, *x;
  hipMalloc(&c, 9L * N * B * 8);
  hipMalloc(&x, N * B * 8);
  hipMemset(c, 0, 9L * N * B * 8);
  Taps taps{};
  for (int m = 0; m < 8; ++m) { taps.a[m] = 0.1 * m; taps.b[m] = 0.2 - 0.01 * m; }
  auto time = [&](auto kern, int C, const char* name) {
    const size_t lds = (size_t)(2 * (Geo<8, 8>::H + 8 * C)) * 8;
    const long steps = 131072 / C + (2048 + C - 1) / C;  // segment + warm-up, as at cfg2
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    dim3 g(8, B);
    kern<<<g, C, lds>>>(c, x, N, steps, taps);
    hipEventRecord(e0);
    for (int i = 0; i < 3; ++i) kern<<<g, C, lds>>>(c, x, N, steps, taps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %8.3f ms\n", name, ms / 3);
  };
  time(inv_nomem<8, 8, true, 256, 256, 2, 2, 7>, 256, "C256 fma, loads+stores ring7");
  time(inv_nomem<8, 8, true, 256, 256, 2, false, 7>, 256, "C256 fma, no HBM ring7");
  time(inv_nomem<8, 8, false, 256, 256, 2, 2, 7>, 256, "C256 strict, loads+stores ring7");
  time(inv_nomem<8, 8, false, 256, 256, 2, false, 7>, 256, "C256 strict, no HBM ring7");

  return 0;
}
