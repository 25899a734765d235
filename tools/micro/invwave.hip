// Compute-only and full timing of the two inverse MODWT kernels (workgroup-shared stream
// `modwt_inv_fast` vs one stream per wave `modwt_inv_wave`) at the cfg2 shape, plus the shader
// clock the box runs at (s_memtime ticks per s_memrealtime 100 MHz tick) -- the inverse's
// compute share scales with that clock, its HBM share does not.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "jw_modwt_fast.hpp"

namespace jw {
void set_error(const char*, ...) {}
int fail(int code, const char*, ...) { return code; }
void clear_error() {}
}  // namespace jw
using namespace jw;

__global__ void clock_probe(unsigned long long* out) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double acc = threadIdx.x;
  for (int i = 0; i < 2000000; ++i) acc = __builtin_fma(acc, 0.999999, 1e-9);
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = c1 - c0; out[1] = r1 - r0; }
  if (acc == 12345.0) out[2] = 1;
}

__global__ void pl_check(unsigned* o) {
  const int l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap((unsigned)l, 100u + l, false, false);
  o[l] = r[0];
  o[64 + l] = r[1];
}

// The inverse's HBM access shape with no math: one wave streams one segment right -> left,
// 9 rows in / 1 out, VEC doubles per lane per row (64*VEC positions per step), D-deep register
// prefetch.  Occupancy is set by the dynamic LDS the launch reserves.
template <int VEC, int D, bool SKEW = false>
__global__ __launch_bounds__(64) void shape_9in1out(const double* __restrict__ c, double* __restrict__ x,
                                                    long N, long seg, long steps, long ld = 0) {
  if (ld == 0) ld = N;
  typedef double dv __attribute__((ext_vector_type(VEC)));
  const int lane = threadIdx.x;
  const long P = (long)blockIdx.x * seg +
                 (SKEW ? (long)((blockIdx.y * 2654435761u) & (unsigned)(seg - 1) & ~63u) : 0);
  const double* cs = c + (long)blockIdx.y * 9 * ld;
  double* xs = x + (long)blockIdx.y * N;
  long a = P + (steps - 1) * 64 * VEC;
  dv S[D][9];
  auto fetch = [&](dv (&dst)[9], long at) {
    long p = ((at % N) + N) % N + lane * VEC;
    p = p >= N ? p - N : p;
#pragma unroll
    for (int j = 0; j < 9; ++j) dst[j] = *(const dv*)(cs + (long)j * ld + p);
  };
#pragma unroll
  for (int q = 0; q < D - 1; ++q) fetch(S[q], a - q * 64 * VEC);
  for (long k = 0; k < steps; k += D) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      fetch(S[(q + D - 1) % D], a - (D - 1) * 64 * VEC);
      dv v = S[q][0];
#pragma unroll
      for (int j = 1; j < 9; ++j) v += S[q][j];
      const long pos = a + lane * VEC;
      if (pos >= P && pos < P + seg) *(dv*)(xs + (pos >= N ? pos - N : pos)) = v;
      a -= 64 * VEC;
    }
  }
}

int main() {
  {
    unsigned* o;
    hipMalloc(&o, 512);
    pl_check<<<1, 64>>>(o);
    unsigned h[128];
    hipMemcpy(h, o, 512, hipMemcpyDeviceToHost);
    printf("permlane32_swap(l, 100+l): r0[0]=%u r0[31]=%u r0[32]=%u r0[63]=%u | r1[0]=%u r1[31]=%u r1[32]=%u r1[63]=%u\n",
           h[0], h[31], h[32], h[63], h[64], h[95], h[96], h[127]);
  }
  const long N = 1L << 20;
  const int B = 1024;
  double *c, *x;
  hipMalloc(&c, 9L * N * B * 8);
  hipMalloc(&x, N * B * 8);
  hipMemset(c, 0, 9L * N * B * 8);
  Taps taps{};
  for (int m = 0; m < 16; ++m) { taps.a[m] = 0.1 * m; taps.b[m] = 0.2 - 0.01 * m; }
  unsigned long long* ck;
  hipMalloc(&ck, 32);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto probe = [&]() {
    clock_probe<<<1024, 256>>>(ck);
    unsigned long long h[2];
    hipMemcpy(h, ck, 16, hipMemcpyDeviceToHost);
    printf("shader clock under FP64 load: %.0f MHz\n", 100.0 * h[0] / h[1]);
  };
  probe();
  auto timeit = [&](const char* name, auto&& launch) {
    launch();
    hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s %8.3f ms\n", name, ms / 5);
  };
  // wave-kernel variants at the library's grid (D sets, U unroll, CP load cache policy)
  auto wave_launch = [&](auto kern, int U) {
    using G = wave::WGeo<8, 8>;
    const long warm = ((long)(G::H + 63) / 64) * 64;
    const long seg = fast::pick_seg(N, B, warm, 64, 8192);
    long steps = seg / 64 + warm / 64;
    steps = ((steps + U - 1) / U) * U;
    const size_t lds = (size_t)G::lds_pairs * 16;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<dim3((unsigned)((N + seg - 1) / seg), B), 64, lds>>>(c, x, N, seg, (steps - 1) * 64,
                                                               steps / U, taps);
  };
  auto fwd_launch = [&](auto kern) {
    using G = fast::GeoF<8, 8, 512>;
    const long warm = ((long)(G::H + 511) / 512) * 512;
    const long seg = fast::pick_seg(N, B, warm, 512);
    const long npairs = ((seg + warm) / 512 + 1) / 2;
    fast::launch(kern, (size_t)G::total * 8, (N + seg - 1) / seg, B, 256, 0, x, N, c, 9 * N, N, seg,
                 warm, npairs, taps);
  };
  for (int rep = 0; rep < 1; ++rep) {
    timeit("fwd fma (product)", [&] { fwd_launch(fast::modwt_fwd_fast<8, 8, true, 256, 0>); });
    timeit("fwd fma nt stores", [&] { fwd_launch(fast::modwt_fwd_fast<8, 8, true, 256, 2>); });
    timeit("wg   fma  (modwt_inv_fast)", [&] { fast::launch_inv_c<8, 8, true, 256, 256, 2, 7>(taps, c, x, N, B, 0); });
    timeit("wave fma D3 U6 (product)", [&] { wave_launch(wave::modwt_inv_wave<8, 8, true, 3, 6, 1, 0>, 6); });
    timeit("wave fma D3 U6 nt loads", [&] { wave_launch(wave::modwt_inv_wave<8, 8, true, 3, 6, 1, 2>, 6); });
    timeit("wave fma D2 U6", [&] { wave_launch(wave::modwt_inv_wave<8, 8, true, 2, 6, 1, 0>, 6); });
    timeit("wave fma D3 U12", [&] { wave_launch(wave::modwt_inv_wave<8, 8, true, 3, 12, 1, 0>, 12); });
    timeit("wave fma compute only", [&] { wave_launch(wave::modwt_inv_wave<8, 8, true, 3, 6, 0, 0>, 6); });
  }
  {
    const long seg = 131072, steps = (seg + 1792) / 64;
    auto k1 = shape_9in1out<1, 2, true>;
    hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, 20 * 1024);
    timeit("shape vec1 20KB, per-signal skew", [&] { k1<<<dim3(N / seg, B), 64, 20 * 1024>>>(c, x, N, seg, steps, 0L); });
    auto k0 = shape_9in1out<1, 2, false>;
    timeit("shape vec1 20KB, row stride N+512 (B=1000)", [&] { k0<<<dim3(N / seg, 1000), 64, 20 * 1024>>>(c, x, N, seg, steps, N + 512); });
    timeit("shape vec1 20KB, row stride N (B=1000)", [&] { k0<<<dim3(N / seg, 1000), 64, 20 * 1024>>>(c, x, N, seg, steps, N); });
  }
  for (int lds_kb : {20, 10}) {
    char nm[96];
    const long seg = 131072, steps = (seg + 1792) / 64;
    auto k1 = shape_9in1out<1, 2>;
    hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024);
    snprintf(nm, sizeof nm, "shape 9in1out vec1 D2, %d KB LDS/wave", lds_kb);
    timeit(nm, [&] { k1<<<dim3(N / seg, B), 64, lds_kb * 1024>>>(c, x, N, seg, steps, 0L); });
    auto k2 = shape_9in1out<2, 2>;
    hipFuncSetAttribute((const void*)k2, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024);
    snprintf(nm, sizeof nm, "shape 9in1out vec2 D2, %d KB LDS/wave", lds_kb);
    timeit(nm, [&] { k2<<<dim3(N / seg, B), 64, lds_kb * 1024>>>(c, x, N, seg, (seg + 1792) / 128, 0L); });
  }
  timeit("wg   sym8 J6 fma", [&] { fast::launch_inv_c<16, 6, true, 256, 256, 2, 7>(taps, c, x, N, B, 0); });
  timeit("wave sym8 J6 fma", [&] { wave::launch_inv_wave<16, 6, true>(taps, c, x, N, B, 0); });
  probe();
  printf("done %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
