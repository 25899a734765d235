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
  // full kernels through the library launchers
  timeit("wg   fma  (modwt_inv_fast)", [&] { fast::launch_inv_c<8, 8, true, 256, 256, 2, 7>(taps, c, x, N, B, 0); });
  timeit("wave fma  (modwt_inv_wave)", [&] { wave::launch_inv_wave<8, 8, true>(taps, c, x, N, B, 0); });
  timeit("wg   strict", [&] { fast::launch_inv_c<8, 8, false, 256, 256, 2, 7>(taps, c, x, N, B, 0); });
  timeit("wave strict", [&] { wave::launch_inv_wave<8, 8, false>(taps, c, x, N, B, 0); });
  timeit("wg   sym8 J6 fma", [&] { fast::launch_inv<16, 6, true>(taps, c, x, N, B, 0); });
  timeit("wave sym8 J6 fma", [&] { wave::launch_inv_wave<16, 6, true>(taps, c, x, N, B, 0); });
  // compute only (wave kernel, MEM = 0) at the same grid
  {
    using G = wave::WGeo<8, 8>;
    const long warm = ((long)(G::H + 63) / 64) * 64;
    const long seg = fast::pick_seg(N, B, warm, 64, 8192);
    long steps = seg / 64 + warm / 64;
    steps = ((steps + 5) / 6) * 6;
    const size_t lds = (size_t)G::lds_pairs * 16;
    auto k = wave::modwt_inv_wave<8, 8, true, 3, 6, 0>;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    timeit("wave fma compute only", [&] {
      k<<<dim3((unsigned)((N + seg - 1) / seg), B), 64, lds>>>(c, x, N, seg, (steps - 1) * 64, steps / 6, taps);
    });
  }
  probe();
  printf("done %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
