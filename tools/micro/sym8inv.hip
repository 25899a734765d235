// Where the Symlet8 J=6 inverse (cfg5) spends its time: the library's wave kernel on zeros vs
// on random coefficients (the clock drops under data-dependent FP64 power), its LDS/VALU work
// alone (MEM = 0), and the shader clock each leaves behind.
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

__global__ void fill_random(double* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned long long z = (unsigned long long)i * 0x9E3779B97F4A7C15ull + 12345;
    z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 27;
    p[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}

int main() {
  const long N = 1L << 20;
  const int B = 1024;
  double *c, *x;
  hipMalloc(&c, 7L * N * B * 8);
  hipMalloc(&x, N * B * 8);
  Taps taps{};
  for (int m = 0; m < 16; ++m) { taps.a[m] = 0.1 * m - 0.7; taps.b[m] = 0.2 - 0.01 * m; }
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
  auto timeit = [&](const char* name, auto&& launch) {
    launch();
    hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-44s %8.3f ms\n", name, ms / 5);
  };
  auto wave_launch = [&](auto kern) {
    using G = wave::WGeo<16, 6>;
    constexpr int U = 6;
    const long warm = ((long)(G::H + 63) / 64) * 64;
    const long seg = fast::pick_seg(N, B, warm, 64, 8192);
    long steps = seg / 64 + warm / 64;
    steps = ((steps + U - 1) / U) * U;
    const size_t lds = (size_t)G::lds_pairs * 16;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<dim3((unsigned)((N + seg - 1) / seg), B), 64, lds>>>(c, x, N, seg, (steps - 1) * 64,
                                                               steps / U, taps);
  };
  probe();
  hipMemset(c, 0, 7L * N * B * 8);
  timeit("sym8 J6 fma    zeros", [&] { wave_launch(wave::modwt_inv_wave<16, 6, true, 3, 6, 1, 0>); });
  timeit("sym8 J6 strict zeros", [&] { wave_launch(wave::modwt_inv_wave<16, 6, false, 3, 6, 1, 0>); });
  fill_random<<<4096, 256>>>(c, 7L * N * B);
  hipDeviceSynchronize();
  timeit("sym8 J6 fma    random", [&] { wave_launch(wave::modwt_inv_wave<16, 6, true, 3, 6, 1, 0>); });
  probe();
  timeit("sym8 J6 strict random", [&] { wave_launch(wave::modwt_inv_wave<16, 6, false, 3, 6, 1, 0>); });
  timeit("sym8 J6 fma    compute only (no HBM)", [&] { wave_launch(wave::modwt_inv_wave<16, 6, true, 3, 6, 0, 0>); });
  timeit("sym8 J6 strict compute only (no HBM)", [&] { wave_launch(wave::modwt_inv_wave<16, 6, false, 3, 6, 0, 0>); });
  timeit("db4 J8 (as sym8 grid) fma random", [&] {
    using G = wave::WGeo<8, 8>;
    constexpr int U = 6;
    auto kern = wave::modwt_inv_wave<8, 8, true, 3, 6, 1, 0>;
    const long warm = ((long)(G::H + 63) / 64) * 64;
    const long seg = fast::pick_seg(N, 512, warm, 64, 8192);
    long steps = ((seg / 64 + warm / 64 + U - 1) / U) * U;
    const size_t lds = (size_t)G::lds_pairs * 16;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<dim3((unsigned)((N + seg - 1) / seg), 512), 64, lds>>>(c, x, N, seg, (steps - 1) * 64, steps / U, taps);
  });
  probe();
  printf("done %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
