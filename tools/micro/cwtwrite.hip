// cwtwrite.hip -- the CWT coefficient write shape without any FFT: how fast can 512-thread
// workgroups write one (signal, scale) pair's 2^18 complex outputs (4 MB) when each workgroup
// owns 8 rows n1 of the four-step output t = n1 + 512 n2 (128-byte pieces 8 KB apart, the
// shape of CoefOut behind pass512_tail), against contiguous 64 KB per workgroup.
// Modes: 0 = row pieces, nt stores; 1 = row pieces, plain stores; 2 = contiguous, nt;
//        3 = contiguous, plain; LDS staging as in the kernels (72 KB per workgroup) in all modes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o cwtwrite_bin cwtwrite.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double nt2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(512) void wr(double2* out, long pairs) {
  __shared__ double2 tile[4608];
  const int tid = threadIdx.x;
  const long rg = blockIdx.x & 63, pair = blockIdx.x >> 6;
  if (pair >= pairs) return;
  // something to stage: a value per element, through LDS like the real tail
#pragma unroll
  for (int i = 0; i < 8; ++i) tile[tid + 512 * i] = make_double2(tid + i, rg);
  __syncthreads();
  double2* o = out + pair * (1L << 18);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = (tid >> 3) + 64 * i, cc = tid & 7;
    const double2 v = tile[8 * n + cc];
    long t;
    if constexpr (MODE <= 1) {
      t = (rg * 8 + cc) + 512L * n;  // row pieces
    } else {
      t = rg * 4096 + tid + 512L * i;  // contiguous 64 KB
    }
    if constexpr (MODE == 0 || MODE == 2) {
      nt2 w = {v.x, v.y};
      __builtin_nontemporal_store(w, (nt2*)&o[t]);
    } else {
      o[t] = v;
    }
  }
}

int main() {
  const long pairs = 2048;  // 8 GB of output
  double2* out;
  if (hipMalloc(&out, pairs * (1L << 18) * sizeof(double2)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name) {
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(pairs * 64), dim3(512), 0, 0, out, pairs);
    hipEventRecord(e0);
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(kern, dim3(pairs * 64), dim3(512), 0, 0, out, pairs);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double bytes = pairs * (double)(1L << 18) * 16;
    printf("%-28s %8.3f ms  %6.2f TB/s  %.3f us/pair\n", name, ms, bytes / ms / 1e9, ms * 1e3 / pairs);
  };
  run(wr<0>, "row pieces, nt");
  run(wr<1>, "row pieces, plain");
  run(wr<2>, "contiguous, nt");
  run(wr<3>, "contiguous, plain");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
