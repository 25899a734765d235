// Does a buffer written by one kernel get re-read from the 256 MB Infinity Cache (MALL) by the
// next, or from HBM?  The CWT's two-pass scales round-trip a workspace A (pass 1 writes it, pass 2
// reads it back while writing the coefficients); if a small A re-reads faster than HBM, a
// smaller, better-scheduled workspace would cut the two-pass chain's time.
//   write  : W bytes, 16 B per lane, grid-stride (plain or non-temporal stores)
//   read   : the same W bytes right after the write (sum per lane, one store per workgroup)
//   pass2  : read the W bytes and write W bytes elsewhere (NT), the two-pass pass-2 shape
// Usage: mallbench   (prints one line per size)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ __launch_bounds__(256) void kwrite(d2v* p, long n, double v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const d2v w = {v + (double)i, v};
    if (NT) __builtin_nontemporal_store(w, p + i); else p[i] = w;
  }
}

__global__ __launch_bounds__(256) void kread(const d2v* p, long n, double* out) {
  d2v acc = {0.0, 0.0};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc += p[i];
  __shared__ double red[256];
  red[threadIdx.x] = acc.x + acc.y;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int t = 0; t < 256; ++t) s += red[t];
    out[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(256) void kpass2(const d2v* p, d2v* q, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    d2v v = p[i];
    v.x += 1.0;
    __builtin_nontemporal_store(v, q + i);
  }
}

int main() {
  const long big = 4L << 30;  // 4 GiB pool: windows are taken from a rotating offset
  d2v *A = nullptr, *O = nullptr;
  double* sums = nullptr;
  CK(hipMalloc(&A, big));
  CK(hipMalloc(&O, big));
  CK(hipMalloc(&sums, 1 << 20));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  const int grid = 256 * 16;
  // warm the clocks
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kwrite<false>, dim3(grid), dim3(256), 0, 0, A, big / 16, 1.0);
  CK(hipDeviceSynchronize());
  const long sizes_mb[] = {8, 16, 32, 64, 96, 128, 192, 256, 512, 1024};
  for (int nt = 0; nt < 2; ++nt) {
    for (long mb : sizes_mb) {
      const long bytes = mb << 20, n = bytes / 16;
      const int reps = (int)(big / bytes) < 8 ? (int)(big / bytes) : 8;
      float tw = 0, tr = 0, tp = 0;
      for (int r = 0; r < reps; ++r) {
        d2v* a = A + (long)r * n;  // a fresh window each rep (nothing left from the last one)
        CK(hipEventRecord(e0));
        if (nt) hipLaunchKernelGGL(kwrite<true>, dim3(grid), dim3(256), 0, 0, a, n, 2.0 + r);
        else hipLaunchKernelGGL(kwrite<false>, dim3(grid), dim3(256), 0, 0, a, n, 2.0 + r);
        CK(hipEventRecord(e1));
        hipLaunchKernelGGL(kread, dim3(grid), dim3(256), 0, 0, a, n, sums);
        CK(hipEventRecord(e2));
        CK(hipEventSynchronize(e2));
        float x, y;
        CK(hipEventElapsedTime(&x, e0, e1));
        CK(hipEventElapsedTime(&y, e1, e2));
        tw += x;
        tr += y;
        // pass-2 shape: rewrite the window, then read it while writing elsewhere
        hipLaunchKernelGGL(kwrite<false>, dim3(grid), dim3(256), 0, 0, a, n, 3.0 + r);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kpass2, dim3(grid), dim3(256), 0, 0, a, O + (long)r * n, n);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&x, e0, e1));
        tp += x;
      }
      tw /= reps;
      tr /= reps;
      tp /= reps;
      printf("%-3s W=%5ld MB  write %8.1f us %7.1f GB/s | read-after-write %8.1f us %7.1f GB/s | "
             "pass2 (read W + NT write W) %8.1f us %7.1f GB/s\n",
             nt ? "NT" : "pl", mb, tw * 1e3, bytes / (tw * 1e-3) / 1e9, tr * 1e3,
             bytes / (tr * 1e-3) / 1e9, tp * 1e3, 2.0 * bytes / (tp * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  // cold read: a window not touched for GBs
  {
    const long n = (64L << 20) / 16;
    hipLaunchKernelGGL(kwrite<false>, dim3(grid), dim3(256), 0, 0, A, big / 16, 5.0);
    hipLaunchKernelGGL(kwrite<false>, dim3(grid), dim3(256), 0, 0, O, big / 16, 5.0);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kread, dim3(grid), dim3(256), 0, 0, A, n, sums);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float x;
    CK(hipEventElapsedTime(&x, e0, e1));
    printf("cold read 64 MB %8.1f us %7.1f GB/s\n", x * 1e3, (64L << 20) / (x * 1e-3) / 1e9);
  }
  return 0;
}
