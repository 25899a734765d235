// Does a workspace written by one XCD re-read faster from that same XCD's L2 than from
// another XCD (i.e. from the Infinity Cache / HBM)?  VERDICT r05 item 2(a): if the re-read is
// >= 1.5x faster, the CWT's two-pass chain (pass 1 writes a 4 MB workspace A per (signal, scale)
// pair at N = 2^18, pass 2 reads it back) could run each pair's two passes on one XCD.
//
// Workgroups are grouped by b % 8 (blocks b and b + 8 share an XCD, MI355X_MICROARCH.md
// "Workgroup dispatch"); the probe reads the XCC id too and reports how consistent that is.
//   cross-launch: kernel 1 writes slice g = b % 8 (S bytes per slice) with plain stores; kernel 2
//                 reads slice (b % 8 + shift) % 8 -- shift 0 = the writer's XCD, 1..7 = another.
//   in-kernel:    one launch: write, grid barrier (agent release / acquire, L1 invalidated, L2
//                 kept), then the same read: L2 residency without a launch boundary.
// The read phase is timed on the device (s_memrealtime, 100 MHz): max(end) - min(start) over
// the workgroups.  Usage: xcdbench (one line per configuration).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);            \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
constexpr int kW = 32;  // workgroups per XCD group (one per CU of an XCD)
constexpr int kG = 8 * kW;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

__device__ void write_slice(d2v* p, long per, int g, int i, double v) {
  d2v* s = p + (long)g * per;
  for (long k = (long)i * 256 + threadIdx.x; k < per; k += (long)kW * 256) s[k] = d2v{v + (double)k, v};
}
__device__ double read_slice(const d2v* p, long per, int g, int i) {
  const d2v* s = p + (long)g * per;
  d2v acc = {0.0, 0.0};
#pragma unroll 4
  for (long k = (long)i * 256 + threadIdx.x; k < per; k += (long)kW * 256) acc += s[k];
  return acc.x + acc.y;
}

__global__ __launch_bounds__(256) void kflush(d2v* p, long n) {
  for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < n; k += (long)gridDim.x * 256)
    p[k] = d2v{(double)k, 1.0};
}

__global__ __launch_bounds__(256) void kwrite(d2v* p, long per, double v, int* xcc) {
  const int b = blockIdx.x;
  write_slice(p, per, b % 8, b / 8, v);
  if (threadIdx.x == 0) xcc[b] = xcc_id();
}

__global__ __launch_bounds__(256) void kread(const d2v* p, long per, int shift, double* sink,
                                             unsigned long long* t) {
  const int b = blockIdx.x;
  __syncthreads();
  const unsigned long long t0 = now();
  const double s = read_slice(p, per, (b % 8 + shift) % 8, b / 8);
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  const unsigned long long t1 = now();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int k = 0; k < 256; ++k) a += red[k];
    sink[b] = a;
    t[2 * b] = t0;
    t[2 * b + 1] = t1;
  }
}

// grid barrier over kG co-resident workgroups (one counter, generation-free: used once)
__device__ void grid_barrier(unsigned* ctr) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // bounded spin: every wave leaves even if a workgroup never arrived (then the timing is void)
    for (int it = 0; it < (1 << 22) &&
                     __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)kG;
         ++it)
      __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void kfused(d2v* p, long per, int shift, double v, unsigned* ctr,
                                              double* sink, unsigned long long* t) {
  const int b = blockIdx.x;
  write_slice(p, per, b % 8, b / 8, v);
  grid_barrier(ctr);
  const unsigned long long t0 = now();
  const double s = read_slice(p, per, (b % 8 + shift) % 8, b / 8);
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  const unsigned long long t1 = now();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int k = 0; k < 256; ++k) a += red[k];
    sink[b] = a;
    t[2 * b] = t0;
    t[2 * b + 1] = t1;
  }
}

static double span_us(const std::vector<unsigned long long>& t) {
  unsigned long long lo = ~0ULL, hi = 0;
  for (int b = 0; b < kG; ++b) {
    lo = std::min(lo, t[2 * b]);
    hi = std::max(hi, t[2 * b + 1]);
  }
  return (double)(hi - lo) / 100.0;  // 100 MHz
}

int main() {
  const long max_per = (8L << 20) / 16;  // up to 8 MiB per slice
  d2v* A = nullptr;
  double* sink = nullptr;
  unsigned long long* dt = nullptr;
  unsigned* ctr = nullptr;
  int* xcc = nullptr;
  d2v* flush = nullptr;
  const long flush_n = (512L << 20) / 16;  // 512 MiB: evicts L2 and the Infinity Cache
  CK(hipMalloc(&A, 8 * max_per * 16));
  CK(hipMalloc(&flush, flush_n * 16));
  CK(hipMalloc(&sink, kG * 8));
  CK(hipMalloc(&dt, 2 * kG * 8));
  CK(hipMalloc(&ctr, 4));
  CK(hipMalloc(&xcc, kG * 4));
  std::vector<unsigned long long> t(2 * kG);
  std::vector<int> hx(kG);
  // placement check: does b % 8 name one XCC?
  hipLaunchKernelGGL(kwrite, dim3(kG), dim3(256), 0, 0, A, 1024L, 1.0, xcc);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hx.data(), xcc, kG * 4, hipMemcpyDeviceToHost));
  int consistent = 0;
  for (int b = 0; b < kG; ++b) consistent += hx[b] == hx[b % 8];
  printf("placement: %d of %d blocks on the XCC of block b %% 8\n", consistent, kG);
  const int reps = 9;
  for (long kb : {1024L, 2048L, 3072L, 4096L, 8192L}) {
    const long per = kb * 1024 / 16;
    for (int fused = 0; fused < 2; ++fused) {
      for (int shift : {0, 1, 4}) {
        std::vector<double> us;
        for (int r = 0; r < reps; ++r) {
          // cold start: stream 512 MiB through the caches first
          hipLaunchKernelGGL(kflush, dim3(4096), dim3(256), 0, 0, flush, flush_n);
          if (fused) {
            CK(hipMemset(ctr, 0, 4));
            hipLaunchKernelGGL(kfused, dim3(kG), dim3(256), 0, 0, A, per, shift, 2.0 + r, ctr, sink, dt);
          } else {
            hipLaunchKernelGGL(kwrite, dim3(kG), dim3(256), 0, 0, A, per, 2.0 + r, xcc);
            hipLaunchKernelGGL(kread, dim3(kG), dim3(256), 0, 0, A, per, shift, sink, dt);
          }
          CK(hipDeviceSynchronize());
          CK(hipMemcpy(t.data(), dt, 2 * kG * 8, hipMemcpyDeviceToHost));
          us.push_back(span_us(t));
        }
        std::sort(us.begin(), us.end());
        const double med = us[reps / 2];
        const double bytes = 8.0 * per * 16;
        printf("%-12s slice %5ld KB  shift %d : read %.2f us  (%.2f TB/s over %.0f MB)\n",
               fused ? "in-kernel" : "cross-launch", kb, shift, med, bytes / (med * 1e-6) / 1e12,
               bytes / 1e6);
      }
    }
  }
  return 0;
}
