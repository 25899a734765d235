// What copy shape reaches MI355X_MICROARCH.md's "6.29 TB/s float4 copy"?  Plain 16-byte copies
// of 4 GiB in four organisations (grid-stride, per-workgroup contiguous chunks, non-temporal),
// against the segment-stream shape of the MODWT kernels (tools/micro/membench.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void grid_stride(const d2v* __restrict__ in, d2v* __restrict__ out, long n) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += U * stride) {
    d2v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? (NT ? __builtin_nontemporal_load(&in[i + u * stride]) : in[i + u * stride]) : d2v{0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) if (i + u * stride < n) { if (NT) __builtin_nontemporal_store(v[u], &out[i + u * stride]); else out[i + u * stride] = v[u]; }
  }
}

// each workgroup copies its own contiguous chunk, 256 x U elements per step
template <int U>
__global__ __launch_bounds__(256) void chunked(const d2v* __restrict__ in, d2v* __restrict__ out, long per) {
  const long base = (long)blockIdx.x * per;
  for (long s = 0; s < per; s += 256 * U) {
    d2v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = in[base + s + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) out[base + s + u * 256 + threadIdx.x] = v[u];
  }
}

// the MODWT kernels' row shapes (membench.hip pattern2): RIN rows in, ROUT rows out, one
// segment of seg samples per workgroup, grid (segments, signals) with segments fastest
template <int RIN, int ROUT, int U, bool REV>
__global__ __launch_bounds__(256) void rows(const double* __restrict__ in, double* __restrict__ out,
                                            long N, long seg) {
  constexpr int C = 512;
  const int t = threadIdx.x;
  const double* ib = in + (long)blockIdx.y * RIN * N;
  double* ob = out + (long)blockIdx.y * ROUT * N;
  const long P = (long)blockIdx.x * seg;
  for (long s = 0; s < seg; s += U * C) {
    d2v v[U][RIN > 0 ? RIN : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long a = REV ? P + seg - (s + (u + 1) * C) : P + s + u * C;
#pragma unroll
      for (int r = 0; r < RIN; ++r) v[u][r] = *(const d2v*)&ib[r * N + a + 2 * t];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long a = REV ? P + seg - (s + (u + 1) * C) : P + s + u * C;
      d2v acc = {0.0, 0.0};
#pragma unroll
      for (int r = 0; r < RIN; ++r) acc += v[u][r];
#pragma unroll
      for (int r = 0; r < ROUT; ++r) *(d2v*)&ob[r * N + a + 2 * t] = acc + (double)r;
    }
  }
}

template <class F>
void timeit(const char* name, F launch, double bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) launch();
  CK(hipEventRecord(e0));
  const int it = 10;
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
  printf("%-44s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
}

int main() {
  const long bytes = 4L << 30, n = bytes / 16;
  d2v *in, *out;
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes));
  CK(hipMemset(in, 0, bytes)); CK(hipMemset(out, 0, bytes));
  const double moved = 2.0 * bytes;
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "grid-stride U=4 grid=%d", g);
    timeit(nm, [&] { grid_stride<4, false><<<g, 256>>>(in, out, n); }, moved);
    snprintf(nm, 64, "grid-stride U=4 NT grid=%d", g);
    timeit(nm, [&] { grid_stride<4, true><<<g, 256>>>(in, out, n); }, moved);
  }
  timeit("grid-stride U=1 grid=n/256", [&] { grid_stride<1, false><<<(unsigned)(n / 256), 256>>>(in, out, n); }, moved);
  timeit("grid-stride U=1 NT grid=n/256", [&] { grid_stride<1, true><<<(unsigned)(n / 256), 256>>>(in, out, n); }, moved);
  for (int wg : {2048, 8192, 32768}) {
    char nm[64];
    snprintf(nm, 64, "chunked U=4 wgs=%d", wg);
    timeit(nm, [&] { chunked<4><<<wg, 256>>>(in, out, n / wg); }, moved);
  }
  for (int wg : {131072, 1048576}) {
    char nm[64];
    snprintf(nm, 64, "chunked U=1 wgs=%d", wg);
    timeit(nm, [&] { chunked<1><<<wg, 256>>>(in, out, n / wg); }, moved);
  }
  // MODWT shapes at 1024 signals x 2^20 with shorter segments
  {
    const long N = 1L << 20;
    const int B = 1024;
    double *ri, *ro;
    CK(hipMalloc(&ri, 9L * N * B * 8)); CK(hipMalloc(&ro, 9L * N * B * 8));
    CK(hipMemset(ri, 0, 9L * N * B * 8)); CK(hipMemset(ro, 0, 9L * N * B * 8));
    const double fwd = 80.0 * N * B, inv = 80.0 * N * B;
    for (long seg : {131072L, 32768L, 8192L, 2048L}) {
      char nm[64];
      dim3 g((unsigned)(N / seg), (unsigned)B);
      snprintf(nm, 64, "forward-like 1->9 seg=%ld", seg);
      timeit(nm, [&] { rows<1, 9, 2, false><<<g, 256>>>(ri, ro, N, seg); }, fwd);
      snprintf(nm, 64, "inverse-like 9->1 rev seg=%ld", seg);
      timeit(nm, [&] { rows<9, 1, 2, true><<<g, 256>>>(ri, ro, N, seg); }, inv);
    }
  }
  return 0;
}
