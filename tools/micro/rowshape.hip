// Verdict r03 item 7: does the MODWT row shape (1 row in / 9 rows out, 9 in / 1 out, 1024 signals
// x 2^20) stream faster when every row gets longer contiguous runs per burst?  copybench.hip
// measured the step-major order (per 512-sample step: 4 KB to each of the 9 rows in turn) at
// 5.26-5.42 TB/s against 6.4-6.7 TB/s for one-shot 4 KB workgroups of a plain copy.
//   ORDER 0: step-major (the kernels' order today): for u < U { for r < 9 { 4 KB of row r } }
//   ORDER 1: row-major: for r < 9 { for u < U { 4 KB of row r } } = one U x 4 KB run per row
// and three schedules: a workgroup streams its segment (seg samples) in U x 512-sample blocks;
// or one-shot workgroups of exactly one block (seg = U x 512, grid = all blocks, segments
// fastest); plus the plain 1-row copy for the box's reference rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

template <int RIN, int ROUT, int U, bool REV, int ORDER, int NT = 256>
__global__ __launch_bounds__(NT) void rows(const double* __restrict__ in, double* __restrict__ out,
                                           long N, long seg) {
  constexpr int C = 2 * NT;
  const int t = threadIdx.x;
  const double* ib = in + (long)blockIdx.y * RIN * N;
  double* ob = out + (long)blockIdx.y * ROUT * N;
  const long P = (long)blockIdx.x * seg;
  for (long s = 0; s < seg; s += U * C) {
    d2v v[U][RIN];
    auto pos = [&](int u) { return REV ? P + seg - (s + (u + 1) * C) : P + s + u * C; };
    if (ORDER == 0) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RIN; ++r) v[u][r] = *(const d2v*)&ib[r * N + pos(u) + 2 * t];
    } else {
#pragma unroll
      for (int r = 0; r < RIN; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) v[u][r] = *(const d2v*)&ib[r * N + pos(u) + 2 * t];
    }
    d2v acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc[u] = d2v{0.0, 0.0};
#pragma unroll
      for (int r = 0; r < RIN; ++r) acc[u] += v[u][r];
    }
    if (ORDER == 0) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < ROUT; ++r) *(d2v*)&ob[r * N + pos(u) + 2 * t] = acc[u] + (double)r;
    } else {
#pragma unroll
      for (int r = 0; r < ROUT; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) *(d2v*)&ob[r * N + pos(u) + 2 * t] = acc[u] + (double)r;
    }
  }
}

template <class F>
void timeit(const char* name, F launch, double bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) launch();
  CK(hipEventRecord(e0));
  const int it = 8;
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
  printf("%-52s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  fflush(stdout);
}

template <int U, int ORDER>
void shapes(double* ri, double* ro, long N, int B, const char* tag) {
  const double bytes = 80.0 * N * B;
  char nm[96];
  for (long seg : {131072L, 16384L, (long)U * 512}) {
    dim3 g((unsigned)(N / seg), (unsigned)B);
    snprintf(nm, 96, "1->9 U=%d %s seg=%ld%s", U, tag, seg, seg == U * 512 ? " (one-shot)" : "");
    timeit(nm, [&] { rows<1, 9, U, false, ORDER><<<g, 256>>>(ri, ro, N, seg); }, bytes);
    snprintf(nm, 96, "9->1 U=%d %s seg=%ld%s", U, tag, seg, seg == U * 512 ? " (one-shot)" : "");
    timeit(nm, [&] { rows<9, 1, U, true, ORDER><<<g, 256>>>(ri, ro, N, seg); }, bytes);
  }
}

int main() {
  const long N = 1L << 20;
  const int B = 1024;
  double *ri, *ro;
  CK(hipMalloc(&ri, 9L * N * B * 8)); CK(hipMalloc(&ro, 9L * N * B * 8));
  // random-ish bits, not zeros (no chance of a zero-data shortcut anywhere)
  CK(hipMemset(ri, 0x3c, 9L * N * B * 8)); CK(hipMemset(ro, 0x3c, 9L * N * B * 8));
  {
    const long n = (4L << 30) / 8;
    dim3 g((unsigned)(n / 512), 1);
    timeit("copy 1->1 one-shot 4 KB workgroups (4 GiB)",
           [&] { rows<1, 1, 1, false, 0><<<g, 256>>>(ri, ro, n, 512); }, 2.0 * n * 8);
  }
  shapes<2, 0>(ri, ro, N, B, "step-major");
  shapes<2, 1>(ri, ro, N, B, "row-major ");
  shapes<4, 0>(ri, ro, N, B, "step-major");
  shapes<4, 1>(ri, ro, N, B, "row-major ");
  shapes<8, 1>(ri, ro, N, B, "row-major ");
  // one wave per segment (the inverse wave kernels' shape: 1 KB per row per step)
  {
    const double bytes = 80.0 * N * B;
    for (long seg : {131072L, 16384L}) {
      dim3 g((unsigned)(N / seg), (unsigned)B);
      char nm[96];
      snprintf(nm, 96, "9->1 wave U=2 step-major seg=%ld", seg);
      timeit(nm, [&] { rows<9, 1, 2, true, 0, 64><<<g, 64>>>(ri, ro, N, seg); }, bytes);
      snprintf(nm, 96, "9->1 wave U=4 row-major seg=%ld", seg);
      timeit(nm, [&] { rows<9, 1, 4, true, 1, 64><<<g, 64>>>(ri, ro, N, seg); }, bytes);
      snprintf(nm, 96, "9->1 wave U=8 row-major seg=%ld", seg);
      timeit(nm, [&] { rows<9, 1, 8, true, 1, 64><<<g, 64>>>(ri, ro, N, seg); }, bytes);
    }
  }
  return 0;
}
