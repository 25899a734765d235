// Memory-pattern microbenchmark: the MODWT kernels' HBM access shape without the math.
// Each workgroup streams one segment of one signal, C samples per step, through RIN input
// rows and ROUT output rows (rows N doubles apart, signals (RIN|ROUT)*N apart).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int RIN, int ROUT, int C, int U, bool REV>
__global__ __launch_bounds__(C) void pattern(const double* __restrict__ in, double* __restrict__ out,
                                             long N, long seg) {
  const int t = threadIdx.x;
  const double* ib = in + (long)blockIdx.y * RIN * N;
  double* ob = out + (long)blockIdx.y * ROUT * N;
  const long P = (long)blockIdx.x * seg;
  for (long s = 0; s < seg; s += U * C) {
    double v[U][RIN];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long a = REV ? P + seg - (s + (u + 1) * C) : P + s + u * C;
#pragma unroll
      for (int r = 0; r < RIN; ++r) v[u][r] = ib[r * N + a + t];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long a = REV ? P + seg - (s + (u + 1) * C) : P + s + u * C;
      double acc = 0.0;
#pragma unroll
      for (int r = 0; r < RIN; ++r) acc += v[u][r];
#pragma unroll
      for (int r = 0; r < ROUT; ++r) ob[r * N + a + t] = acc + r;
    }
  }
}

typedef double d2v __attribute__((ext_vector_type(2)));
template <int RIN, int ROUT, int NT, int U, bool REV>
__global__ __launch_bounds__(NT) void pattern2(const double* __restrict__ in, double* __restrict__ out,
                                               long N, long seg) {
  constexpr int C = 2 * NT;
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

template <int RIN, int ROUT, int NT, int U, bool REV>
void run2(const char* name, double* in, double* out, long N, int B, long nseg) {
  const long seg = N / nseg;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  dim3 g((unsigned)nseg, (unsigned)B);
  for (int i = 0; i < 2; ++i) pattern2<RIN, ROUT, NT, U, REV><<<g, NT>>>(in, out, N, seg);
  CK(hipEventRecord(e0));
  const int it = 5;
  for (int i = 0; i < it; ++i) pattern2<RIN, ROUT, NT, U, REV><<<g, NT>>>(in, out, N, seg);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
  const double bytes = 8.0 * (RIN + ROUT) * (double)N * B;
  printf("%-34s NT=%3d U=%d nseg=%3ld  %8.3f ms  %7.1f GB/s\n", name, NT, U, nseg, ms, bytes / ms / 1e6);
}

template <int RIN, int ROUT, int C, int U, bool REV>
void run(const char* name, double* in, double* out, long N, int B, long nseg) {
  const long seg = N / nseg;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  dim3 g((unsigned)nseg, (unsigned)B);
  for (int i = 0; i < 2; ++i) pattern<RIN, ROUT, C, U, REV><<<g, C>>>(in, out, N, seg);
  CK(hipEventRecord(e0));
  const int it = 5;
  for (int i = 0; i < it; ++i) pattern<RIN, ROUT, C, U, REV><<<g, C>>>(in, out, N, seg);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
  const double bytes = 8.0 * (RIN + ROUT) * (double)N * B;
  printf("%-34s C=%3d U=%d nseg=%3ld  %8.3f ms  %7.1f GB/s\n", name, C, U, nseg, ms, bytes / ms / 1e6);
}

int main() {
  const long N = 1L << 20; const int B = 1024;
  double *in, *out;
  CK(hipMalloc(&in, 9L * N * B * 8)); CK(hipMalloc(&out, 9L * N * B * 8));
  CK(hipMemset(in, 0, 9L * N * B * 8)); CK(hipMemset(out, 0, 9L * N * B * 8));
  run<1, 1, 256, 4, false>("copy 1->1", in, out, N, B * 4, 8);
  run<9, 1, 256, 2, true>("inverse-like 9->1 rev", in, out, N, B, 8);
  run<9, 1, 256, 4, true>("inverse-like 9->1 rev", in, out, N, B, 8);
  run<9, 1, 512, 2, true>("inverse-like 9->1 rev", in, out, N, B, 8);
  run<9, 1, 256, 2, false>("inverse-like 9->1 fwd", in, out, N, B, 8);
  run<9, 1, 256, 2, true>("inverse-like 9->1 rev", in, out, N, B, 32);
  run<9, 1, 256, 2, true>("inverse-like 9->1 rev", in, out, N, B, 2);
  run<1, 9, 512, 2, false>("forward-like 1->9", in, out, N, B, 8);
  run<1, 9, 256, 2, false>("forward-like 1->9", in, out, N, B, 8);
  run<9, 0, 256, 2, true>("read-only 9 rows rev", in, out, N, B, 8);
  run<0, 9, 256, 2, false>("write-only 9 rows", in, out, N, B, 8);
  run2<1, 1, 256, 4, false>("copy16 1->1", in, out, N, B * 4, 8);
  run2<9, 1, 256, 2, true>("inverse-like16 9->1 rev", in, out, N, B, 8);
  run2<9, 1, 128, 2, true>("inverse-like16 9->1 rev", in, out, N, B, 8);
  run2<1, 9, 256, 2, false>("forward-like16 1->9", in, out, N, B, 8);
  run2<0, 9, 256, 2, false>("write-only16 9 rows", in, out, N, B, 8);
  run2<0, 1, 256, 4, false>("write-only16 1 row", in, out, N, B * 9, 8);
  // fewer concurrent streams: more lanes per segment (one stream set per workgroup)
  run2<9, 1, 512, 2, true>("inverse-like16 9->1 rev", in, out, N, B, 8);
  run2<9, 1, 1024, 1, true>("inverse-like16 9->1 rev", in, out, N, B, 8);
  run2<9, 1, 1024, 2, true>("inverse-like16 9->1 rev", in, out, N, B, 4);
  run2<9, 1, 256, 4, true>("inverse-like16 9->1 rev", in, out, N, B, 2);
  run2<1, 1, 1024, 2, false>("copy16 1->1", in, out, N, B * 4, 8);
  run2<9, 0, 512, 2, true>("read-only16 9 rows rev", in, out, N, B, 8);
  return 0;
}
