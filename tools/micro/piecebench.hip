// Write (and read) efficiency of the CWT output shape: the 512 x 512 four-step writes every
// (signal, scale) row of 2^18 complex outputs as 512 pieces of L lines x 16 B (8 consecutive
// n1, one n2) at a stride of 512 x 16 B = 8 KB, one workgroup per L lines.  Does a wider piece
// (16, 32, 64 lines: 256 B .. 1 KB) move HBM faster?  Also the same pieces read.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

// grid: (512 / LINES line groups, pairs); 512 threads; each thread writes 16-byte values
// out[pair][n1 + 512 n2] for n1 in the group's LINES lines, n2 < 512
template <int LINES, bool NT, bool READ>
__global__ __launch_bounds__(512) void pieces(d2v* __restrict__ out, const d2v* __restrict__ in) {
  const long pair = blockIdx.y;
  const int g = blockIdx.x;
  d2v* o = out + pair * 262144L;
  const d2v* ip = in + pair * 262144L;
  constexpr int PER = 512 * LINES / 512;  // values per thread
  d2v acc = {0.0, 0.0};
#pragma unroll 8
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + 512 * i;          // element of the group's LINES x 512 block
    const int n1 = g * LINES + e % LINES, n2 = e / LINES;
    const long idx = n1 + 512L * n2;
    if (READ) {
      acc += NT ? __builtin_nontemporal_load(&ip[idx]) : ip[idx];
    } else {
      const d2v v = {(double)idx, (double)pair};
      if (NT) {
        __builtin_nontemporal_store(v, &o[idx]);
      } else {
        o[idx] = v;
      }
    }
  }
  if (READ && acc.x == -1.0) o[0] = acc;  // keep the loads
}

template <class F>
void timeit(const char* name, F launch, double bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) launch();
  CK(hipEventRecord(e0));
  const int it = 6;
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
  printf("%-40s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  fflush(stdout);
}

template <int LINES>
void run(d2v* a, d2v* b, int pairs) {
  const double bytes = (double)pairs * 262144 * 16;
  dim3 g(512 / LINES, pairs);
  char nm[64];
  snprintf(nm, 64, "write %d lines (%d B pieces)", LINES, LINES * 16);
  timeit(nm, [&] { pieces<LINES, false, false><<<g, 512>>>(a, b); }, bytes);
  snprintf(nm, 64, "write %d lines NT", LINES);
  timeit(nm, [&] { pieces<LINES, true, false><<<g, 512>>>(a, b); }, bytes);
  snprintf(nm, 64, "read  %d lines", LINES);
  timeit(nm, [&] { pieces<LINES, false, true><<<g, 512>>>(a, b); }, bytes);
}

int main() {
  const int pairs = 4096;  // 16 GiB
  d2v *a, *b;
  CK(hipMalloc(&a, (size_t)pairs * 262144 * 16));
  CK(hipMalloc(&b, (size_t)pairs * 262144 * 16));
  CK(hipMemset(a, 0, (size_t)pairs * 262144 * 16));
  CK(hipMemset(b, 0x3c, (size_t)pairs * 262144 * 16));
  run<2>(a, b, pairs);
  run<4>(a, b, pairs);
  run<8>(a, b, pairs);
  run<16>(a, b, pairs);
  run<32>(a, b, pairs);
  run<64>(a, b, pairs);
  run<512>(a, b, pairs);  // whole rows: contiguous
  return 0;
}
