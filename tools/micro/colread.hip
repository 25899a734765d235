// Column-tile reads of the STRICT FFT column kernels (jw_jfft.hpp load_cols): items of a [1024][1024]
// complex view, T columns x 1024 rows per 512-thread workgroup (T x 16-byte pieces per row), with
// the kernels' XCD-aware tile order (tile_item: consecutive workgroups of an XCD take adjacent tiles)
// or the plain one (tile fastest).  T = 4 is what the kernels do (64-byte pieces); 8 = 128-byte
// pieces (two phases of 4 columns through the same LDS, the second half held in registers).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
constexpr int LC = 1024, NT = 512;

__device__ __forceinline__ void tile_item(int ntiles, long nitems, bool xcd, int* tile, long* item) {
  const long b = blockIdx.x;
  if (xcd && (ntiles & 7) == 0) {
    const int x = (int)(b & 7), per = ntiles >> 3;
    const long q = b >> 3;
    *tile = x * per + (int)(q % per);
    *item = q / per;
  } else {
    *tile = (int)(b % ntiles);
    *item = b / ntiles;
  }
}

// T columns per workgroup; EPT = T * LC / NT values per thread
template <int T>
__global__ __launch_bounds__(NT) void colread(const d2v* __restrict__ z, d2v* __restrict__ out,
                                              long nitems, int xcd) {
  constexpr int EPT = T * LC / NT;
  __shared__ d2v lds[4 * (LC + LC / 16 + 1)];
  int tile;
  long item;
  tile_item(LC / T, nitems, xcd != 0, &tile, &item);
  const d2v* zi = z + item * (long)LC * LC;
  d2v v[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int f = threadIdx.x + NT * k;
    v[k] = zi[(long)(f / T) * LC + tile * T + f % T];
  }
  d2v acc = {0.0, 0.0};
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int f = threadIdx.x + NT * k;
    if ((f % T) < 4) lds[(f % T) * (LC + LC / 16 + 1) + f / T] = v[k];
    acc += v[k];
  }
  __syncthreads();
  acc += lds[threadIdx.x];
  if (acc.x == -1.0) out[0] = acc;
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
  printf("%-44s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  fflush(stdout);
}

int main() {
  const long items = 64;  // 64 x 16 MiB
  d2v *z, *o;
  CK(hipMalloc(&z, items * LC * LC * 16));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(z, 0x3c, items * LC * LC * 16));
  const double bytes = (double)items * LC * LC * 16;
  for (int xcd = 0; xcd < 2; ++xcd) {
    char nm[64];
    snprintf(nm, 64, "T=2 (32 B) %s", xcd ? "xcd-adjacent" : "plain");
    timeit(nm, [&] { colread<2><<<(unsigned)(LC / 2 * items), NT>>>(z, o, items, xcd); }, bytes);
    snprintf(nm, 64, "T=4 (64 B) %s", xcd ? "xcd-adjacent" : "plain");
    timeit(nm, [&] { colread<4><<<(unsigned)(LC / 4 * items), NT>>>(z, o, items, xcd); }, bytes);
    snprintf(nm, 64, "T=8 (128 B) %s", xcd ? "xcd-adjacent" : "plain");
    timeit(nm, [&] { colread<8><<<(unsigned)(LC / 8 * items), NT>>>(z, o, items, xcd); }, bytes);
    snprintf(nm, 64, "T=16 (256 B) %s", xcd ? "xcd-adjacent" : "plain");
    timeit(nm, [&] { colread<16><<<(unsigned)(LC / 16 * items), NT>>>(z, o, items, xcd); }, bytes);
  }
  return 0;
}
