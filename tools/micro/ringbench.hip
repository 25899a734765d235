// Can a two-pass transform keep its workspace in the 256 MB Infinity Cache?  The CWT's two-pass
// scales write a 4 MB workspace per (signal, scale) pair (pass 1), read it back (pass 2) and write
// 4 MB of coefficients.  Launched as kernels, the write and the read of a workspace line are
// separated by ~300 MB of other traffic and both go to HBM.  Here one launch runs the whole
// chain: workgroups take tickets in dispatch order (atomic counter), ticket -> (role, chunk,
// part) interleaves the producers of chunk k with the consumers of chunk k - LAG, producers of a
// chunk signal a per-chunk counter (release), consumers wait for it (acquire), and the
// workspace is a ring of R chunk slots (a producer also waits until slot k mod R was consumed).
// With R chunks of 4 MB small enough, the ring should stay resident in the Infinity Cache.
//   ringbench RING_CHUNKS LAG [NC [MODE]]   (RING_CHUNKS = 0: no ring, every chunk its own slot)
// Prints the time per chunk and the effective rate over the 12 MB a chunk moves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
constexpr int kThreads = 256;
constexpr long kChunk = 4L << 20;           // bytes per chunk (one pair's workspace)
constexpr int kParts = 64;                  // workgroups per chunk and role
constexpr long kPart = kChunk / kParts;     // 64 KB per workgroup
constexpr int kSpin = 1 << 22;              // bounded waits: every wave exits

__device__ bool wait_geq(unsigned* p, unsigned v, unsigned* err) {
  for (int i = 0; i < kSpin; ++i) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= v) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  atomicAdd(err, 1u);
  return false;
}

__global__ __launch_bounds__(kThreads) void ring(d2v* ws, d2v* out, unsigned* ticket,
                                                 unsigned* produced, unsigned* consumed,
                                                 unsigned* err, int nc, int rchunks, int lag,
                                                 int mode) {
  // mode 0: tickets from an atomic counter; 1: blockIdx as the ticket (in-order dispatch);
  // 2: blockIdx, waits without the release/acquire fences (timing only); 3: no waits at all
  __shared__ unsigned s_t;
  if (mode == 0) {
    if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
  }
  const unsigned t = mode == 0 ? s_t : blockIdx.x;
  // ticket order: step k = [producers of chunk k][consumers of chunk k - lag]
  const unsigned step = t / (2 * kParts), r = t % (2 * kParts);
  const bool prod = r < kParts;
  const int part = r % kParts;
  const long chunk = prod ? (long)step : (long)step - lag;
  if (chunk < 0 || chunk >= nc) return;
  const long slot = rchunks ? chunk % rchunks : chunk;
  d2v* w = ws + (slot * kChunk + part * kPart) / 16;
  if (prod) {
    if (rchunks && chunk >= rchunks && mode < 3) {
      if (threadIdx.x == 0) wait_geq(&consumed[chunk - rchunks], kParts, err);
      __syncthreads();
    }
    for (long i = threadIdx.x; i < kPart / 16; i += kThreads) w[i] = d2v{(double)chunk, (double)i};
    __syncthreads();
    if (threadIdx.x == 0) {
      if (mode < 2) __threadfence();
      atomicAdd(&produced[chunk], 1u);
    }
  } else {
    if (threadIdx.x == 0 && mode < 3) wait_geq(&produced[chunk], kParts, err);
    __syncthreads();
    if (mode < 2) __atomic_thread_fence(__ATOMIC_ACQUIRE);
    d2v* o = out + (chunk * kChunk + part * kPart) / 16;
    for (long i = threadIdx.x; i < kPart / 16; i += kThreads) {
      d2v v = w[i];
      v.x += 1.0;
      __builtin_nontemporal_store(v, o + i);
    }
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&consumed[chunk], 1u);
  }
}

int main(int argc, char** argv) {
  const int rchunks = argc > 1 ? atoi(argv[1]) : 16;
  const int lag = argc > 2 ? atoi(argv[2]) : 2;
  const int nc = argc > 3 ? atoi(argv[3]) : 1536;  // 6 GB of output
  const int mode = argc > 4 ? atoi(argv[4]) : 1;
  const long wsb = (rchunks ? rchunks : nc) * kChunk;
  d2v *ws = nullptr, *out = nullptr;
  unsigned* ctr = nullptr;
  CK(hipMalloc(&ws, wsb));
  CK(hipMalloc(&out, nc * kChunk));
  CK(hipMalloc(&ctr, (2L * nc + 2) * sizeof(unsigned)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned blocks = (unsigned)((long)(nc + lag) * 2 * kParts);
  float best = 1e30f;
  unsigned herr = 0;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipMemset(ctr, 0, (2L * nc + 2) * sizeof(unsigned)));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(ring, dim3(blocks), dim3(kThreads), 0, 0, ws, out, ctr, ctr + 2,
                       ctr + 2 + nc, ctr + 1, nc, rchunks, lag, mode);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
    unsigned e;
    CK(hipMemcpy(&e, ctr + 1, 4, hipMemcpyDeviceToHost));
    herr += e;
  }
  printf("mode %d ring %3d chunks (%5ld MB) lag %d: %8.3f ms for %d chunks = %6.2f us/chunk, "
         "%6.2f TB/s over 12 MB/chunk, %6.2f TB/s output-only, wait timeouts %u\n",
         mode, rchunks, wsb >> 20, lag, best, nc, best * 1e3 / nc, 3.0 * nc * kChunk / (best * 1e-3) / 1e12,
         1.0 * nc * kChunk / (best * 1e-3) / 1e12, herr);
  return 0;
}
