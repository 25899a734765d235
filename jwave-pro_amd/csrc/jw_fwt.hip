// jw_fwt.hip -- Fast Wavelet Transform (filter-bank cascade), 1-D and 2-D, for gfx950.
//
// Reference semantics (src/main/java/jwave/):
//   transforms/wavelets/Wavelet.java:236-260  forward(arr, h): for i < h/2
//       out[i]     = sum_j arr[(2i+j) wrap h] * sD[j]      (j ascending, from +0.0)
//       out[i+h/2] = sum_j arr[(2i+j) wrap h] * wD[j]
//   transforms/wavelets/Wavelet.java:277-303  reverse(arr, h): a SCATTER, i outer, j inner
//       out[(2i+j) wrap h] += (arr[i]*sR[j]) + (arr[i+h/2]*wR[j])
//   haar/Haar1Orthogonal.java:175-207 reverse: out[k] += 0.5 * ((a*sR) + (d*wR))
//   transforms/FastWaveletTransform.java:71-153  the cascade over h = n, n/2, ... (forward)
//       and h = tw << (log2 n - level) ... n (reverse)
//   transforms/BasicTransform.java:361-474  2-D: rows (lvlN) then columns (lvlM); reverse
//       columns then rows.
//
// The reverse scatter is evaluated here as a gather that adds, for each output k, exactly
// the contributions the Java loop adds to out[k], in the Java loop's order (i ascending,
// then j): bit-identical in JW_ARITH_STRICT.  Derivation: for h >= M every (i,j) wraps at
// most once, the j with 2i+j == k (i = (k-j)/2) come first in descending j, then the
// wrapped ones (2i+j == k+h) in descending j.  For h < M (multi-wrap) the Java loop is
// replayed per output.
#include <cstdlib>
#include <utility>

#include "jw_fwt_common.hpp"
#include "jw_internal.hpp"

namespace jw {
namespace {

constexpr int kNT = 256;
constexpr int kLdsN = 4096;              // signals up to this length run one workgroup each
constexpr int kPer = kLdsN / kNT;        // outputs per thread per level (max)

using fwtc::Filters;
using fwtc::madd;
using fwtc::contrib;
using fwtc::rev_acc;

// Wavelet.forward output pair (i, i + h/2) from in[0..h).
template <bool FMA>
__device__ __forceinline__ void fwd_pair(const double* in, int h, int i, int M, const Filters& f,
                                         double& lo, double& hi) {
  lo = 0.;
  hi = 0.;
  for (int j = 0; j < M; ++j) {
    int k = (i << 1) + j;
    while (k >= h) k -= h;
    const double x = in[k];
    lo = madd<FMA>(lo, f.sD[j], x);
    hi = madd<FMA>(hi, f.wD[j], x);
  }
}

// Wavelet.reverse output k from in[0..h) (gather in the scatter's order).
template <bool FMA>
__device__ __forceinline__ double rev_out(const double* in, int h, int k, int M, int kind,
                                          const double* sR, const double* wR) {
  const int half = h >> 1;
  double acc = 0.;
  if (h >= M) {
    const int p = k & 1;
    int jn = k < M - 1 ? k : M - 1;
    if ((jn & 1) != p) --jn;
    for (int j = jn; j >= p; j -= 2) {
      const int i = (k - j) >> 1;
      acc += contrib<FMA>(in[i], in[i + half], sR[j], wR[j], kind);
    }
    int jw = M - 1;
    if ((jw & 1) != p) --jw;
    for (int j = jw; j > k; j -= 2) {
      const int i = (k + h - j) >> 1;
      acc += contrib<FMA>(in[i], in[i + half], sR[j], wR[j], kind);
    }
  } else {
    // multi-wrap (h < M, h a power of two): for each i ascending, the j with
    // (2i + j) mod h == k ascending -- exactly the Java loop's additions, without the scan
    for (int i = 0; i < half; ++i)
      for (int j = (k - (i << 1)) & (h - 1); j < M; j += h)
        acc += contrib<FMA>(in[i], in[i + half], sR[j], wR[j], kind);
  }
  return acc;
}

// One workgroup per signal, whole cascade in LDS (n <= kLdsN).
template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_fwd_lds(const double* __restrict__ x,
                                                   double* __restrict__ y, int n, int level,
                                                   int M, int tw, Filters f) {
  __shared__ double buf[kLdsN];
  const int tid = threadIdx.x;
  const double* xs = x + (long)blockIdx.x * n;
  double* ys = y + (long)blockIdx.x * n;
  for (int i = tid; i < n; i += kNT) buf[i] = xs[i];
  __syncthreads();
  int l = 0;
  for (int h = n; h >= tw && l < level; h >>= 1, ++l) {
    const int half = h >> 1;
    double lo[kPer / 2], hi[kPer / 2];
#pragma unroll
    for (int r = 0; r < kPer / 2; ++r) {
      const int i = tid + r * kNT;
      if (i < half) fwd_pair<FMA>(buf, h, i, M, f, lo[r], hi[r]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPer / 2; ++r) {
      const int i = tid + r * kNT;
      if (i < half) {
        buf[i] = lo[r];
        buf[i + half] = hi[r];
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += kNT) ys[i] = buf[i];
}

template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_rev_lds(const double* __restrict__ y,
                                                   double* __restrict__ x, int n, int h0, int M,
                                                   int tw, int kind, Filters f) {
  __shared__ double buf[kLdsN];
  __shared__ double tsR[kMaxTaps], twR[kMaxTaps];  // taps in LDS: indexed per output below
  const int tid = threadIdx.x;
  const double* ys = y + (long)blockIdx.x * n;
  double* xs = x + (long)blockIdx.x * n;
  for (int i = tid; i < n; i += kNT) buf[i] = ys[i];
  if (tid < M) {
    tsR[tid] = f.sR[tid];
    twR[tid] = f.wR[tid];
  }
  __syncthreads();
  for (int h = h0; h <= n && h >= tw; h <<= 1) {
    double o[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int k = tid + r * kNT;
      if (k < h) o[r] = rev_out<FMA>(buf, h, k, M, kind, tsR, twR);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int k = tid + r * kNT;
      if (k < h) buf[k] = o[r];
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += kNT) xs[i] = buf[i];
}

// ---------------------------------------------------------------------------------------
// Fast LDS cascades for power-of-two n <= 4096 and even M (every orthogonal wavelet):
//  * forward: (2i + j) mod h == (2i + j) & (h - 1); taps read as 16-byte pairs
//    (x[2i+2t], x[2i+2t+1]) -- bank-conflict free, no wrap branch, j ascending as in Java.
//  * reverse: a thread owns outputs (2u, 2u+1); for 2u >= M - 2 every contributing (i, j)
//    has 2i + j = k, i = u - t for tap pairs (j = 2t, 2t+1), and Java's scatter adds them in
//    i ascending = t descending order.  The first outputs (2u < M - 2, or h < M) replay the
//    general wrapped order (rev_out).
// ---------------------------------------------------------------------------------------
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int kNT2 = 256;               // fast LDS cascades: 4 waves per row

// Outputs (2U, 2U+1) of a multi-wrap level h = H < M, H and U compile-time: for each i
// ascending the j with (2i + j) mod H == 2U + p are j = p + 2((U - i) mod H/2) + mH ascending
// (Java's scatter order, M/2 terms per output), so the taps and LDS offsets are constants.
template <bool FMA, int M, int KIND, int H, int U>
__device__ __forceinline__ d2 rev_pair_mw(const double* buf, const Filters& f) {
  constexpr int half = H / 2;
  double acc[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    double a = 0.;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const double av = buf[i], dv = buf[i + half];
      const int s = ((U - i) % half + half) % half;
#pragma unroll
      for (int j = p + 2 * s; j < M; j += H) a += contrib<FMA>(av, dv, f.sR[j], f.wR[j], KIND);
    }
    acc[p] = a;
  }
  return d2{acc[0], acc[1]};
}

// rev_pair_mw for a runtime pair u < H/2: one compile-time block per u (the level's H/2 lanes
// take one each).  The predicated form below evaluated all M taps for every i and made the
// levels h = 2, 4, 8 of the 2-D column tail cost more than its whole memory traffic.
template <bool FMA, int M, int KIND, int H>
__device__ __forceinline__ d2 rev_pair_mw_u(const double* buf, int u, const Filters& f) {
  d2 o = d2{0., 0.};
  [&]<int... Us>(std::integer_sequence<int, Us...>) {
    ((u == Us ? (o = rev_pair_mw<FMA, M, KIND, H, Us>(buf, f), 0) : 0), ...);
  }(std::make_integer_sequence<int, H / 2>{});
  return o;
}

// Outputs (2u, 2u+1) that see wrapped taps, in Java's scatter order (i ascending, then j),
// with compile-time M: fully unrolled, predicated (select, not "+ 0.0") so the sums are
// bit-identical to the reference's.
template <bool FMA, int M, int KIND, bool ENUM = false>
__device__ __forceinline__ d2 rev_pair_wrapped(const double* buf, int h, int u,
                                               const Filters& f, const d2* tp = nullptr) {
  // ENUM (STRICT, runtime h: the line cascades): the multi-wrap terms enumerated, M/2 per
  // output, taps from LDS -- the column tail 789 -> 686 us (profiles/r05/ab/tail_mw); with a
  // compile-time h (the row kernels) the predicated form below folds better
  if constexpr (ENUM && !FMA) {
    if (h < M) {
      const int half = h >> 1;
      double acc[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int k = 2 * u + p;
        double a = 0.;
        for (int i = 0; i < half; ++i) {
          const double av = buf[i], dv = buf[i + half];
          for (int j = (k - (i << 1)) & (h - 1); j < M; j += h) {
            const d2 sr = tp[j & ~1], wr = tp[(j & ~1) + 1];
            a += contrib<FMA>(av, dv, p ? sr.y : sr.x, p ? wr.y : wr.x, KIND);
          }
        }
        acc[p] = a;
      }
      return d2{acc[0], acc[1]};
    }
  }
  // multi-wrap levels h = 2 .. 16 as compile-time blocks; FMA only: in STRICT (separate
  // multiplies, taps as SGPR operands) the blocks pushed the taps into VGPR lanes (~900
  // v_readlane) and the column tail went 0.79 -> 1.3 ms
  if constexpr (FMA && M <= 20) {
    if (h < M) {
      if (h == 2) return rev_pair_mw_u<FMA, M, KIND, 2>(buf, u, f);
      if constexpr (M > 4) if (h == 4) return rev_pair_mw_u<FMA, M, KIND, 4>(buf, u, f);
      if constexpr (M > 8) if (h == 8) return rev_pair_mw_u<FMA, M, KIND, 8>(buf, u, f);
      if constexpr (M > 16) if (h == 16) return rev_pair_mw_u<FMA, M, KIND, 16>(buf, u, f);
    }
  }
  const int half = h >> 1;
  double acc[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int k = 2 * u + p;
    double a = 0.;
    if (h >= M) {
      // non-wrapped j <= k (i = (k - j)/2) by j descending, then wrapped j > k
      // (i = (k + h - j)/2) by j descending
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int t = M / 2 - 1; t >= 0; --t) {
          const int j = 2 * t + p;
          const bool take = pass == 0 ? j <= k : j > k;
          const int i = ((pass == 0 ? k : k + h) - j) >> 1;
          const int ii = take ? i : 0;
          const double c = contrib<FMA>(buf[ii], buf[ii + half], f.sR[j], f.wR[j], KIND);
          a = take ? a + c : a;
        }
      }
    } else {
      // multi-wrap: every (i, j) in Java order with (2i + j) mod h == k
      for (int i = 0; i < half; ++i) {
        const double av = buf[i], dv = buf[i + half];
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const bool take = (((i << 1) + j) & (h - 1)) == k;
          const double c = contrib<FMA>(av, dv, f.sR[j], f.wR[j], KIND);
          a = take ? a + c : a;
        }
      }
    }
    acc[p] = a;
  }
  return d2{acc[0], acc[1]};
}

// Taps of the reverse, in LDS, for the wrapped pairs' lane-dependent tap order:
// tp[2t] = (sR[2t], sR[2t+1]), tp[2t+1] = (wR[2t], wR[2t+1]).  Filled by threads tid < M/2.
template <int M>
__device__ __forceinline__ void fill_rev_taps(d2* tp, int tid, const Filters& f) {
  if (tid < M / 2) {
    tp[2 * tid] = d2{f.sR[2 * tid], f.sR[2 * tid + 1]};
    tp[2 * tid + 1] = d2{f.wR[2 * tid], f.wR[2 * tid + 1]};
  }
}

// Wrapped pair (2u, 2u+1), u < M/2 - 1, h >= M: the same additions as rev_pair_wrapped in
// the same order -- Java's scatter adds i ascending: the unwrapped taps t = u .. 0
// (i = u - t), then the wrapped t = M/2-1 .. u+1 (i = u - t + h/2).  Step s of that order
// is t = (u - s) mod M/2 with i = (u - t) mod h/2, so a uniform 8-step loop replaces the
// predicated 2 x M/2 passes per output (taps from LDS: t is lane-dependent).
template <bool FMA, int M, int KIND>
__device__ __forceinline__ d2 rev_pair_rot(const double* buf, int h, int u, const d2* tp) {
  constexpr int T2 = M / 2;
  const int half = h >> 1;
  // pairs past the wrap (u >= M/2 - 1) start at t = M/2 - 1: the plain descending order, so
  // a whole wave can take this path (cascade_rev)
  const int t0 = u < T2 - 1 ? u : T2 - 1;
  double a0 = 0., a1 = 0.;
#pragma unroll
  for (int st = 0; st < T2; ++st) {
    const int t = t0 - st >= 0 ? t0 - st : t0 - st + T2;
    const int i = u - t >= 0 ? u - t : u - t + half;
    const double av = buf[i], dv = buf[i + half];
    const d2 sr = tp[2 * t], wr = tp[2 * t + 1];
    a0 = rev_acc<FMA, KIND>(a0, av, dv, sr.x, wr.x);
    a1 = rev_acc<FMA, KIND>(a1, av, dv, sr.y, wr.y);
  }
  return d2{a0, a1};
}

// Level barrier of the line cascades: workgroup-wide, or (WS) wave-level when every line's
// threads sit in one wavefront (NTL divides 64), whose DS instructions execute in issue order
// -- a wave-scope fence pair around a wave barrier keeps the compiler from moving LDS accesses
// across it.
#ifndef JW_TAIL_WSYNC  // A/B builds: 0 = workgroup barriers in the column tails too
#define JW_TAIL_WSYNC 1
#endif
template <bool WS>
__device__ __forceinline__ void line_sync() {
  if constexpr (WS) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// The forward cascade on one line held in LDS (buf), by NTL threads (tid < NTL).  The
// barriers are workgroup-wide (every line of the workgroup runs the same levels), or wave-level
// with WS.
template <bool FMA, int M, int NTL, int LEN = kLdsN, bool WS = false>
__device__ __forceinline__ void cascade_fwd(double* buf, int n, int level, int tw, int tid,
                                            const Filters& f) {
  static_assert(!WS || (NTL <= 64 && 64 % NTL == 0), "wave-level syncs: one line per wave part");
  constexpr int P = (LEN / NTL / 2) < 1 ? 1 : LEN / NTL / 2;  // pairs per thread, first level
  int l = 0;
  for (int h = n; h >= tw && h >= 2 && l < level; h >>= 1, ++l) {
    const int half = h >> 1, mask = h - 1;
    double lo[P], hi[P];
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int i = tid + r * NTL;
      lo[r] = 0.;
      hi[r] = 0.;
      if (i < half) {
#pragma unroll
        for (int t = 0; t < (M >> 1); ++t) {
          const d2 v = *(const d2*)&buf[(2 * i + 2 * t) & mask];
          lo[r] = madd<FMA>(lo[r], f.sD[2 * t], v.x);
          hi[r] = madd<FMA>(hi[r], f.wD[2 * t], v.x);
          lo[r] = madd<FMA>(lo[r], f.sD[2 * t + 1], v.y);
          hi[r] = madd<FMA>(hi[r], f.wD[2 * t + 1], v.y);
        }
      }
      if (i + NTL >= half) break;
    }
    line_sync<WS>();
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int i = tid + r * NTL;
      if (i < half) {
        buf[i] = lo[r];
        buf[i + half] = hi[r];
      }
    }
    line_sync<WS>();
  }
}

template <bool FMA, int M>
__global__ __launch_bounds__(kNT2) void fwt_fwd_lds2(const double* __restrict__ x,
                                                    double* __restrict__ y, int n, int level,
                                                    int tw, Filters f) {
  __shared__ __attribute__((aligned(16))) double buf[kLdsN];
  const int tid = threadIdx.x;
  const double* xs = x + (long)blockIdx.x * n;
  double* ys = y + (long)blockIdx.x * n;
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&buf[i] = *(const d2*)&xs[i];
  __syncthreads();
  cascade_fwd<FMA, M, kNT2>(buf, n, level, tw, tid, f);
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&ys[i] = *(const d2*)&buf[i];
}

template <bool FMA, int M, int KIND, int NTL, int LEN = kLdsN, bool WS = false>
__device__ __forceinline__ void cascade_rev(double* buf, int n, int h0, int tw, int tid,
                                            const Filters& f, const d2* tp,
                                            double* gout = nullptr) {
  static_assert(!WS || (NTL <= 64 && 64 % NTL == 0), "wave-level syncs: one line per wave part");
  constexpr int P = (LEN / NTL / 2) < 1 ? 1 : LEN / NTL / 2;
  for (int h = h0; h <= n && h >= tw && h >= 2; h <<= 1) {
    const int half = h >> 1;
    // pairs u < nslow see wrapped taps: all of them when h < M, else the first M/2 - 1; they
    // are all thread tid = u of the first pass (nslow <= 32)
    const int nslow = h < M ? half : (M >> 1) - 1 < half ? (M >> 1) - 1 : half;
    d2 o[P];
    // STRICT: the wave holding the wrapped pairs (u < nslow, all in the first 64 threads'
    // first pass) runs that pass in the rotated order for all its lanes -- one pass with LDS
    // taps instead of the plain pass plus a second one for 7 lanes, which held every barrier.
    // FMA (a tolerance contract, the order is free): every pair, wrapped or not, takes the
    // plain descending tap order with its index taken mod h/2, so no lane is special.
    const bool fma_wrap = FMA && h >= M;
    const bool rot_wave = !fma_wrap && h >= M && NTL >= 64 && (tid >> 6) == 0;
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int u = tid + r * NTL;
      if (r == 0 && rot_wave) {
        if (u < half) o[0] = rev_pair_rot<FMA, M, KIND>(buf, h, u, tp);
      } else if (u < half && (fma_wrap || u >= nslow)) {
        double a0 = 0., a1 = 0.;
#pragma unroll
        for (int t = (M >> 1) - 1; t >= 0; --t) {
          const int i = fma_wrap ? (u - t) & (half - 1) : u - t;
          const double av = buf[i], dv = buf[i + half];
          a0 = rev_acc<FMA, KIND>(a0, av, dv, f.sR[2 * t], f.wR[2 * t]);  // KIND: compile-time
          a1 = rev_acc<FMA, KIND>(a1, av, dv, f.sR[2 * t + 1], f.wR[2 * t + 1]);
        }
        o[r] = d2{a0, a1};
      }
      if (u + NTL >= half) break;
    }
    if (tid < nslow && !rot_wave && !fma_wrap)
      o[0] = h >= M ? rev_pair_rot<FMA, M, KIND>(buf, h, tid, tp)
                    : rev_pair_wrapped<FMA, M, KIND, true>(buf, h, tid, f, tp);
    if (gout && h == n) {
      // last level straight to global memory (lane-consecutive 16-byte stores): no LDS
      // round trip, no barriers; the caller skips its copy-out
#pragma unroll
      for (int r = 0; r < P; ++r) {
        const int u = tid + r * NTL;
        if (u < half) *(d2*)&gout[2 * u] = o[r];
      }
      return;
    }
    line_sync<WS>();
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int u = tid + r * NTL;
      if (u < half) *(d2*)&buf[2 * u] = o[r];
    }
    line_sync<WS>();
  }
}

template <bool FMA, int M, int KIND>
__global__ __launch_bounds__(kNT2) void fwt_rev_lds2(const double* __restrict__ y,
                                                    double* __restrict__ x, int n, int h0, int tw,
                                                    int kind, Filters f) {
  __shared__ __attribute__((aligned(16))) double buf[kLdsN];
  __shared__ d2 tp[M];
  const int tid = threadIdx.x;
  const double* ys = y + (long)blockIdx.x * n;
  double* xs = x + (long)blockIdx.x * n;
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&buf[i] = *(const d2*)&ys[i];
  fill_rev_taps<M>(tp, tid, f);
  __syncthreads();
  // the last level (h = n) stores to xs itself when the cascade reaches it
  const bool to_global = [&] {
    int h = h0;
    while (h < n && h >= tw && h >= 2) h <<= 1;
    return h == n && h >= tw && h >= 2;
  }();
  cascade_rev<FMA, M, KIND, kNT2>(buf, n, h0, tw, tid, f, tp, to_global ? xs : nullptr);
  if (!to_global)
    for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&xs[i] = *(const d2*)&buf[i];
}

// ---------------------------------------------------------------------------------------
// 4096-sample rows (the cfg4 2-D row pass, and 1-D signals of that length): the cascades
// above with every level size a compile-time constant (the levels are unrolled), so each
// thread's LDS reads come off one base address with immediate offsets -- the mask and shift
// per tap pair of the runtime-h loops was ~40 % of their VALU instructions.
//  * forward: the circular wrap (2i + j) mod h is a copy of the level's first M - 2 inputs
//    after its end (buf[h .. h + M - 2)), written by the level before; the details of every
//    level go from registers straight to global memory (they are final), only the
//    approximations return to LDS.
//  * reverse: the wrapped pairs (u < M/2 - 1) all lie in wave 0's first pass; that wave
//    takes the wrapped order (STRICT) or the masked index (FMA), the others plain u - t.
// Same sums in the same order as cascade_fwd / cascade_rev (bit-identical in STRICT).
// ---------------------------------------------------------------------------------------
constexpr int kRowN = 4096;
constexpr int kRowMaxM = 20;  // longer filters keep the runtime-level kernels (compile time)
#ifndef JW_REV_PAIRS2
#define JW_REV_PAIRS2 1
#endif
#ifndef JW_REV_SMALL_WAVE
#define JW_REV_SMALL_WAVE 1
#endif
// row reverse: levels 2 .. 128 on one wave with wave-level syncs (A/B builds: 0)
constexpr bool kRevSmallWave = JW_REV_SMALL_WAVE;
#ifndef JW_FWT_NOROT
#define JW_FWT_NOROT 0  // timing-only A/B builds: STRICT wrapped pairs in the plain order
#endif
constexpr bool kRevPairs2 = JW_REV_PAIRS2;  // row kernels: two outputs per lane (A/B builds: 0)

template <bool FMA, int M, int H>
__device__ __forceinline__ void row_fwd_level(double* buf, double* ys, int tid, const Filters& f) {
  constexpr int half = H / 2, P = half >= kNT2 ? half / kNT2 : 1, PAD = M - 2;
  constexpr bool padded = H >= PAD;  // single wrap, read from the copy after the end
  if constexpr (padded && P >= 2 && kRevPairs2) {
    // two adjacent outputs (2v, 2v + 1) per lane, v = tid + r kNT2: output i reads
    // buf[2i .. 2i + M), so the pair shares M - 2 inputs and the lane loads M/2 + 1 aligned
    // 16-byte pairs instead of M; each sum keeps the one-output order (bit-identical)
    double lo[P], hi[P];
#pragma unroll
    for (int r = 0; r < P / 2; ++r) {
      const int i0 = 2 * (tid + r * kNT2);
      double v[M + 2];
#pragma unroll
      for (int q = 0; q <= M / 2; ++q) {
        const d2 w = *(const d2*)&buf[2 * i0 + 2 * q];
        v[2 * q] = w.x;
        v[2 * q + 1] = w.y;
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        double l = 0., h = 0.;
#pragma unroll
        for (int t = 0; t < (M >> 1); ++t) {
          const double x0 = v[2 * e + 2 * t], x1 = v[2 * e + 2 * t + 1];
          l = madd<FMA>(l, f.sD[2 * t], x0);
          h = madd<FMA>(h, f.wD[2 * t], x0);
          l = madd<FMA>(l, f.sD[2 * t + 1], x1);
          h = madd<FMA>(h, f.wD[2 * t + 1], x1);
        }
        lo[2 * r + e] = l;
        hi[2 * r + e] = h;
      }
    }
    __syncthreads();  // every read of buf[0 .. H + PAD) is done
#pragma unroll
    for (int r = 0; r < P / 2; ++r) {
      const int i0 = 2 * (tid + r * kNT2);
      *(d2*)&buf[i0] = d2{lo[2 * r], lo[2 * r + 1]};
      *(d2*)&ys[half + i0] = d2{hi[2 * r], hi[2 * r + 1]};
    }
    // the next level's wrap copy (its first PAD inputs are this level's lo[0 .. PAD))
    if constexpr (PAD > 0 && half >= PAD) {
      if (2 * tid < PAD) *(d2*)&buf[half + 2 * tid] = d2{lo[0], lo[1]};
    }
    __syncthreads();
    return;
  }
  double lo[P], hi[P];
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const int i = tid + r * kNT2;
    lo[r] = 0.;
    hi[r] = 0.;
    if (half >= kNT2 || i < half) {
#pragma unroll
      for (int t = 0; t < (M >> 1); ++t) {
        const int k = padded ? 2 * i + 2 * t : (2 * i + 2 * t) & (H - 1);
        const d2 v = *(const d2*)&buf[k];
        lo[r] = madd<FMA>(lo[r], f.sD[2 * t], v.x);
        hi[r] = madd<FMA>(hi[r], f.wD[2 * t], v.x);
        lo[r] = madd<FMA>(lo[r], f.sD[2 * t + 1], v.y);
        hi[r] = madd<FMA>(hi[r], f.wD[2 * t + 1], v.y);
      }
    }
  }
  __syncthreads();  // every read of buf[0 .. H + PAD) is done
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const int i = tid + r * kNT2;
    if (half >= kNT2 || i < half) {
      buf[i] = lo[r];
      ys[half + i] = hi[r];
    }
  }
  // the next level's wrap copy (its first PAD inputs are this level's lo[0 .. PAD))
  if constexpr (PAD > 0 && half >= PAD) {
    if (tid < PAD) buf[half + tid] = lo[0];
  }
  __syncthreads();
}

// Levels H, H/2, ... while level and tw allow; returns the length of the part left in buf.
template <bool FMA, int M, int H>
__device__ __forceinline__ int row_fwd_from(double* buf, double* ys, int tid, int level, int tw,
                                            const Filters& f) {
  if constexpr (H < 2) {
    return H;
  } else {
    if (level <= 0 || H < tw) return H;
    row_fwd_level<FMA, M, H>(buf, ys, tid, f);
    return row_fwd_from<FMA, M, H / 2>(buf, ys, tid, level - 1, tw, f);
  }
}

template <bool FMA, int M>
__global__ __launch_bounds__(kNT2) void fwt_fwd_row(const double* x, double* y, int level, int tw,
                                                   Filters f) {
  constexpr int PAD = M - 2;
  __shared__ __attribute__((aligned(16))) double buf[kRowN + PAD + 2];
  const int tid = threadIdx.x;
  const double* xs = x + (long)blockIdx.x * kRowN;
  double* ys = y + (long)blockIdx.x * kRowN;
#pragma unroll
  for (int r = 0; r < kRowN / (2 * kNT2); ++r) {
    const int i = 2 * (tid + r * kNT2);
    *(d2*)&buf[i] = *(const d2*)&xs[i];
  }
  if (PAD > 0 && tid < PAD) buf[kRowN + tid] = xs[tid];
  __syncthreads();
  const int hcur = row_fwd_from<FMA, M, kRowN>(buf, ys, tid, level, tw, f);
  for (int i = tid; i < hcur; i += kNT2) ys[i] = buf[i];
}

// Two adjacent pairs (u, u + 1) of an unwrapped reverse level from one lane: pair u reads
// buf[u - t] and buf[u - t + half] for t < M/2, pair u + 1 the same shifted by one, so the lane
// loads the M/2 + 1 values of each half once, as aligned 16-byte pairs (u even), instead of
// 2 x M/2 eight-byte reads per pair.  Each output's sum runs t = M/2 - 1 .. 0 as in the
// one-pair form (bit-identical).
template <bool FMA, int M, int KIND>
__device__ __forceinline__ void rev_two_pairs(const double* buf, int half, int u, const Filters& f,
                                              d2& o0, d2& o1) {
  constexpr int T2 = M / 2;
  constexpr int LO = (T2 & 1) ? T2 - 1 : T2;  // base u - LO: even, <= u - T2 + 1
  constexpr int NV = (LO + 2) / 2;            // 16-byte pairs covering [u - LO, u + 1]
  double a[2 * NV], d[2 * NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const d2 va = *(const d2*)&buf[u - LO + 2 * q];
    const d2 vd = *(const d2*)&buf[u - LO + 2 * q + half];
    a[2 * q] = va.x;
    a[2 * q + 1] = va.y;
    d[2 * q] = vd.x;
    d[2 * q + 1] = vd.y;
  }
  double a0 = 0., a1 = 0., b0 = 0., b1 = 0.;
#pragma unroll
  for (int t = T2 - 1; t >= 0; --t) {
    const int i = LO - t;  // buf[u - t] at a[LO - t], buf[u + 1 - t] at a[LO - t + 1]
    a0 = rev_acc<FMA, KIND>(a0, a[i], d[i], f.sR[2 * t], f.wR[2 * t]);
    a1 = rev_acc<FMA, KIND>(a1, a[i], d[i], f.sR[2 * t + 1], f.wR[2 * t + 1]);
    b0 = rev_acc<FMA, KIND>(b0, a[i + 1], d[i + 1], f.sR[2 * t], f.wR[2 * t]);
    b1 = rev_acc<FMA, KIND>(b1, a[i + 1], d[i + 1], f.sR[2 * t + 1], f.wR[2 * t + 1]);
  }
  o0 = d2{a0, a1};
  o1 = d2{b0, b1};
}

// Within one wavefront the DS instructions execute in issue order: a wave-scope fence pair
// around a wave barrier keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One reverse level of a 4096-sample row.  WAVE: a level with half <= 64 output pairs run by
// wave 0 alone with wave-level syncs (the caller issues one workgroup barrier after the last
// such level), instead of two workgroup barriers per level.
template <bool FMA, int M, int KIND, int H, bool WAVE = false>
__device__ __forceinline__ void row_rev_level(double* buf, double* xs, int tid, const Filters& f,
                                              const d2* tp) {
  static_assert(!WAVE || H <= 128, "wave-level reverse levels: half <= 64");
  constexpr int half = H / 2, P = half >= kNT2 ? half / kNT2 : 1;
  d2 o[P];
  if constexpr (FMA && H >= M && P >= 2 && kRevPairs2) {
    // lanes take pairs (2v, 2v + 1), v = tid + r kNT2; the wave holding the wrapped pairs
    // (u < M/2 - 1, r = 0, tid < 64) keeps the one-pair forms.  FMA contract only: in STRICT
    // (four FP64 instructions per tap instead of two) the blocked form measured slower, 5.08 ->
    // 5.24 ms per cfg4 reverse, against 3.67 -> 3.37 ms with FMA (profiles/r03/ab_revpairs.log)
#pragma unroll
    for (int r = 0; r < P / 2; ++r) {
      const int u = 2 * (tid + r * kNT2);
      if (r == 0 && tid < 64) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int ue = u + e;
          if constexpr (FMA) {
            double a0 = 0., a1 = 0.;
#pragma unroll
            for (int t = (M >> 1) - 1; t >= 0; --t) {
              const int i = (ue - t) & (half - 1);
              const double av = buf[i], dv = buf[i + half];
              a0 = rev_acc<FMA, KIND>(a0, av, dv, f.sR[2 * t], f.wR[2 * t]);
              a1 = rev_acc<FMA, KIND>(a1, av, dv, f.sR[2 * t + 1], f.wR[2 * t + 1]);
            }
            o[2 * r + e] = d2{a0, a1};
          } else {
            o[2 * r + e] = rev_pair_rot<FMA, M, KIND>(buf, H, ue, tp);
          }
        }
      } else {
        rev_two_pairs<FMA, M, KIND>(buf, half, u, f, o[2 * r], o[2 * r + 1]);
      }
    }
    if constexpr (H == kRowN) {  // last level: straight to global memory
#pragma unroll
      for (int r = 0; r < P / 2; ++r) {
        const int u = 2 * (tid + r * kNT2);
        *(d2*)&xs[2 * u] = o[2 * r];
        *(d2*)&xs[2 * u + 2] = o[2 * r + 1];
      }
      return;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < P / 2; ++r) {
      const int u = 2 * (tid + r * kNT2);
      *(d2*)&buf[2 * u] = o[2 * r];
      *(d2*)&buf[2 * u + 2] = o[2 * r + 1];
    }
    __syncthreads();
    return;
  }
  if constexpr (H < M) {  // multi-wrap: Java's loop replayed per output
    if constexpr (M <= 20) {  // compile-time blocks per pair (rev_pair_mw), STRICT too here
      if (tid < half) o[0] = rev_pair_mw_u<FMA, M, KIND, H>(buf, tid, f);
    } else {
      if (tid < half) o[0] = rev_pair_wrapped<FMA, M, KIND>(buf, H, tid, f);
    }
  } else {
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int u = tid + r * kNT2;
      if (half >= kNT2 || u < half) {
        if (r == 0 && tid < 64) {  // wave-uniform: the wave holding u < M/2 - 1 (<= 19)
          if constexpr (FMA || JW_FWT_NOROT) {  // JW_FWT_NOROT: timing-only builds (wrong order)
            double a0 = 0., a1 = 0.;
#pragma unroll
            for (int t = (M >> 1) - 1; t >= 0; --t) {
              const int i = (u - t) & (half - 1);
              const double av = buf[i], dv = buf[i + half];
              a0 = rev_acc<FMA, KIND>(a0, av, dv, f.sR[2 * t], f.wR[2 * t]);
              a1 = rev_acc<FMA, KIND>(a1, av, dv, f.sR[2 * t + 1], f.wR[2 * t + 1]);
            }
            o[r] = d2{a0, a1};
          } else {
            o[r] = rev_pair_rot<FMA, M, KIND>(buf, H, u, tp);
          }
        } else {
          double a0 = 0., a1 = 0.;
#pragma unroll
          for (int t = (M >> 1) - 1; t >= 0; --t) {
            const double av = buf[u - t], dv = buf[u - t + half];
            a0 = rev_acc<FMA, KIND>(a0, av, dv, f.sR[2 * t], f.wR[2 * t]);
            a1 = rev_acc<FMA, KIND>(a1, av, dv, f.sR[2 * t + 1], f.wR[2 * t + 1]);
          }
          o[r] = d2{a0, a1};
        }
      }
    }
  }
  if constexpr (H == kRowN) {  // last level: straight to global memory
#pragma unroll
    for (int r = 0; r < P; ++r) *(d2*)&xs[2 * (tid + r * kNT2)] = o[r];
    return;
  }
  if constexpr (WAVE) {
    wave_sync();
  } else {
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const int u = tid + r * kNT2;
    if (half >= kNT2 || u < half) *(d2*)&buf[2 * u] = o[r];
  }
  if constexpr (WAVE) {
    wave_sync();
  } else {
    __syncthreads();
  }
}

// Levels H, 2H, .., 128 from h0 on, wave 0 only (WAVE levels)
template <bool FMA, int M, int KIND, int H>
__device__ __forceinline__ void row_rev_small(double* buf, int tid, int h0, const Filters& f,
                                              const d2* tp) {
  if constexpr (H <= 128) {
    if (H >= h0) row_rev_level<FMA, M, KIND, H, true>(buf, nullptr, tid, f, tp);
    row_rev_small<FMA, M, KIND, 2 * H>(buf, tid, h0, f, tp);
  }
}

// Levels H, 2H, ..., kRowN from h0 on (h0 a power of two); true when the last one stored to xs.
template <bool FMA, int M, int KIND, int H>
__device__ __forceinline__ bool row_rev_from(double* buf, double* xs, int tid, int h0,
                                             const Filters& f, const d2* tp) {
  if constexpr (H > kRowN) {
    return false;
  } else {
    if (H >= h0) {
      row_rev_level<FMA, M, KIND, H>(buf, xs, tid, f, tp);
      if constexpr (H == kRowN) return true;
    }
    return row_rev_from<FMA, M, KIND, 2 * H>(buf, xs, tid, h0, f, tp);
  }
}

template <bool FMA, int M, int KIND>
__global__ __launch_bounds__(kNT2) void fwt_rev_row(const double* y, double* x, int h0, int tw,
                                                   Filters f) {
  __shared__ __attribute__((aligned(16))) double buf[kRowN];
  __shared__ d2 tp[M];
  const int tid = threadIdx.x;
  const double* ys = y + (long)blockIdx.x * kRowN;
  double* xs = x + (long)blockIdx.x * kRowN;
#pragma unroll
  for (int r = 0; r < kRowN / (2 * kNT2); ++r) {
    const int i = 2 * (tid + r * kNT2);
    *(d2*)&buf[i] = *(const d2*)&ys[i];
  }
  // fill_rev_taps with compile-time tap indices: a thread-indexed read of the kernel-argument
  // filters made the compiler copy all 2 KB of them to scratch and read every tap from there
#pragma unroll
  for (int t = 0; t < M / 2; ++t) {
    if (tid == t) {
      tp[2 * t] = d2{f.sR[2 * t], f.sR[2 * t + 1]};
      tp[2 * t + 1] = d2{f.wR[2 * t], f.wR[2 * t + 1]};
    }
  }
  __syncthreads();
  // cascade_rev's loop: h = h0, 2 h0, ... while h <= n, h >= tw, h >= 2 (h0 >= tw here)
  const bool run = h0 >= tw && h0 >= 2 && h0 <= kRowN;
  bool stored = false;
  if (run) {
    if (kRevSmallWave) {  // levels 2 .. 128 by wave 0, then one workgroup barrier
      if (h0 <= 128) {
        if (tid < 64) row_rev_small<FMA, M, KIND, 2>(buf, tid, h0, f, tp);
        __syncthreads();
      }
      stored = row_rev_from<FMA, M, KIND, 256>(buf, xs, tid, h0, f, tp);
    } else {
      stored = row_rev_from<FMA, M, KIND, 2>(buf, xs, tid, h0, f, tp);
    }
  }
  if (!stored)
    for (int i = 2 * tid; i < kRowN; i += 2 * kNT2) *(d2*)&xs[i] = *(const d2*)&buf[i];
}

// ---------------------------------------------------------------------------------------
// Wavelet packet transform (WaveletPacketTransform.java:60-191): every level applies
// Wavelet.forward / reverse to each of the n/h packets of length h, not just the first.
// Same per-packet arithmetic as the FWT cascades above (bit-identical in STRICT).
// ---------------------------------------------------------------------------------------
template <bool FMA, int M>
__global__ __launch_bounds__(kNT2) void wpt_fwd_lds(const double* __restrict__ x,
                                                   double* __restrict__ y, int n, int level, int tw,
                                                   Filters f) {
  __shared__ __attribute__((aligned(16))) double buf[kLdsN];
  constexpr int P = kLdsN / kNT2 / 2;
  const int tid = threadIdx.x;
  const double* xs = x + (long)blockIdx.x * n;
  double* ys = y + (long)blockIdx.x * n;
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&buf[i] = *(const d2*)&xs[i];
  __syncthreads();
  const int npairs = n >> 1;
  int l = 0;
  for (int h = n; h >= tw && h >= 2 && l < level; h >>= 1, ++l) {
    const int half = h >> 1, mask = h - 1, lh = 31 - __builtin_clz(half);
    double lo[P], hi[P];
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int q = tid + r * kNT2;
      lo[r] = 0.;
      hi[r] = 0.;
      if (q < npairs) {
        const int base = (q >> lh) * h, i = q & (half - 1);
#pragma unroll
        for (int t = 0; t < (M >> 1); ++t) {
          const d2 v = *(const d2*)&buf[base + ((2 * i + 2 * t) & mask)];
          lo[r] = madd<FMA>(lo[r], f.sD[2 * t], v.x);
          hi[r] = madd<FMA>(hi[r], f.wD[2 * t], v.x);
          lo[r] = madd<FMA>(lo[r], f.sD[2 * t + 1], v.y);
          hi[r] = madd<FMA>(hi[r], f.wD[2 * t + 1], v.y);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int q = tid + r * kNT2;
      if (q < npairs) {
        const int base = (q >> lh) * h, i = q & (half - 1);
        buf[base + i] = lo[r];
        buf[base + i + half] = hi[r];
      }
    }
    __syncthreads();
  }
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&ys[i] = *(const d2*)&buf[i];
}

template <bool FMA, int M, int KIND>
__global__ __launch_bounds__(kNT2) void wpt_rev_lds(const double* __restrict__ y,
                                                   double* __restrict__ x, int n, int h0, int tw,
                                                   Filters f) {
  __shared__ __attribute__((aligned(16))) double buf[kLdsN];
  __shared__ d2 tp[M];
  constexpr int P = kLdsN / kNT2 / 2;
  const int tid = threadIdx.x;
  const double* ys = y + (long)blockIdx.x * n;
  double* xs = x + (long)blockIdx.x * n;
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&buf[i] = *(const d2*)&ys[i];
  fill_rev_taps<M>(tp, tid, f);
  __syncthreads();
  const int npairs = n >> 1;
  for (int h = h0; h <= n && h >= tw && h >= 2; h <<= 1) {
    const int half = h >> 1, lh = 31 - __builtin_clz(half);
    const int nslow = h < M ? half : (M >> 1) - 1 < half ? (M >> 1) - 1 : half;
    d2 o[P];
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int q = tid + r * kNT2;
      if (q < npairs) {
        const int base = (q >> lh) * h, u = q & (half - 1);
        if (u >= nslow) {
          double a0 = 0., a1 = 0.;
#pragma unroll
          for (int t = (M >> 1) - 1; t >= 0; --t) {
            const double av = buf[base + u - t], dv = buf[base + u - t + half];
            a0 = rev_acc<FMA, KIND>(a0, av, dv, f.sR[2 * t], f.wR[2 * t]);
            a1 = rev_acc<FMA, KIND>(a1, av, dv, f.sR[2 * t + 1], f.wR[2 * t + 1]);
          }
          o[r] = d2{a0, a1};
        } else {
          o[r] = h >= M ? rev_pair_rot<FMA, M, KIND>(buf + base, h, u, tp)
                        : rev_pair_wrapped<FMA, M, KIND>(buf + base, h, u, f);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int q = tid + r * kNT2;
      if (q < npairs) {
        const int base = (q >> lh) * h, u = q & (half - 1);
        *(d2*)&buf[base + 2 * u] = o[r];
      }
    }
    __syncthreads();
  }
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&xs[i] = *(const d2*)&buf[i];
}

// One WPT level on global memory (any M, any power-of-two n): out-of-place.
template <bool FMA>
__global__ __launch_bounds__(kNT) void wpt_fwd_level(const double* __restrict__ in,
                                                     double* __restrict__ out, long n, int h, int M,
                                                     Filters f) {
  const long q = (long)blockIdx.x * kNT + threadIdx.x;
  if (q >= (n >> 1)) return;
  const int half = h >> 1;
  const long base = (q / half) * h;
  const int i = (int)(q % half);
  const double* src = in + (long)blockIdx.y * n + base;
  double* dst = out + (long)blockIdx.y * n + base;
  double lo, hi;
  fwd_pair<FMA>(src, h, i, M, f, lo, hi);
  dst[i] = lo;
  dst[i + half] = hi;
}

template <bool FMA>
__global__ __launch_bounds__(kNT) void wpt_rev_level(const double* __restrict__ in,
                                                     double* __restrict__ out, long n, int h, int M,
                                                     int kind, Filters f) {
  const long k = (long)blockIdx.x * kNT + threadIdx.x;
  if (k >= n) return;
  const long base = (k / h) * h;
  out[(long)blockIdx.y * n + k] =
      rev_out<FMA>(in + (long)blockIdx.y * n + base, h, (int)(k - base), M, kind, f.sR, f.wR);
}

// ---------------------------------------------------------------------------------------
// 2-D passes with the transpose fused in: a workgroup (1024 threads) transforms 4 lines of
// one matrix at once, one 256-thread group per line.  READ_T: the lines are columns of the
// [len][nlines] input (read as 4 consecutive doubles per row); WRITE_T: line i is written as
// column i of the [len][nlines] output.  The 32-byte pieces of neighbouring workgroups fill
// whole 128-byte lines in L2 because consecutive tiles go to the same XCD (tile remap below).
// ---------------------------------------------------------------------------------------
constexpr int kLines = 4;
constexpr int kLinePad = kLdsN + 4;  // row stride in LDS: the 4 lines hit different banks

template <bool FMA, int M, bool REV, int KIND, bool READ_T, bool WRITE_T, int NL>
__global__ __launch_bounds__(NL * 256) void fwt_lines4(const double* in,
                                                           double* out, int len,
                                                           int nlines, int lvl_h0, int tw,
                                                           long tiles, Filters f) {
  __shared__ __attribute__((aligned(16))) double bufs[NL * kLinePad];
  __shared__ d2 tp[M];
  const int tid = threadIdx.x, g = tid >> 8, lt = tid & 255;
  if (REV) fill_rev_taps<M>(tp, tid, f);
  // XCD-aware tile order: workgroup b runs on XCD b % 8; give each XCD a contiguous range
  const long b = blockIdx.x;
  const long tile = (tiles % 8 == 0) ? (b % 8) * (tiles / 8) + b / 8 : b;
  const long per_mat = nlines / NL;
  const long mat = tile / per_mat;
  const int line0 = (int)(tile - mat * per_mat) * NL;
  const double* src = in + mat * (long)len * nlines;
  double* dst = out + mat * (long)len * nlines;
  double* buf = bufs + g * kLinePad;
  if (READ_T) {
    for (int k = tid; k < len * NL; k += NL * 256) {
      const int i = k / NL, c = k % NL;
      bufs[c * kLinePad + i] = src[(long)i * nlines + line0 + c];
    }
  } else {
    const double* row = src + (long)(line0 + g) * len;
    for (int i = 2 * lt; i < len; i += 512) *(d2*)&buf[i] = *(const d2*)&row[i];
  }
  __syncthreads();
  if (REV) {
    cascade_rev<FMA, M, KIND, 256>(buf, len, lvl_h0, tw, lt, f, tp);
  } else {
    cascade_fwd<FMA, M, 256>(buf, len, lvl_h0, tw, lt, f);
  }
  if (WRITE_T) {
    for (int k = tid; k < len * NL; k += NL * 256) {
      const int i = k / NL, c = k % NL;
      dst[(long)i * nlines + line0 + c] = bufs[c * kLinePad + i];
    }
  } else {
    double* row = dst + (long)(line0 + g) * len;
    for (int i = 2 * lt; i < len; i += 512) *(d2*)&row[i] = *(const d2*)&buf[i];
  }
}

// ---------------------------------------------------------------------------------------
// 2-D column pass for tall matrices (rows > the tail length): the first S levels of every
// column run as "strip" kernels that work on whole row segments -- a workgroup owns kSW = 64
// columns (512-byte row pieces, fully coalesced) and kST output rows of one level, staged
// through LDS -- and the remaining levels run on the top rows >> S rows with the LDS
// cascade, kTailNL columns per workgroup (fwt_cols_tail).  Same sums, same order as
// Wavelet.forward/reverse per column (bit-identical in STRICT).
// ---------------------------------------------------------------------------------------
constexpr int kSW = 64;      // columns per strip workgroup (32 lanes x 2 columns)
constexpr int kST = 32;      // output rows per strip workgroup
constexpr int kTailNL = 16;  // columns per tail workgroup (128-byte row pieces)
constexpr int kTailLen = 256;
constexpr int kTailNT = 512; // threads per tail workgroup (32 per column): 1024 held one per CU

struct Strip {  // one level's buffers, each [rows][cols] per matrix with its own matrix stride
  const double* src;  // forward: level input rows [0, h); reverse: approximations rows [0, h/2)
  const double* srcd; // reverse: details rows [0, h/2)
  double* dsta;       // forward: approximations rows [0, h/2); reverse: output rows [0, h)
  double* dstd;       // forward: details rows [0, h/2)
  long ms_src, ms_srcd, ms_dsta, ms_dstd;
  int cols, h;
};

// Forward level on rows [0, h) of every column: approximation row i -> dsta, detail -> dstd.
template <bool FMA, int M>
__global__ __launch_bounds__(256) void fwt_strip_fwd(Strip s, Filters f) {
  constexpr int NR = 2 * kST + M - 2;  // input rows of one strip
  __shared__ __attribute__((aligned(16))) double tile[NR * kSW];
  const int tid = threadIdx.x, cp = tid & 31, rl = tid >> 5;
  const int nchunk = s.cols / kSW;
  const int chunk = blockIdx.x % nchunk, strip = blockIdx.x / nchunk;
  const long mat = blockIdx.y;
  const int c0 = chunk * kSW, i0 = strip * kST, mask = s.h - 1;
  const double* src = s.src + mat * s.ms_src + c0;
  for (int r = rl; r < NR; r += 8) {
    const int row = (2 * i0 + r) & mask;  // (2i + j) mod h, h a power of two
    *(d2*)&tile[r * kSW + 2 * cp] = *(const d2*)&src[(long)row * s.cols + 2 * cp];
  }
  __syncthreads();
  double* da = s.dsta + mat * s.ms_dsta + c0 + 2 * cp;
  double* dd = s.dstd + mat * s.ms_dstd + c0 + 2 * cp;
#pragma unroll
  for (int q = 0; q < kST / 8; ++q) {
    const int i = rl + 8 * q;
    double l0 = 0., l1 = 0., h0 = 0., h1 = 0.;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const d2 v = *(const d2*)&tile[(2 * i + j) * kSW + 2 * cp];
      l0 = madd<FMA>(l0, f.sD[j], v.x);
      h0 = madd<FMA>(h0, f.wD[j], v.x);
      l1 = madd<FMA>(l1, f.sD[j], v.y);
      h1 = madd<FMA>(h1, f.wD[j], v.y);
    }
    *(d2*)&da[(long)(i0 + i) * s.cols] = d2{l0, l1};
    *(d2*)&dd[(long)(i0 + i) * s.cols] = d2{h0, h1};
  }
}

// Reverse level: output rows [0, h) from approximations a and details d (rows [0, h/2) each),
// Wavelet.reverse's scatter gathered per output in the scatter's order: output pair
// (2u, 2u+1) adds the taps t (i = u - t mod h/2) by t descending, except that the outputs
// whose taps wrap (u < M/2 - 1) add the unwrapped i first, i ascending, then the wrapped i
// (near h/2), i ascending: t = u, ..., 0, M/2 - 1, ..., u + 1.  Needs h/2 >= M.
template <bool FMA, int M, int KIND>
__global__ __launch_bounds__(256) void fwt_strip_rev(Strip s, Filters f) {
  constexpr int T2 = M / 2;
  constexpr int NI = kST / 2 + T2 - 1;  // a/d rows of one strip
  __shared__ __attribute__((aligned(16))) double ta[NI * kSW], td[NI * kSW];
  __shared__ d2 tp[M];
  const int tid = threadIdx.x, cp = tid & 31, rl = tid >> 5;
  fill_rev_taps<M>(tp, tid, f);
  const int nchunk = s.cols / kSW;
  const int chunk = blockIdx.x % nchunk, strip = blockIdx.x / nchunk;
  const long mat = blockIdx.y;
  const int c0 = chunk * kSW, k0 = strip * kST, half = s.h >> 1;
  const int ibase = k0 / 2 - (T2 - 1);  // tile row r holds i = ibase + r (mod h/2)
  const double* sa = s.src + mat * s.ms_src + c0;
  const double* sd = s.srcd + mat * s.ms_srcd + c0;
  for (int r = rl; r < NI; r += 8) {
    const int row = (ibase + r) & (half - 1);
    *(d2*)&ta[r * kSW + 2 * cp] = *(const d2*)&sa[(long)row * s.cols + 2 * cp];
    *(d2*)&td[r * kSW + 2 * cp] = *(const d2*)&sd[(long)row * s.cols + 2 * cp];
  }
  __syncthreads();
  double* dst = s.dsta + mat * s.ms_dsta + c0 + 2 * cp;
  // Strips past the first (k0/2 >= kST/2 >= T2 - 1) never wrap: compile-time taps t
  // descending.  The first strip takes the rotated order (tstart = u there) with LDS taps.
  const bool first = k0 / 2 < T2 - 1;
#pragma unroll
  for (int q = 0; q < kST / 16; ++q) {
    const int ul = rl + 8 * q;  // local output pair: rows k0 + 2ul, k0 + 2ul + 1
    const int u = k0 / 2 + ul;
    double e0 = 0., e1 = 0., o0 = 0., o1 = 0.;  // (even, odd row) x (column 0, column 1)
    auto tap = [&](int t, double sr0, double wr0, double sr1, double wr1) {
      const int r = ul + (T2 - 1) - t;  // tile row of i = u - t
      const d2 av = *(const d2*)&ta[r * kSW + 2 * cp];
      const d2 dv = *(const d2*)&td[r * kSW + 2 * cp];
      e0 = rev_acc<FMA, KIND>(e0, av.x, dv.x, sr0, wr0);
      e1 = rev_acc<FMA, KIND>(e1, av.y, dv.y, sr0, wr0);
      o0 = rev_acc<FMA, KIND>(o0, av.x, dv.x, sr1, wr1);
      o1 = rev_acc<FMA, KIND>(o1, av.y, dv.y, sr1, wr1);
    };
    if (!first) {
#pragma unroll
      for (int t = T2 - 1; t >= 0; --t) tap(t, f.sR[2 * t], f.wR[2 * t], f.sR[2 * t + 1], f.wR[2 * t + 1]);
    } else {
      const int tstart = u >= T2 - 1 ? T2 - 1 : u;
#pragma unroll
      for (int tt = 0; tt < T2; ++tt) {
        int t = tstart - tt;
        t = t < 0 ? t + T2 : t;
        const d2 sr = tp[2 * t], wr = tp[2 * t + 1];
        tap(t, sr.x, wr.x, sr.y, wr.y);
      }
    }
    *(d2*)&dst[(long)(k0 + 2 * ul) * s.cols] = d2{e0, e1};
    *(d2*)&dst[(long)(k0 + 2 * ul + 1) * s.cols] = d2{o0, o1};
  }
}

// The remaining levels of kTailNL columns on rows [0, len) (len <= kTailLen), in LDS:
// forward levels lvl_h0 = level count from h = len; reverse from h = lvl_h0 up to len.
template <bool FMA, int M, bool REV, int KIND>
__global__ __launch_bounds__(kTailNT) void fwt_cols_tail(const double* in, double* out, int len,
                                                      int cols, long ms_in, long ms_out,
                                                      int lvl_h0, int tw, Filters f) {
  constexpr int NTL = kTailNT / kTailNL;
  constexpr int PAD = kTailLen + 2;  // 16-byte aligned lines; the transposed stores spread banks
  __shared__ __attribute__((aligned(16))) double bufs[kTailNL * PAD];
  __shared__ d2 tp[M];
  const int tid = threadIdx.x, g = tid / NTL, lt = tid % NTL;
  if (REV) fill_rev_taps<M>(tp, tid, f);
  const int nchunk = cols / kTailNL;
  const long mat = blockIdx.x / nchunk;
  const int line0 = (int)(blockIdx.x % nchunk) * kTailNL;
  const double* src = in + mat * ms_in + line0;
  double* dst = out + mat * ms_out + line0;
  // every load issued before the first LDS write (a load-then-store loop waited out one HBM
  // latency per row piece: fwt_cols_tail ran at 1.7-3.0 TB/s)
  constexpr int KL = kTailLen * kTailNL / kTailNT;
  double v[KL];
#pragma unroll
  for (int q = 0; q < KL; ++q) {
    const int k = tid + q * kTailNT, i = k / kTailNL, c = k % kTailNL;
    v[q] = i < len ? src[(long)i * cols + c] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < KL; ++q) {
    const int k = tid + q * kTailNT, i = k / kTailNL, c = k % kTailNL;
    if (i < len) bufs[c * PAD + i] = v[q];
  }
  __syncthreads();
  double* buf = bufs + g * PAD;
  // each column's NTL = 32 threads are half a wavefront: its levels sync at wave level, and
  // only the loads and stores across columns take workgroup barriers (cfg4 -0.5..-1 %,
  // profiles/r04/ab/fwt_tail_wsync_j.log)
  constexpr bool WS = JW_TAIL_WSYNC != 0;
  if (REV) {
    cascade_rev<FMA, M, KIND, NTL, kTailLen, WS>(buf, len, lvl_h0, tw, lt, f, tp);
  } else {
    cascade_fwd<FMA, M, NTL, kTailLen, WS>(buf, len, lvl_h0, tw, lt, f);
  }
  if (WS) __syncthreads();  // the stores below read other waves' columns
#pragma unroll
  for (int q = 0; q < KL; ++q) {
    const int k = tid + q * kTailNT, i = k / kTailNL, c = k % kTailNL;
    v[q] = i < len ? bufs[c * PAD + i] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < KL; ++q) {
    const int k = tid + q * kTailNT, i = k / kTailNL, c = k % kTailNL;
    if (i < len) dst[(long)i * cols + c] = v[q];
  }
}

// One level on global memory (long signals): out[0..h) of every signal from in[0..h).
template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_fwd_level(const double* __restrict__ in,
                                                     double* __restrict__ out, long stride, int h,
                                                     int M, Filters f) {
  const int i = blockIdx.x * kNT + threadIdx.x;
  if (i >= (h >> 1)) return;
  const double* src = in + (long)blockIdx.y * stride;
  double* dst = out + (long)blockIdx.y * stride;
  double lo, hi;
  fwd_pair<FMA>(src, h, i, M, f, lo, hi);
  dst[i] = lo;
  dst[i + (h >> 1)] = hi;
}

template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_rev_level(const double* __restrict__ in,
                                                     double* __restrict__ out, long stride, int h,
                                                     int M, int kind, Filters f) {
  const int k = blockIdx.x * kNT + threadIdx.x;
  if (k >= h) return;
  out[(long)blockIdx.y * stride + k] =
      rev_out<FMA>(in + (long)blockIdx.y * stride, h, k, M, kind, f.sR, f.wR);
}

// Tiled out-of-place transpose of `batch` rows x cols matrices (the 2-D column pass runs as
// transpose -> row cascade -> transpose).
__global__ __launch_bounds__(kNT) void transpose_kernel(const double* __restrict__ in,
                                                        double* __restrict__ out, int rows,
                                                        int cols) {
  __shared__ double tile[32][33];
  const long mat = (long)blockIdx.z * rows * cols;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int rr = r0 + r, cc = c0 + tx;
    if (rr < rows && cc < cols) tile[r][tx] = in[mat + (long)rr * cols + cc];
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int cc = c0 + r, rr = r0 + tx;
    if (cc < cols && rr < rows) out[mat + (long)cc * rows + rr] = tile[tx][r];
  }
}

// Even filter lengths with a compiled fast kernel; others use fwt_fwd_lds / fwt_rev_lds.
#ifndef JW_FWT_LENGTHS  // (a one-length build for ISA inspection: -D'JW_FWT_LENGTHS(X)=X(16)')
#define JW_FWT_LENGTHS(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22) X(24) \
  X(26) X(28) X(30) X(32) X(34) X(36) X(38) X(40)
#endif

// 4096-sample rows use fwt_fwd_row / fwt_rev_row; env JW_FWT_ROW=0 keeps the runtime-level
// cascades (A/B runs, tests).
bool row_kernels() {
  const char* e = knob("JW_FWT_ROW");
  return !(e && e[0] == '0');
}

template <bool FMA>
bool launch_fwd2(int M, dim3 g, hipStream_t s, const double* x, double* y, int n, int level,
                 int tw, const Filters& f) {
  const bool row = n == kRowN && row_kernels();
  switch (M) {
#define JW_C(MM)                                                                          \
  case MM:                                                                                \
    if constexpr (MM <= kRowMaxM) {                                                       \
      if (row) {                                                                          \
        hipLaunchKernelGGL((fwt_fwd_row<FMA, MM>), g, dim3(kNT2), 0, s, x, y, level, tw, f); \
        return true;                                                                      \
      }                                                                                   \
    }                                                                                     \
    hipLaunchKernelGGL((fwt_fwd_lds2<FMA, MM>), g, dim3(kNT2), 0, s, x, y, n, level, tw, f); \
    return true;
    JW_FWT_LENGTHS(JW_C)
#undef JW_C
    default:
      return false;
  }
}

template <bool FMA>
bool launch_rev2(int M, dim3 g, hipStream_t s, const double* y, double* x, int n, int h0, int tw,
                 int kind, const Filters& f) {
  // the compile-time-level row kernel runs levels h0, 2 h0, ..., n: h0 a power of two
  const bool row = n == kRowN && (h0 & (h0 - 1)) == 0 && row_kernels();
  switch (M) {
#define JW_C(MM)                                                                           \
  case MM:                                                                                 \
    if constexpr (MM <= kRowMaxM) {                                                        \
      if (row) {                                                                           \
        if (kind == JW_WAVELET_HAAR_ORTH)                                                  \
          hipLaunchKernelGGL((fwt_rev_row<FMA, MM, JW_WAVELET_HAAR_ORTH>), g, dim3(kNT2), 0, s, \
                             y, x, h0, tw, f);                                             \
        else                                                                               \
          hipLaunchKernelGGL((fwt_rev_row<FMA, MM, JW_WAVELET_GENERIC>), g, dim3(kNT2), 0, s, \
                             y, x, h0, tw, f);                                             \
        return true;                                                                       \
      }                                                                                    \
    }                                                                                      \
    if (kind == JW_WAVELET_HAAR_ORTH)                                                      \
      hipLaunchKernelGGL((fwt_rev_lds2<FMA, MM, JW_WAVELET_HAAR_ORTH>), g, dim3(kNT2), 0, s, y, \
                         x, n, h0, tw, kind, f);                                           \
    else                                                                                   \
      hipLaunchKernelGGL((fwt_rev_lds2<FMA, MM, JW_WAVELET_GENERIC>), g, dim3(kNT2), 0, s, y,  \
                         x, n, h0, tw, kind, f);                                           \
    return true;
    JW_FWT_LENGTHS(JW_C)
#undef JW_C
    default:
      return false;
  }
}

// Column pass of a 2-D transform in place (no transposes): lines = columns of each
// [rows][cols] matrix.  Returns false if (M, shape) has no fused kernel.
template <bool FMA, int NL>
bool launch_cols_nl(int M, int kind, bool rev, hipStream_t s, const double* in, double* out,
                    int rows, int cols, int lvl_h0, int tw, int batch, const Filters& f) {
  if (rows > kLdsN || cols % NL != 0) return false;
  const long tiles = (long)batch * (cols / NL);
  const dim3 g((unsigned)tiles), b(NL * 256);
  switch (M) {
#define JW_C(MM)                                                                                 \
  case MM:                                                                                       \
    if (!rev)                                                                                    \
      hipLaunchKernelGGL((fwt_lines4<FMA, MM, false, 0, true, true, NL>), g, b, 0, s, in, out,    \
                         rows, cols, lvl_h0, tw, tiles, f);                                       \
    else if (kind == JW_WAVELET_HAAR_ORTH)                                                        \
      hipLaunchKernelGGL((fwt_lines4<FMA, MM, true, JW_WAVELET_HAAR_ORTH, true, true, NL>), g, b, \
                         0, s, in, out, rows, cols, lvl_h0, tw, tiles, f);                        \
    else                                                                                         \
      hipLaunchKernelGGL((fwt_lines4<FMA, MM, true, JW_WAVELET_GENERIC, true, true, NL>), g, b, 0, \
                         s, in, out, rows, cols, lvl_h0, tw, tiles, f);                           \
    return true;
    JW_FWT_LENGTHS(JW_C)
#undef JW_C
    default:
      return false;
  }
}

// Columns per workgroup: measured best 4 for the forward, 2 for the reverse (its cascade
// needs more registers and barriers per level); env JW_FWT_LINES = 2 | 4 overrides.
template <bool FMA>
bool launch_cols(int M, int kind, bool rev, hipStream_t s, const double* in, double* out, int rows,
                 int cols, int lvl_h0, int tw, int batch, const Filters& f) {
  const char* e = knob("JW_FWT_LINES");
  if (e ? e[0] == '2' : rev)
    return launch_cols_nl<FMA, 2>(M, kind, rev, s, in, out, rows, cols, lvl_h0, tw, batch, f);
  return launch_cols_nl<FMA, 4>(M, kind, rev, s, in, out, rows, cols, lvl_h0, tw, batch, f);
}

// Strip / tail column kernels (filter lengths with compiled instances).
#define JW_STRIP_LENGTHS(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20)

template <bool FMA>
bool launch_strip(int M, int kind, bool rev, hipStream_t s, const Strip& st, int batch,
                  const Filters& f) {
  const int rows_out = rev ? st.h : st.h / 2;  // output rows of the level (per kind of output)
  const dim3 g((unsigned)((st.cols / kSW) * (rows_out / kST)), (unsigned)batch), b(256);
  switch (M) {
#define JW_C(MM)                                                                              \
  case MM:                                                                                    \
    if (!rev)                                                                                 \
      hipLaunchKernelGGL((fwt_strip_fwd<FMA, MM>), g, b, 0, s, st, f);                        \
    else if (kind == JW_WAVELET_HAAR_ORTH)                                                    \
      hipLaunchKernelGGL((fwt_strip_rev<FMA, MM, JW_WAVELET_HAAR_ORTH>), g, b, 0, s, st, f);  \
    else                                                                                      \
      hipLaunchKernelGGL((fwt_strip_rev<FMA, MM, JW_WAVELET_GENERIC>), g, b, 0, s, st, f);    \
    return true;
    JW_STRIP_LENGTHS(JW_C)
#undef JW_C
    default:
      return false;
  }
}

template <bool FMA>
bool launch_tail(int M, int kind, bool rev, hipStream_t s, const double* in, double* out, int len,
                 int cols, long ms_in, long ms_out, int lvl_h0, int tw, int batch,
                 const Filters& f) {
  const dim3 g((unsigned)((long)batch * (cols / kTailNL))), b(kTailNT);
  switch (M) {
#define JW_C(MM)                                                                                \
  case MM:                                                                                      \
    if (!rev)                                                                                   \
      hipLaunchKernelGGL((fwt_cols_tail<FMA, MM, false, 0>), g, b, 0, s, in, out, len, cols,     \
                         ms_in, ms_out, lvl_h0, tw, f);                                         \
    else if (kind == JW_WAVELET_HAAR_ORTH)                                                      \
      hipLaunchKernelGGL((fwt_cols_tail<FMA, MM, true, JW_WAVELET_HAAR_ORTH>), g, b, 0, s, in,   \
                         out, len, cols, ms_in, ms_out, lvl_h0, tw, f);                         \
    else                                                                                        \
      hipLaunchKernelGGL((fwt_cols_tail<FMA, MM, true, JW_WAVELET_GENERIC>), g, b, 0, s, in, out, \
                         len, cols, ms_in, ms_out, lvl_h0, tw, f);                              \
    return true;
    JW_STRIP_LENGTHS(JW_C)
#undef JW_C
    default:
      return false;
  }
}

Filters make_filters(const FwtPlan& p) {
  Filters f{};
  for (int i = 0; i < p.M; ++i) {
    f.sD[i] = p.sD[i];
    f.wD[i] = p.wD[i];
    f.sR[i] = p.sR[i];
    f.wR[i] = p.wR[i];
  }
  return f;
}

int log2_exact(long n) {
  int e = 0;
  while ((1L << e) < n) ++e;
  return e;
}

template <bool FMA>
int forward_t(const FwtPlan& p, const double* x, double* y, long n, int level, long batch,
              hipStream_t s) {
  const Filters f = make_filters(p);
  if (n <= kLdsN) {
    const bool fast = p.M % 2 == 0 && n >= 2 && !knob("JW_FWT_GENERIC");
    for (long b0 = 0; b0 < batch; b0 += 1L << 30) {
      const long nb = batch - b0 < (1L << 30) ? batch - b0 : (1L << 30);
      if (!fast || !launch_fwd2<FMA>(p.M, dim3((unsigned)nb), s, x + b0 * n, y + b0 * n, (int)n,
                                     level, p.tw, f)) {
        hipLaunchKernelGGL(fwt_fwd_lds<FMA>, dim3((unsigned)nb), dim3(kNT), 0, s, x + b0 * n,
                           y + b0 * n, (int)n, level, p.M, p.tw, f);
      }
    }
    JW_HIP_TRY(hipGetLastError());
    return JW_OK;
  }
  double* tmp = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&tmp, sizeof(double) * (size_t)(n * batch)));
  if (y != x) JW_HIP_TRY(hipMemcpyAsync(y, x, sizeof(double) * n * batch, hipMemcpyDeviceToDevice, s));
  int l = 0;
  for (long h = n; h >= p.tw && l < level; h >>= 1, ++l) {
    for (long b0 = 0; b0 < batch; b0 += 65535) {
      const long nb = batch - b0 < 65535 ? batch - b0 : 65535;
      dim3 grid((unsigned)(((h >> 1) + kNT - 1) / kNT), (unsigned)nb);
      hipLaunchKernelGGL(fwt_fwd_level<FMA>, grid, dim3(kNT), 0, s, y + b0 * n, tmp + b0 * n, n,
                         (int)h, p.M, f);
    }
    JW_HIP_TRY(hipMemcpy2DAsync(y, sizeof(double) * n, tmp, sizeof(double) * n,
                                sizeof(double) * h, batch, hipMemcpyDeviceToDevice, s));
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

template <bool FMA>
int reverse_t(const FwtPlan& p, const double* y, double* x, long n, int level, long batch,
              hipStream_t s) {
  const Filters f = make_filters(p);
  long h0 = p.tw;
  const int steps = log2_exact(n);
  for (int l = level; l < steps; ++l) h0 <<= 1;  // FastWaveletTransform.java:137-141
  if (n <= kLdsN) {
    const bool fast = p.M % 2 == 0 && n >= 2 && !knob("JW_FWT_GENERIC");
    for (long b0 = 0; b0 < batch; b0 += 1L << 30) {
      const long nb = batch - b0 < (1L << 30) ? batch - b0 : (1L << 30);
      if (!fast || !launch_rev2<FMA>(p.M, dim3((unsigned)nb), s, y + b0 * n, x + b0 * n, (int)n,
                                     (int)h0, p.tw, p.kind, f)) {
        hipLaunchKernelGGL(fwt_rev_lds<FMA>, dim3((unsigned)nb), dim3(kNT), 0, s, y + b0 * n,
                           x + b0 * n, (int)n, (int)h0, p.M, p.tw, p.kind, f);
      }
    }
    JW_HIP_TRY(hipGetLastError());
    return JW_OK;
  }
  double* tmp = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&tmp, sizeof(double) * (size_t)(n * batch)));
  if (x != y) JW_HIP_TRY(hipMemcpyAsync(x, y, sizeof(double) * n * batch, hipMemcpyDeviceToDevice, s));
  for (long h = h0; h <= n && h >= p.tw; h <<= 1) {
    for (long b0 = 0; b0 < batch; b0 += 65535) {
      const long nb = batch - b0 < 65535 ? batch - b0 : 65535;
      dim3 grid((unsigned)((h + kNT - 1) / kNT), (unsigned)nb);
      hipLaunchKernelGGL(fwt_rev_level<FMA>, grid, dim3(kNT), 0, s, x + b0 * n, tmp + b0 * n, n,
                         (int)h, p.M, p.kind, f);
    }
    JW_HIP_TRY(hipMemcpy2DAsync(x, sizeof(double) * n, tmp, sizeof(double) * n,
                                sizeof(double) * h, batch, hipMemcpyDeviceToDevice, s));
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

int transpose(const double* in, double* out, int rows, int cols, int batch, hipStream_t s) {
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32), (unsigned)batch);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(kNT), 0, s, in, out, rows, cols);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace

int fwt_forward_device(const FwtPlan& p, const double* x, double* y, long n, int level, int batch,
                       hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? forward_t<true>(p, x, y, n, level, batch, s)
                                 : forward_t<false>(p, x, y, n, level, batch, s);
}

int fwt_reverse_device(const FwtPlan& p, const double* y, double* x, long n, int level, int batch,
                       hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? reverse_t<true>(p, y, x, n, level, batch, s)
                                 : reverse_t<false>(p, y, x, n, level, batch, s);
}

namespace {

template <bool FMA>
bool launch_wpt_lds(bool rev, int M, int kind, dim3 g, hipStream_t s, const double* in,
                    double* out, int n, int lvl_h0, int tw, const Filters& f) {
  switch (M) {
#define JW_C(MM)                                                                                \
  case MM:                                                                                      \
    if (!rev)                                                                                   \
      hipLaunchKernelGGL((wpt_fwd_lds<FMA, MM>), g, dim3(kNT2), 0, s, in, out, n, lvl_h0, tw, f); \
    else if (kind == JW_WAVELET_HAAR_ORTH)                                                       \
      hipLaunchKernelGGL((wpt_rev_lds<FMA, MM, JW_WAVELET_HAAR_ORTH>), g, dim3(kNT2), 0, s, in, \
                         out, n, lvl_h0, tw, f);                                                 \
    else                                                                                        \
      hipLaunchKernelGGL((wpt_rev_lds<FMA, MM, JW_WAVELET_GENERIC>), g, dim3(kNT2), 0, s, in,    \
                         out, n, lvl_h0, tw, f);                                                 \
    return true;
    JW_FWT_LENGTHS(JW_C)
#undef JW_C
    default:
      return false;
  }
}

template <bool FMA>
int wpt_t(const FwtPlan& p, bool rev, const double* in, double* out, long n, int level, long batch,
          hipStream_t s) {
  const Filters f = make_filters(p);
  long h0 = p.tw;
  if (rev)
    for (int l = level; l < log2_exact(n); ++l) h0 <<= 1;  // WaveletPacketTransform.java:160-162
  const int lvl_h0 = rev ? (int)h0 : level;
  if (n <= kLdsN && n >= 2 && p.M % 2 == 0 && !knob("JW_FWT_GENERIC")) {
    bool ok = true;
    for (long b0 = 0; b0 < batch && ok; b0 += 1L << 30) {
      const long nb = batch - b0 < (1L << 30) ? batch - b0 : (1L << 30);
      ok = launch_wpt_lds<FMA>(rev, p.M, p.kind, dim3((unsigned)nb), s, in + b0 * n, out + b0 * n,
                               (int)n, lvl_h0, p.tw, f);
    }
    if (ok) {
      JW_HIP_TRY(hipGetLastError());
      return JW_OK;
    }
  }
  // per-level global kernels, ping-pong between out and a workspace
  double* tmp = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&tmp, sizeof(double) * (size_t)(n * batch)));
  if (out != in) JW_HIP_TRY(hipMemcpyAsync(out, in, sizeof(double) * n * batch, hipMemcpyDeviceToDevice, s));
  double *a = out, *b = tmp;
  int l = 0;
  for (long h = rev ? h0 : n; rev ? (h <= n && h >= p.tw) : (h >= p.tw && l < level);
       h = rev ? h << 1 : h >> 1, ++l) {
    if (h < 2) break;
    for (long b0 = 0; b0 < batch; b0 += 65535) {
      const long nb = batch - b0 < 65535 ? batch - b0 : 65535;
      if (rev) {
        hipLaunchKernelGGL(wpt_rev_level<FMA>, dim3((unsigned)((n + kNT - 1) / kNT), (unsigned)nb),
                           dim3(kNT), 0, s, a + b0 * n, b + b0 * n, n, (int)h, p.M, p.kind, f);
      } else {
        hipLaunchKernelGGL(wpt_fwd_level<FMA>,
                           dim3((unsigned)(((n >> 1) + kNT - 1) / kNT), (unsigned)nb), dim3(kNT),
                           0, s, a + b0 * n, b + b0 * n, n, (int)h, p.M, f);
      }
    }
    double* t = a;
    a = b;
    b = t;
  }
  if (a != out)
    JW_HIP_TRY(hipMemcpyAsync(out, a, sizeof(double) * n * batch, hipMemcpyDeviceToDevice, s));
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace

int wpt_forward_device(const FwtPlan& p, const double* x, double* y, long n, int level, int batch,
                       hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? wpt_t<true>(p, false, x, y, n, level, batch, s)
                                 : wpt_t<false>(p, false, x, y, n, level, batch, s);
}

int wpt_reverse_device(const FwtPlan& p, const double* y, double* x, long n, int level, int batch,
                       hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? wpt_t<true>(p, true, y, x, n, level, batch, s)
                                 : wpt_t<false>(p, true, y, x, n, level, batch, s);
}

// Column levels that run as strips for a [rows][cols] 2-D pass (0: use fwt_lines4).  Strips
// run while h > the tail length (env JW_FWT_TAIL overrides it, for tests; JW_FWT_STRIP=0
// disables the strips).  Transform wavelength 2 keeps the reverse's first level at
// rows >> (lvlM - 1) (FastWaveletTransform.java:137-141).
int strip_levels(const FwtPlan& p, int rows, int cols, int lvlM) {
  const char* e = knob("JW_FWT_STRIP");
  if ((e && e[0] == '0') || knob("JW_FWT_GENERIC")) return 0;
  if (p.M % 2 || p.M > 20 || p.tw != 2 || cols % kSW || cols > kLdsN || (rows & (rows - 1)))
    return 0;
  const char* te = knob("JW_FWT_TAIL");
  long tail = te ? std::atol(te) : kTailLen;
  if (tail > kTailLen) tail = kTailLen;
  if (tail < 2 * kST) tail = 2 * kST;
  int S = 0;
  long h = rows;
  while (S < lvlM && h > tail && h / 2 >= p.M) {
    ++S;
    h >>= 1;
  }
  if (S < lvlM && h > kTailLen) return 0;  // the remaining levels would not fit the tail
  return S;
}

template <bool FMA>
int fwt2d_forward_strips(const FwtPlan& p, int S, const double* x, double* y, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  const long mat = (long)rows * cols, half = mat / 2;
  double *T = nullptr, *B = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&T, sizeof(double) * mat * batch));
  JW_HIP_TRY(mem.alloc(&B, sizeof(double) * half * batch));
  int st = fwt_forward_device(p, x, T, cols, lvlN, rows * batch, s);  // rows -> T
  const Filters f = make_filters(p);
  const int tail_lv = lvlM - S;
  // levels 1..4 of every column in one pass (T -> y), then the tail in place on y
  if (st == JW_OK && fwtc::launch_stream_fwd<FMA>(p.M, S, s, T, y, rows, cols, mat, batch, f)) {
    if (tail_lv > 0 && !launch_tail<FMA>(p.M, p.kind, false, s, y, y, rows >> S, cols, mat, mat,
                                         tail_lv, p.tw, batch, f))
      st = fail(JW_ERR_UNSUPPORTED, "no 2-D strip kernel for filter length %d", p.M);
    if (st == JW_OK) JW_HIP_TRY(hipGetLastError());
    return st;
  }
  double* bufs[2] = {T, B};
  const long ms[2] = {mat, half};
  int cur = 0;  // buffer holding the current level's input (approximations)
  for (int l = 0; l < S && st == JW_OK; ++l) {
    const int h = rows >> l;
    const bool to_y = l == S - 1 && tail_lv == 0;
    const Strip sp{bufs[cur], nullptr, to_y ? y : bufs[cur ^ 1], y + (long)(h / 2) * cols,
                   ms[cur], 0, to_y ? mat : ms[cur ^ 1], mat, cols, h};
    if (!launch_strip<FMA>(p.M, p.kind, false, s, sp, batch, f)) st = fail(JW_ERR_UNSUPPORTED, "no 2-D strip kernel for filter length %d", p.M);
    cur ^= 1;
  }
  if (st == JW_OK && tail_lv > 0 &&
      !launch_tail<FMA>(p.M, p.kind, false, s, bufs[cur], y, rows >> S, cols, ms[cur], mat, tail_lv,
                        p.tw, batch, f))
    st = fail(JW_ERR_UNSUPPORTED, "no 2-D strip kernel for filter length %d", p.M);
  if (st == JW_OK) JW_HIP_TRY(hipGetLastError());
  return st;
}

template <bool FMA>
int fwt2d_reverse_strips(const FwtPlan& p, int S, const double* y, double* x, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  const long mat = (long)rows * cols, half = mat / 2;
  double *T = nullptr, *B = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&T, sizeof(double) * mat * batch));
  JW_HIP_TRY(mem.alloc(&B, sizeof(double) * half * batch));
  const Filters f = make_filters(p);
  const int tail_lv = lvlM - S;
  // level l (h = rows >> l) writes rows [0, h) of O_l: O_0 = T, then alternating with B.
  // The streaming pass writes T from the tail's output, so that output goes to B then.
  const bool stream = fwtc::launch_stream_rev<FMA>(p.M, p.kind, S, s, nullptr, 0, nullptr,
                                                   nullptr, rows, cols, mat, batch, f);
  auto obuf = [&](int l) { return stream && l == S ? B : (l & 1) ? B : T; };
  auto oms = [&](int l) { return stream && l == S ? half : (l & 1) ? half : mat; };
  int st = JW_OK;
  const double* a = y;  // approximations of the next (finer) level
  long ms_a = mat;
  if (tail_lv > 0) {
    long h0 = p.tw;
    for (int l = lvlM; l < log2_exact(rows); ++l) h0 <<= 1;  // FastWaveletTransform.java:137-141
    if (!launch_tail<FMA>(p.M, p.kind, true, s, y, obuf(S), rows >> S, cols, mat, oms(S), (int)h0,
                          p.tw, batch, f))
      st = fail(JW_ERR_UNSUPPORTED, "no 2-D strip kernel for filter length %d", p.M);
    a = obuf(S);
    ms_a = oms(S);
  }
  // levels 4..1 of every column in one pass (a + the details of y -> T)
  if (st == JW_OK && stream &&
      fwtc::launch_stream_rev<FMA>(p.M, p.kind, S, s, a, ms_a, y, T, rows, cols, mat, batch, f)) {
    JW_HIP_TRY(hipGetLastError());
    return fwt_reverse_device(p, T, x, cols, lvlN, rows * batch, s);  // rows
  }
  for (int l = S - 1; l >= 0 && st == JW_OK; --l) {
    const int h = rows >> l;
    const Strip sp{a, y + (long)(h / 2) * cols, obuf(l), nullptr, ms_a, mat, oms(l), 0, cols, h};
    if (!launch_strip<FMA>(p.M, p.kind, true, s, sp, batch, f)) st = fail(JW_ERR_UNSUPPORTED, "no 2-D strip kernel for filter length %d", p.M);
    a = obuf(l);
    ms_a = oms(l);
  }
  if (st == JW_OK) JW_HIP_TRY(hipGetLastError());
  if (st == JW_OK) st = fwt_reverse_device(p, T, x, cols, lvlN, rows * batch, s);  // rows
  return st;
}

// 2-D (BasicTransform.java:361-399): every row with lvlN, then every column with lvlM.
// Tall matrices (rows > 1024): rows with the LDS cascade, then the strip levels and the LDS
// tail of the columns (fwt2d_forward_strips).  Otherwise, fused path (power-of-two sides <=
// 4096, even M): rows with the LDS cascade, then the columns in place with fwt_lines4 -- two
// passes over HBM.  Otherwise rows -> transpose -> rows -> transpose.
int fwt2d_forward_device(const FwtPlan& p, const double* x, double* y, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  if (const int S = strip_levels(p, rows, cols, lvlM); S > 0 && cols <= kLdsN) {
    return p.arith == JW_ARITH_FMA
               ? fwt2d_forward_strips<true>(p, S, x, y, rows, cols, lvlM, lvlN, batch, s)
               : fwt2d_forward_strips<false>(p, S, x, y, rows, cols, lvlM, lvlN, batch, s);
  }
  const bool fused = p.M % 2 == 0 && rows <= kLdsN && cols <= kLdsN && cols % kLines == 0 &&
                     rows >= 2 && !knob("JW_FWT_GENERIC");
  if (fused) {
    int st = fwt_forward_device(p, x, y, cols, lvlN, rows * batch, s);
    if (st != JW_OK) return st;
    const Filters f = make_filters(p);
    const bool ok = p.arith == JW_ARITH_FMA
                        ? launch_cols<true>(p.M, p.kind, false, s, y, y, rows, cols, lvlM, p.tw, batch, f)
                        : launch_cols<false>(p.M, p.kind, false, s, y, y, rows, cols, lvlM, p.tw, batch, f);
    if (ok) {
      JW_HIP_TRY(hipGetLastError());
      return JW_OK;
    }
    // no fused kernel for this M: finish with the transpose path on y
    const size_t elems = (size_t)rows * cols * batch;
    double* t = nullptr;
    StreamAllocs mem(s);
    JW_HIP_TRY(mem.alloc(&t, sizeof(double) * elems));
    st = transpose(y, t, rows, cols, batch, s);
    if (st == JW_OK) st = fwt_forward_device(p, t, t, rows, lvlM, cols * batch, s);
    if (st == JW_OK) st = transpose(t, y, cols, rows, batch, s);
    return st;
  }
  const size_t elems = (size_t)rows * cols * batch;
  double* t = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&t, sizeof(double) * elems));
  int st = fwt_forward_device(p, x, y, cols, lvlN, rows * batch, s);
  if (st == JW_OK) st = transpose(y, t, rows, cols, batch, s);
  if (st == JW_OK) st = fwt_forward_device(p, t, t, rows, lvlM, cols * batch, s);
  if (st == JW_OK) st = transpose(t, y, cols, rows, batch, s);
  return st;
}

// 2-D reverse (BasicTransform.java:436-474): every column with lvlM, then every row with lvlN.
int fwt2d_reverse_device(const FwtPlan& p, const double* y, double* x, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  if (const int S = strip_levels(p, rows, cols, lvlM); S > 0) {
    return p.arith == JW_ARITH_FMA
               ? fwt2d_reverse_strips<true>(p, S, y, x, rows, cols, lvlM, lvlN, batch, s)
               : fwt2d_reverse_strips<false>(p, S, y, x, rows, cols, lvlM, lvlN, batch, s);
  }
  const bool fused = p.M % 2 == 0 && rows <= kLdsN && cols <= kLdsN && cols % kLines == 0 &&
                     rows >= 2 && !knob("JW_FWT_GENERIC");
  if (fused) {
    long h0 = p.tw;
    for (int l = lvlM; l < log2_exact(rows); ++l) h0 <<= 1;  // FastWaveletTransform.java:137-141
    const Filters f = make_filters(p);
    const bool ok = p.arith == JW_ARITH_FMA
                        ? launch_cols<true>(p.M, p.kind, true, s, y, x, rows, cols, (int)h0, p.tw, batch, f)
                        : launch_cols<false>(p.M, p.kind, true, s, y, x, rows, cols, (int)h0, p.tw, batch, f);
    if (ok) {
      JW_HIP_TRY(hipGetLastError());
      return fwt_reverse_device(p, x, x, cols, lvlN, rows * batch, s);
    }
  }
  const size_t elems = (size_t)rows * cols * batch;
  double* t = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&t, sizeof(double) * elems));
  int st = transpose(y, t, rows, cols, batch, s);
  if (st == JW_OK) st = fwt_reverse_device(p, t, t, rows, lvlM, cols * batch, s);
  if (st == JW_OK) st = transpose(t, x, cols, rows, batch, s);
  if (st == JW_OK) st = fwt_reverse_device(p, x, x, cols, lvlN, rows * batch, s);
  return st;
}

// ---------------------------------------------------------------------------------------
// 3-D (BasicTransform.java:509-565 forward, :602-659 reverse).  The space is [R][C][H]
// (Java's spc[i][j][k]), batch-major.  Forward: every slab i gets the 2-D forward with
// (lvlP, lvlQ) -- rows of H samples with lvlQ, then columns of C samples with lvlP -- and
// then every (j, k) line along i (R samples, stride C*H) gets the 1-D forward with lvlR.
// Reverse: the 2-D reverse per slab first, then the 1-D reverse along i (the reference's
// order, not the mirror of the forward's).  The slabs are a batch of R*batch matrices for
// the 2-D kernels; the lines along i are the columns of the [R][C*H] matrix.
// ---------------------------------------------------------------------------------------
namespace {
// Columns of `batch` row-major [rows][cols] matrices: level lvl (forward) or the reverse of
// level lvl, in -> out (in == out allowed).
int fwt_columns(const FwtPlan& p, bool rev, const double* in, double* out, int rows, long cols,
                int lvl, int batch, hipStream_t s) {
  const size_t elems = (size_t)rows * cols * batch;
  if (rows < 2 || lvl == 0) {  // forward(arr, 0) / reverse(arr, 0) copy the line
    if (in != out) JW_HIP_TRY(hipMemcpyAsync(out, in, elems * sizeof(double), hipMemcpyDeviceToDevice, s));
    return JW_OK;
  }
  if (p.M % 2 == 0 && rows <= kLdsN && cols % kLines == 0 && cols <= (1L << 30) &&
      !knob("JW_FWT_GENERIC")) {
    int arg = lvl;
    if (rev) {  // h0 = tw << (log2 rows - lvl), FastWaveletTransform.java:137-141
      long h0 = p.tw;
      for (int l = lvl; l < log2_exact(rows); ++l) h0 <<= 1;
      arg = (int)h0;
    }
    const Filters f = make_filters(p);
    const bool ok =
        p.arith == JW_ARITH_FMA
            ? launch_cols<true>(p.M, p.kind, rev, s, in, out, rows, (int)cols, arg, p.tw, batch, f)
            : launch_cols<false>(p.M, p.kind, rev, s, in, out, rows, (int)cols, arg, p.tw, batch, f);
    if (ok) {
      JW_HIP_TRY(hipGetLastError());
      return JW_OK;
    }
  }
  double* t = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&t, sizeof(double) * elems));
  int st = transpose(in, t, rows, (int)cols, batch, s);
  if (st == JW_OK)
    st = rev ? fwt_reverse_device(p, t, t, rows, lvl, (int)(cols * batch), s)
             : fwt_forward_device(p, t, t, rows, lvl, (int)(cols * batch), s);
  if (st == JW_OK) st = transpose(t, out, (int)cols, rows, batch, s);
  return st;
}
}  // namespace

int fwt3d_forward_device(const FwtPlan& p, const double* x, double* y, int R, int C, int H,
                         int lvlP, int lvlQ, int lvlR, int batch, hipStream_t s) {
  int st = fwt2d_forward_device(p, x, y, C, H, lvlP, lvlQ, R * batch, s);
  if (st != JW_OK) return st;
  return fwt_columns(p, false, y, y, R, (long)C * H, lvlR, batch, s);
}

int fwt3d_reverse_device(const FwtPlan& p, const double* y, double* x, int R, int C, int H,
                         int lvlP, int lvlQ, int lvlR, int batch, hipStream_t s) {
  int st = fwt2d_reverse_device(p, y, x, C, H, lvlP, lvlQ, R * batch, s);
  if (st != JW_OK) return st;
  return fwt_columns(p, true, x, x, R, (long)C * H, lvlR, batch, s);
}

}  // namespace jw
