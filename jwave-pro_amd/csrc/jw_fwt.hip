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

#include "jw_internal.hpp"

namespace jw {
namespace {

constexpr int kNT = 256;
constexpr int kLdsN = 4096;              // signals up to this length run one workgroup each
constexpr int kPer = kLdsN / kNT;        // outputs per thread per level (max)

struct Filters {
  double sD[kMaxTaps], wD[kMaxTaps], sR[kMaxTaps], wR[kMaxTaps];
};

template <bool FMA>
__device__ __forceinline__ double madd(double acc, double f, double v) {
  if constexpr (FMA) return __builtin_fma(f, v, acc);
  else return acc + f * v;
}

template <bool FMA>
__device__ __forceinline__ double contrib(double a, double d, double sr, double wr, int kind) {
  double c;
  if constexpr (FMA) c = __builtin_fma(a, sr, d * wr);
  else c = (a * sr) + (d * wr);
  return kind == JW_WAVELET_HAAR_ORTH ? .5 * c : c;
}

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

// Outputs (2u, 2u+1) that see wrapped taps, in Java's scatter order (i ascending, then j),
// with compile-time M: fully unrolled, predicated (select, not "+ 0.0") so the sums are
// bit-identical to the reference's.
template <bool FMA, int M, int KIND>
__device__ __forceinline__ d2 rev_pair_wrapped(const double* buf, int h, int u,
                                               const Filters& f) {
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

// The forward cascade on one line held in LDS (buf), by NTL threads (tid < NTL).  The
// barriers are workgroup-wide: every line of the workgroup runs the same levels.
template <bool FMA, int M, int NTL>
__device__ __forceinline__ void cascade_fwd(double* buf, int n, int level, int tw, int tid,
                                            const Filters& f) {
  constexpr int P = kLdsN / NTL / 2;  // pairs per thread at the first level (max)
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
    __syncthreads();
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int i = tid + r * NTL;
      if (i < half) {
        buf[i] = lo[r];
        buf[i + half] = hi[r];
      }
    }
    __syncthreads();
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

template <bool FMA, int M, int KIND, int NTL>
__device__ __forceinline__ void cascade_rev(double* buf, int n, int h0, int tw, int tid,
                                            const Filters& f) {
  constexpr int P = kLdsN / NTL / 2;
  for (int h = h0; h <= n && h >= tw && h >= 2; h <<= 1) {
    const int half = h >> 1;
    // pairs u < nslow see wrapped taps: all of them when h < M, else the first M/2 - 1; they
    // are all thread tid = u of the first pass (nslow <= 32)
    const int nslow = h < M ? half : (M >> 1) - 1 < half ? (M >> 1) - 1 : half;
    d2 o[P];
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int u = tid + r * NTL;
      if (u < half && u >= nslow) {
        double a0 = 0., a1 = 0.;
#pragma unroll
        for (int t = (M >> 1) - 1; t >= 0; --t) {
          const double av = buf[u - t], dv = buf[u - t + half];
          a0 += contrib<FMA>(av, dv, f.sR[2 * t], f.wR[2 * t], KIND);  // KIND: compile-time
          a1 += contrib<FMA>(av, dv, f.sR[2 * t + 1], f.wR[2 * t + 1], KIND);
        }
        o[r] = d2{a0, a1};
      }
      if (u + NTL >= half) break;
    }
    if (tid < nslow) o[0] = rev_pair_wrapped<FMA, M, KIND>(buf, h, tid, f);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int u = tid + r * NTL;
      if (u < half) *(d2*)&buf[2 * u] = o[r];
    }
    __syncthreads();
  }
}

template <bool FMA, int M, int KIND>
__global__ __launch_bounds__(kNT2) void fwt_rev_lds2(const double* __restrict__ y,
                                                    double* __restrict__ x, int n, int h0, int tw,
                                                    int kind, Filters f) {
  __shared__ __attribute__((aligned(16))) double buf[kLdsN];
  const int tid = threadIdx.x;
  const double* ys = y + (long)blockIdx.x * n;
  double* xs = x + (long)blockIdx.x * n;
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&buf[i] = *(const d2*)&ys[i];
  __syncthreads();
  cascade_rev<FMA, M, KIND, kNT2>(buf, n, h0, tw, tid, f);
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&xs[i] = *(const d2*)&buf[i];
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
  constexpr int P = kLdsN / kNT2 / 2;
  const int tid = threadIdx.x;
  const double* ys = y + (long)blockIdx.x * n;
  double* xs = x + (long)blockIdx.x * n;
  for (int i = 2 * tid; i < n; i += 2 * kNT2) *(d2*)&buf[i] = *(const d2*)&ys[i];
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
            a0 += contrib<FMA>(av, dv, f.sR[2 * t], f.wR[2 * t], KIND);
            a1 += contrib<FMA>(av, dv, f.sR[2 * t + 1], f.wR[2 * t + 1], KIND);
          }
          o[r] = d2{a0, a1};
        } else {
          o[r] = rev_pair_wrapped<FMA, M, KIND>(buf + base, h, u, f);
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
  const int tid = threadIdx.x, g = tid >> 8, lt = tid & 255;
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
    cascade_rev<FMA, M, KIND, 256>(buf, len, lvl_h0, tw, lt, f);
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
#define JW_FWT_LENGTHS(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22) X(24) \
  X(26) X(28) X(30) X(32) X(34) X(36) X(38) X(40)

template <bool FMA>
bool launch_fwd2(int M, dim3 g, hipStream_t s, const double* x, double* y, int n, int level,
                 int tw, const Filters& f) {
  switch (M) {
#define JW_C(MM)                                                                          \
  case MM:                                                                                \
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
  switch (M) {
#define JW_C(MM)                                                                           \
  case MM:                                                                                 \
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
  const char* e = std::getenv("JW_FWT_LINES");
  if (e ? e[0] == '2' : rev)
    return launch_cols_nl<FMA, 2>(M, kind, rev, s, in, out, rows, cols, lvl_h0, tw, batch, f);
  return launch_cols_nl<FMA, 4>(M, kind, rev, s, in, out, rows, cols, lvl_h0, tw, batch, f);
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
    const bool fast = p.M % 2 == 0 && n >= 2 && !std::getenv("JW_FWT_GENERIC");
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
  JW_HIP_TRY(hipMallocAsync((void**)&tmp, sizeof(double) * (size_t)(n * batch), s));
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
  JW_HIP_TRY(hipFreeAsync(tmp, s));
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
    const bool fast = p.M % 2 == 0 && n >= 2 && !std::getenv("JW_FWT_GENERIC");
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
  JW_HIP_TRY(hipMallocAsync((void**)&tmp, sizeof(double) * (size_t)(n * batch), s));
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
  JW_HIP_TRY(hipFreeAsync(tmp, s));
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
  if (n <= kLdsN && n >= 2 && p.M % 2 == 0 && !std::getenv("JW_FWT_GENERIC")) {
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
  JW_HIP_TRY(hipMallocAsync((void**)&tmp, sizeof(double) * (size_t)(n * batch), s));
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
  JW_HIP_TRY(hipFreeAsync(tmp, s));
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

// 2-D (BasicTransform.java:361-399): every row with lvlN, then every column with lvlM.
// Fused path (power-of-two sides <= 4096, even M): rows with the LDS cascade, then the columns
// in place with fwt_lines4 -- two passes over HBM.  Otherwise rows -> transpose -> rows ->
// transpose.
int fwt2d_forward_device(const FwtPlan& p, const double* x, double* y, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  const bool fused = p.M % 2 == 0 && rows <= kLdsN && cols <= kLdsN && cols % kLines == 0 &&
                     rows >= 2 && !std::getenv("JW_FWT_GENERIC");
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
    JW_HIP_TRY(hipMallocAsync((void**)&t, sizeof(double) * elems, s));
    st = transpose(y, t, rows, cols, batch, s);
    if (st == JW_OK) st = fwt_forward_device(p, t, t, rows, lvlM, cols * batch, s);
    if (st == JW_OK) st = transpose(t, y, cols, rows, batch, s);
    JW_HIP_TRY(hipFreeAsync(t, s));
    return st;
  }
  const size_t elems = (size_t)rows * cols * batch;
  double* t = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&t, sizeof(double) * elems, s));
  int st = fwt_forward_device(p, x, y, cols, lvlN, rows * batch, s);
  if (st == JW_OK) st = transpose(y, t, rows, cols, batch, s);
  if (st == JW_OK) st = fwt_forward_device(p, t, t, rows, lvlM, cols * batch, s);
  if (st == JW_OK) st = transpose(t, y, cols, rows, batch, s);
  JW_HIP_TRY(hipFreeAsync(t, s));
  return st;
}

// 2-D reverse (BasicTransform.java:436-474): every column with lvlM, then every row with lvlN.
int fwt2d_reverse_device(const FwtPlan& p, const double* y, double* x, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  const bool fused = p.M % 2 == 0 && rows <= kLdsN && cols <= kLdsN && cols % kLines == 0 &&
                     rows >= 2 && !std::getenv("JW_FWT_GENERIC");
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
  JW_HIP_TRY(hipMallocAsync((void**)&t, sizeof(double) * elems, s));
  int st = transpose(y, t, rows, cols, batch, s);
  if (st == JW_OK) st = fwt_reverse_device(p, t, t, rows, lvlM, cols * batch, s);
  if (st == JW_OK) st = transpose(t, x, cols, rows, batch, s);
  if (st == JW_OK) st = fwt_reverse_device(p, x, x, cols, lvlN, rows * batch, s);
  JW_HIP_TRY(hipFreeAsync(t, s));
  return st;
}

}  // namespace jw
