// jw_modwt.hip -- MODWT forward / inverse (direct circular convolution) for gfx950.
//
// Reference semantics (src/main/java/jwave/transforms/MODWTTransform.java):
//   forwardMODWT :256-306   W_j = h_j (*) V_{j-1},  V_j = g_j (*) V_{j-1},  V_0 = x
//   inverseMODWT :337-375   V_{j-1} = (g_j^T V_j) + (h_j^T W_j)   for j = J..1
//   circularConvolve :677-690        y[n] = sum_m x[floorMod(n - m, N)] * f[m]
//   circularConvolveAdjoint :703-716 y[n] = sum_m x[floorMod(n + m, N)] * f[m]
// f = upsample(base, j) (:618-630): base taps at m = k * 2^(j-1), zeros elsewhere.  A zero
// tap adds x*0 = +-0 to a running sum that starts at +0.0 and is never -0.0, which leaves
// the sum bit-identical, so only the L non-zero taps are evaluated here -- in the same
// ascending order, starting from +0.0, without FMA (JW_ARITH_STRICT): the JVM's exact
// IEEE sequence for finite inputs.
//
// Non-finite inputs.  Java multiplies the zero taps too, and 0 * +-Inf = 0 * NaN = NaN, so an
// output whose window holds a non-finite sample on a zero tap is NaN in JWave; otherwise the
// zero taps add +-0 and the non-zero-tap sum stands.  Level by level, that is exactly the
// reference (checked against the faithful every-tap oracle, tests/test_modwt_nonfinite_gpu.py).
// The fast paths skip the zero taps and flag a signal whose final row holds a non-finite value
// (fast::nonfinite_flag: a non-finite sample anywhere in the cascade reaches that row); the
// generic streaming kernel then runs again for the flagged signals only, in FIX mode, which
// adds the zero-tap test to every output (modwt_fwd_fused / modwt_inv_fused <.., true>).  The
// per-level kernels test the zero taps themselves when their input row is flagged.  All of it
// stays on the stream: a clean signal costs a flag word, a memset and an early-exit launch.
//
// Design (DESIGN.md "MODWT kernels"): one workgroup streams a segment of one signal through
// all J levels in LDS.  The signal is walked in chunks of C samples; every level keeps the
// (L-1)*2^(j-1) samples of history its dilated filter needs in an LDS buffer, so each
// sample is read from HBM once and each coefficient row written once: the HBM traffic is
// the algorithmic 8*(1 + (J+1)) bytes/sample forward and 8*((J+1) + 1) inverse.
// Forward streams left->right (history on the left), inverse right->left (history on the
// right).  A segment starts with a warm-up of ceil(H/C) chunks, H = (L-1)(2^J - 1), whose
// outputs are not stored.  Positions are taken modulo N, so any N >= 1 (multi-wrap
// filters included) follows the reference's floorMod semantics.
#include <cstdlib>
#include <cstring>

#include "jw_internal.hpp"
#include "jw_modwt_fast.hpp"

namespace jw {
namespace {

constexpr int kC = 512;                  // chunk: samples per level per step
constexpr int kNT = 256;                 // threads per workgroup (4 waves)
constexpr int kHistPer = 16;             // history samples a thread moves per step (max)
constexpr int kHistMax = kHistPer * kNT; // fused path needs H <= this
constexpr int kWinPer = 16;              // W-window samples a thread stages (max)
constexpr int kWinMax = kWinPer * kNT;   // fused inverse needs C + hist_J <= this
constexpr int kLoad = kC / kNT;          // chunk samples per thread

template <bool FMA>
__device__ __forceinline__ double madd(double acc, double f, double v) {
  if constexpr (FMA) {
    return __builtin_fma(f, v, acc);
  } else {
    return acc + f * v;  // built with -ffp-contract=off: rounded product, rounded sum (Java)
  }
}

__device__ __forceinline__ long wrap(long p, long N) {
  if (p >= 0 && p < N) return p;
  long r = p % N;
  return r < 0 ? r + N : r;
}

__host__ __device__ constexpr long hist_of(int L, int j) { return (long)(L - 1) << (j - 1); }

// True when a zero tap of the up-sampled window at p meets a non-finite sample: taps m in
// [1, M) with m mod d != 0, at p[-m] (circularConvolve, DIR = -1) or p[+m] (adjoint, +1).
// Literal walk over the window in LDS (FIX mode only).
template <int DIR>
__device__ __forceinline__ bool zero_tap_nonfinite(const double* p, int d, int M) {
  bool hit = false;
  if (d > 1) {
    for (int m = 1; m < M; ++m)
      if ((m & (d - 1)) != 0) hit |= !__builtin_isfinite(p[DIR * m]);
  }
  return hit;
}

// The same test for the per-level kernels, whose window lives in global memory (M up to
// 39 * 4096 + 1): a wave covers outputs n0 .. n0 + 63 (lane l: n = n0 + l) and walks the union
// of their windows 64 positions at a time; each non-finite position found (ballot) is checked
// against every lane's window.  ADJ: window n .. n + M - 1, else n - M + 1 .. n.  Every lane
// of the wave must take part (dead tail lanes included).
template <bool ADJ>
__device__ bool zero_tap_nonfinite_wave(const double* v, long N, long n, long M, long d) {
  const int lane = threadIdx.x & 63;
  const long n0 = n - lane;
  const long lo = ADJ ? n0 : n0 - (M - 1);
  const long hi = ADJ ? n0 + 63 + (M - 1) : n0 + 63;
  bool hit = false;
  for (long base = lo; base <= hi; base += 64) {
    const long q = base + lane;
    const bool bad = q <= hi && !__builtin_isfinite(v[wrap(q, N)]);
    unsigned long long mask = __ballot(bad);
    while (mask != 0) {
      const int b = __builtin_ctzll(mask);
      mask &= mask - 1;
      const long m = ADJ ? (base + b) - n : n - (base + b);
      if (m > 0 && m < M && (m & (d - 1)) != 0) hit = true;
    }
  }
  return hit;
}

constexpr double kNaN = __builtin_nan("");

// flags[r * fstride + b] = 1 when row r of signal b holds a non-finite value (rows r < nrows at
// row_stride within a signal, signals at sig_stride).  Vector stores of the constant 1.
__global__ __launch_bounds__(256) void modwt_nonfinite_rows(const double* __restrict__ p,
                                                            long sig_stride, long row_stride,
                                                            int nrows, long N,
                                                            int* __restrict__ flags,
                                                            long fstride) {
  const double* ps = p + (long)blockIdx.y * sig_stride;
  for (int r = 0; r < nrows; ++r) {
    bool bad = false;
    for (long n = (long)blockIdx.x * 256 + threadIdx.x; n < N; n += (long)gridDim.x * 256)
      bad |= !__builtin_isfinite(ps[(long)r * row_stride + n]);
    if (bad) flags[(long)r * fstride + blockIdx.y] = 1;
  }
}

// Flat history index e -> level j (1-based): level j owns e in [(L-1)(2^(j-1)-1), (L-1)(2^j-1)).
template <int L>
__device__ __forceinline__ int level_of(int e) {
  const unsigned q = (unsigned)(e / (L - 1)) + 1u;
  return 32 - __builtin_clz(q);
}

// ---------------------------------------------------------------------------------------
// Fused forward.  LDS: for j = 1..J a buffer B_{j-1} = [hist_j | C] holding V_{j-1} at
// stream positions [a - hist_j, a + C).  After the J levels of a step, the last hist_j
// samples of every buffer move to its front (the history of the next chunk).
// B_{j-1} starts at (L-1)(2^(j-1)-1) + (j-1)*C.
// FIX = false: the generic path; nf (nullable) receives the signal's non-finite flag.
// FIX = true: the zero-tap pass; only signals whose nf is set run, every output gets the
// zero-tap test (NaN on a hit), and all rows of the signal are rewritten.
// ---------------------------------------------------------------------------------------
template <int L, bool FMA, bool FIX>
__global__ __launch_bounds__(kNT) void modwt_fwd_fused(const double* __restrict__ x,
                                                       double* __restrict__ coeffs, long N, int J,
                                                       long seg_len, long warm, Taps taps,
                                                       int* __restrict__ nf) {
  if constexpr (FIX) {
    if (nf[blockIdx.y] == 0) return;  // workgroup-uniform: a clean signal
  }
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x;
  const long P = (long)blockIdx.x * seg_len;
  const long seg_end = min(P + seg_len, N);
  const double* xs = x + (long)blockIdx.y * N;
  double* cs = coeffs + (long)blockIdx.y * (long)(J + 1) * N;
  const int H = (L - 1) * ((1 << J) - 1);
  const int total = H + J * kC;
  for (int i = tid; i < total; i += kNT) lds[i] = 0.0;

  double pre[kLoad];
  bool bad = false;
  long a = P - warm;
  {
    const long base = wrap(a, N);
#pragma unroll
    for (int r = 0; r < kLoad; ++r) {
      const long p = base + tid + r * kNT;
      pre[r] = xs[p < N ? p : wrap(p, N)];
    }
  }
  __syncthreads();

  for (; a < seg_end; a += kC) {
    // Land the prefetched chunk of V_0 = x in B_0's chunk region, then prefetch the next.
#pragma unroll
    for (int r = 0; r < kLoad; ++r) lds[(L - 1) + tid + r * kNT] = pre[r];
    if (a + kC < seg_end) {
      const long base = wrap(a + kC, N);
#pragma unroll
      for (int r = 0; r < kLoad; ++r) {
        const long p = base + tid + r * kNT;
        pre[r] = xs[p < N ? p : wrap(p, N)];
      }
    }
    __syncthreads();

    int off = 0;
    for (int j = 1; j <= J; ++j) {
      const int d = 1 << (j - 1);
      const int hist = (L - 1) * d;
      const double* src = lds + off;
      const int off_next = off + hist + kC;
      double* dst = lds + off_next + (L - 1) * (d << 1);  // chunk region of B_j
      double* W = cs + (long)(j - 1) * N;
      double* VJ = cs + (long)J * N;
      const bool last = (j == J);
      auto emit = [&](int i, double w, double v) {
        if constexpr (FIX) {
          if (zero_tap_nonfinite<-1>(src + hist + i, d, hist + 1)) w = v = kNaN;
        }
        const long pos = a + i;
        const bool keep = pos >= P && pos < seg_end;
        if (keep) W[pos] = w;
        if (!last) {
          dst[i] = v;
        } else {
          if (keep) VJ[pos] = v;
          bad |= !__builtin_isfinite(v);
        }
      };
      if (2 * d <= kC) {
        // Pair (i1, i1+d): the two outputs share L-1 of their L taps -> L+1 LDS reads.
        for (int t = tid; t < kC / 2; t += kNT) {
          const int i1 = ((t >> (j - 1)) << j) + (t & (d - 1));
          const double* s0 = src + hist + i1 + d;
          double v[L + 1];
#pragma unroll
          for (int k = 0; k <= L; ++k) v[k] = s0[-k * d];
          double w1 = 0.0, g1 = 0.0, w2 = 0.0, g2 = 0.0;
#pragma unroll
          for (int m = 0; m < L; ++m) {
            w1 = madd<FMA>(w1, taps.b[m], v[m + 1]);
            g1 = madd<FMA>(g1, taps.a[m], v[m + 1]);
            w2 = madd<FMA>(w2, taps.b[m], v[m]);
            g2 = madd<FMA>(g2, taps.a[m], v[m]);
          }
          emit(i1, w1, g1);
          emit(i1 + d, w2, g2);
        }
      } else {
        for (int i = tid; i < kC; i += kNT) {
          const double* s0 = src + hist + i;
          double w = 0.0, g = 0.0;
#pragma unroll
          for (int m = 0; m < L; ++m) {
            const double xv = s0[-m * d];
            w = madd<FMA>(w, taps.b[m], xv);
            g = madd<FMA>(g, taps.a[m], xv);
          }
          emit(i, w, g);
        }
      }
      __syncthreads();
      off = off_next;
    }

    // History shift: B_{j-1}[C .. C+hist_j) -> B_{j-1}[0 .. hist_j) for every level.  The
    // ranges overlap when hist_j > C, so all reads complete before any write.  Flat index
    // e: B_{j-1} starts at flat offset + (j-1)*C, so src = e + j*C and dst = e + (j-1)*C.
    // The next step's chunk store touches only B_0[hist_1 ..), disjoint from every history
    // write, and the level reads that follow it sit behind a barrier.
    if constexpr (L > 1) {
      double hv[kHistPer];
#pragma unroll
      for (int r = 0; r < kHistPer; ++r) {
        const int e = tid + r * kNT;
        if (e < H) hv[r] = lds[e + level_of<L>(e) * kC];
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kHistPer; ++r) {
        const int e = tid + r * kNT;
        if (e < H) lds[e + (level_of<L>(e) - 1) * kC] = hv[r];
      }
    }
  }
  if constexpr (!FIX) fast::nonfinite_flag(nf, bad);
}

// ---------------------------------------------------------------------------------------
// Fused inverse.  LDS: for j = 1..J a buffer VB_j = [C | hist_j] with V_j at positions
// [a, a + C + hist_j) (VB_j starts at (j-1)*C + (L-1)(2^(j-1)-1)), then two W staging
// buffers of C + hist_J samples.
// ---------------------------------------------------------------------------------------
template <int L, bool FMA, bool FIX>
__global__ __launch_bounds__(kNT) void modwt_inv_fused(const double* __restrict__ coeffs,
                                                       double* __restrict__ x, long N, int J,
                                                       long seg_len, long warm, Taps taps,
                                                       int* __restrict__ nf) {
  if constexpr (FIX) {
    if (nf[blockIdx.y] == 0) return;
  }
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x;
  const long P = (long)blockIdx.x * seg_len;
  const long seg_end = min(P + seg_len, N);
  const double* cs = coeffs + (long)blockIdx.y * (long)(J + 1) * N;
  double* xs = x + (long)blockIdx.y * N;
  const int H = (L - 1) * ((1 << J) - 1);
  const int vtotal = H + J * kC;
  const int wcap = kC + (L - 1) * (1 << (J - 1));
  double* const wst0 = lds + vtotal;
  double* const wst1 = lds + vtotal + wcap;
  for (int i = tid; i < vtotal + 2 * wcap; i += kNT) lds[i] = 0.0;

  auto vb = [&](int j) -> double* { return lds + (j - 1) * kC + (L - 1) * ((1 << (j - 1)) - 1); };

  const long nchunks = (seg_end - P + kC - 1) / kC;
  const long steps = nchunks + warm / kC;
  double pre[kLoad];
  double wreg[kWinPer];
  bool bad = false;

  auto load_chunk = [&](const double* row, long a0) {
    const long base = wrap(a0, N);
#pragma unroll
    for (int r = 0; r < kLoad; ++r) {
      const long p = base + tid + r * kNT;
      pre[r] = row[p < N ? p : wrap(p, N)];
    }
  };
  // W_j window [a, a + C + hist_j) -> registers.
  auto load_window = [&](int j, long a0) {
    const double* row = cs + (long)(j - 1) * N;
    const int win = kC + (L - 1) * (1 << (j - 1));
    const long base = wrap(a0, N);
#pragma unroll
    for (int r = 0; r < kWinPer; ++r) {
      const int e = tid + r * kNT;
      if (e < win) {
        const long p = base + e;
        wreg[r] = row[p < N ? p : wrap(p, N)];
      }
    }
  };
  auto store_window = [&](int j, double* w) {
    const int win = kC + (L - 1) * (1 << (j - 1));
#pragma unroll
    for (int r = 0; r < kWinPer; ++r) {
      const int e = tid + r * kNT;
      if (e < win) w[e] = wreg[r];
    }
  };

  long a = P + (steps - 1) * kC;
  load_chunk(cs + (long)J * N, a);
  __syncthreads();

  for (long s = 0; s < steps; ++s, a -= kC) {
    // V_J chunk into VB_J[0..C); W_J window into staging 0.
    double* vJ = vb(J);
#pragma unroll
    for (int r = 0; r < kLoad; ++r) vJ[tid + r * kNT] = pre[r];
    load_window(J, a);
    store_window(J, wst0);
    if (s + 1 < steps) load_chunk(cs + (long)J * N, a - kC);
    __syncthreads();

    bool cur0 = true;
    for (int j = J; j >= 1; --j) {
      const int d = 1 << (j - 1);
      const double* vsrc = vb(j);
      const double* wsrc = cur0 ? wst0 : wst1;
      if (j > 1) load_window(j - 1, a);  // in flight during this level's arithmetic
      double* vdst = (j > 1) ? vb(j - 1) : nullptr;
      auto emit = [&](int i, double v) {
        if constexpr (FIX) {
          // vFromApprox and vFromDetail (:366-369) are NaN on a zero-tap hit of their window
          if (zero_tap_nonfinite<1>(vsrc + i, d, (L - 1) * d + 1) ||
              zero_tap_nonfinite<1>(wsrc + i, d, (L - 1) * d + 1))
            v = kNaN;
        }
        if (j > 1) {
          vdst[i] = v;
        } else {
          const long pos = a + i;
          if (pos >= P && pos < seg_end) xs[pos] = v;
          bad |= !__builtin_isfinite(v);
        }
      };
      if (2 * d <= kC) {
        for (int t = tid; t < kC / 2; t += kNT) {
          const int i1 = ((t >> (j - 1)) << j) + (t & (d - 1));
          double vv[L + 1], ww[L + 1];
#pragma unroll
          for (int k = 0; k <= L; ++k) {
            vv[k] = vsrc[i1 + k * d];
            ww[k] = wsrc[i1 + k * d];
          }
          double a1 = 0.0, d1 = 0.0, a2 = 0.0, d2 = 0.0;
#pragma unroll
          for (int m = 0; m < L; ++m) {
            a1 = madd<FMA>(a1, taps.a[m], vv[m]);
            d1 = madd<FMA>(d1, taps.b[m], ww[m]);
            a2 = madd<FMA>(a2, taps.a[m], vv[m + 1]);
            d2 = madd<FMA>(d2, taps.b[m], ww[m + 1]);
          }
          emit(i1, a1 + d1);
          emit(i1 + d, a2 + d2);
        }
      } else {
        for (int i = tid; i < kC; i += kNT) {
          double ap = 0.0, dp = 0.0;
#pragma unroll
          for (int m = 0; m < L; ++m) {
            ap = madd<FMA>(ap, taps.a[m], vsrc[i + m * d]);
            dp = madd<FMA>(dp, taps.b[m], wsrc[i + m * d]);
          }
          emit(i, ap + dp);
        }
      }
      if (j > 1) store_window(j - 1, cur0 ? wst1 : wst0);
      __syncthreads();
      cur0 = !cur0;
    }

    // History shift: VB_j[0 .. hist_j) -> VB_j[C .. C + hist_j) (V_j at [a, a+hist_j) is
    // the right-hand history of the next chunk [a - C, a)).  Flat index e: VB_j starts at
    // flat offset + (j-1)*C, so src = e + (j-1)*C and dst = e + j*C.
    if constexpr (L > 1) {
      double hv[kHistPer];
#pragma unroll
      for (int r = 0; r < kHistPer; ++r) {
        const int e = tid + r * kNT;
        if (e < H) hv[r] = lds[e + (level_of<L>(e) - 1) * kC];
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kHistPer; ++r) {
        const int e = tid + r * kNT;
        if (e < H) lds[e + level_of<L>(e) * kC] = hv[r];
      }
    }
    __syncthreads();
  }
  if constexpr (!FIX) fast::nonfinite_flag(nf, bad);
}

// ---------------------------------------------------------------------------------------
// Per-level kernels: any N, L, J (used when the fused buffers exceed the LDS budget).
// ---------------------------------------------------------------------------------------
// fin (nullable): per-signal flag "the input row holds a non-finite value"; when set, every
// output gets the zero-tap test.  fout (nullable): set when the V output holds one.
template <int L, bool FMA>
__global__ __launch_bounds__(kNT) void modwt_fwd_level(const double* __restrict__ v, long v_stride,
                                                       double* __restrict__ w, long w_stride,
                                                       double* __restrict__ vn, long vn_stride,
                                                       long N, long d, Taps taps,
                                                       const int* __restrict__ fin,
                                                       int* __restrict__ fout) {
  const long n = (long)blockIdx.x * kNT + threadIdx.x;
  const bool live = n < N;  // dead tail lanes stay for the wave-wide zero-tap walk
  const long nn = live ? n : N - 1;
  const double* vs = v + (long)blockIdx.y * v_stride;
  double wa = 0.0, ga = 0.0;
#pragma unroll
  for (int m = 0; m < L; ++m) {
    const double xv = vs[wrap(nn - m * d, N)];
    wa = madd<FMA>(wa, taps.b[m], xv);
    ga = madd<FMA>(ga, taps.a[m], xv);
  }
  if (fin != nullptr && fin[blockIdx.y] != 0) {
    if (zero_tap_nonfinite_wave<false>(vs, N, n, (long)(L - 1) * d + 1, d)) wa = ga = kNaN;
  }
  if (!live) return;
  w[(long)blockIdx.y * w_stride + n] = wa;
  vn[(long)blockIdx.y * vn_stride + n] = ga;
  if (fout != nullptr && !__builtin_isfinite(ga)) fout[blockIdx.y] = 1;
}

// fa / fb (nullable): flags of the V_j / W_j input rows; fout: set when the output holds a
// non-finite value.
template <int L, bool FMA>
__global__ __launch_bounds__(kNT) void modwt_inv_level(const double* __restrict__ v, long v_stride,
                                                       const double* __restrict__ w, long w_stride,
                                                       double* __restrict__ out, long out_stride,
                                                       long N, long d, Taps taps,
                                                       const int* __restrict__ fa,
                                                       const int* __restrict__ fb,
                                                       int* __restrict__ fout) {
  const long n = (long)blockIdx.x * kNT + threadIdx.x;
  const bool live = n < N;
  const long nn = live ? n : N - 1;
  const double* vs = v + (long)blockIdx.y * v_stride;
  const double* ws = w + (long)blockIdx.y * w_stride;
  double ap = 0.0, dp = 0.0;
#pragma unroll
  for (int m = 0; m < L; ++m) {
    const long idx = wrap(nn + m * d, N);
    ap = madd<FMA>(ap, taps.a[m], vs[idx]);
    dp = madd<FMA>(dp, taps.b[m], ws[idx]);
  }
  double o = ap + dp;
  if ((fa != nullptr && fa[blockIdx.y] != 0) || (fb != nullptr && fb[blockIdx.y] != 0)) {
    const long M = (long)(L - 1) * d + 1;
    const bool hv = zero_tap_nonfinite_wave<true>(vs, N, n, M, d);
    const bool hw = zero_tap_nonfinite_wave<true>(ws, N, n, M, d);
    if (hv || hw) o = kNaN;
  }
  if (!live) return;
  out[(long)blockIdx.y * out_stride + n] = o;
  if (fout != nullptr && !__builtin_isfinite(o)) fout[blockIdx.y] = 1;
}

// ---------------------------------------------------------------------------------------
// Host-side dispatch
// ---------------------------------------------------------------------------------------
constexpr size_t kMaxFusedLds = 80 * 1024;
constexpr size_t kMaxFixLds = 160 * 1024;  // the zero-tap pass may take a CU's whole LDS

size_t fused_lds_bytes(int L, int J, bool inverse) {
  const long H = (long)(L - 1) * ((1L << J) - 1);
  long doubles = H + (long)J * kC;
  if (inverse) doubles += 2 * (kC + hist_of(L, J));
  return (size_t)doubles * sizeof(double);
}

bool fused_fits(int L, int J, bool inverse, size_t max_lds) {
  const long H = (long)(L - 1) * ((1L << J) - 1);
  if (H > kHistMax) return false;
  if (inverse && kC + hist_of(L, J) > kWinMax) return false;
  return fused_lds_bytes(L, J, inverse) <= max_lds;
}
bool fused_ok(int L, int J, bool inverse) { return fused_fits(L, J, inverse, kMaxFusedLds); }
// The streaming kernels (fast or generic) may run only where their zero-tap pass can follow.
bool fix_ok(int L, int J, bool inverse) { return fused_fits(L, J, inverse, kMaxFixLds); }

// Segment length: whole chunks, long enough that the warm-up is a small fraction, short
// enough that the grid has several workgroups per CU.
long pick_segment(long N, int batch, long warm) {
  const long nchunks = (N + kC - 1) / kC;
  long min_chunks = (8 * warm) / kC;
  if (min_chunks < 1) min_chunks = 1;
  long seg_chunks = nchunks;
  const long want_blocks = 4096;
  while (seg_chunks > min_chunks &&
         (long)batch * ((nchunks + seg_chunks - 1) / seg_chunks) < want_blocks)
    seg_chunks = (seg_chunks + 1) / 2;
  if (seg_chunks < min_chunks) seg_chunks = min_chunks < nchunks ? min_chunks : nchunks;
  return seg_chunks * kC;
}

template <int L>
Taps make_taps(const ModwtPlan& p) {
  Taps t{};
  for (int i = 0; i < L; ++i) {
    t.a[i] = p.g[i];
    t.b[i] = p.h[i];
  }
  return t;
}

// JW_MODWT_KERNEL=generic forces the runtime-J kernels (A/B and parity testing).
bool fast_enabled() {
  const char* e = knob("JW_MODWT_KERNEL");
  return !(e && std::strcmp(e, "generic") == 0);
}

int try_fast_forward(int L, const Taps& t, bool fma, const double* x, double* c, long N, int J,
                     int B, hipStream_t s, int* nf) {
  if (!fast_enabled()) return fast::kNotHandled;
  switch (L) {
#define JW_CASE(LL) \
  case LL:          \
    return fast::forward<LL>(t, fma, x, c, N, J, B, s, nf);
    JW_FAST_LENGTHS(JW_CASE)
#undef JW_CASE
    default:
      return fast::kNotHandled;
  }
}

int try_fast_inverse(int L, const Taps& t, bool fma, const double* c, double* x, long N, int J,
                     int B, hipStream_t s, int* nf) {
  if (!fast_enabled()) return fast::kNotHandled;
  switch (L) {
#define JW_CASE(LL) \
  case LL:          \
    return fast::inverse<LL>(t, fma, c, x, N, J, B, s, nf);
    JW_FAST_LENGTHS(JW_CASE)
#undef JW_CASE
    default:
      return fast::kNotHandled;
  }
}

// `count` zeroed per-signal flag words, stream-ordered.
int alloc_flags(StreamAllocs& mem, int** f, size_t count, hipStream_t s) {
  JW_HIP_TRY(mem.alloc(f, count * sizeof(int)));
  JW_HIP_TRY(hipMemsetAsync(*f, 0, count * sizeof(int), s));
  return JW_OK;
}

// flags[r * batch + b] for rows r0 .. r0 + nrows - 1 of every signal (signal stride sig).
int scan_rows(const double* p, long sig, long row_stride, int nrows, long N, int batch,
              int* flags, hipStream_t s) {
  long gx = (N + 255) / 256;
  const long want = 4096 / (batch > 0 ? batch : 1);
  if (gx > want) gx = want < 1 ? 1 : want;
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    hipLaunchKernelGGL(modwt_nonfinite_rows, dim3((unsigned)gx, (unsigned)nb), dim3(256), 0, s,
                       p + (long)b0 * sig, sig, row_stride, nrows, N, flags + b0, (long)batch);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

// The generic streaming kernels, main (FIX = false, nf = out flags or null) or zero-tap pass.
template <int L, bool FMA, bool FIX>
int launch_fused_fwd(const Taps& t, const double* x, double* coeffs, long N, int J, int batch,
                     int* nf, hipStream_t s) {
  const size_t lds = fused_lds_bytes(L, J, false);
  const long H = (long)(L - 1) * ((1L << J) - 1);
  const long warm = ((H + kC - 1) / kC) * kC;
  const long seg = pick_segment(N, batch, warm);
  const long nseg = (N + seg - 1) / seg;
  const long rstride = (long)(J + 1) * N;
  auto kern = modwt_fwd_fused<L, FMA, FIX>;
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    hipLaunchKernelGGL(kern, dim3((unsigned)nseg, (unsigned)nb), dim3(kNT), lds, s,
                       x + (long)b0 * N, coeffs + (long)b0 * rstride, N, J, seg, warm, t,
                       nf ? nf + b0 : nullptr);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

template <int L, bool FMA, bool FIX>
int launch_fused_inv(const Taps& t, const double* coeffs, double* x, long N, int J, int batch,
                     int* nf, hipStream_t s) {
  const size_t lds = fused_lds_bytes(L, J, true);
  const long H = (long)(L - 1) * ((1L << J) - 1);
  const long warm = ((H + kC - 1) / kC) * kC;
  const long seg = pick_segment(N, batch, warm);
  const long nseg = (N + seg - 1) / seg;
  const long rstride = (long)(J + 1) * N;
  auto kern = modwt_inv_fused<L, FMA, FIX>;
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    hipLaunchKernelGGL(kern, dim3((unsigned)nseg, (unsigned)nb), dim3(kNT), lds, s,
                       coeffs + (long)b0 * rstride, x + (long)b0 * N, N, J, seg, warm, t,
                       nf ? nf + b0 : nullptr);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

template <int L, bool FMA>
int forward_impl(const ModwtPlan& p, const double* x, double* coeffs, long N, int J, int batch,
                 hipStream_t s) {
  const Taps t = make_taps<L>(p);
  const long rstride = (long)(J + 1) * N;
  StreamAllocs mem(s);
  const bool zt = J >= 2 && L > 1;  // level 1 has no zero taps
  if (!zt || fix_ok(L, J, false)) {
    int* nf = nullptr;
    if (zt) {
      if (int st = alloc_flags(mem, &nf, (size_t)batch, s); st != JW_OK) return st;
    }
    int st = try_fast_forward(L, t, FMA, x, coeffs, N, J, batch, s, nf);
    if (st == fast::kNotHandled && fused_ok(L, J, false))
      st = launch_fused_fwd<L, FMA, false>(t, x, coeffs, N, J, batch, nf, s);
    if (st != fast::kNotHandled) {
      if (st != JW_OK || !zt) return st;
      return launch_fused_fwd<L, FMA, true>(t, x, coeffs, N, J, batch, nf, s);
    }
  }
  // Per-level path: V_j ping-pongs between coefficient row J and a workspace row so that
  // V_J lands in row J.  fl[j] = "V_j of the signal holds a non-finite value".
  double* tmp = nullptr;
  int* fl = nullptr;
  JW_HIP_TRY(mem.alloc(&tmp, sizeof(double) * (size_t)N * batch));
  if (int st = alloc_flags(mem, &fl, (size_t)(J + 1) * batch, s); st != JW_OK) return st;
  const double* vin = x;
  long vin_stride = N;
  for (int j = 1; j <= J; ++j) {
    const bool to_row = ((J - j) % 2) == 0;
    double* vout = to_row ? coeffs + (long)J * N : tmp;
    const long vout_stride = to_row ? rstride : N;
    const int* fin = j >= 2 ? fl + (long)(j - 1) * batch : nullptr;
    int* fout = j < J ? fl + (long)j * batch : nullptr;
    for (int b0 = 0; b0 < batch; b0 += 65535) {
      const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
      dim3 grid((unsigned)((N + kNT - 1) / kNT), (unsigned)nb);
      hipLaunchKernelGGL((modwt_fwd_level<L, FMA>), grid, dim3(kNT), 0, s, vin + b0 * vin_stride,
                         vin_stride, coeffs + (long)(j - 1) * N + b0 * rstride, rstride,
                         vout + b0 * vout_stride, vout_stride, N, 1L << (j - 1), t,
                         fin ? fin + b0 : nullptr, fout ? fout + b0 : nullptr);
    }
    JW_HIP_TRY(hipGetLastError());
    vin = vout;
    vin_stride = vout_stride;
  }
  return JW_OK;
}

template <int L, bool FMA>
int inverse_impl(const ModwtPlan& p, const double* coeffs, double* x, long N, int J, int batch,
                 hipStream_t s) {
  const Taps t = make_taps<L>(p);
  const long rstride = (long)(J + 1) * N;
  StreamAllocs mem(s);
  const bool zt = J >= 2 && L > 1;
  if (!zt || fix_ok(L, J, true)) {
    int* nf = nullptr;
    if (zt) {
      if (int st = alloc_flags(mem, &nf, (size_t)batch, s); st != JW_OK) return st;
    }
    int st = try_fast_inverse(L, t, FMA, coeffs, x, N, J, batch, s, nf);
    if (st == fast::kNotHandled && fused_ok(L, J, true))
      st = launch_fused_inv<L, FMA, false>(t, coeffs, x, N, J, batch, nf, s);
    if (st != fast::kNotHandled) {
      if (st != JW_OK || !zt) return st;
      return launch_fused_inv<L, FMA, true>(t, coeffs, x, N, J, batch, nf, s);
    }
  }
  // Per-level path.  fr[r] = "coefficient row r holds a non-finite value" (one scan),
  // fv[j] = "V_j (level j+1's output) does".
  double* tmp = nullptr;
  int *fr = nullptr, *fv = nullptr;
  JW_HIP_TRY(mem.alloc(&tmp, sizeof(double) * (size_t)N * batch));
  if (int st = alloc_flags(mem, &fr, (size_t)(2 * J + 1) * batch, s); st != JW_OK) return st;
  fv = fr + (long)(J + 1) * batch - (long)batch;  // fv[j] at fv + j*batch, j = 1..J-1
  if (int st = scan_rows(coeffs, rstride, N, J + 1, N, batch, fr, s); st != JW_OK) return st;
  const double* vin = coeffs + (long)J * N;
  long vin_stride = rstride;
  for (int j = J; j >= 1; --j) {
    const bool to_out = ((j - 1) % 2) == 0;
    double* vout = to_out ? x : tmp;
    const int* fa = j == 1 ? nullptr : j == J ? fr + (long)J * batch : fv + (long)j * batch;
    const int* fb = j == 1 ? nullptr : fr + (long)(j - 1) * batch;
    int* fout = j > 1 ? fv + (long)(j - 1) * batch : nullptr;
    for (int b0 = 0; b0 < batch; b0 += 65535) {
      const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
      dim3 grid((unsigned)((N + kNT - 1) / kNT), (unsigned)nb);
      hipLaunchKernelGGL((modwt_inv_level<L, FMA>), grid, dim3(kNT), 0, s, vin + b0 * vin_stride,
                         vin_stride, coeffs + (long)(j - 1) * N + b0 * rstride, rstride,
                         vout + b0 * N, N, N, 1L << (j - 1), t, fa ? fa + b0 : nullptr,
                         fb ? fb + b0 : nullptr, fout ? fout + b0 : nullptr);
    }
    JW_HIP_TRY(hipGetLastError());
    vin = vout;
    vin_stride = N;
  }
  return JW_OK;
}

#define JW_MODWT_LENGTHS(X)                                                                  \
  X(1) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22) X(24) X(26) X(28) X(30) \
  X(32) X(34) X(36) X(38) X(40)

template <bool FMA>
int forward_dispatch(const ModwtPlan& p, const double* x, double* c, long N, int J, int B,
                     hipStream_t s) {
  switch (p.L) {
#define JW_CASE(LL) \
  case LL:          \
    return forward_impl<LL, FMA>(p, x, c, N, J, B, s);
    JW_MODWT_LENGTHS(JW_CASE)
#undef JW_CASE
    default:
      return fail(JW_ERR_UNSUPPORTED, "MODWT: filter length %d is not built into this library",
                  p.L);
  }
}

template <bool FMA>
int inverse_dispatch(const ModwtPlan& p, const double* c, double* x, long N, int J, int B,
                     hipStream_t s) {
  switch (p.L) {
#define JW_CASE(LL) \
  case LL:          \
    return inverse_impl<LL, FMA>(p, c, x, N, J, B, s);
    JW_MODWT_LENGTHS(JW_CASE)
#undef JW_CASE
    default:
      return fail(JW_ERR_UNSUPPORTED, "MODWT: filter length %d is not built into this library",
                  p.L);
  }
}

// One DIRECT level of the AUTO / STRICT level schedule (jw_jfft*.hip): its input rows may come
// from an FFT level, so they are scanned for non-finite values first (levels >= 2 only).
template <int L, bool FMA>
int level_forward(const ModwtPlan& p, int j, const double* v, long vs, double* w, long ws,
                  double* vn, long vns, long N, int batch, hipStream_t s) {
  const Taps t = make_taps<L>(p);
  StreamAllocs mem(s);
  int* fin = nullptr;
  if (j >= 2 && L > 1) {
    if (int st = alloc_flags(mem, &fin, (size_t)batch, s); st != JW_OK) return st;
    if (int st = scan_rows(v, vs, 0, 1, N, batch, fin, s); st != JW_OK) return st;
  }
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    dim3 grid((unsigned)((N + kNT - 1) / kNT), (unsigned)nb);
    hipLaunchKernelGGL((modwt_fwd_level<L, FMA>), grid, dim3(kNT), 0, s, v + b0 * vs, vs,
                       w + b0 * ws, ws, vn + b0 * vns, vns, N, 1L << (j - 1), t,
                       fin ? fin + b0 : nullptr, nullptr);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

template <int L, bool FMA>
int level_inverse(const ModwtPlan& p, int j, const double* v, long vs, const double* w, long ws,
                  double* out, long os, long N, int batch, hipStream_t s) {
  const Taps t = make_taps<L>(p);
  StreamAllocs mem(s);
  int* f = nullptr;
  if (j >= 2 && L > 1) {
    if (int st = alloc_flags(mem, &f, (size_t)2 * batch, s); st != JW_OK) return st;
    if (int st = scan_rows(v, vs, 0, 1, N, batch, f, s); st != JW_OK) return st;
    if (int st = scan_rows(w, ws, 0, 1, N, batch, f + batch, s); st != JW_OK) return st;
  }
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    dim3 grid((unsigned)((N + kNT - 1) / kNT), (unsigned)nb);
    hipLaunchKernelGGL((modwt_inv_level<L, FMA>), grid, dim3(kNT), 0, s, v + b0 * vs, vs,
                       w + b0 * ws, ws, out + b0 * os, os, N, 1L << (j - 1), t,
                       f ? f + b0 : nullptr, f ? f + batch + b0 : nullptr, nullptr);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace

int modwt_level_forward_device(const ModwtPlan& p, int j, const double* v, long vs, double* w,
                               long ws, double* vn, long vns, long N, int batch, hipStream_t s) {
  const bool fma = p.arith == JW_ARITH_FMA;
  switch (p.L) {
#define JW_CASE(LL)                                                                        \
  case LL:                                                                                 \
    return fma ? level_forward<LL, true>(p, j, v, vs, w, ws, vn, vns, N, batch, s)         \
               : level_forward<LL, false>(p, j, v, vs, w, ws, vn, vns, N, batch, s);
    JW_MODWT_LENGTHS(JW_CASE)
#undef JW_CASE
    default:
      return fail(JW_ERR_UNSUPPORTED, "MODWT: filter length %d is not built into this library",
                  p.L);
  }
}

int modwt_level_inverse_device(const ModwtPlan& p, int j, const double* v, long vs,
                               const double* w, long ws, double* out, long os, long N, int batch,
                               hipStream_t s) {
  const bool fma = p.arith == JW_ARITH_FMA;
  switch (p.L) {
#define JW_CASE(LL)                                                                        \
  case LL:                                                                                 \
    return fma ? level_inverse<LL, true>(p, j, v, vs, w, ws, out, os, N, batch, s)         \
               : level_inverse<LL, false>(p, j, v, vs, w, ws, out, os, N, batch, s);
    JW_MODWT_LENGTHS(JW_CASE)
#undef JW_CASE
    default:
      return fail(JW_ERR_UNSUPPORTED, "MODWT: filter length %d is not built into this library",
                  p.L);
  }
}

int modwt_forward_device(const ModwtPlan& p, const double* x, double* coeffs, long n, int J,
                         int batch, hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? forward_dispatch<true>(p, x, coeffs, n, J, batch, s)
                                 : forward_dispatch<false>(p, x, coeffs, n, J, batch, s);
}

int modwt_inverse_device(const ModwtPlan& p, const double* coeffs, double* x, long n, int J,
                         int batch, hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? inverse_dispatch<true>(p, coeffs, x, n, J, batch, s)
                                 : inverse_dispatch<false>(p, coeffs, x, n, J, batch, s);
}

}  // namespace jw
