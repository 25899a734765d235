// jw_jfft_host.hpp -- host-side helpers of the JW_ARITH_STRICT FFT paths (jw_jfft.hip,
// jw_jfft_bs.hip): twiddle tables, launch helpers, functors, natural-order transforms of rows.
#pragma once
#include <algorithm>
#include <type_traits>

#include "jw_jfft.hpp"

namespace jw {
namespace jf {

constexpr long kLineMax = 4096;  // whole transform in one column up to here

constexpr size_t kCacheBytes = 2UL << 30;  // per table cache

struct Tw {
  long n = 0;
  int lc1 = 0;
  const cplx* p1 = nullptr;
  const cplx* p2 = nullptr;
};

// pass-1 length of an n-point transform (n itself when it runs in one column)
inline int split_lc1(long n) { return n <= kLineMax ? (int)n : 1 << (ilog2(n) / 2); }

// Power-of-two transforms from here on run as three column passes (n = A x B x C, each a
// column of 64 .. 4096 points): the two-pass split stops at 4096 x 4096 = 2^24.  2^25 by
// default; env JW_JFFT_3PASS_MIN (a power of two >= 2^18) lowers it, so the tests can check the
// three-pass code against the oracle at sizes the oracle finishes quickly.
long three_pass_min();
// Plain transforms (jw_fft STRICT, filter spectra, Bluestein's b) switch earlier: from 2^23 the
// three-pass split (columns of 2^11..2^12 x 2^6 x 2^6) beats the two 2^11..2^12-point column
// passes: 4.43 -> 3.18 ms at 2^23, 4.82 -> 3.54 ms at 2^24 per 128 Mi points, equal at 2^22
// (profiles/r06/ab/ept_big/fft3.txt).  MODWT's fused levels and Bluestein's fused convolution
// stay two-pass up to three_pass_min(): unfused three passes measured slower there (AUTO db4 J=4
// at 2^22: 1,922 vs 1,273 Msamples/s; Bluestein m = 2^23: 2.73 vs 3.19 ms).
inline long plain_three_pass_min() { return std::min(three_pass_min(), 1L << 23); }
constexpr long kStrictPow2Max = kStrictFftPow2Max;  // the longest power-of-two STRICT transform
// bits of A, B, C for a three-pass n = 2^lg (18 <= lg <= 36)
inline void split3(int lg, int* a, int* b, int* c) {
  *a = std::min(12, lg - 12);
  const int rem = lg - *a;
  *b = std::max(6, rem - 12);
  *c = rem - *b;
}

// Twiddles of an n-point transform in the reference's recurrence order, laid out for a split
// with pass-1 length lc1 (jw_jfft.hip); cached per (device, n, direction, lc1).
int twiddles(long n, bool inverse, int lc1, Tw* out, StreamAllocs& mem, hipStream_t s);

// Twiddles of a three-pass transform: p1 = Tw[0 .. A) (pass 1, natural), pm[l B + m] =
// Tw[m A + l] (pass 2 over planes of [B][A], l < A, m < B), p3[l C + m] = Tw[m A B + l] (pass 3,
// l < A B, m < C); Tw in the reference's recurrence order.
struct Tw3 {
  long n = 0;
  int A = 0, B = 0, C = 0;
  const cplx* p1 = nullptr;
  const cplx* pm = nullptr;
  const cplx* p3 = nullptr;
};
int twiddles3(long n, bool inverse, Tw3* out, StreamAllocs& mem, hipStream_t s);

// ---------------------------------------------------------------------------------------
// Launch helpers: runtime column length -> template instantiation
// ---------------------------------------------------------------------------------------
#define JF_CASE(V) \
  case V:          \
    return f(std::integral_constant<int, V>{});

template <class F>
inline int with_lc(long lc, F&& f) {
  switch (lc) {
    JF_CASE(2) JF_CASE(4) JF_CASE(8) JF_CASE(16) JF_CASE(32) JF_CASE(64) JF_CASE(128)
    JF_CASE(256) JF_CASE(512) JF_CASE(1024) JF_CASE(2048) JF_CASE(4096)
    default:
      return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: line length %ld unsupported", lc);
  }
}
template <class F>
inline int with_big_lc(long lc, F&& f) {
  switch (lc) {
    JF_CASE(64) JF_CASE(128) JF_CASE(256) JF_CASE(512) JF_CASE(1024) JF_CASE(2048) JF_CASE(4096)
    default:
      return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: column length %ld unsupported", lc);
  }
}
#undef JF_CASE

template <int LC, int E = 0, class K, class... A>
int launch_grid(K kern, long blocks, hipStream_t s, A... args) {
  const size_t lds = Geo<LC, E>::LDS_BYTES;
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  if (blocks <= 0) return JW_OK;
  if (blocks >= (1L << 24))
    return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: grid of %ld workgroups", blocks);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kNT), lds, s, args...);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

// kp2p_w (1024-point columns, 8 per workgroup): its own LDS size
template <class K, class... A>
int launch_wcol(K kern, long blocks, hipStream_t s, A... args) {
  const size_t lds = wcol::LDS_BYTES;
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  if (blocks <= 0) return JW_OK;
  if (blocks >= (1L << 24))
    return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: grid of %ld workgroups", blocks);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kNT), lds, s, args...);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}
// JW_AUTO_WCOL=1 (A/B setting): kp2p's 1024-point columns through kp2p_w
inline bool use_wcol() {
  const char* e = knob("JW_AUTO_WCOL");
  return e && e[0] == '1';
}

// ---------------------------------------------------------------------------------------
// Functors (natural indices; see jw_jfft.hpp)
// ---------------------------------------------------------------------------------------
struct RowsR {  // real rows -> Complex(x, 0) (:766-769)
  const double* p;
  long st;
  __device__ cplx operator()(long it, long i) const { return make_double2(p[it * st + i], 0.0); }
};
struct RowsC {
  const cplx* p;
  long st;
  __device__ cplx operator()(long it, long i) const { return p[it * st + i]; }
};
struct OutC {
  cplx* p;
  long st;
  __device__ void operator()(long it, long i, cplx v) const { p[it * st + i] = v; }
};
struct OutCS {  // x[i].mul(1.0 / n) for a reverse transform (FastFourierTransform.java:207-211)
  cplx* p;
  long st;
  double sc;
  int do_scale;
  __device__ void operator()(long it, long i, cplx v) const {
    p[it * st + i] = do_scale ? jscale(v, sc) : v;
  }
};
struct OutR {
  double* p;
  long st;
  __device__ void operator()(long it, long i, double v) const { p[it * st + i] = v; }
};
// result[i].mul(1.0 / n).getReal() of a reverse transform (:207-211, :781-783) into a real row;
// ADD: added to the value already there (vFromApprox[i] + vFromDetail[i], :366-369)
template <bool ADD>
struct OutRe {
  double* p;
  long st;
  double sc;
  __device__ void operator()(long it, long i, cplx v) const {
    const double r = v.x * sc;
    if constexpr (ADD) {
      p[it * st + i] = p[it * st + i] + r;
    } else {
      p[it * st + i] = r;
    }
  }
};
// the middle pass of a three-pass transform: item it' = item * C + plane o, natural index
// i = h A + l of the plane's [B][A] view at o A B + i of the item's n points (read and written
// in place: a workgroup writes exactly the points it read)
struct Plane {
  cplx* p;
  long n, ab;
  int cbits;
  __device__ cplx operator()(long it, long i) const {
    return p[(it >> cbits) * n + (it & ((1L << cbits) - 1)) * ab + i];
  }
  __device__ void operator()(long it, long i, cplx v) const {
    p[(it >> cbits) * n + (it & ((1L << cbits) - 1)) * ab + i] = v;
  }
};
// NF row outputs, stream f at p + f * fst
struct OutF {
  cplx* p;
  long st, fst;
  __device__ void operator()(int f, long it, long j, cplx v) const { p[f * fst + it * st + j] = v; }
};
// NIN column inputs, stream s at p + s * sst
struct InS {
  const cplx* p;
  long st, sst;
  __device__ cplx operator()(int s, long it, long i) const { return p[s * sst + it * st + i]; }
};
struct PowPost {  // result[i].mul(1.0 / n).getReal() (:207-211, :781-783)
  double inv_n;
  __device__ double operator()(int, long, long, cplx v) const { return v.x * inv_n; }
};
// forward level, one filter per item: item 2 sig + f reads signal sig's spectrum (Z rows of
// sig) and takes signalFFT[i].mul(filterFFT[i]) with f = 0 -> h_j (W_j), 1 -> g_j (V_j)
// (:775-778).  The two items of a signal are adjacent, so they run back to back on one XCD
// (tile_item) and the second one's Z column tile comes from L2.
struct ZPair {
  const cplx* p;
  long st;
  __device__ cplx operator()(long it, long i) const { return p[(it >> 1) * st + i]; }
};
struct FwdMid {
  const cplx* fh;
  const cplx* fg;
  __device__ cplx operator()(int, long it, long i, cplx x) const {
    return jmul(x, ((it & 1) ? fg : fh)[i]);
  }
};
// The same products with the filter spectra stored per column of the kp2p view (FT[l C + h] =
// F[h R + l], l < R columns, h < C points; jw_jfft.hip spectra_t): the lanes of a column read
// consecutive entries instead of one 16-byte value per 16 KB row (natural order).
struct FwdMidT {
  const cplx* fh;
  const cplx* fg;
  int rbits;
  long C;
  __device__ cplx operator()(int, long it, long i, cplx x) const {
    const long t = (i & ((1L << rbits) - 1)) * C + (i >> rbits);
    return jmul(x, ((it & 1) ? fg : fh)[t]);
  }
};
struct AdjMidT {
  const cplx* fg;
  const cplx* fh;
  long nb;
  int rbits;
  long C;
  __device__ cplx operator()(int, long it, long i, cplx x) const {
    const long t = (i & ((1L << rbits) - 1)) * C + (i >> rbits);
    const cplx f = (it < nb ? fg : fh)[t];
    return jmul(x, make_double2(f.x, -f.y));
  }
};
struct OutPair {  // item 2 sig + f -> stream f's row sig
  cplx* p;
  long st, fst;
  __device__ void operator()(int, long it, long j, cplx v) const {
    p[(it & 1) * fst + (it >> 1) * st + j] = v;
  }
};
// adjoint: signalFFT[i].mul(filterFFT[i].conjugate()) (:820-824); items [0, nb) are V_j (g_j),
// [nb, 2 nb) are W_j (h_j)
struct AdjMid {
  const cplx* fg;
  const cplx* fh;
  long nb;
  __device__ cplx operator()(int, long it, long i, cplx x) const {
    const cplx f = (it < nb ? fg : fh)[i];
    return jmul(x, make_double2(f.x, -f.y));
  }
};
// line kernels (n <= kLineMax)
struct LineIn {
  const double* p0;
  long st0;
  const double* p1;
  long st1;
  __device__ double operator()(int s, long ln, int r) const {
    return s == 0 ? p0[ln * st0 + r] : p1[ln * st1 + r];
  }
};
struct LineOut {
  double* p0;
  long st0;
  double* p1;
  long st1;
  __device__ void operator()(int f, long ln, int r, double v) const {
    if (f == 0) {
      p0[ln * st0 + r] = v;
    } else {
      p1[ln * st1 + r] = v;
    }
  }
};
struct LineFwdMid {
  const cplx* fh;
  const cplx* fg;
  __device__ cplx operator()(int, int f, long i, cplx x) const { return jmul(x, (f ? fg : fh)[i]); }
};
struct LineAdjMid {  // s = 0: V_j with g_j, s = 1: W_j with h_j
  const cplx* fg;
  const cplx* fh;
  __device__ cplx operator()(int s, int, long i, cplx x) const {
    const cplx f = (s ? fh : fg)[i];
    return jmul(x, make_double2(f.x, -f.y));
  }
};

// ---------------------------------------------------------------------------------------
// Natural-order transforms of `items` rows: in (RowsR / RowsC) -> out (OutCS)
// ---------------------------------------------------------------------------------------
// Three column passes (n >= three_pass_min()): pass 1 = the first log A stages on the
// bit-reversed blocks of A points (kp1, rows of Z), pass 2 = the next log B stages on columns of
// stride A within each plane of A B points (kp2s in place), pass 3 = the last log C stages on
// columns of stride A B (kp2s into Out).  Same butterflies, same twiddles, same order as the
// two-pass split: stage t pairs positions p, p + 2^t with Tw[2^t + p mod 2^t] whatever the
// pass boundaries (jw_jfft.hpp).
template <class In, class Out>
inline int fft_rows3(long n, bool inverse, long items, In in, Out out, StreamAllocs& mem,
                     hipStream_t s) {
  Tw3 tw;
  int st = twiddles3(n, inverse, &tw, mem, s);
  if (st != JW_OK) return st;
  const int abits = ilog2(tw.A), cbits = ilog2(tw.C);
  const long ab = (long)tw.A * tw.B;
  const long chunk = std::max(1L, std::min<long>(items, (1L << 30) / (n * (long)sizeof(cplx))));
  cplx* Z = nullptr;
  JW_HIP_TRY(mem.alloc(&Z, (size_t)chunk * n * sizeof(cplx)));
  for (long i0 = 0; i0 < items && st == JW_OK; i0 += chunk) {
    const long ni = std::min(chunk, items - i0);
    In in_c = in;
    in_c.p += i0 * in.st;
    Out out_c = out;
    out_c.p += i0 * out.st;
    st = with_big_lc(tw.A, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC, kPlainEPT<LC>>(kp1<LC, In, OutC, kPlainEPT<LC>>,
                                            (n / tw.A / PlainGeo<LC>::T) * ni, s, in_c,
                                            OutC{Z, n}, ilog2(n / tw.A), ni, tw.p1);
    });
    if (st != JW_OK) break;
    st = with_big_lc(tw.B, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      const Plane pl{Z, n, ab, cbits};
      return launch_grid<LC, kPlainEPT<LC>>(kp2s<LC, Plane, Plane, kPlainEPT<LC>>,
                                            (tw.A / PlainGeo<LC>::T) * ni * tw.C, s, pl, pl,
                                            abits, ni * tw.C, tw.pm);
    });
    if (st != JW_OK) break;
    st = with_big_lc(tw.C, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC, kPlainEPT<LC>>(kp2s<LC, RowsC, Out, kPlainEPT<LC>>,
                                            (ab / PlainGeo<LC>::T) * ni, s, RowsC{Z, n}, out_c,
                                            ilog2(ab), ni, tw.p3);
    });
  }
  return st;
}

template <class In, class Out = OutCS>
inline int fft_rows(long n, bool inverse, long items, In in, Out out, StreamAllocs& mem,
             hipStream_t s) {
  if (n > kLineMax && n >= plain_three_pass_min())
    return fft_rows3(n, inverse, items, in, out, mem, s);
  const int lc1 = split_lc1(n);
  Tw tw;
  int st = twiddles(n, inverse, lc1, &tw, mem, s);
  if (st != JW_OK) return st;
  if (n <= kLineMax) {
    return with_lc(n, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC, kLineEPT<LC>>(kline_fft<LC, In, Out>,
                                           (items + LineGeo<LC>::T - 1) / LineGeo<LC>::T, s,
                             in, out, items, tw.p1, 1.0, 0);
    });
  }
  const long lc2 = n / lc1;
  const long chunk = std::max(1L, std::min<long>(items, (1L << 30) / (n * (long)sizeof(cplx))));
  cplx* Z = nullptr;
  JW_HIP_TRY(mem.alloc(&Z, (size_t)chunk * n * sizeof(cplx)));
  for (long i0 = 0; i0 < items && st == JW_OK; i0 += chunk) {
    const long ni = std::min(chunk, items - i0);
    In in_c = in;
    in_c.p += i0 * in.st;
    Out out_c = out;
    out_c.p += i0 * out.st;
    st = with_big_lc(lc1, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC, kPlainEPT<LC>>(kp1<LC, In, OutC, kPlainEPT<LC>>,
                                            (lc2 / PlainGeo<LC>::T) * ni, s, in_c, OutC{Z, n},
                                            ilog2(lc2), ni, tw.p1);
    });
    if (st != JW_OK) break;
    st = with_big_lc(lc2, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC, kPlainEPT<LC>>(kp2s<LC, RowsC, Out, kPlainEPT<LC>>,
                                            (lc1 / PlainGeo<LC>::T) * ni, s, RowsC{Z, n},
                                            out_c, ilog2(lc1), ni, tw.p2);
    });
  }
  return st;
}

// Lengths that are not powers of two (jw_jfft_bs.hip): the reference's Bluestein transform.
int bs_spectra_real(long n, long items, const double* rows, cplx* out, StreamAllocs& mem,
                    hipStream_t s);
int bs_fft_strict(bool inverse, const cplx* in, cplx* out, long n, long batch, hipStream_t s);
int modwt_strict_bs(bool inverse, const ModwtPlan& p, const double* in, double* out, long N,
                    int J, int batch, const bool* fft, const cplx* F, StreamAllocs& mem,
                    hipStream_t s);

}  // namespace jf
}  // namespace jw
