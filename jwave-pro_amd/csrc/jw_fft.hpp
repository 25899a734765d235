// jw_fft.hpp -- power-of-two complex FFT building blocks for the FFT paths (CWT transformFFT,
// MODWT FFT convolution).  Replaces FastFourierTransform.forward/reverse
// (src/main/java/jwave/transforms/FastFourierTransform.java:112-212) for power-of-two n.
//
// Layout: complex double as double2 (re, im), interleaved, batch-major.
// Direction S: -1 forward (e^{-2 pi i nk/N}), +1 reverse (e^{+2 pi i nk/N}, then x 1/N like
// FastFourierTransform.reverse :207-211).  The reference computes twiddles by recurrence
// (w_n = w_n * w, :188-201); this engine uses correctly rounded tables (cos/sin in long double
// on the host), so it is at least as accurate -- results agree to ~1e-12 normwise at 2^18.
//
// Long transforms use the four-step split N = N1 * N2 (input index k = N2*k1 + k2, output index
// n = n1 + N1*n2):
//   pass 1: for every column k2, an N1-point FFT over k1, times W_N^(n1*k2)   -> A[n1][k2]
//   pass 2: for every row n1, an N2-point FFT over k2                          -> x[n1 + N1*n2]
// Sub-transforms of 512 points run on one wavefront each (radix 8 x 8 x 8 in registers, two
// LDS transposes); other sizes use a workgroup radix-2 kernel (correct, not tuned).
#pragma once
#include "jw_internal.hpp"

namespace jw {
namespace fft {

using cplx = double2;

__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cplx csub(cplx a, cplx b) { return make_double2(a.x - b.x, a.y - b.y); }
// a * w^S for a table entry w = e^{+i theta} (S = -1 uses the conjugate).  This engine is the
// exact-twiddle one (tolerance contract, not the reference's operation order -- that is
// jw_jfft.hpp), so the complex products use fused multiply-adds: two FP64 instructions fewer per
// product, and at FP64 every wave64 VALU instruction holds its SIMD four cycles.
template <int S>
__device__ __forceinline__ cplx cmul_tw(cplx a, cplx w) {
  const double wy = S > 0 ? w.y : -w.y;
  return make_double2(__builtin_fma(a.x, w.x, -(a.y * wy)), __builtin_fma(a.x, wy, a.y * w.x));
}
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
  return make_double2(__builtin_fma(a.x, b.x, -(a.y * b.y)), __builtin_fma(a.x, b.y, a.y * b.x));
}

// In-register 8-point DFT, v[q] <- sum_r v[r] e^{S 2 pi i r q / 8} (radix-2 DIF, bit-reversed
// positions undone at the end).
template <int S>
__device__ __forceinline__ void dft8(cplx (&v)[8]) {
  constexpr double h = 0.70710678118654752440;
  cplx t[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    t[r] = cadd(v[r], v[r + 4]);
    t[r + 4] = csub(v[r], v[r + 4]);
  }
  // t[4+r] *= W8^r
  {
    const cplx a = t[5];
    t[5] = make_double2(h * (a.x - S * a.y), h * (S * a.x + a.y));
    const cplx b = t[6];
    t[6] = make_double2(-S * b.y, S * b.x);
    const cplx c = t[7];
    t[7] = make_double2(h * (-c.x - S * c.y), h * (S * c.x - c.y));
  }
#pragma unroll
  for (int hb = 0; hb < 8; hb += 4) {
    const cplx a0 = t[hb], a1 = t[hb + 1], a2 = t[hb + 2], a3 = t[hb + 3];
    t[hb] = cadd(a0, a2);
    t[hb + 1] = cadd(a1, a3);
    t[hb + 2] = csub(a0, a2);
    const cplx d = csub(a1, a3);
    t[hb + 3] = make_double2(-S * d.y, S * d.x);  // * W4^1
  }
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    const cplx a = t[k], b = t[k + 1];
    t[k] = cadd(a, b);
    t[k + 1] = csub(a, b);
  }
  v[0] = t[0]; v[1] = t[4]; v[2] = t[2]; v[3] = t[6];
  v[4] = t[1]; v[5] = t[5]; v[6] = t[3]; v[7] = t[7];
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// 512-point FFT on one wavefront.  In: a[r] = x[lane + 64 r].  Out: a[k2] = X[q + 8 k1 + 64 k2]
// with q = lane >> 3, k1 = lane & 7.  xb: this wave's 576-entry LDS exchange buffer (padded
// so both transposes are bank-conflict free); tw: W_512^j = e^{+2 pi i j/512}, j < 512.
constexpr int kXbuf = 576;
template <int S>
__device__ __forceinline__ void fft512_wave(cplx (&a)[8], cplx* xb, const cplx* __restrict__ tw,
                                            int lane) {
  dft8<S>(a);
#pragma unroll
  for (int q = 1; q < 8; ++q) a[q] = cmul_tw<S>(a[q], tw[lane * q]);
  wave_sync();
#pragma unroll
  for (int q = 0; q < 8; ++q) xb[q * 72 + lane] = a[q];
  wave_sync();
  const int q = lane >> 3, l1 = lane & 7;
#pragma unroll
  for (int l2 = 0; l2 < 8; ++l2) a[l2] = xb[q * 72 + l1 + 8 * l2];
  dft8<S>(a);
#pragma unroll
  for (int k1 = 1; k1 < 8; ++k1) a[k1] = cmul_tw<S>(a[k1], tw[8 * l1 * k1]);
  wave_sync();
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) xb[q * 72 + l1 * 9 + k1] = a[k1];
  wave_sync();
  const int k1 = lane & 7;
#pragma unroll
  for (int m = 0; m < 8; ++m) a[m] = xb[q * 72 + m * 9 + k1];
  dft8<S>(a);
}

// The same transform with the two transposes through a buffer of doubles (576 per wave, half
// the bytes): real parts first, then imaginary parts, through the same conflict-free index
// maps.  Twice the LDS instructions, half the LDS footprint: the 512-point passes that use it
// fit three workgroups per CU instead of two.
template <int S, class WF, class RF>
__device__ __forceinline__ void exchange_split(cplx (&a)[8], double* xb, WF widx, RF ridx) {
  double t[8];
  wave_sync();
#pragma unroll
  for (int q = 0; q < 8; ++q) xb[widx(q)] = a[q].x;
  wave_sync();
#pragma unroll
  for (int q = 0; q < 8; ++q) t[q] = xb[ridx(q)];
  wave_sync();
#pragma unroll
  for (int q = 0; q < 8; ++q) xb[widx(q)] = a[q].y;
  wave_sync();
#pragma unroll
  for (int q = 0; q < 8; ++q) a[q] = make_double2(t[q], xb[ridx(q)]);
}

template <int S>
__device__ __forceinline__ void fft512_wave_split(cplx (&a)[8], double* xb,
                                                  const cplx* __restrict__ tw, int lane) {
  dft8<S>(a);
#pragma unroll
  for (int q = 1; q < 8; ++q) a[q] = cmul_tw<S>(a[q], tw[lane * q]);
  const int q8 = lane >> 3, l1 = lane & 7;
  exchange_split<S>(a, xb, [&](int q) { return q * 72 + lane; },
                    [&](int l2) { return q8 * 72 + l1 + 8 * l2; });
  dft8<S>(a);
#pragma unroll
  for (int k1 = 1; k1 < 8; ++k1) a[k1] = cmul_tw<S>(a[k1], tw[8 * l1 * k1]);
  exchange_split<S>(a, xb, [&](int k1) { return q8 * 72 + l1 * 9 + k1; },
                    [&](int m) { return q8 * 72 + m * 9 + l1; });
  dft8<S>(a);
}

// Device twiddle tables for a length-N transform (cached per N for the library's lifetime):
//   w512[j] = e^{2 pi i j/512}           (j < 512)      -- the wave engine's table
//   lo[j]   = e^{2 pi i j/N}             (j < Q)        -- Q = 2^ceil(log2 N / 2)
//   hi[j]   = e^{2 pi i Q j/N}           (j < N/Q)      -- W_N^m = hi[m / Q] * lo[m % Q]
struct Tables {
  long N = 0;
  int logQ = 0;
  const cplx* w512 = nullptr;
  const cplx* lo = nullptr;
  const cplx* hi = nullptr;
};
int tables(long N, Tables* out);  // thread-safe, JW_OK or JW_ERR_*

__device__ __forceinline__ cplx twiddle(const Tables& T, long m) {  // e^{+2 pi i m/N}, m < N
  return cmul(T.hi[m >> T.logQ], T.lo[m & ((1L << T.logQ) - 1)]);
}

}  // namespace fft
}  // namespace jw
