// jw_fwt_common.hpp -- the FWT arithmetic shared by the cascade kernels (jw_fwt.hip) and the
// streaming column kernels (jw_fwt_stream.hip): filter sets and the per-tap operations in the
// reference's order (Wavelet.java:236-303).
#pragma once
#include "jw_internal.hpp"

namespace jw {
namespace fwtc {

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

// acc + contrib: STRICT keeps Java's acc + ((a*sR) + (d*wR)); FMA folds both products into
// the running sum, fma(d, wR, fma(a, sR, acc)) -- same taps, same order, 2 instead of 3
// double ops per tap pair (the reverse cascades are VALU-heavy).
template <bool FMA, int KIND>
__device__ __forceinline__ double rev_acc(double acc, double a, double d, double sr, double wr) {
  if constexpr (FMA && KIND != JW_WAVELET_HAAR_ORTH) {
    return __builtin_fma(d, wr, __builtin_fma(a, sr, acc));
  } else {
    return acc + contrib<FMA>(a, d, sr, wr, KIND);
  }
}

// Streaming column passes of a 2-D transform with 4096-row (2^S-level) columns
// (jw_fwt_stream.hip).  Return false when (M, S, shape) has no streaming kernel; the reverse
// with A == nullptr only answers whether it would run.
template <bool FMA>
bool launch_stream_fwd(int M, int S, hipStream_t s, const double* T, double* y, int rows,
                       int cols, long mat, int batch, const Filters& f);
template <bool FMA>
bool launch_stream_rev(int M, int kind, int S, hipStream_t s, const double* A, long ms_a,
                       const double* y, double* T, int rows, int cols, long mat, int batch,
                       const Filters& f);

}  // namespace fwtc
}  // namespace jw
