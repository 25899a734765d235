// jw_modwt_fft.hip -- MODWT with FFT convolution on the GPU (ConvolutionMethod.FFT,
// src/main/java/jwave/transforms/MODWTTransform.java:640-664, circularConvolveFFT :752-786,
// circularConvolveFFTAdjoint :798-837, wrapFilterToSignalLength :729-741).
//
// The reference convolves level by level: W_j = Re IFFT(FFT(V_{j-1}) FFT(wrap h_j)).  The FFT
// of the up-sampled, wrapped filter is the base filter's DFT at a scaled frequency,
// FFT(wrap h_j)(k) = H(2^(j-1) k mod N) with H(f) = sum_m h[m] e^{-2 pi i f m / N}, so the whole
// pyramid is diagonal in frequency:
//   forward:  W_j = IFFT(X . H_j . prod_{i<j} G_i),   V_J = IFFT(X . prod_{i<=J} G_i)
//   inverse:  S_J = FFT(V_J);  S_{j-1} = conj(G_j) S_j + conj(H_j) FFT(W_j);  x = IFFT(S_0)
// (real parts taken at the end instead of per level: the same values up to rounding, inside
// the FFT path's tolerance class).  Power-of-two N only (the four-step engine); other N are
// served by the direct kernels, whose results are exact.
#include <algorithm>

#include "jw_fft_passes.hpp"

namespace jw {
namespace {

using fft::cplx;
using fft::Tables;

// R[0][f] = G(f), R[1][f] = H(f), f < N
__global__ void filter_response(cplx* R, Taps taps, int L, long N, Tables T) {
  const long f = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= N) return;
  cplx g = make_double2(0.0, 0.0), h = make_double2(0.0, 0.0);
  for (int m = 0; m < L; ++m) {
    const cplx w = fft::twiddle(T, (f * m) & (N - 1));  // e^{+2 pi i f m / N}; use conj
    g.x += taps.a[m] * w.x;
    g.y -= taps.a[m] * w.y;
    h.x += taps.b[m] * w.x;
    h.y -= taps.b[m] * w.y;
  }
  R[f] = g;
  R[N + f] = h;
}

struct RealIn {  // row `item` of a real array, element k = N2 k1 + col (strided pass 1)
  static constexpr bool kStrided = true;
  const double* x;
  long N, N2;
  __device__ cplx operator()(long item, long k1, long col) const {
    return make_double2(x[item * N + N2 * k1 + col], 0.0);
  }
};

struct RealOut {  // out row `item`: Re(v) / N at t = line + N1 idx
  double* out;
  long N, N1;
  double inv_n;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    out[item * N + line + N1 * idx] = v.x * inv_n;
  }
};

// Forward: item = signal * (J+1) + row; row r < J is W_{r+1}, row J is V_J.
struct FwdIn {
  static constexpr bool kStrided = false;
  const cplx* X;  // column-major spectra, one per signal
  const cplx* R;
  long N, N1, N2;
  int J;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long sig = item / (J + 1);
    const int r = (int)(item - sig * (J + 1));
    const long k = N2 * k1 + col;
    // W_{r+1} = X H_{r+1} prod_{i<=r} G_i  (r < J);  V_J = X prod_{i<=J} G_i  (r = J)
    const int ng = r < J ? r : J - 1;
    cplx f = make_double2(1.0, 0.0);
    for (int i = 1; i <= ng; ++i) f = fft::cmul(f, R[(k << (i - 1)) & (N - 1)]);  // G_i
    f = fft::cmul(f, R[(r < J ? N : 0) + ((k << ng) & (N - 1))]);  // H_{r+1} or G_J
    return fft::cmul(X[sig * N + col * N1 + k1], f);
  }
};

// Inverse: item = signal; C = column-major spectra of the J+1 rows of every signal.
struct InvIn {
  static constexpr bool kStrided = false;
  const cplx* C;
  const cplx* R;
  long N, N1, N2;
  int J;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long k = N2 * k1 + col, t = col * N1 + k1;
    const cplx* c = C + item * (long)(J + 1) * N;
    cplx s = c[(long)J * N + t];  // S_J = FFT(V_J)
    for (int j = J; j >= 1; --j) {
      const long f = (k << (j - 1)) & (N - 1);
      const cplx g = R[f], h = R[N + f];
      const cplx w = c[(long)(j - 1) * N + t];  // FFT(W_j)
      s = make_double2(g.x * s.x + g.y * s.y + h.x * w.x + h.y * w.y,  // conj(G) S + conj(H) W
                       g.x * s.y - g.y * s.x + h.x * w.y - h.y * w.x);
    }
    return s;
  }
};

int prepare(long N, const ModwtPlan& p, Tables* T, cplx** R, hipStream_t s) {
  int st = fft::tables(N, T);
  if (st != JW_OK) return st;
  Taps taps;
  for (int m = 0; m < p.L; ++m) {
    taps.a[m] = p.g[m];
    taps.b[m] = p.h[m];
  }
  JW_HIP_TRY(hipMallocAsync((void**)R, (size_t)2 * N * sizeof(cplx), s));
  hipLaunchKernelGGL(filter_response, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, *R,
                     taps, p.L, N, *T);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

// signals per chunk so that the spectra + pass workspace stay near 1 GB
long chunk_signals(long N, int J, int batch) {
  const long per_sig = (long)(2 * (J + 1) + 1) * N * (long)sizeof(cplx);
  return std::max(1L, std::min<long>(batch, (1L << 30) / per_sig));
}

}  // namespace

bool modwt_fft_supported(long N) { return N >= 2 && (N & (N - 1)) == 0 && N <= (1L << 24); }

int modwt_forward_fft_device(const ModwtPlan& p, const double* x, double* coeffs, long N, int J,
                             int batch, hipStream_t s) {
  Tables T;
  cplx* R = nullptr;
  int st = prepare(N, p, &T, &R, s);
  if (st != JW_OK) return st;
  const long N1 = fft::split_n1(N), N2 = N / N1;
  const long bc = chunk_signals(N, J, batch);
  cplx *X = nullptr, *A = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&X, (size_t)bc * N * sizeof(cplx), s));
  JW_HIP_TRY(hipMallocAsync((void**)&A, (size_t)bc * (J + 1) * N * sizeof(cplx), s));
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += bc) {
    const long nb = std::min<long>(bc, batch - b0);
    st = fft::run_fft<-1>(N, nb, RealIn{x + b0 * N, N, N2}, fft::SpecOut1{X, N, 0},
                          fft::SpecOut{X, N, N1, N2, 0}, A, s, T, false);
    if (st != JW_OK) break;
    const double inv = 1.0 / (double)N;
    double* o = coeffs + b0 * (long)(J + 1) * N;
    st = fft::run_fft<1>(N, nb * (J + 1), FwdIn{X, R, N, N1, N2, J}, RealOut{o, N, 1, inv},
                         RealOut{o, N, N1, inv}, A, s, T, false);
  }
  (void)hipFreeAsync(A, s);
  (void)hipFreeAsync(X, s);
  (void)hipFreeAsync(R, s);
  return st;
}

int modwt_inverse_fft_device(const ModwtPlan& p, const double* coeffs, double* x, long N, int J,
                             int batch, hipStream_t s) {
  Tables T;
  cplx* R = nullptr;
  int st = prepare(N, p, &T, &R, s);
  if (st != JW_OK) return st;
  const long N1 = fft::split_n1(N), N2 = N / N1;
  const long bc = chunk_signals(N, J, batch);
  cplx *C = nullptr, *A = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&C, (size_t)bc * (J + 1) * N * sizeof(cplx), s));
  JW_HIP_TRY(hipMallocAsync((void**)&A, (size_t)bc * (J + 1) * N * sizeof(cplx), s));
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += bc) {
    const long nb = std::min<long>(bc, batch - b0);
    st = fft::run_fft<-1>(N, nb * (J + 1), RealIn{coeffs + b0 * (long)(J + 1) * N, N, N2},
                          fft::SpecOut1{C, N, 0}, fft::SpecOut{C, N, N1, N2, 0}, A, s, T, false);
    if (st != JW_OK) break;
    const double inv = 1.0 / (double)N;
    st = fft::run_fft<1>(N, nb, InvIn{C, R, N, N1, N2, J}, RealOut{x + b0 * N, N, 1, inv},
                         RealOut{x + b0 * N, N, N1, inv}, A, s, T, false);
  }
  (void)hipFreeAsync(A, s);
  (void)hipFreeAsync(C, s);
  (void)hipFreeAsync(R, s);
  return st;
}

}  // namespace jw
