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
// the FFT path's tolerance class).  Power-of-two N run the four-step engine directly; other N
// (the reference's Bluestein lengths) run every length-N DFT as a chirp-z transform on it.
#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "jw_fft_passes.hpp"

namespace jw {
namespace {

using fft::cplx;
using fft::Tables;

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

// The pyramid's per-row filter products, once per call (signal independent):
//   F[r][k] = H_{r+1}(k) prod_{i<=r} G_i(k)  (r < J, row W_{r+1}),   F[J][k] = prod_{i<=J} G_i(k)
// with G_i(k) = G(2^(i-1) k mod N), G(f) = sum_m g[m] z^m, z = e^{-2 pi i f/N} (exact table
// twiddle for power-of-two N, sincospi of the reduced angle otherwise), by Horner's rule.
// Stored at position t = pos(k) -- the spectra's own layout -- so the IFFT/FFT functors read
// F with the same sequential index as the spectra (a response table indexed at the scaled
// frequencies 2^(i-1) k would cost one cache line per element and level).
__device__ __forceinline__ cplx fresp(const double* c, int L, cplx z) {
  cplx v = make_double2(c[L - 1], 0.0);
  for (int m = L - 2; m >= 0; --m) {
    v = fft::cmul(v, z);
    v.x += c[m];
  }
  return v;
}

template <bool POW2>
__global__ void filter_products(cplx* __restrict__ F, Taps taps, int L, long N, int J, long N1,
                                long N2, Tables T) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  const long t = POW2 ? fft::tpos(k, N1, N2) : k;
  cplx p = make_double2(1.0, 0.0);
  for (int i = 1; i <= J; ++i) {
    cplx z;
    if constexpr (POW2) {
      const cplx w = fft::twiddle(T, (k << (i - 1)) & (N - 1));
      z = make_double2(w.x, -w.y);
    } else {
      double sn, cs;
      sincospi(2.0 * (double)(long)(((__int128)k << (i - 1)) % N) / (double)N, &sn, &cs);
      z = make_double2(cs, -sn);
    }
    F[(long)(i - 1) * N + t] = fft::cmul(p, fresp(taps.b, L, z));  // H_i prod_{<i} G
    p = fft::cmul(p, fresp(taps.a, L, z));
  }
  F[(long)J * N + t] = p;
}

// Inverse adjoint sum S_0 = sum_r conj(F_r) C_r, C_r = FFT(row r) (the nested recursion
// S_{j-1} = conj(G_j) S_j + conj(H_j) FFT(W_j) multiplied out).
__device__ __forceinline__ cplx adjoint_sum(const cplx* c, const cplx* F, long N, int J, long t) {
  cplx s = make_double2(0.0, 0.0);
  for (int r = J; r >= 0; --r) {
    const cplx f = F[(long)r * N + t], w = c[(long)r * N + t];
    s.x += f.x * w.x + f.y * w.y;  // conj(f) w
    s.y += f.x * w.y - f.y * w.x;
  }
  return s;
}

Taps taps_of(const ModwtPlan& p) {
  Taps taps{};
  for (int m = 0; m < p.L; ++m) {
    taps.a[m] = p.g[m];
    taps.b[m] = p.h[m];
  }
  return taps;
}

// F: (J+1) x N filter products at the spectra's positions (power-of-two N: column-major
// for the split N1 x N2; other N: natural order, N1 = N2 = 0)
int products(const ModwtPlan& p, long N, int J, long N1, long N2, const Tables& T, cplx** F,
             StreamAllocs& mem, hipStream_t s) {
  JW_HIP_TRY(mem.alloc(F, (size_t)(J + 1) * N * sizeof(cplx)));
  const unsigned nb = (unsigned)((N + 255) / 256);
  if (N1 > 0) {
    hipLaunchKernelGGL(filter_products<true>, dim3(nb), dim3(256), 0, s, *F, taps_of(p), p.L, N,
                       J, N1, N2, T);
  } else {
    hipLaunchKernelGGL(filter_products<false>, dim3(nb), dim3(256), 0, s, *F, taps_of(p), p.L, N,
                       J, 1L, 1L, T);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}


// ---------------------------------------------------------------------------------------
// Other lengths (FastFourierTransform.java:259-324 takes them through Bluestein): the same
// frequency-domain pyramid on natural-order spectra, each length-N DFT a chirp-z transform
// over the power-of-two engine, M = 2^ceil(log2(2N - 1)):
//   X_k = c_k^S * sum_n (x_n c_n^S) b_{k-n},  c_n = e^{i pi n^2 / N},  b_m = c_|m|^-S
// (c^S: the conjugate for the forward transform, S = -1), the convolution as
// IFFT_M(FFT_M(a) FFT_M(b)) / M.  Chirp angles are reduced exactly (n^2 mod 2N) on the host.
// ---------------------------------------------------------------------------------------
struct NatIn {  // complex rows of length M (natural order), element k = N2 k1 + col
  static constexpr bool kStrided = true;
  const cplx* a;
  long M, N2;
  __device__ cplx operator()(long item, long k1, long col) const {
    return a[item * M + N2 * k1 + col];
  }
};
struct NatOut1 {  // single pass: out[item][idx]
  cplx* o;
  long M;
  __device__ void operator()(long item, long idx, long, cplx v) const { o[item * M + idx] = v; }
};
struct NatOut {  // four-step: out[item][n1 + N1 n2]
  cplx* o;
  long M, N1;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    o[item * M + line + N1 * idx] = v;
  }
};

__device__ __forceinline__ cplx chirp(const cplx* w, long n, int S) {  // c_n^S
  const cplx c = w[n];
  return S < 0 ? make_double2(c.x, -c.y) : c;
}

// a[item][m] = m < N ? in[item][m] c_m^S : 0, m < M
__global__ void bs_pre(const cplx* __restrict__ in, cplx* __restrict__ a, const cplx* w, long N,
                       long M, long items, int S) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= items * M) return;
  const long item = i / M, m = i - item * M;
  a[i] = m < N ? fft::cmul(in[item * N + m], chirp(w, m, S)) : make_double2(0.0, 0.0);
}
// (elementwise, so any layout both spectra share: the column-major one of fft_to_spec)
__global__ void bs_mul(cplx* __restrict__ a, const cplx* __restrict__ bh, long M, long items) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= items * M) return;
  a[i] = fft::cmul(a[i], bh[i % M]);
}
// out[item][k] = c_k^S conv[item][k] / M, k < N
__global__ void bs_post(const cplx* __restrict__ conv, cplx* __restrict__ out, const cplx* w,
                        long N, long M, long items, int S) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= items * N) return;
  const long item = i / N, k = i - item * N;
  const cplx v = fft::cmul(conv[item * M + k], chirp(w, k, S));
  const double inv = 1.0 / (double)M;
  out[i] = make_double2(v.x * inv, v.y * inv);
}

struct Bluestein {
  long N = 0, M = 0;
  Tables T;
  const cplx* w = nullptr;   // c_n, n < N (cached per device and N)
  const cplx* bh[2] = {};    // FFT_M(b) for S = -1 (index 0) and S = +1 (index 1), cached
  cplx* ws = nullptr;        // 3 x items x M workspace (the caller's StreamAllocs)
  long ws_items = 0;
};

unsigned blocks(long n) { return (unsigned)((n + 255) / 256); }

// Column-major spectra of length M (element k at tpos(k, N1c, N2c), the layout the inverse's
// pass 1 reads as contiguous columns; natural order for M <= 4096).
struct TposIn {
  static constexpr bool kStrided = false;
  const cplx* a;
  long M, N1, N2;
  __device__ cplx operator()(long item, long k1, long col) const {
    return a[item * M + col * N1 + k1];
  }
};

// FFT_M of natural-order rows -> column-major spectra
int fft_to_spec(long M, long items, const cplx* in, cplx* out, cplx* A, hipStream_t s,
                const Tables& T) {
  const long N1n = fft::split_n1(M, true), N1c = fft::split_n1(M, false);
  return fft::run_fft<-1>(M, items, NatIn{in, M, M / N1n}, NatOut1{out, M},
                          fft::SpecOut{out, M, N1n, N1c, M / N1c, 0}, A, s, T, false);
}
// IFFT_M (no 1/M) of column-major spectra -> natural-order rows
int ifft_from_spec(long M, long items, const cplx* in, cplx* out, cplx* A, hipStream_t s,
                   const Tables& T) {
  const long N1c = fft::split_n1(M, false);
  return fft::run_fft<1>(M, items, TposIn{in, M, N1c, M / N1c}, NatOut1{out, M},
                         NatOut{out, M, N1c}, A, s, T, false);
}

// c_n = e^{i pi n^2 / N}, the angle reduced exactly (n^2 mod 2N, n < 2^23 so n^2 < 2^46)
__global__ void chirp_table(cplx* w, long N) {
  const long n = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const long r = (n * n) % (2 * N);
  double sn, cs;
  sincospi((double)r / (double)N, &sn, &cs);
  w[n] = make_double2(cs, sn);
}
// b for both signs, zero-padded to M: b_m = c_|m| (m < N, M - m < N), q = 1 conjugated
__global__ void chirp_b(cplx* b, const cplx* w, long N, long M) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * M) return;
  const long q = i / M, m = i - q * M;
  const long j = m < N ? m : (M - m < N ? M - m : -1);
  cplx c = j >= 0 ? w[j] : make_double2(0.0, 0.0);
  if (q == 1) c.y = -c.y;
  b[i] = c;
}

// The chirp tables and FFT_M(b) depend on N alone: built once per (device, N) on the device
// (the first call for a length synchronises its stream once) and kept, within a 2 GiB budget
// (past it a call builds its own), until jw_release_caches().  One buffer per key:
// [c_n, n < N | FFT_M(b) for S = -1 | for S = +1].
DevCache<std::pair<int, long>> g_bs(2UL << 30);

int bluestein_init(Bluestein* B, long N, long max_items, StreamAllocs& mem, hipStream_t s) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  B->N = N;
  B->M = 1;
  while (B->M < 2 * N - 1) B->M <<= 1;
  const long M = B->M;
  int st = fft::tables(M, &B->T);
  if (st != JW_OK) return st;
  const void* tab = nullptr;
  st = cached_table(g_bs, std::make_pair(dev, N), (size_t)(N + 2 * M) * sizeof(cplx), mem, s, &tab,
                    [&](void* d) -> int {
                      cplx* w = (cplx*)d;
                      cplx* bh = w + N;
                      cplx* tmp = nullptr;
                      JW_HIP_TRY(mem.alloc(&tmp, (size_t)4 * M * sizeof(cplx)));
                      hipLaunchKernelGGL(chirp_table, dim3(blocks(N)), dim3(256), 0, s, w, N);
                      hipLaunchKernelGGL(chirp_b, dim3(blocks(2 * M)), dim3(256), 0, s, tmp, w, N, M);
                      JW_HIP_TRY(hipGetLastError());
                      // column-major, as bs_mul reads it
                      return fft_to_spec(M, 2, tmp, bh, tmp + 2 * M, s, B->T);
                    });
  if (st != JW_OK) return st;
  B->w = (const cplx*)tab;
  B->bh[0] = (const cplx*)tab + N;
  B->bh[1] = (const cplx*)tab + N + M;
  B->ws_items = max_items;
  JW_HIP_TRY(mem.alloc(&B->ws, (size_t)3 * max_items * M * sizeof(cplx)));
  return JW_OK;
}

// items length-N DFTs (S = -1 forward, +1 reverse without 1/N), natural order in -> out
int bluestein_dft(const Bluestein& B, int S, long items, const cplx* in, cplx* out, hipStream_t s) {
  const long N = B.N, M = B.M;
  for (long i0 = 0; i0 < items; i0 += B.ws_items) {
    const long ni = std::min(B.ws_items, items - i0);
    // the inverse FFT reads column-major c and its pass 1 writes rows: its own workspace p
    cplx *a = B.ws, *c = B.ws + ni * M, *p = B.ws + 2 * ni * M;
    hipLaunchKernelGGL(bs_pre, dim3(blocks(ni * M)), dim3(256), 0, s, in + i0 * N, a, B.w, N, M,
                       ni, S);
    int st = fft_to_spec(M, ni, a, c, a, s, B.T);  // FFT_M(a) -> c (a is the pass workspace)
    if (st != JW_OK) return st;
    hipLaunchKernelGGL(bs_mul, dim3(blocks(ni * M)), dim3(256), 0, s, c, B.bh[S < 0 ? 0 : 1], M, ni);
    st = ifft_from_spec(M, ni, c, a, p, s, B.T);  // IFFT_M (no 1/M) -> a, natural order
    if (st != JW_OK) return st;
    hipLaunchKernelGGL(bs_post, dim3(blocks(ni * N)), dim3(256), 0, s, a, out + i0 * N, B.w, N, M,
                       ni, S);
    JW_HIP_TRY(hipGetLastError());
  }
  return JW_OK;
}

__global__ void real_to_cplx(const double* __restrict__ x, cplx* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = make_double2(x[i], 0.0);
}
__global__ void cplx_re_scaled(const cplx* __restrict__ y, double* __restrict__ x, long n,
                               double inv) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = y[i].x * inv;
}
// forward pyramid in frequency, natural order: Y[sig][r][k] = X[sig][k] F_r(k)
__global__ void fwd_combine(const cplx* __restrict__ X, const cplx* __restrict__ F,
                            cplx* __restrict__ Y, long N, int J, long nsig) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsig * (J + 1) * N) return;
  const long k = i % N, item = i / N, sig = item / (J + 1);
  const long r = item - sig * (J + 1);
  Y[i] = fft::cmul(X[sig * N + k], F[r * N + k]);
}
// inverse: S[sig][k] = sum_r conj(F_r(k)) C[sig][r][k], C[sig][r] = FFT(row r)
__global__ void inv_combine(const cplx* __restrict__ C, const cplx* __restrict__ F,
                            cplx* __restrict__ Sout, long N, int J, long nsig) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsig * N) return;
  const long sig = i / N, k = i - sig * N;
  Sout[i] = adjoint_sum(C + sig * (long)(J + 1) * N, F, N, J, k);
}

// per-chunk signals for the general path: rows, spectra and the chirp workspace ~1 GB
long chunk_any(long N, long M, int J, int batch) {
  const long per_sig = ((long)(J + 1) * (2 * N + 3 * M) + 2 * N) * (long)sizeof(cplx);
  return std::max(1L, std::min<long>(batch, (1L << 30) / per_sig));
}

int forward_any(const ModwtPlan& p, const double* x, double* coeffs, long N, int J, int batch,
                hipStream_t s) {
  StreamAllocs mem(s);
  cplx* R = nullptr;  // filter products, natural order
  int st = products(p, N, J, 0, 0, Tables{}, &R, mem, s);
  if (st != JW_OK) return st;
  long M = 1;
  while (M < 2 * N - 1) M <<= 1;
  const long bc = chunk_any(N, M, J, batch);
  Bluestein B;
  st = bluestein_init(&B, N, bc * (J + 1), mem, s);
  if (st != JW_OK) return st;
  cplx *X = nullptr, *Y = nullptr;
  JW_HIP_TRY(mem.alloc(&X, (size_t)bc * N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&Y, (size_t)bc * (J + 1) * N * sizeof(cplx)));
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += bc) {
    const long nb = std::min<long>(bc, batch - b0);
    hipLaunchKernelGGL(real_to_cplx, dim3(blocks(nb * N)), dim3(256), 0, s, x + b0 * N, Y, nb * N);
    st = bluestein_dft(B, -1, nb, Y, X, s);
    if (st != JW_OK) break;
    hipLaunchKernelGGL(fwd_combine, dim3(blocks(nb * (J + 1) * N)), dim3(256), 0, s, X, R, Y, N, J, nb);
    st = bluestein_dft(B, 1, nb * (J + 1), Y, Y, s);
    if (st != JW_OK) break;
    hipLaunchKernelGGL(cplx_re_scaled, dim3(blocks(nb * (J + 1) * N)), dim3(256), 0, s, Y,
                       coeffs + b0 * (long)(J + 1) * N, nb * (J + 1) * N, 1.0 / (double)N);
    JW_HIP_TRY(hipGetLastError());
  }
  return st;
}

int inverse_any(const ModwtPlan& p, const double* coeffs, double* x, long N, int J, int batch,
                hipStream_t s) {
  StreamAllocs mem(s);
  cplx* R = nullptr;  // filter products, natural order
  int st = products(p, N, J, 0, 0, Tables{}, &R, mem, s);
  if (st != JW_OK) return st;
  long M = 1;
  while (M < 2 * N - 1) M <<= 1;
  const long bc = chunk_any(N, M, J, batch);
  Bluestein B;
  st = bluestein_init(&B, N, bc * (J + 1), mem, s);
  if (st != JW_OK) return st;
  cplx *C = nullptr, *S = nullptr;
  JW_HIP_TRY(mem.alloc(&C, (size_t)bc * (J + 1) * N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&S, (size_t)bc * N * sizeof(cplx)));
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += bc) {
    const long nb = std::min<long>(bc, batch - b0);
    hipLaunchKernelGGL(real_to_cplx, dim3(blocks(nb * (J + 1) * N)), dim3(256), 0, s,
                       coeffs + b0 * (long)(J + 1) * N, C, nb * (J + 1) * N);
    st = bluestein_dft(B, -1, nb * (J + 1), C, C, s);
    if (st != JW_OK) break;
    hipLaunchKernelGGL(inv_combine, dim3(blocks(nb * N)), dim3(256), 0, s, C, R, S, N, J, nb);
    st = bluestein_dft(B, 1, nb, S, S, s);
    if (st != JW_OK) break;
    hipLaunchKernelGGL(cplx_re_scaled, dim3(blocks(nb * N)), dim3(256), 0, s, S, x + b0 * N,
                       nb * N, 1.0 / (double)N);
    JW_HIP_TRY(hipGetLastError());
  }
  return st;
}

// FastFourierTransform.forward/reverse(Complex[]) front-end (jw_fft_forward / jw_fft_reverse):
// natural-order interleaved lines, the reverse scaled by 1/n (:207-211).
struct NatOut1S {  // single pass: out[item][idx] * scale
  cplx* o;
  long M;
  double scale;
  __device__ void operator()(long item, long idx, long, cplx v) const {
    o[item * M + idx] = make_double2(v.x * scale, v.y * scale);
  }
};
struct NatOutS {  // four-step: out[item][n1 + N1 n2] * scale
  cplx* o;
  long M, N1;
  double scale;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    o[item * M + line + N1 * idx] = make_double2(v.x * scale, v.y * scale);
  }
};
__global__ void cplx_scale(cplx* __restrict__ a, long n, double f) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = make_double2(a[i].x * f, a[i].y * f);
}

}  // namespace

int fft_device(int S, const double* in, double* out, long n, long batch, hipStream_t s) {
  if (n == 0 || batch == 0) return JW_OK;
  const cplx* x = (const cplx*)in;
  cplx* y = (cplx*)out;
  if (n == 1) {  // forward/reverse return a copy (:117-119, :146-148)
    if (in != out) JW_HIP_TRY(hipMemcpyAsync(out, in, (size_t)batch * sizeof(cplx),
                                             hipMemcpyDeviceToDevice, s));
    return JW_OK;
  }
  StreamAllocs mem(s);
  if ((n & (n - 1)) == 0) {  // Cooley-Tukey lengths: the four-step engine (exact twiddles)
    Tables T;
    int st = fft::tables(n, &T);
    if (st != JW_OK) return st;
    const long N1 = fft::split_n1(n), N2 = n / N1;
    const double scale = S > 0 ? 1.0 / (double)n : 1.0;
    // lines per launch: grid y <= 32768 and a pass workspace of at most 512 MiB
    const long chunk = std::max(1L, std::min<long>({batch, 32768L,
                                                   (512L << 20) / (n * (long)sizeof(cplx))}));
    cplx* A = nullptr;
    if (n > 4096) JW_HIP_TRY(mem.alloc(&A, (size_t)chunk * n * sizeof(cplx)));
    for (long b0 = 0; b0 < batch && st == JW_OK; b0 += chunk) {
      const long nb = std::min(chunk, batch - b0);
      const NatIn fin{x + b0 * n, n, N2};
      const NatOut1S o1{y + b0 * n, n, scale};
      const NatOutS o2{y + b0 * n, n, N1, scale};
      // natural order in and out: the legacy split (long_ok = false)
      st = S < 0 ? fft::run_fft<-1>(n, nb, fin, o1, o2, A, s, T, false, false)
                 : fft::run_fft<1>(n, nb, fin, o1, o2, A, s, T, false, false);
    }
    return st;
  }
  // Bluestein lengths (:259-324): the chirp-z transform over the power-of-two engine
  if (n > (1L << 23)) return fail(JW_ERR_UNSUPPORTED, "FFT length %ld > 2^23 (not a power of 2)", n);
  long M = 1;
  while (M < 2 * n - 1) M <<= 1;
  const long items = std::max(2L, std::min<long>(batch, (1L << 30) / (3 * M * (long)sizeof(cplx))));
  Bluestein B;
  int st = bluestein_init(&B, n, items, mem, s);
  if (st != JW_OK) return st;
  st = bluestein_dft(B, S < 0 ? -1 : 1, batch, x, y, s);
  if (st == JW_OK && S > 0) {
    hipLaunchKernelGGL(cplx_scale, dim3(blocks(batch * n)), dim3(256), 0, s, y, batch * n,
                       1.0 / (double)n);
    JW_HIP_TRY(hipGetLastError());
  }
  return st;
}

static bool is_pow2(long N) { return (N & (N - 1)) == 0; }

// power-of-two N: the four-step pyramid; other N (< 2^23): the chirp-z pyramid
bool modwt_fft_supported(long N) { return N >= 2 && N <= kPyramidFftMax; }

namespace {
// ---------------------------------------------------------------------------------------
// Power-of-two N: two real rows per complex transform.  Every spectrum of the pyramid is
// Hermitian (real signals, real filters), so rows a = 2q and b = 2q+1 share one complex FFT:
//   forward:  W_a + i W_b = IFFT(X (F_a + i F_b))                 (P1_q = F_a + i F_b)
//   inverse:  Z_q = FFT(row_a + i row_b),  FFT(row_a) = (Z_q[k] + conj Z_q[-k]) / 2,
//             FFT(row_b) = (Z_q[k] - conj Z_q[-k]) / 2i, so the adjoint sum is
//             S_0[k] = 1/2 sum_q conj(P1_q[k]) Z_q[k] + conj(P2_q[k]) conj(Z_q[-k])
//                                                                  (P2_q = F_a - i F_b)
// An odd last row pairs with zero (F_b = 0).  Half the transforms of the row-by-row pyramid;
// the same values up to rounding (the FFT path's tolerance class, 1e-10 of DIRECT).
// ---------------------------------------------------------------------------------------
__global__ void pair_products(cplx* __restrict__ P, const cplx* __restrict__ F, long N, int J) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N) return;
  const int Q = (J + 2) / 2;
  for (int q = 0; q < Q; ++q) {
    const cplx fa = F[(long)(2 * q) * N + t];
    const cplx fb = 2 * q + 1 <= J ? F[(long)(2 * q + 1) * N + t] : make_double2(0.0, 0.0);
    P[(long)q * N + t] = make_double2(fa.x - fb.y, fa.y + fb.x);             // F_a + i F_b
    P[(long)(Q + q) * N + t] = make_double2(fa.x + fb.y, fa.y - fb.x);       // F_a - i F_b
  }
}

struct FwdIn2 {  // item = signal * Q + q: X * P1_q
  static constexpr bool kStrided = false;
  const cplx* X;
  const cplx* P;
  long N, N1, N2;
  int Q;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long sig = item / Q, q = item - sig * Q, t = col * N1 + k1;
    return fft::cmul(X[sig * N + t], P[q * N + t]);
  }
};
struct RealOut2 {  // rows 2q <- Re v / N, 2q+1 <- Im v / N (if it exists), t = line + N1 idx
  double* out;
  long N, N1;
  int J, Q;
  double inv_n;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    const long sig = item / Q, q = item - sig * Q, t = line + N1 * idx;
    double* o = out + (sig * (J + 1) + 2 * q) * N + t;
    o[0] = v.x * inv_n;
    if (2 * q + 1 <= J) o[N] = v.y * inv_n;
  }
};
struct RealIn2 {  // item = signal * Q + q: row 2q + i row 2q+1, element k = N2 k1 + col
  static constexpr bool kStrided = true;
  const double* x;
  long N, N2;
  int J, Q;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long sig = item / Q, q = item - sig * Q, k = N2 * k1 + col;
    const double* r = x + (sig * (J + 1) + 2 * q) * N + k;
    return make_double2(r[0], 2 * q + 1 <= J ? r[N] : 0.0);
  }
};
struct InvIn2 {  // item = signal; Z: Q column-major spectra per signal
  static constexpr bool kStrided = false;
  const cplx* Z;
  const cplx* P;
  long N, N1, N2;
  int Q;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long k = N2 * k1 + col, t = col * N1 + k1;
    const long km = (N - k) & (N - 1), tm = fft::tpos(km, N1, N2);
    const cplx* z = Z + item * (long)Q * N;
    cplx s = make_double2(0.0, 0.0);
    for (int q = Q - 1; q >= 0; --q) {
      const cplx p1 = P[(long)q * N + t], p2 = P[(long)(Q + q) * N + t];
      const cplx zk = z[(long)q * N + t], zm = z[(long)q * N + tm];
      // conj(p1) zk + conj(p2) conj(zm)
      s.x += p1.x * zk.x + p1.y * zk.y + p2.x * zm.x - p2.y * zm.y;
      s.y += p1.x * zk.y - p1.y * zk.x - p2.x * zm.y - p2.y * zm.x;
    }
    return make_double2(0.5 * s.x, 0.5 * s.y);
  }
};

// ---------------------------------------------------------------------------------------
// Other lengths N, the fast option: the same pyramid over a power-of-two length P >= N + H
// (H = (L - 1)(2^J - 1), the longest cumulative filter minus one) instead of a chirp-z
// transform per DFT.  Every row is a circular convolution of length N with a filter of at most
// H + 1 taps, so with x_ext[i] = x[(i - H) mod N] (i < N + H; 0 up to P)
//   (x (*)_N f)[t] = (x_ext (*)_P f)[t + H],   t < N
// -- no index of the window wraps modulo P -- and the adjoint (correlation) likewise reads
// c_ext[i] = c[i mod N] (i < N + H) and keeps t < N.  F_P(k), the filters' P-point responses,
// are the power-of-two pair tables of length P.  One P-point FFT per transform instead of two
// M-point ones (M >= 2N), the same values up to rounding.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ long wrap_index(long i, long N) {
  if (i >= N) {
    i -= N;
  } else if (i < 0) {
    i += N;
  }
  if (i < 0 || i >= N) i = ((i % N) + N) % N;  // filters longer than the signal
  return i;
}
struct RealInExt {  // x_ext[k] = x[(k - H) mod N] (k < N + H), element k = N2 k1 + col
  static constexpr bool kStrided = true;
  const double* x;
  long N, N2, H;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long k = N2 * k1 + col;
    return make_double2(k < N + H ? x[item * N + wrap_index(k - H, N)] : 0.0, 0.0);
  }
};
struct RealOut2Ext {  // window [H, H + N) of the P-point rows 2q, 2q + 1
  double* out;
  long N, N1, H;
  int J, Q;
  double inv_p;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    const long sig = item / Q, q = item - sig * Q, t = line + N1 * idx - H;
    if (t < 0 || t >= N) return;
    double* o = out + (sig * (J + 1) + 2 * q) * N + t;
    o[0] = v.x * inv_p;
    if (2 * q + 1 <= J) o[N] = v.y * inv_p;
  }
};
struct RealIn2Ext {  // rows 2q + i 2q+1 extended: c_ext[k] = c[k mod N] (k < N + H)
  static constexpr bool kStrided = true;
  const double* x;
  long N, N2, H;
  int J, Q;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long sig = item / Q, q = item - sig * Q, k = N2 * k1 + col;
    if (k >= N + H) return make_double2(0.0, 0.0);
    const double* r = x + (sig * (J + 1) + 2 * q) * N + wrap_index(k, N);
    return make_double2(r[0], 2 * q + 1 <= J ? r[N] : 0.0);
  }
};
struct RealOutExt {  // window [0, N) of the P-point row
  double* out;
  long N, N1;
  double inv_p;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    const long t = line + N1 * idx;
    if (t < N) out[item * N + t] = v.x * inv_p;
  }
};

// filter products F ((J+1) rows, scratch) -> pair tables P (2Q rows), spectra layout.
// P depends on the filters, N and J alone, so it is built once per (device, filters, N, J)
// and kept, like the twiddle and chirp-z tables: the first call for a key synchronises its
// stream once (other streams may read the table right after), later calls launch no table
// kernels (the two took ~0.4 ms per call at N = 2^20, J = 8).  At most kPairCacheBytes of
// tables are kept; past that a new key gets a per-call table.
struct PairKey {
  int dev, L, J;
  long N, N1;
  std::vector<double> taps;  // g then h, L each: the plan's content, not its address
  bool operator<(const PairKey& o) const {
    return std::tie(dev, L, J, N, N1, taps) < std::tie(o.dev, o.L, o.J, o.N, o.N1, o.taps);
  }
};
DevCache<PairKey> g_pair(4UL << 30);

int build_pair_tables(const ModwtPlan& p, long N, int J, long N1, long N2, const Tables& T,
                      cplx* P, StreamAllocs& mem, hipStream_t s) {
  cplx* F = nullptr;
  int st = products(p, N, J, N1, N2, T, &F, mem, s);
  if (st != JW_OK) return st;
  hipLaunchKernelGGL(pair_products, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, P, F, N, J);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

int pair_tables(const ModwtPlan& p, long N, int J, long N1, long N2, const Tables& T, cplx** P,
                StreamAllocs& mem, hipStream_t s) {
  const int Q = (J + 2) / 2;
  const size_t bytes = (size_t)2 * Q * N * sizeof(cplx);
  PairKey key{0, p.L, J, N, N1, {}};
  JW_HIP_TRY(hipGetDevice(&key.dev));
  key.taps.assign(p.g, p.g + p.L);
  key.taps.insert(key.taps.end(), p.h, p.h + p.L);
  const void* tab = nullptr;
  const int st = cached_table(g_pair, key, bytes, mem, s, &tab, [&](void* d) -> int {
    return build_pair_tables(p, N, J, N1, N2, T, (cplx*)d, mem, s);
  });
  *P = (cplx*)tab;
  return st;
}

// signals per chunk: spectra + pass workspace of about 4 GB (HBM holds 288 GB; bigger chunks
// mean fewer, fuller launches)
long chunk_pairs(long N, int J, int batch) {
  const int Q = (J + 2) / 2;
  const long per_sig = (long)(2 * Q + 1) * N * (long)sizeof(cplx);
  return std::max(1L, std::min<long>(batch, (4L << 30) / per_sig));
}
}  // namespace

namespace {
// history of the deepest cumulative filter (the padded path's H)
long pyramid_hist(const ModwtPlan& p, int J) { return (long)(p.L - 1) * ((1L << J) - 1); }
// the padded path's length for a length N that is not a power of two (0: use the chirp-z one)
long padded_len(const ModwtPlan& p, long N, int J) {
  const long need = N + pyramid_hist(p, J);
  long P = 1;
  while (P < need) P <<= 1;
  return P <= (1L << 23) ? P : 0;
}
}  // namespace

int modwt_forward_fft_device(const ModwtPlan& p, const double* x, double* coeffs, long N, int J,
                             int batch, hipStream_t s) {
  const long P = is_pow2(N) ? N : padded_len(p, N, J);
  if (P == 0) return forward_any(p, x, coeffs, N, J, batch, s);
  const long H = P == N ? 0 : pyramid_hist(p, J);
  StreamAllocs mem(s);
  Tables T;
  int st = fft::tables(P, &T);
  if (st != JW_OK) return st;
  // forward FFTs read natural-order rows (split N1n), the inverse FFTs column-major spectra
  // (split N1 x N2, the spectra's layout)
  const long N1n = fft::split_n1(P, true), N1 = fft::split_n1(P, false), N2 = P / N1;
  const int Q = (J + 2) / 2;
  cplx* PT = nullptr;
  st = pair_tables(p, P, J, N1, N2, T, &PT, mem, s);
  if (st != JW_OK) return st;
  const long bc = chunk_pairs(P, J, batch);
  cplx *X = nullptr, *A = nullptr;
  JW_HIP_TRY(mem.alloc(&X, (size_t)bc * P * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&A, (size_t)bc * Q * P * sizeof(cplx)));
  const double inv = 1.0 / (double)P;
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += bc) {
    const long nb = std::min<long>(bc, batch - b0);
    double* o = coeffs + b0 * (long)(J + 1) * N;
    if (H == 0) {
      st = fft::run_fft<-1>(P, nb, RealIn{x + b0 * N, N, P / N1n}, fft::SpecOut1{X, P, 0},
                            fft::SpecOut{X, P, N1n, N1, N2, 0}, A, s, T, false);
      if (st != JW_OK) break;
      st = fft::run_fft<1>(P, nb * Q, FwdIn2{X, PT, P, N1, N2, Q}, RealOut2{o, N, 1, J, Q, inv},
                           RealOut2{o, N, N1, J, Q, inv}, A, s, T, false);
    } else {
      st = fft::run_fft<-1>(P, nb, RealInExt{x + b0 * N, N, P / N1n, H}, fft::SpecOut1{X, P, 0},
                            fft::SpecOut{X, P, N1n, N1, N2, 0}, A, s, T, false);
      if (st != JW_OK) break;
      st = fft::run_fft<1>(P, nb * Q, FwdIn2{X, PT, P, N1, N2, Q},
                           RealOut2Ext{o, N, 1, H, J, Q, inv}, RealOut2Ext{o, N, N1, H, J, Q, inv},
                           A, s, T, false);
    }
  }
  return st;
}

int modwt_inverse_fft_device(const ModwtPlan& p, const double* coeffs, double* x, long N, int J,
                             int batch, hipStream_t s) {
  const long P = is_pow2(N) ? N : padded_len(p, N, J);
  if (P == 0) return inverse_any(p, coeffs, x, N, J, batch, s);
  const long H = P == N ? 0 : pyramid_hist(p, J);
  StreamAllocs mem(s);
  Tables T;
  int st = fft::tables(P, &T);
  if (st != JW_OK) return st;
  const long N1n = fft::split_n1(P, true), N1 = fft::split_n1(P, false), N2 = P / N1;
  const int Q = (J + 2) / 2;
  cplx* PT = nullptr;
  st = pair_tables(p, P, J, N1, N2, T, &PT, mem, s);
  if (st != JW_OK) return st;
  const long bc = chunk_pairs(P, J, batch);
  cplx *Z = nullptr, *A = nullptr;
  JW_HIP_TRY(mem.alloc(&Z, (size_t)bc * Q * P * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&A, (size_t)bc * Q * P * sizeof(cplx)));
  const double inv = 1.0 / (double)P;
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += bc) {
    const long nb = std::min<long>(bc, batch - b0);
    const double* c = coeffs + b0 * (long)(J + 1) * N;
    if (H == 0) {
      st = fft::run_fft<-1>(P, nb * Q, RealIn2{c, N, P / N1n, J, Q}, fft::SpecOut1{Z, P, 0},
                            fft::SpecOut{Z, P, N1n, N1, N2, 0}, A, s, T, false);
      if (st != JW_OK) break;
      st = fft::run_fft<1>(P, nb, InvIn2{Z, PT, P, N1, N2, Q}, RealOut{x + b0 * N, N, 1, inv},
                           RealOut{x + b0 * N, N, N1, inv}, A, s, T, false);
    } else {
      st = fft::run_fft<-1>(P, nb * Q, RealIn2Ext{c, N, P / N1n, H, J, Q}, fft::SpecOut1{Z, P, 0},
                            fft::SpecOut{Z, P, N1n, N1, N2, 0}, A, s, T, false);
      if (st != JW_OK) break;
      st = fft::run_fft<1>(P, nb, InvIn2{Z, PT, P, N1, N2, Q}, RealOutExt{x + b0 * N, N, 1, inv},
                           RealOutExt{x + b0 * N, N, N1, inv}, A, s, T, false);
    }
  }
  return st;
}

}  // namespace jw
