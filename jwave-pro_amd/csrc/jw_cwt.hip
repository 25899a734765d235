// jw_cwt.hip -- ContinuousWaveletTransform.transformFFT on the GPU
// (src/main/java/jwave/transforms/ContinuousWaveletTransform.java:183-229; the scale-parallel
// transformFFTParallel :511-565 computes the same values).
//
// Per signal: pad to Np = nextPowerOfTwo(n) (padSignal :269-306), X = FFT(padded) once; per
// scale a: coeff[a][t] = IFFT(X * conj(psi_hat(omega, a, 0)))[t] for t < n, with
// omega[i] = 2 pi i fs / Np - [i > Np/2] 2 pi fs (createFrequencyAxis :450-459) and
// psi_hat(omega, a, 0) = F(a omega) sqrt(a) (ContinuousWavelet.fourierTransform :122-141).
// psi_hat is real for Morlet (MorletWavelet.java:112-124) and Mexican Hat
// (MexicanHatWavelet.java:107-119), evaluated per bin inside the first IFFT pass (never stored).
//
// HBM: the spectra X (B x Np complex) stay resident; each (signal, scale) IFFT is two passes
// through a group workspace A (G pairs x Np complex) that the Infinity Cache mostly absorbs;
// the coefficients (B x ns x n complex) are written once -- that write is the roofline.
#include <algorithm>
#include <cstdlib>

#include "jw_fft.hpp"

namespace jw {
namespace {

using fft::cplx;
using fft::Tables;

constexpr double kPi = 3.14159265358979323846;  // Math.PI
typedef double nt2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void nt_store(cplx* p, cplx v) {
  nt2 w = {v.x, v.y};
  __builtin_nontemporal_store(w, (nt2*)p);
}

struct WaveletFT {
  int kind;        // JW_CWT_MORLET / JW_CWT_MEXHAT
  double p0, p1;   // Morlet (fb, fc); Mexican Hat (sigma, unused)
  double norm;     // Morlet sqrt(2 pi fb); Mexican Hat ftNorm = nc sigma sqrt(2 pi)
};

// F(a omega) * sqrt(a), in the reference's operation order.
__device__ __forceinline__ double psi_hat(const WaveletFT& w, double omega, double scale,
                                          double sqrt_scale) {
  const double om = scale * omega;  // fourierTransform(scale * omega)
  double v;
  if (w.kind == JW_CWT_MORLET) {
    const double f = om / (2.0 * kPi);
    const double e = -2.0 * kPi * kPi * w.p0 * (f - w.p1) * (f - w.p1);
    v = e < -746.0 ? 0.0 : w.norm * exp(e);  // exp underflows to +0 below -745.2 anyway
  } else {
    const double om2 = om * om;
    const double e = -0.5 * w.p0 * w.p0 * om2;
    v = e < -746.0 ? 0.0 : w.norm * om2 * exp(e);
  }
  return v * sqrt_scale;  // ft.mul(Math.sqrt(scale))
}

// ---------------------------------------------------------------------------------------
// Pass kernels.  Pass 1 ("columns"): item, column col < N2; inputs k = N2*k1 + col, k1 < N1;
// outputs n1 < N1, multiplied by W_N^(S n1 col) when N2 > 1.  Pass 2 ("rows"): item, row n1;
// inputs k2 < N2 of that row; outputs n2 < N2.  In/Out are functors:
//   cplx in(long item, long idx_in_line, long line)     (idx = k1 or k2, line = col or n1)
//   void out(long item, long idx_out, long line, cplx v)
// Fast kernels: 512-point lines, 8 lines per workgroup, one per wavefront, staged through a
// padded LDS tile so global reads/writes move 8 consecutive complex values (128 bytes).
// ---------------------------------------------------------------------------------------
constexpr int kT = 8;                  // lines per workgroup (fast kernels)
constexpr int kTile = 512 * (kT + 1);  // padded tile, also holds the 8 exchange buffers
static_assert(kTile >= kT * fft::kXbuf, "tile must hold the exchange buffers");

// IN_TILE: the line's inputs are strided (pass 1 over a natural-order array): stage 8 lines
// through the tile.  TWID: apply the four-step twiddle W_N^(S n1 col) (pass 1).
template <int S, bool IN_TILE, bool TWID, class In, class Out>
__global__ __launch_bounds__(512) void pass512(In in, Out out, long N, long N2, Tables T) {
  __shared__ cplx tile[kTile];
  const int tid = threadIdx.x, lane = tid & 63, c = tid >> 6;
  const long item = blockIdx.y;
  const long line0 = (long)blockIdx.x * kT;
  cplx a[8];
  if (IN_TILE) {
    // tile[k1][c] <- in(k1, line0 + c): 8 consecutive columns per row, coalesced
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k1 = (tid >> 3) + 64 * i, cc = tid & 7;
      tile[k1 * (kT + 1) + cc] = in(item, k1, line0 + cc);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r] = tile[(lane + 64 * r) * (kT + 1) + c];
    __syncthreads();
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r] = in(item, lane + 64 * r, line0 + c);
  }
  fft::fft512_wave<S>(a, tile + c * fft::kXbuf, T.w512, lane);
  const int q = lane >> 3, k1 = lane & 7;
  if (TWID && N2 > 1) {
    // W_N^(n1 col) for n1 = q + 8 k1 + 64 k2: one table lookup per lane, then the
    // wave-uniform step W_N^(64 col) applied k2 times (7 products: ~1e-15 relative)
    const long col = line0 + c;
    cplx w = fft::twiddle(T, ((long)(q + 8 * k1) * col) & (N - 1));
    const cplx step = fft::twiddle(T, (64 * col) & (N - 1));
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      a[k2] = fft::cmul_tw<S>(a[k2], w);
      if (k2 < 7) w = fft::cmul(w, step);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) tile[(q + 8 * k1 + 64 * k2) * (kT + 1) + c] = a[k2];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = (tid >> 3) + 64 * i, cc = tid & 7;
    out(item, n, line0 + cc, tile[n * (kT + 1) + cc]);
  }
}

// Generic line FFT of M = 2^logM <= 4096 points, one workgroup per line: bit-reversed load,
// in-place radix-2 stages in LDS.
template <int S, bool COLS, class In, class Out>
__global__ __launch_bounds__(256) void pass_generic(In in, Out out, long N, long N2, int logM,
                                                    Tables T) {
  extern __shared__ cplx buf[];
  const int tid = threadIdx.x;
  const int M = 1 << logM;
  const long item = blockIdx.y, line = blockIdx.x;
  for (int j = tid; j < M; j += 256) {
    const int r = logM ? (int)(__brev((unsigned)j) >> (32 - logM)) : 0;
    buf[r] = in(item, j, line);
  }
  __syncthreads();
  for (int len = 2; len <= M; len <<= 1) {
    const int half = len >> 1;
    const long step = N / len;
    for (int b = tid; b < (M >> 1); b += 256) {
      const int pos = b & (half - 1);
      const int i0 = (b - pos) * 2 + pos, i1 = i0 + half;
      const cplx w = fft::twiddle(T, pos * step);
      const cplx u = buf[i0], v = fft::cmul_tw<S>(buf[i1], w);
      buf[i0] = fft::cadd(u, v);
      buf[i1] = fft::csub(u, v);
    }
    __syncthreads();
  }
  for (int j = tid; j < M; j += 256) {
    cplx v = buf[j];
    if (COLS && N2 > 1) v = fft::cmul_tw<S>(v, fft::twiddle(T, ((long)j * line) & (N - 1)));
    out(item, j, line, v);
  }
}

// ---------------------------------------------------------------------------------------
// Functors
// ---------------------------------------------------------------------------------------
// Spectra are stored "column-major" for the inverse's four-step: element k at
// (k mod N2) * N1 + k / N2, so each pass-1 column is contiguous.
__device__ __forceinline__ long tpos(long k, long N1, long N2) { return (k % N2) * N1 + k / N2; }

struct PadIn {  // padded real signal, element k (padSignal :269-306)
  static constexpr bool kStrided = true;
  const double* x;
  long n, N2;
  int padding;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long k = N2 * k1 + col;
    const double* xs = x + item * n;
    double v = 0.0;
    if (k < n) {
      v = xs[k];
    } else if (padding == JW_PAD_SYMMETRIC) {
      const long mi = 2 * n - k - 2;
      if (mi >= 0 && mi < n) v = xs[mi];
    } else if (padding == JW_PAD_PERIODIC) {
      v = xs[k % n];
    } else if (padding == JW_PAD_CONSTANT) {
      v = xs[n - 1];
    }
    return make_double2(v, 0.0);
  }
};
struct RowIn {  // A[item][n1 * N2 + k2]
  const cplx* A;
  long N, N2;
  __device__ cplx operator()(long item, long k2, long n1) const {
    return A[item * N + n1 * N2 + k2];
  }
};
struct ColOut {  // A[item][n1 * N2 + col]
  cplx* A;
  long N, N2;
  bool nt;  // non-temporal stores
  __device__ void operator()(long item, long n1, long col, cplx v) const {
    if (nt) {  // streamed once: keep it from evicting the spectra out of L2
      nt_store(&A[item * N + n1 * N2 + col], v);
    } else {
      A[item * N + n1 * N2 + col] = v;
    }
  }
};
struct SpecOut {  // X[item][k], k = n1 + N1 * n2, at its column-major position
  cplx* X;
  long N, N1, N2;
  long item0;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    X[(item0 + item) * N + tpos(line + N1 * idx, N1, N2)] = v;
  }
};
struct SpecOut1 {  // single pass: X[item][idx]
  cplx* X;
  long N, item0;
  __device__ void operator()(long item, long idx, long, cplx v) const {
    X[(item0 + item) * N + idx] = v;
  }
};
struct ScaleIn {  // X[sig][k] * psi_hat(omega_k, a_s), k = N2 k1 + col; item = pair in group
  static constexpr bool kStrided = false;  // column-major spectra: contiguous columns
  const cplx* X;
  const double* scales;
  WaveletFT w;
  long N, N1, N2, pair0;
  int ns;
  double fs;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long p = pair0 + item, sig = p / ns;
    const int s = (int)(p - sig * ns);
    const long k = N2 * k1 + col;
    double om = 2.0 * kPi * (double)k * fs / (double)N;  // createFrequencyAxis :453-456
    if (k > N / 2) om -= 2.0 * kPi * fs;
    const double a = scales[s];
    const double wv = psi_hat(w, om, a, sqrt(a));
    if (wv == 0.0) return make_double2(0.0, 0.0);  // exp underflowed: skip the X read
    const cplx xv = X[sig * N + col * N1 + k1];
    return make_double2(xv.x * wv, xv.y * wv);  // signalFFT[i].mul(conj(waveletFFT[i]))
  }
};
struct CoefOut {  // out[pair][t] = v / N for t = line + N1 * idx < n  (reverse :207-211)
  double* out;  // interleaved (re, im), B x ns x n
  long n, N1, pair0;
  double inv_n;
  bool nt;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    const long t = line + N1 * idx;
    if (t < n) {
      cplx* o = (cplx*)(out + 2 * ((pair0 + item) * n + t));
      const cplx r = make_double2(v.x * inv_n, v.y * inv_n);
      if (nt) {
        nt_store(o, r);
      } else {
        *o = r;
      }
    }
  }
};

// One full FFT (forward or reverse) of `items` lines of length N: in(item, k) -> out.
template <int S, class In1, class Out1, class Out2>
int run_fft(long N, long items, In1 in1, Out1 out_single, Out2 out_final, cplx* A, hipStream_t s,
            const Tables& T, bool a_nt) {
  int logN = 0;
  while ((1L << logN) < N) ++logN;
  if (N <= 4096) {  // one pass, N2 = 1
    hipLaunchKernelGGL((pass_generic<S, true, In1, Out1>), dim3(1, (unsigned)items), dim3(256),
                       (size_t)N * sizeof(cplx), s, in1, out_single, N, 1L, logN, T);
    JW_HIP_TRY(hipGetLastError());
    return JW_OK;
  }
  const int log1 = (logN + 1) / 2, log2 = logN - log1;
  const long N1 = 1L << log1, N2 = 1L << log2;
  ColOut a_out{A, N, N2, a_nt};
  RowIn a_in{A, N, N2};
  if (N1 == 512) {
    hipLaunchKernelGGL((pass512<S, In1::kStrided, true, In1, ColOut>),
                       dim3((unsigned)(N2 / kT), (unsigned)items), dim3(512), 0, s, in1, a_out, N,
                       N2, T);
  } else {
    hipLaunchKernelGGL((pass_generic<S, true, In1, ColOut>), dim3((unsigned)N2, (unsigned)items),
                       dim3(256), (size_t)N1 * sizeof(cplx), s, in1, a_out, N, N2, log1, T);
  }
  JW_HIP_TRY(hipGetLastError());
  if (N2 == 512) {
    hipLaunchKernelGGL((pass512<S, false, false, RowIn, Out2>),
                       dim3((unsigned)(N1 / kT), (unsigned)items), dim3(512), 0, s, a_in, out_final,
                       N, N2, T);
  } else {
    hipLaunchKernelGGL((pass_generic<S, false, RowIn, Out2>), dim3((unsigned)N1, (unsigned)items),
                       dim3(256), (size_t)N2 * sizeof(cplx), s, a_in, out_final, N, N2, log2, T);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace

// Group sizes: signals per forward chunk and (signal, scale) pairs per inverse group, so the
// workspace A stays ~128 MB (Infinity Cache sized) at N = 2^18.
int cwt_fft_device(int wavelet, const double* params, const double* x, long n,
                   const double* scales_host, int ns, double fs, int padding, double* out,
                   int batch, hipStream_t s) {
  if (n == 0 || ns == 0 || batch == 0) return JW_OK;
  long N = 1;
  while (N < n) N <<= 1;  // MathUtils.nextPowerOfTwo :46-49
  if (N > (1L << 24)) return fail(JW_ERR_UNSUPPORTED, "CWT padded length %ld > 2^24", N);
  Tables T;
  int st = fft::tables(N, &T);
  if (st != JW_OK) return st;
  WaveletFT w;
  w.kind = wavelet;
  w.p0 = params[0];
  w.p1 = wavelet == JW_CWT_MORLET ? params[1] : 0.0;
  if (wavelet == JW_CWT_MORLET) {
    w.norm = std::sqrt(2.0 * kPi * w.p0);  // MorletWavelet.java:117
  } else {
    const double nc = 2.0 / (std::sqrt(3.0 * w.p0) * std::pow(kPi, 0.25));  // :72
    w.norm = nc * w.p0 * std::sqrt(2.0 * kPi);                              // :111
  }
  const char* gnt = std::getenv("JW_CWT_NT");  // A/B runs: bit 1 = NT stores of A, 2 = of coeffs
  const int ntm = gnt ? std::atoi(gnt) : 2;  // measured best: NT coefficient stores only
  const char* gmb = std::getenv("JW_CWT_GROUP_MB");  // A/B runs: workspace size in MiB
  const long ws = (gmb ? std::atol(gmb) : 128L) << 20;
  const long per = std::max(1L, ws / (N * (long)sizeof(cplx)));
  const long gsig = std::min<long>(batch, per), gpair = std::min<long>((long)batch * ns, per);
  cplx *X = nullptr, *A = nullptr;
  double* dsc = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&X, (size_t)batch * N * sizeof(cplx), s));
  JW_HIP_TRY(hipMallocAsync((void**)&A, (size_t)std::max(gsig, gpair) * N * sizeof(cplx), s));
  JW_HIP_TRY(hipMallocAsync((void**)&dsc, (size_t)ns * sizeof(double), s));
  JW_HIP_TRY(hipMemcpyAsync(dsc, scales_host, (size_t)ns * sizeof(double), hipMemcpyHostToDevice, s));
  int logN = 0;
  while ((1L << logN) < N) ++logN;
  const long N1 = N <= 4096 ? N : 1L << ((logN + 1) / 2);
  // forward FFT of the padded signals, gsig at a time
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += gsig) {
    const long nb = std::min<long>(gsig, batch - b0);
    PadIn in{x + b0 * n, n, N <= 4096 ? 1 : N / N1, padding};
    st = run_fft<-1>(N, nb, in, SpecOut1{X, N, b0}, SpecOut{X, N, N1, N / N1, b0}, A, s, T,
                     (ntm & 1) != 0);
  }
  // per (signal, scale) pair: IFFT(X * psi_hat) -> coefficients
  const long pairs = (long)batch * ns;
  for (long p0 = 0; p0 < pairs && st == JW_OK; p0 += gpair) {
    const long np_ = std::min<long>(gpair, pairs - p0);
    ScaleIn in{X, dsc, w, N, N1, N <= 4096 ? 1 : N / N1, p0, ns, fs};
    CoefOut o{out, n, N <= 4096 ? 1 : N1, p0, 1.0 / (double)N, (ntm & 2) != 0};
    CoefOut o1{out, n, 1, p0, 1.0 / (double)N, (ntm & 2) != 0};
    st = run_fft<1>(N, np_, in, o1, o, A, s, T, (ntm & 1) != 0);
  }
  (void)hipFreeAsync(dsc, s);
  (void)hipFreeAsync(A, s);
  (void)hipFreeAsync(X, s);
  return st;
}

}  // namespace jw
