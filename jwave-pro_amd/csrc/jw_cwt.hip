// jw_cwt.hip -- ContinuousWaveletTransform.transformFFT on the GPU
// (src/main/java/jwave/transforms/ContinuousWaveletTransform.java:183-229; the scale-parallel
// transformFFTParallel :511-565 computes the same values).
//
// Per signal: pad to Np = nextPowerOfTwo(n) (padSignal :269-306), X = FFT(padded) once; per
// scale a: coeff[a][t] = IFFT(X * conj(psi_hat(omega, a, 0)))[t] for t < n, with
// omega[i] = 2 pi i fs / Np - [i > Np/2] 2 pi fs (createFrequencyAxis :450-459) and
// psi_hat(omega, a, 0) = F(a omega) sqrt(a) (ContinuousWavelet.fourierTransform :122-141).
// psi_hat is evaluated per bin inside the first IFFT pass (never stored): real for Morlet
// (MorletWavelet.java:112-124), Mexican Hat (MexicanHatWavelet.java:107-119) and Paul
// (PaulWavelet.java:152-164), complex for DOG (DOGWavelet.java:187-220, odd n) and Meyer
// (MeyerWavelet.java:223-253).
//
// HBM: the spectra X (B x Np complex) stay resident; each (signal, scale) IFFT is two passes
// through a group workspace A (G pairs x Np complex) that the Infinity Cache mostly absorbs;
// the coefficients (B x ns x n complex) are written once -- that write is the roofline.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <type_traits>
#include <vector>

#include "jw_fft_passes.hpp"

namespace jw {
namespace {

using fft::cplx;
using fft::Tables;
using fft::ColOut;
using fft::RowIn;
using fft::SpecOut;
using fft::SpecOut1;
using fft::SpecOutBoth;
using fft::nt_store;
using fft::run_fft;
using fft::tpos;

constexpr double kPi = 3.14159265358979323846;  // Math.PI

struct WaveletFT {
  int kind;        // JW_CWT_*
  int ord;         // Paul m, DOG n
  double p0, p1;   // Morlet (fb, fc); Mexican Hat and DOG (sigma, unused)
  double p2;       // exponent factor: Morlet -2 pi^2 fb; Mexican Hat -0.5 sigma^2
  double norm;     // Morlet sqrt(2 pi fb); Mexican Hat ftNorm = nc sigma sqrt(2 pi);
                   // Paul and Meyer sqrt(2 pi); DOG sqrt(2 pi) sigma^(n+1)
  double norm2;    // DOG _normConstant (computeNormalizationConstant :357-366)
};

// Meyer transition polynomial nu(x) = x^4 (35 - 84x + 70x^2 - 20x^3) (MeyerWavelet.java:279-295)
__device__ __forceinline__ double meyer_nu(double x) {
  if (x <= 0) return 0.0;
  if (x >= 1) return 1.0;
  const double x2 = x * x, x3 = x2 * x, x4 = x3 * x;
  return x4 * (35.0 + -84.0 * x + 70.0 * x2 + -20.0 * x3);
}

// psi_hat(omega, a, 0) = sqrt(a) F(a omega) as (re, im), in the reference's operation order.
// The exp arguments below -746 give +0 in Java as here; the test only skips the exp call.
template <int K>
__device__ __forceinline__ cplx psi_hat(const WaveletFT& w, double omega, double scale,
                                        double sqrt_scale) {
  const double om = scale * omega;  // fourierTransform(scale * omega)
  double re = 0.0, im = 0.0;
  if constexpr (K == JW_CWT_MORLET) {  // MorletWavelet.java:114-124
    const double f = om / (2.0 * kPi);
    const double e = -2.0 * kPi * kPi * w.p0 * (f - w.p1) * (f - w.p1);
    re = e < -746.0 ? 0.0 : w.norm * exp(e);
  } else if constexpr (K == JW_CWT_MEXHAT) {  // MexicanHatWavelet.java:107-119
    const double om2 = om * om;
    const double e = -0.5 * w.p0 * w.p0 * om2;
    re = e < -746.0 ? 0.0 : w.norm * om2 * exp(e);
  } else if constexpr (K == JW_CWT_PAUL) {
    // PaulWavelet.fourierTransform(omega, scale, b) override :152-164: no sqrt(a) afterwards
    if (omega <= 0) return make_double2(0.0, 0.0);
    if (-om < -746.0) return make_double2(0.0, 0.0);
    return make_double2(sqrt_scale * w.norm * pow(om, (double)w.ord) * exp(-om), 0.0);
  } else if constexpr (K == JW_CWT_DOG) {  // DOGWavelet.java:187-220
    const double e = -0.5 * w.p0 * w.p0 * om * om;
    double mag = e < -746.0 ? 0.0 : w.norm * pow(fabs(om), (double)w.ord) * exp(e);
    mag *= w.norm2;
    const double sg = om > 0 ? 1.0 : (om < 0 ? -1.0 : om);  // Math.signum
    switch (w.ord & 3) {
      case 0: re = mag; break;
      case 1: im = mag * sg; break;
      case 2: re = -mag; break;
      default: im = -mag * sg; break;
    }
  } else {  // Meyer, MeyerWavelet.java:223-253
    constexpr double lo = 2.0 * kPi / 3.0, mid = 4.0 * kPi / 3.0, hi = 8.0 * kPi / 3.0;
    const double a = fabs(om);
    if (a < lo || a > hi) return make_double2(0.0, 0.0);
    double v;
    if (a <= mid) {
      v = sin(kPi / 2.0 * meyer_nu(3.0 * a / (2.0 * kPi) - 1.0));
    } else {
      v = cos(kPi / 2.0 * meyer_nu(3.0 * a / (4.0 * kPi) - 1.0));
    }
    v *= w.norm;
    double sn, cs;
    sincos(om / 2.0, &sn, &cs);
    re = v * cs;
    im = v * sn;
  }
  return make_double2(re * sqrt_scale, im * sqrt_scale);  // ft.mul(Math.sqrt(scale))
}


// ---------------------------------------------------------------------------------------
// Functors
// ---------------------------------------------------------------------------------------

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
// psi_hat of (scale s, bin k) exactly as the inverse FFT's first pass uses it: for Morlet and
// Mexican hat the per-bin divisions hoisted into per-scale constants: the bin's signed index
// kk = k or k - N (createFrequencyAxis :453-456) times
//   Morlet:      f = a*omega/(2 pi) = kk * (a fs / N)            (MorletWavelet :114-124)
//   Mexican hat: a*omega = kk * (2 pi a fs / N)                  (MexicanHatWavelet :107-119)
// (a few ulps from the reference's operation order; the tests bound it at 1e-12).
// sc: per scale {bin step, norm * sqrt(a)}, see cwt_fft_device.
template <int K>
__device__ __forceinline__ cplx psi_bin(const WaveletFT& w, const double* scales, const double* sc,
                                        int s, long k, long N, double fs) {
  if constexpr (K == JW_CWT_MORLET || K == JW_CWT_MEXHAT) {
    const double kk = (double)(k > N / 2 ? k - N : k);
    const double step = sc[2 * s], amp = sc[2 * s + 1];
    double e, m = amp;
    if constexpr (K == JW_CWT_MORLET) {
      const double d = kk * step - w.p1;
      e = w.p2 * d * d;  // p2 = -2 pi^2 fb
    } else {
      const double om = kk * step, om2 = om * om;
      e = w.p2 * om2;  // p2 = -0.5 sigma^2
      m *= om2;
    }
    // Bins past the underflow point are exact zeros (as Math.exp gives): no exp, no X
    // read.  A narrow band leaves whole 64-bin wave blocks zero, so the branch skips them.
    if (e < -746.0) return make_double2(0.0, 0.0);
    return make_double2(m * exp(e), 0.0);
  } else {
    double om = 2.0 * kPi * (double)k * fs / (double)N;  // createFrequencyAxis :453-456
    if (k > N / 2) om -= 2.0 * kPi * fs;
    const double a = scales[s];
    return psi_hat<K>(w, om, a, sqrt(a));
  }
}

// Pair q of a (sub)set of the (signal, scale) pairs: signal q / nsub, scale smap[q % nsub]
// (smap == nullptr: all ns scales, q = signal * ns + scale).
// Pair counts stay below 2^31 (checked on the host): 32-bit division, which the scalar unit
// does in a fraction of the 64-bit sequence.
struct PairMap {
  const int* smap;
  int nsub, ns;
  __device__ __forceinline__ void split(long q, long& sig, int& s) const {
    const unsigned uq = (unsigned)q, un = (unsigned)nsub, sg = uq / un;
    const int r = (int)(uq - sg * un);
    sig = sg;
    s = smap ? smap[r] : r;
  }
  __device__ __forceinline__ long out_pair(long q) const {  // signal * ns + scale
    if (!smap) return q;
    long sig;
    int s;
    split(q, sig, s);
    return sig * ns + s;
  }
};

template <int K>
struct ScaleIn {  // X[sig][k] * conj(psi_hat(omega_k, a_s)), k = N2 k1 + col; item = pair in group
  static constexpr bool kStrided = false;  // column-major spectra: contiguous columns
  const cplx* X;
  const double* scales;
  WaveletFT w;
  long N, N1, N2, pair0;
  PairMap pm;
  double fs;
  const double* sc;  // per scale (MORLET, MEXHAT): {bin step, norm * sqrt(a)}, see cwt_fft_device
  const double* band;  // per scale (MORLET, MEXHAT): signed bins {lo, hi} of the e^-60 band
  bool early;  // A/B runs (JW_CWT_EARLY): X read issued before psi_hat's exp (same values)
  __device__ cplx operator()(long item, long k1, long col) const {
    long sig;
    int s;
    pm.split(pair0 + item, sig, s);
    const long k = N2 * k1 + col;
    if constexpr (K == JW_CWT_MORLET || K == JW_CWT_MEXHAT) {
      // bins where psi_hat is below e^-60 of its peak (cwt_band, the band kernel's cut): zero,
      // without the exp or the X read
      const double kk = (double)(k > N / 2 ? k - N : k);
      if (kk < band[2 * s] || kk > band[2 * s + 1]) return make_double2(0.0, 0.0);
      if (early) {
        // inside the band psi_hat never underflows, so the X read does not wait for the exp
        const cplx xv = X[sig * N + col * N1 + k1];
        const double wv = psi_bin<K>(w, scales, sc, s, k, N, fs).x;
        return make_double2(xv.x * wv, xv.y * wv);
      }
    }
    const cplx wv = psi_bin<K>(w, scales, sc, s, k, N, fs);
    if (wv.x == 0.0 && wv.y == 0.0) return make_double2(0.0, 0.0);  // skip the X read
    const cplx xv = X[sig * N + col * N1 + k1];
    if constexpr (K == JW_CWT_DOG || K == JW_CWT_MEYER) {
      const double cr = wv.x, ci = -wv.y;  // waveletFFT[i].conjugate(); signalFFT[i].mul(...)
      return make_double2(xv.x * cr - xv.y * ci, xv.x * ci + xv.y * cr);
    } else {  // real psi_hat: the imaginary products are exact zeros
      return make_double2(xv.x * wv.x, xv.y * wv.x);
    }
  }
};
struct CoefRow {  // CoefOut with the output pair resolved: one coefficient row
  double* row;
  long n, N1;
  double inv_n;
  bool nt;
  __device__ void operator()(long idx, long line, cplx v) const {
    const long t = line + N1 * idx;
    if (t < n) {
      cplx* o = (cplx*)(row + 2 * t);
      const cplx r = make_double2(v.x * inv_n, v.y * inv_n);
      if (nt) {
        nt_store(o, r);
      } else {
        *o = r;
      }
    }
  }
};
struct CoefOut {  // out[pair][t] = v / N for t = line + N1 * idx < n  (reverse :207-211)
  double* out;  // interleaved (re, im), B x ns x n
  long n, N1, pair0;
  double inv_n;
  bool nt;
  PairMap pm;  // item -> (signal, scale) of the output
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    const long t = line + N1 * idx;
    const long pr = pm.out_pair(pair0 + item);
    if (t < n) {
      cplx* o = (cplx*)(out + 2 * (pr * n + t));
      const cplx r = make_double2(v.x * inv_n, v.y * inv_n);
      if (nt) {
        nt_store(o, r);
      } else {
        *o = r;
      }
    }
  }
  __device__ CoefRow bind(long item) const {  // fft::bind_out: the pair looked up once per line
    return CoefRow{out + 2 * pm.out_pair(pair0 + item) * n, n, N1, inv_n, nt};
  }
  // the band kernel's output for (launch item, signal, scale): coefficient row sig * ns + s
  __device__ CoefOut at(long, long sig, int s) const {
    CoefOut o = *this;
    o.pair0 = sig * pm.ns + s;
    return o;
  }
};
// The band kernel run on a coarse grid (cwt_interp below): row `item` of the workspace U
// (M complex per launch item, natural order), unscaled, plain stores (U is read back next).
struct CoarseRow {  // u[t], t = line + N1 idx < M: unscaled, every index in range
  cplx* u;
  long N1;
  __device__ void operator()(long idx, long line, cplx v) const { u[line + N1 * idx] = v; }
};
struct CoarseOut {
  double* U;
  long M, N1, row;
  __device__ CoarseOut at(long item, long, int) const { return CoarseOut{U, M, N1, item}; }
  __device__ CoarseRow bind(long) const { return CoarseRow{(cplx*)(U + 2 * row * M), N1}; }
};


// ---------------------------------------------------------------------------------------
// Band-limited scales in one pass.  With N = N1 x 512 (input k = 512 k1 + k2, output
// t = n1 + N1 n2) the inverse FFT's row n1 is the 512-point FFT over k2 of
//   A[n1][k2] = W_N^(n1 k2) sum_k1 Z[512 k1 + k2] W_N1^(k1 n1),   Z = X conj(psi_hat).
// For a large scale, psi_hat is above e^-60 of its peak only in a few consecutive 512-bin
// blocks k1 = b0 .. b0 + nb - 1 (mod N1); below that it lies ten orders of magnitude under the
// rounding of the spectrum X itself, and those bins are dropped.  A[n1][.] then costs nb
// complex multiply-adds per element, computed in registers from the band, so the row needs
// no workspace: one pass, 16 B written per output and 24 B read per band bin (L2-resident).
// ---------------------------------------------------------------------------------------
constexpr double kBandE = 60.0;  // bins with |psi_hat| < e^-60 |psi_hat|max are dropped

struct BandScale {
  long b0;       // first 512-bin block of the band (mod N1) in the transform's own spectrum
  long psi_off;  // offset of this scale's psi_hat band in the table (nb x 512 entries)
  int nb;        // blocks in the band
  int s;         // scale index
  long fb0;      // first block in the signal's spectrum (mod Nx / 512): b0 unless coarse
  long kc;       // coarse grid (cwt_interp): signed bin of the signal's spectrum at coarse bin 0
};

// psi_hat of every bin of every band block, as the two-pass path evaluates it (psi_bin)
template <int K>
__global__ __launch_bounds__(256) void cwt_band_psi(const BandScale* bands, double* psi,
                                                    WaveletFT w, const double* scales,
                                                    const double* sc, long N, long N1, double fs) {
  const BandScale b = bands[blockIdx.y];
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)b.nb * 512) return;
  const long k = 512 * ((b.b0 + (e >> 9)) & (N1 - 1)) + (e & 511);
  psi[b.psi_off + e] = psi_bin<K>(w, scales, sc, b.s, k, N, fs).x;
}

// e^{+2 pi i m / N1} = W_N^(512 m), m < N1: the band kernel's wave-uniform twiddles
// stored as {cos, sin, cos + sin, 0} for the three-product complex multiply-add (Gauss)
__global__ __launch_bounds__(256) void cwt_band_roots(double4* w, long N, long N1, Tables T) {
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  if (m < N1) {
    const cplx r = fft::twiddle(T, 512 * m);
    w[m] = make_double4(r.x, r.y, r.x + r.y, 0.0);
  }
}

// One workgroup = 8 consecutive rows n1 of one band pair (sig, band scale): thread k2 sums the
// band for all 8 rows, the rows go through the tile into the wavefront FFT (one row per wave)
// and leave as 8-row (128-byte) output pieces.  Xn: natural-order spectra.  The twiddles
// W_N1^(k1 n1) are uniform over the workgroup: scalar loads from the N1-entry root table.
// Placement: the rpp = N1/8 workgroups of a pair share blockIdx % 8 (one XCD under the
// round-robin dispatch), so the pair's band of X is fetched into one L2, not eight (speed only).
typedef double d4v __attribute__((ext_vector_type(4)));

// MF: band sums on the matrix cores (else VALU, Gauss form); PF: the next block pair's loads
// issued before the current pair's MFMAs; WPE: waves per SIMD the registers are fitted to (6 =
// three workgroups per CU, one row group each; 4 = two, R row groups each).
// Out: CoefOut (the coefficients) or CoarseOut (a coarse-grid transform for cwt_interp, where
// N = M is the coarse length and the band is read from the signal's spectrum of length Nx).
template <bool MF, bool PF, int WPE, class Out>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE))) void cwt_band512(
    const cplx* __restrict__ Xn, const double* __restrict__ psi,
    const BandScale* __restrict__ bands, int nband, const double4* __restrict__ wN1, long N,
    long N1, long items, Out out, Tables T, int R, long Nx) {
  __shared__ double tile[fft::kTileD];  // re/im-split staging (36.9 KB)
  // 32-bit index math (the scalar unit runs 64-bit division as a ~100-instruction sequence)
  const unsigned lrpp = (unsigned)__builtin_ctzl(N1 / (fft::kT * R)), local = blockIdx.x >> 3;
  const unsigned slot = local >> lrpp;
  const unsigned item = slot * 8 + (blockIdx.x & 7);
  const unsigned rg = local - (slot << lrpp);
  if (item >= (unsigned long)items) return;
  const unsigned sig = item / (unsigned)nband;
  const BandScale b = bands[item - sig * (unsigned)nband];
  // R row groups per workgroup, one after the other: the output stores of one group drain
  // while the band sums of the next run
  const int tid = threadIdx.x, lane = tid & 63, c = tid >> 6;
  for (int it = 0; it < (WPE > 4 ? 1 : R); ++it) {  // WPE > 4: one group (registers)
  const long r0 = ((long)rg * R + it) * fft::kT;
  double im[8];  // this thread's 8 elements of the 8 rows of A: imaginary parts (re: the tile)
  __syncthreads();  // the previous group's staging reads are done with the tile
  // thread (h, kp): columns kp and kp + 256, rows r0 + 4h .. r0 + 4h + 3 (h uniform per wave,
  // so each wave-uniform twiddle feeds two columns)
  const unsigned m1 = (unsigned)N1 - 1, mx = (unsigned)(Nx >> 9) - 1;
  if constexpr (!MF) {
  const int h = tid >> 8, kp = tid & 255;
  const unsigned rr = __builtin_amdgcn_readfirstlane((unsigned)r0 + 4 * h);  // wave-uniform
  // sum_j z w as three real sums (Gauss): s1 = sum zr c, s2 = sum zi d, s3 = sum (zr+zi)(c+d);
  // re = s1 - s2, im = s3 - s1 - s2: three multiply-adds per term instead of four
  double s1[2][4], s2[2][4], s3[2][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 2; ++q) s1[q][t] = s2[q][t] = s3[q][t] = 0.0;
  const cplx* xs = Xn + (long)sig * Nx + kp;
  const double* ps = psi + b.psi_off + kp;
  constexpr int kU = 4;  // blocks whose loads are in flight together
  for (int j0 = 0; j0 < b.nb; j0 += kU) {
    cplx xv[kU][2];
    double p[kU][2];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int j = j0 + u < b.nb ? j0 + u : b.nb - 1;  // clamped; skipped below
      const unsigned kx = ((unsigned)b.fb0 + j) & mx;
      xv[u][0] = xs[512 * kx];
      xv[u][1] = xs[512 * kx + 256];
      p[u][0] = ps[512 * j];
      p[u][1] = ps[512 * j + 256];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (j0 + u >= b.nb) break;
      const unsigned k1 = ((unsigned)b.b0 + j0 + u) & m1;
      double zr[2], zi[2], zs[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        zr[q] = xv[u][q].x * p[u][q];
        zi[q] = xv[u][q].y * p[u][q];
        zs[q] = zr[q] + zi[q];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double4 w = wN1[(k1 * (rr + t)) & m1];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          s1[q][t] = fma(zr[q], w.x, s1[q][t]);
          s2[q][t] = fma(zi[q], w.y, s2[q][t]);
          s3[q][t] = fma(zs[q], w.z, s3[q][t]);
        }
      }
    }
  }
  // four-step twiddle W_N^(n1 k2), then row n1 - r0 of the tile: for column kp
  // W_N^((rr + t) kp) = W_N^(rr kp) (W_N^kp)^t (two lookups per lane, three products), for
  // column kp + 256 times the wave-uniform W_N^(256 (rr + t))
  cplx w0 = fft::twiddle(T, ((long)rr * kp) & (N - 1));
  const cplx st = fft::twiddle(T, kp);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const cplx u = fft::twiddle(T, (256L * (rr + t)) & (N - 1));  // uniform: scalar loads
    const cplx v0 = make_double2(s1[0][t] - s2[0][t], s3[0][t] - s1[0][t] - s2[0][t]);
    const cplx v1 = make_double2(s1[1][t] - s2[1][t], s3[1][t] - s1[1][t] - s2[1][t]);
    const cplx r0v = fft::cmul(v0, w0), r1v = fft::cmul(v1, fft::cmul(w0, u));
    tile[(4 * h + t) * 512 + kp] = r0v.x;
    tile[(4 * h + t) * 512 + kp + 256] = r1v.x;
    im[t] = r0v.y;
    im[4 + t] = r1v.y;
    if (t < 3) w0 = fft::cmul(w0, st);
  }
  } else {
  // The same sums as a real GEMM on the matrix cores (v_mfma_f64_16x16x4_f64): rows 0..7 are
  // Re A[r0 + t][.], rows 8..15 Im A[r0 + t][.]; K runs over (block j, re/im of Z_j):
  //   [Re; Im] A = [[Re W, -Im W], [Im W, Re W]] [Re Z; Im Z],   W_tj = W_N1^(k1_j (r0 + t)).
  // Wave c owns columns 64c .. 64c + 63 (four 16-column tiles); one MFMA per tile consumes two
  // blocks.  Lane l holds A[l & 15][k = l >> 4] and B[k = l >> 4][col l & 15] (the f32
  // 16x16x4 operand maps), and D[row (l >> 4) + 4 r][col l & 15] (the f64 C/D map).
  const int tr = lane & 15, kq = lane >> 4;  // A row / B column, K index
  const int t = tr & 7, im_row = tr >> 3, jo = kq >> 1, zc = kq & 1;
  d4v acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = d4v{0.0, 0.0, 0.0, 0.0};
  // each lane loads only the part of Z it feeds (re for kq even, im for kq odd): 8-byte loads
  const double* xs = (const double*)(Xn + (long)sig * Nx + 64 * c + tr) + zc;
  const double* ps = psi + b.psi_off + 64 * c + tr;
  // loads of the next block pair are issued before the current pair's MFMAs (the L2 latency of
  // one pair hides under the other's arithmetic); past the band the index clamps to nb - 1 and
  // the twiddle row is zeroed
  auto load = [&](int j0, double (&xv)[4], double (&pv)[4], double& av) {
    const int j = j0 + jo;
    const bool in = j < b.nb;
    const int jj = in ? j : b.nb - 1;
    const unsigned k1 = ((unsigned)b.b0 + jj) & m1, kx = ((unsigned)b.fb0 + jj) & mx;
    const double4 w = wN1[(k1 * ((unsigned)r0 + t)) & m1];
    // A[tr][kq]: Re row: (Re W, -Im W) for (Re Z, Im Z); Im row: (Im W, Re W)
    av = im_row ? (zc ? w.x : w.y) : (zc ? -w.y : w.x);
    av = in ? av : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xv[q] = xs[2 * (512L * kx + 16 * q)];
      pv[q] = ps[512 * jj + 16 * q];
    }
  };
  double xv[4], pv[4], av;
  load(0, xv, pv, av);
  for (int j0 = 0; j0 < b.nb; j0 += 2) {
    double xn[4], pn[4], an;
    if (PF) load(j0 + 2, xn, pn, an);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double bv = xv[q] * pv[q];
      acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
    }
    if (PF) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xv[q] = xn[q];
        pv[q] = pn[q];
      }
      av = an;
    } else {
      load(j0 + 2, xv, pv, av);
    }
  }
  // lane: D rows (l >> 4) + 4 r -> Re of rows t0, t0 + 4 (r = 0, 1), Im of them (r = 2, 3);
  // four-step twiddle W_N^(n1 col), col = 64 c + 16 q + tr, by a step of 16 columns per tile
  const int t0 = lane >> 4;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const long n1 = r0 + t0 + 4 * e, col0 = 64 * c + tr;
    cplx w0 = fft::twiddle(T, (n1 * col0) & (N - 1));
    const cplx st = fft::twiddle(T, (16 * n1) & (N - 1));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const cplx v = fft::cmul(make_double2(acc[q][e], acc[q][e + 2]), w0);
      tile[(t0 + 4 * e) * 512 + (int)col0 + 16 * q] = v.x;  // re now, im after the first read
      im[4 * e + q] = v.y;
      if (q < 3) w0 = fft::cmul(w0, st);
    }
  }
  }
  // rows r0 .. r0 + 7 of A through the tile (re, then im) into wave c's line r0 + c
  cplx a[8];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; ++r) a[r].x = tile[c * 512 + lane + 64 * r];
  __syncthreads();
  if constexpr (!MF) {
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[(4 * (tid >> 8) + (i & 3)) * 512 + (tid & 255) + 256 * (i >> 2)] = im[i];
  } else {
    const int t0 = lane >> 4, col0 = 64 * c + (lane & 15);
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[(t0 + 4 * (i >> 2)) * 512 + col0 + 16 * (i & 3)] = im[i];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; ++r) a[r].y = tile[c * 512 + lane + 64 * r];
  __syncthreads();
  const Out o = out.at(item, sig, b.s);  // one output row per workgroup
  fft::pass512_tail_split<1, false>(a, o, N, 512L, T, 0L, r0, tile);
  }
}


// The band kernel for grids of N1 >= 16 rows, two row groups per workgroup: rows r0 .. r0 + 7
// and r0 + N1/2 .. r0 + N1/2 + 7.  W_N1^(k1 (n1 + N1/2)) = (-1)^k1 W_N1^(k1 n1), so with the
// band's sums split by the parity of the block index k1,
//   A[n1] ~ S_even(n1) + S_odd(n1),   A[n1 + N1/2] ~ S_even(n1) - S_odd(n1),
// the MFMAs of one row group give both (half the band-sum work per row).  Each MFMA takes two
// blocks of one parity (j and j + 2).  MFMA only; one workgroup = 16 rows, 2 per CU (WPE 4).
#ifndef JW_CWT_PAR_PF
#define JW_CWT_PAR_PF 1
#endif
// The lane's twiddles by recurrence (one complex product per block group, VALU that is ~7 % busy
// here) instead of a dependent table gather: cfg3 2,374 -> 2,395 Msamples/s same box, accuracy
// unchanged at the tests' bars (profiles/r06/ab/cwt_par_rec/); 0 = the table (A/B builds).
#ifndef JW_CWT_PAR_REC
#define JW_CWT_PAR_REC 1
#endif
template <class Out>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void cwt_band512_par(
    const cplx* __restrict__ Xn, const double* __restrict__ psi,
    const BandScale* __restrict__ bands, int nband, const double4* __restrict__ wN1, long N,
    long N1, long items, Out out, Tables T, long Nx) {
  __shared__ double tile[fft::kTileD];
  const unsigned lrpp = (unsigned)__builtin_ctzl(N1 / (2 * fft::kT)), local = blockIdx.x >> 3;
  const unsigned slot = local >> lrpp;
  const unsigned item = slot * 8 + (blockIdx.x & 7);
  const unsigned rg = local - (slot << lrpp);
  if (item >= (unsigned long)items) return;
  const unsigned sig = item / (unsigned)nband;
  const BandScale b = bands[item - sig * (unsigned)nband];
  const int tid = threadIdx.x, lane = tid & 63, c = tid >> 6;
  const long r0 = (long)rg * fft::kT;
  const unsigned m1 = (unsigned)N1 - 1, mx = (unsigned)(Nx >> 9) - 1;
  const int tr = lane & 15, kq = lane >> 4;
  const int t = tr & 7, im_row = tr >> 3, jo = kq >> 1, zc = kq & 1;
  const double* xs = (const double*)(Xn + (long)sig * Nx + 64 * c + tr) + zc;
  const double* ps = psi + b.psi_off + 64 * c + tr;
  // blocks j0 + 2 jo (jo = 0, 1: two blocks of one parity per MFMA)
#if JW_CWT_PAR_REC
  // the lane's twiddle W_N1^(k1 (r0 + t)) by recurrence over its blocks (k1 steps by 4 per
  // call of load; at most nb / 4 <= 31 products: ~1e-14 relative)
  cplx wr = make_double2(0.0, 0.0), ws = make_double2(0.0, 0.0);
  auto rec_init = [&](int par) {
    const unsigned e = (((unsigned)b.b0 + par + 2 * jo) * ((unsigned)r0 + t)) & m1;
    const double4 w0 = wN1[e], s4 = wN1[(4u * ((unsigned)r0 + t)) & m1];
    wr = make_double2(w0.x, w0.y);
    ws = make_double2(s4.x, s4.y);
  };
#endif
  auto load = [&](int j0, double (&xv)[4], double (&pv)[4], double& av) {
    const int j = j0 + 2 * jo;
    const bool in = j < b.nb;
    const int jj = in ? j : b.nb - 1;
    const unsigned kx = ((unsigned)b.fb0 + jj) & mx;
#if JW_CWT_PAR_REC
    const cplx w = wr;
    wr = fft::cmul(wr, ws);
#else
    const unsigned k1 = ((unsigned)b.b0 + jj) & m1;
    const double4 w = wN1[(k1 * ((unsigned)r0 + t)) & m1];
#endif
    av = im_row ? (zc ? w.x : w.y) : (zc ? -w.y : w.x);
    av = in ? av : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xv[q] = xs[2 * (512L * kx + 16 * q)];
      pv[q] = ps[512 * jj + 16 * q];
    }
  };
  auto sums = [&](int par, d4v (&acc)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = d4v{0.0, 0.0, 0.0, 0.0};
    double xv[4], pv[4], av;
#if JW_CWT_PAR_REC
    rec_init(par);
#endif
    load(par, xv, pv, av);
    for (int j0 = par; j0 < b.nb; j0 += 4) {
#if JW_CWT_PAR_PF  // the next pair's loads before this pair's MFMAs (16 more VGPRs)
      double xn[4], pn[4], an;
      load(j0 + 4, xn, pn, an);
#endif
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, xv[q] * pv[q], acc[q], 0, 0, 0);
#if JW_CWT_PAR_PF
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xv[q] = xn[q];
        pv[q] = pn[q];
      }
      av = an;
#else
      load(j0 + 4, xv, pv, av);
#endif
    }
  };
  d4v lo[4], hi[4];
  sums(0, lo);
  sums(1, hi);
  // j even <-> k1 parity of b0 (N1 is even): hi = +-(S_j-even - S_j-odd)
  const double sg = (b.b0 & 1) ? -1.0 : 1.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const d4v e = lo[q], o = hi[q];
    lo[q] = e + o;
    hi[q] = sg * (e - o);
  }
  const Out o = out.at(item, sig, b.s);
  auto finish = [&](const d4v (&acc)[4], long rb) {
    double im[8];
    const int t0 = lane >> 4;
    __syncthreads();  // the previous group's staging reads are done with the tile
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const long n1 = rb + t0 + 4 * e, col0 = 64 * c + tr;
      cplx w0 = fft::twiddle(T, (n1 * col0) & (N - 1));
      const cplx st = fft::twiddle(T, (16 * n1) & (N - 1));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const cplx v = fft::cmul(make_double2(acc[q][e], acc[q][e + 2]), w0);
        tile[(t0 + 4 * e) * 512 + (int)col0 + 16 * q] = v.x;
        im[4 * e + q] = v.y;
        if (q < 3) w0 = fft::cmul(w0, st);
      }
    }
    cplx a[8];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r].x = tile[c * 512 + lane + 64 * r];
    __syncthreads();
    const int col0 = 64 * c + (lane & 15);
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[(t0 + 4 * (i >> 2)) * 512 + col0 + 16 * (i & 3)] = im[i];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r].y = tile[c * 512 + lane + 64 * r];
    __syncthreads();
    fft::pass512_tail_split<1, false>(a, o, N, 512L, T, 0L, rb, tile);
  };
  finish(lo, r0);
  // nothing of the second group's tail may be hoisted into the first's (its values would be live
  // through the first tail: spills)
  __builtin_amdgcn_sched_barrier(0);
  finish(hi, r0 + N1 / 2);
}

// ---------------------------------------------------------------------------------------
// Band scales on a coarse grid.  A scale whose band (signed bins lo .. hi, centred on the
// 512-aligned bin kc) fits in |m| <= M/4 of an M-point spectrum, M = N / P, gives
//   y[t] = (1/N) sum_k Z[k] e^{2 pi i k t / N} = e^{2 pi i kc t / N} f(t / P) / N,
//   f(tau) = sum_m Z[kc + m] e^{2 pi i m tau / M}      (a band-limited, M-periodic function),
// and f is interpolated from the coarse samples u[s] = sum_m (Z[kc + m] / Phi(m / M)) e^{2 pi i m s / M}
// (an M-point inverse DFT, run by the band kernel on the coarse grid) with a Kaiser-Bessel kernel
// phi of width W: f(tau) = sum_s u[s] phi(tau - s) up to the kernel's aliasing, Phi being phi's
// Fourier transform (the deconvolution; Jackson et al. 1991).  Oversampling M >= 2.5 |m|max
// (sigma = 1.25) with W = 18 bounds that error near 1e-14 of the scale's peak (numpy prototype
// over the cfg3 scales: <= 1.2e-14; tests/test_cwt_gpu.py).  The coarse transform is P times
// smaller than the scale's N-point one; the interpolation reads it from L2 and writes each
// coefficient once, in 1 KB pieces per wave.
// ---------------------------------------------------------------------------------------
constexpr int kInterpW = 18;                   // kernel width (coarse samples)
constexpr int kInterpHalf = kInterpW / 2;
constexpr int kInterpTaps = 2 * kInterpHalf + 1;  // taps per output: s0 - 9 .. s0 + 9
constexpr int kInterpStride = 20;              // weights per r in the table
constexpr double kInterpSigma = 1.25;           // minimum oversampling of the band on the grid
// beta = pi sqrt((W / sigma)^2 (sigma - 1/2)^2 - 0.8) (Beatty et al. 2005)
constexpr double kInterpBeta = 33.812645176356604;

// Phi(nu) = W sinh(sqrt(beta^2 - (pi W nu)^2)) / sqrt(...), the transform of
// phi(x) = I0(beta sqrt(1 - (2x/W)^2)), |x| <= W/2 (|nu| <= 1/2 here, so the root is real)
__device__ __forceinline__ double kb_phi_hat(double nu) {
  const double a = kPi * kInterpW * nu;
  const double q = sqrt(kInterpBeta * kInterpBeta - a * a);
  return kInterpW * sinh(q) / q;
}

// psi_hat of every bin of every band block (as psi_bin evaluates it) divided by Phi at the bin's
// coarse frequency m / M, m = kk - kc
template <int K>
__global__ __launch_bounds__(256) void cwt_interp_psi(const BandScale* bands, double* psi,
                                                      WaveletFT w, const double* scales,
                                                      const double* sc, long N, long N1, double fs,
                                                      long M) {
  const BandScale b = bands[blockIdx.y];
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)b.nb * 512) return;
  const long k = 512 * ((b.fb0 + (e >> 9)) & (N1 - 1)) + (e & 511);
  const long kk = k > N / 2 ? k - N : k;
  psi[b.psi_off + e] = psi_bin<K>(w, scales, sc, b.s, k, N, fs).x / kb_phi_hat((double)(kk - b.kc) / (double)M);
}

// One workgroup = interp_tc<LOGP>() = min(1024 P, 8192) consecutive coefficients t of one (signal, scale)
// pair from its coarse row U[item] (M = N / P samples, P = 2^LOGP): the 1024 + 19 coarse samples
// the chunk needs are staged in LDS.  Lane l of wave v takes t = t0 + v TC / 4 + l + 64 i, so
// its r = t mod P is fixed (P <= 64) and its 19 weights phi(r / P + 9 - k) / N (wtab, host-made)
// stay in registers; the lanes of one s0 = t / P read the same samples (LDS broadcast).  The
// phase e^{2 pi i kc t / N} is a table lookup per lane every 32 outputs and a wave-uniform step
// per 64 positions in between.  (Chunks of 4096 for every P ran the P = 32, 64 grids at 5.3-5.4
// TB/s against 6.2-6.3 for P = 4, 8; 65536 for P = 64 took it 1116 -> 1062 us, 8192 -> 1000 us:
// the per-workgroup start -- the weight loads, the staging, the phase lookups -- amortised over
// more outputs, with enough workgroups left for an even finish; profiles/r05/ab/cwt_interp_tc_z.txt)
#ifndef JW_INTERP_TCMAX  // A/B builds: the largest chunk
#define JW_INTERP_TCMAX 8192
#endif
template <int LOGP>
constexpr long interp_tc() {
  return (1024L << LOGP) < JW_INTERP_TCMAX ? (1024L << LOGP) : JW_INTERP_TCMAX;
}
template <int LOGP>
__global__ __launch_bounds__(256) void cwt_interp(const cplx* __restrict__ U, long M,
                                                  const BandScale* __restrict__ bands, int nsc,
                                                  const double* __restrict__ wtab, long N, long n,
                                                  int ns, long sig0, double* __restrict__ out,
                                                  bool nt, Tables T, int chunks) {
  constexpr int P = 1 << LOGP;
  constexpr long TC = interp_tc<LOGP>();
  constexpr int NU = (int)(TC / P) + kInterpTaps, PER = (int)(TC / 4 / 64), RS = 32;
  static_assert(PER % RS == 0 || PER < RS, "phase resync period");
  __shared__ cplx us[NU];
  const unsigned bid = blockIdx.x, item = bid / (unsigned)chunks;
  const unsigned chunk = bid - item * (unsigned)chunks;
  const unsigned sl = item / (unsigned)nsc;
  const BandScale b = bands[item - sl * (unsigned)nsc];
  const long t0 = (long)chunk * TC;
  const cplx* u = U + (long)item * M;
  const long s_lo = (t0 >> LOGP) - kInterpHalf;  // first staged sample (mod M)
  for (int j = threadIdx.x; j < NU; j += 256) {
    long q = s_lo + j;
    q = q < 0 ? q + M : (q >= M ? q - M : q);
    us[j] = u[q];
  }
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long tl = t0 + (long)wv * (TC / 4) + lane;  // this lane's first output
  const int r = (int)(tl & (P - 1));
  double wr[kInterpTaps];
#pragma unroll
  for (int k = 0; k < kInterpTaps; ++k) wr[k] = wtab[r * kInterpStride + k];
  const long kcu = ((b.kc % N) + N) % N;
  const cplx st = fft::twiddle(T, (kcu * 64) & (N - 1));
  double* row = out + 2 * ((sig0 + sl) * ns + b.s) * n;
  __syncthreads();
  const int base0 = (int)((tl >> LOGP) - (t0 >> LOGP));
  for (int i0 = 0; i0 < PER; i0 += RS) {
    cplx ph = fft::twiddle(T, (kcu * (tl + 64L * i0)) & (N - 1));
#pragma unroll 4
    for (int i = i0; i < i0 + (PER < RS ? PER : RS); ++i) {
      const long t = tl + 64 * i;
      const int base = base0 + ((64 * i) >> LOGP);
      double ar = 0.0, ai = 0.0;
#pragma unroll
      for (int k = 0; k < kInterpTaps; ++k) {
        const cplx v = us[base + k];
        ar = __builtin_fma(wr[k], v.x, ar);
        ai = __builtin_fma(wr[k], v.y, ai);
      }
      const cplx y = fft::cmul(make_double2(ar, ai), ph);
      if (t < n) {
        cplx* o = (cplx*)(row + 2 * t);
        if (nt) {
          fft::nt_store(o, y);
        } else {
          *o = y;
        }
      }
      ph = fft::cmul(ph, st);
    }
  }
}

}  // namespace

// A second stream per (host thread, device) for the band kernel, so that it runs beside the
// two-pass pipeline instead of before it: the band kernel is FP64-issue and latency bound
// (§5.4 of DESIGN.md), the two-pass passes mostly HBM bound, and run together they share the
// CUs.  fork: the band kernel waits for everything queued on the caller's stream so far; join:
// the caller's stream waits for the band kernel before anything after it (and before the
// stream-ordered frees of the call's buffers).
struct SideStream {
  int dev = -1;
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  ~SideStream() {
    if (dev < 0) return;
    (void)hipSetDevice(dev);
    if (s) (void)hipStreamSynchronize(s);
    for (hipEvent_t e : {fork, join})
      if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
  }
};
static int side_stream(SideStream** out) {
  static thread_local std::vector<std::unique_ptr<SideStream>> sides;  // by device ordinal
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  if ((int)sides.size() <= dev) sides.resize(dev + 1);
  if (!sides[dev]) {
    auto ss = std::make_unique<SideStream>();
    ss->dev = dev;
    JW_HIP_TRY(hipStreamCreateWithFlags(&ss->s, hipStreamNonBlocking));
    JW_HIP_TRY(hipEventCreateWithFlags(&ss->fork, hipEventDisableTiming));
    JW_HIP_TRY(hipEventCreateWithFlags(&ss->join, hipEventDisableTiming));
    sides[dev] = std::move(ss);
  }
  *out = sides[dev].get();
  return JW_OK;
}
// Destroyed before the StreamAllocs declared ahead of it: the caller's stream waits for the side
// stream's work before the buffers that work reads are freed.  The join event is recorded here,
// at scope exit, behind everything the call queued on the side stream, so an early error return
// after some side launches joins them too (no stale or never-recorded event).
struct JoinGuard {
  hipStream_t s = nullptr;
  SideStream* side = nullptr;
  ~JoinGuard() {
    if (!side) return;
    (void)hipEventRecord(side->join, side->s);
    (void)hipStreamWaitEvent(s, side->join, 0);
  }
};

// The band of scale a (bins whose psi_hat is above e^-kBandE of its peak) as 512-bin blocks
// b0 .. b0 + nb - 1 mod N1; false when the band is not known in closed form (Paul, DOG,
// Meyer) or wraps the whole spectrum.  Morlet: |f - fc| <= sqrt(E / (2 pi^2 fb)) with
// f = kk a fs / N; Mexican hat: u = sigma^2 om^2 / 2 with u - ln u <= E + 1 (om^2 e^-u
// against its peak 2/(e sigma^2)), om = 2 pi kk a fs / N.  Two bins of margin each side.
static bool cwt_band(int wavelet, const WaveletFT& w, double a, double fs, long N, long* b0,
                     int* nb, double* lo_out = nullptr, double* hi_out = nullptr) {
  double lo, hi;
  if (wavelet == JW_CWT_MORLET) {
    const double step = a * fs / (double)N;
    if (!(w.p0 > 0) || !(step > 0)) return false;
    const double d = std::sqrt(kBandE / (2.0 * kPi * kPi * w.p0));
    lo = std::floor((w.p1 - d) / step) - 2;
    hi = std::ceil((w.p1 + d) / step) + 2;
  } else if (wavelet == JW_CWT_MEXHAT) {
    const double step = 2.0 * kPi * a * fs / (double)N;
    if (!(w.p0 > 0) || !(step > 0)) return false;
    const double u = kBandE + 2.0 + std::log(kBandE + 1.0 + std::log(kBandE + 1.0));
    const double W = std::ceil(std::sqrt(2.0 * u) / w.p0 / step) + 2;
    lo = -W;
    hi = W;
  } else {
    return false;
  }
  if (!(lo > -(double)(N / 2)) || !(hi < (double)(N / 2))) return false;
  if (lo_out) *lo_out = lo;
  if (hi_out) *hi_out = hi;
  const long blo = (long)std::floor(lo / 512.0), bhi = (long)std::floor(hi / 512.0);
  const long N1 = N / 512;
  *nb = (int)(bhi - blo + 1);
  *b0 = ((blo % N1) + N1) % N1;
  return true;
}

// The coarse grid of a band (signed bins lo .. hi of the N-point spectrum) for cwt_interp:
// centre kc on a 512-bin block boundary (so the coarse blocks are the signal's blocks), and the
// smallest power of two M >= 4096 with the band inside |m| <= M / (2 kInterpSigma) (the
// oversampling the kernel's error bound assumes) and its whole 512-bin blocks inside [-M/2, M/2).
// cb0 = the band's first block on the coarse grid (mod M / 512).  P = N / M <= 64 (the
// interpolation kernel's lane mapping).
static bool coarse_grid(double lo, double hi, long N, long* M_out, long* kc_out, long* cb0) {
  const long blo = (long)std::floor(lo / 512.0), bhi = (long)std::floor(hi / 512.0);
  long s2 = blo + bhi + 1;  // floor((blo + bhi + 1) / 2)
  const long kcb = s2 >= 0 ? s2 / 2 : -((-s2 + 1) / 2);
  const long kc = 512 * kcb;
  const double hw = std::max((double)kc - lo, hi - (double)kc);
  long M = std::max(4096L, N / 64);
  while (M <= N && ((double)M < 2.0 * kInterpSigma * hw || 512 * (kcb - blo) > M / 2 ||
                     512 * (bhi + 1 - kcb) > M / 2))
    M <<= 1;
  if (M > N / 2) return false;
  const long n1 = M / 512;
  *M_out = M;
  *kc_out = kc;
  *cb0 = (((blo - kcb) % n1) + n1) % n1;
  return true;
}

struct CoarseGroup {
  long M;
  int first, n, nb_hi;
};

// phi(x) / N at x = r / P + kInterpHalf - k for r < P, k < kInterpTaps (zero outside |x| <=
// W / 2): the interpolation weights of cwt_interp, phi(x) = I0(beta sqrt(1 - (2x/W)^2))
static void interp_weights(long P, long N, std::vector<double>& wt) {
  wt.assign((size_t)P * kInterpStride, 0.0);
  for (long r = 0; r < P; ++r)
    for (int k = 0; k < kInterpTaps; ++k) {
      const long double x = (long double)r / P + kInterpHalf - k;
      const long double z = 1.0L - (2.0L * x / kInterpW) * (2.0L * x / kInterpW);
      if (z < 0) continue;
      const long double b = (long double)kInterpBeta * std::sqrt(z), q = b * b / 4.0L;
      long double term = 1.0L, sum = 1.0L;  // I0(b) = sum (b^2/4)^j / (j!)^2
      for (int j = 1; j < 200 && term > sum * 1e-22L; ++j) {
        term *= q / ((long double)j * j);
        sum += term;
      }
      wt[(size_t)r * kInterpStride + k] = (double)(sum / (long double)N);
    }
}

// One interpolation launch of the coarse-grid path: `items` rows of U (from row 0), signals
// from sg0, of one group of equal M.
struct InterpJob {
  const cplx* U;
  long M, P, sg0, items;
  const BandScale* gb;
  int gn;
  const double* gw;
};

// Which path each scale of a jw_cwt_fft call takes (band kernel, coarse grid, two-pass), with
// the wavelet's spectrum parameters: the rule cwt_fft_device runs and jw_cwt_fft_paths reports.
struct CwtSplit {
  WaveletFT w{};
  std::vector<BandScale> bands, coarse;  // coarse sorted by M, grouped in groups
  std::vector<int> full;                 // two-pass scales
  std::vector<CoarseGroup> groups;
  long psi_total = 0;
  int nb_hi = 0;
};
static void cwt_split(int wavelet, const double* params, long N, const double* scales_host, int ns,
                      double fs, CwtSplit* sp) {
  WaveletFT& w = sp->w;
  w = WaveletFT{};
  w.kind = wavelet;
  if (wavelet == JW_CWT_MORLET) {
    w.p0 = params[0];
    w.p1 = params[1];
    w.norm = std::sqrt(2.0 * kPi * w.p0);  // MorletWavelet.java:117
  } else if (wavelet == JW_CWT_MEXHAT) {
    w.p0 = params[0];
    const double nc = 2.0 / (std::sqrt(3.0 * w.p0) * std::pow(kPi, 0.25));  // :72
    w.norm = nc * w.p0 * std::sqrt(2.0 * kPi);                              // :111
  } else if (wavelet == JW_CWT_PAUL) {
    w.ord = (int)params[0];
    w.norm = std::sqrt(2.0 * kPi);  // PaulWavelet.java:159
  } else if (wavelet == JW_CWT_DOG) {
    w.ord = (int)params[0];
    w.p0 = params[1];
    w.norm = std::sqrt(2.0 * kPi) * std::pow(w.p0, w.ord + 1);  // DOGWavelet.java:189-190
    double df = 1.0;  // doubleFactorial(2n - 1) :376-382
    for (int i = 2 * w.ord - 1; i > 0; i -= 2) df *= i;
    w.norm2 = std::sqrt(df / (std::pow(2, w.ord) * std::sqrt(kPi) *
                              std::pow(w.p0, 2 * w.ord + 1)));  // :357-366
  } else {
    w.norm = std::sqrt(2.0 * kPi);  // MeyerWavelet.java:244
  }
  w.p2 = wavelet == JW_CWT_MORLET ? -2.0 * kPi * kPi * w.p0 : -0.5 * w.p0 * w.p0;
  // Scales whose band spans at most nbmax 512-bin blocks run in one pass (cwt_band512); the
  // rest through the two-pass FFT.  One pass costs ~1.1 us per (signal, scale) pair at N = 2^18
  // plus ~0.05 us per block, two passes ~3 us: the measured optimum at cfg3 is nbmax = 32
  // (profiles/r02/cwt_band_sweep_r02.log).  env JW_CWT_BAND (A/B runs): nbmax, 0 = all two-pass.
  // Before either, a band scale whose band fits a coarse grid of M = N / P points with P >=
  // pmin runs there (cwt_interp): env JW_CWT_INTERP (A/B runs and tests) = pmin, 0 = never.
  const char* gbd = knob("JW_CWT_BAND");
  const int nbmax = gbd ? std::atoi(gbd) : 32;
  const char* gip = knob("JW_CWT_INTERP");
  const long pmin = gip ? std::atol(gip) : 4;
  const long N1b = N / 512;
  auto& bands = sp->bands;
  auto& coarse = sp->coarse;  // sorted by M below
  std::vector<long> coarse_m;
  auto& full = sp->full;
  long& psi_total = sp->psi_total;
  int& nb_hi = sp->nb_hi;
  for (int i = 0; i < ns; ++i) {
    long b0 = 0;
    int nb = 0;
    double lo = 0.0, hi = 0.0;
    // (band and coarse-grid paths up to 2^26; the three-pass lengths run every scale two-pass)
    const bool bandok = N >= 8192 && N <= (1L << 26) &&
                        cwt_band(wavelet, w, scales_host[i], fs, N, &b0, &nb, &lo, &hi) &&
                        nb <= N1b;
    if (bandok && pmin > 0) {
      long M = 0, kc = 0, cb0 = 0;
      if (coarse_grid(lo, hi, N, &M, &kc, &cb0) && M <= N / pmin) {
        coarse.push_back(BandScale{cb0, 0, nb, i, b0, kc});
        coarse_m.push_back(M);
        continue;
      }
    }
    if (bandok && nbmax > 0 && nb <= nbmax) {
      bands.push_back(BandScale{b0, psi_total, nb, i, b0, 0});
      psi_total += 512L * nb;
      nb_hi = std::max(nb_hi, nb);
    } else {
      full.push_back(i);
    }
  }
  // coarse scales grouped by M (one band-kernel and one interpolation launch per group)
  auto& groups = sp->groups;
  {
    std::vector<int> ord(coarse.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int)i;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return coarse_m[a] < coarse_m[b]; });
    std::vector<BandScale> sorted;
    for (int k : ord) {
      BandScale b = coarse[k];
      b.psi_off = psi_total;
      psi_total += 512L * b.nb;
      if (groups.empty() || groups.back().M != coarse_m[k])
        groups.push_back(CoarseGroup{coarse_m[k], (int)sorted.size(), 0, 0});
      groups.back().n++;
      groups.back().nb_hi = std::max(groups.back().nb_hi, b.nb);
      sorted.push_back(b);
    }
    coarse = std::move(sorted);
  }
}

// Group sizes: signals per forward chunk and (signal, scale) pairs per inverse group, so the
// workspace A stays ~96 MB at N = 2^18 (two of them when pipelined).
int cwt_fft_device(int wavelet, const double* params, const double* x, long n,
                   const double* scales_host, int ns, double fs, int padding, double* out,
                   int batch, hipStream_t s) {
  if (n == 0 || ns == 0 || batch == 0) return JW_OK;
  long N = 1;
  while (N < n) N <<= 1;  // MathUtils.nextPowerOfTwo :46-49
  // 2^25 and 2^26 run the generic four-step passes (8192-point lines in 128 KB of LDS), 2^27
  // and 2^28 three passes (fft::run_fft: the 16384 / 32768-point rows as FFTs of their own,
  // through a second workspace), every scale two-pass
  if (N > (1L << 28)) return fail(JW_ERR_UNSUPPORTED, "CWT padded length %ld > 2^28", N);
  const bool three = N > (1L << 26);
  if ((long)batch * ns >= (1L << 31))
    return fail(JW_ERR_UNSUPPORTED, "CWT batch x scales = %ld >= 2^31", (long)batch * ns);
  Tables T;
  int st = fft::tables(N, &T);
  if (st != JW_OK) return st;
  CwtSplit sp;
  cwt_split(wavelet, params, N, scales_host, ns, fs, &sp);
  const WaveletFT& w = sp.w;
  const auto& bands = sp.bands;
  const auto& coarse = sp.coarse;
  const auto& full = sp.full;
  const auto& groups = sp.groups;
  const long psi_total = sp.psi_total;
  const int nb_hi = sp.nb_hi;
  const long N1b = N / 512;
  const char* gnt = knob("JW_CWT_NT");  // A/B runs: bit 1 = NT stores of A, 2 = of coeffs
  const int ntm = gnt ? std::atoi(gnt) : 2;  // measured best: NT coefficient stores only
  const int nband = (int)bands.size(), nfull = (int)full.size();
  const char* gmb = knob("JW_CWT_GROUP_MB");  // A/B runs: workspace size in MiB
  const long ws = (gmb ? std::atol(gmb) : 96L) << 20;  // 96 MB: profiles/r05/ab/cwt_group_p.txt
  const long per = std::max(1L, ws / (N * (long)sizeof(cplx)));
  const long pairs = (long)batch * nfull;  // two-pass pairs
  // two-pass groups of whole signals (all of a signal's two-pass scales in one group) when they
  // fit the workspace: the group's pass 1 then reads one signal's spectrum, which stays cached
  // (cfg3, 24 two-pass scales: 24-pair groups in a 96 MB workspace 27.7-27.9 ms against 32-pair
  // groups in 128 MB 29.0-29.2 ms; 80 / 112 MB 29.1 / 28.5 ms; profiles/r05/ab/cwt_group_*.txt)
  const long per_g = nfull > 0 && per >= nfull ? per / nfull * nfull : per;
  const long gsig = std::min<long>(batch, per), gpair = std::max(1L, std::min<long>(pairs, per_g));
  // N = 2^18 (512 x 512): the pairs' inverse FFTs are software-pipelined over two workspaces
  // (run_fft512_pipelined); env JW_CWT_PIPE=0 runs the groups one after the other (A/B runs).
  const char* gpp = knob("JW_CWT_PIPE");
  const char* gel = knob("JW_CWT_EARLY");
  const bool early = !(gel && gel[0] == '0');
  const bool pipe = N == (1L << 18) && pairs > gpair && !(gpp && gpp[0] == '0');
  StreamAllocs mem(s);
  JoinGuard join{s, nullptr};  // declared after mem: joins before mem's frees
  cplx *X = nullptr, *A = nullptr, *Xn = nullptr;
  double4* wN1 = nullptr;
  double *dsc = nullptr, *psi = nullptr;
  BandScale* dbands = nullptr;
  int* dsmap = nullptr;
  const long a_items = std::max(gsig, pipe ? 2 * gpair : gpair);
  JW_HIP_TRY(mem.alloc(&X, (size_t)batch * N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&A, (size_t)a_items * N * sizeof(cplx)));
  cplx* Bw = nullptr;  // the three-pass lengths' second workspace (fft::run_fft)
  if (three) JW_HIP_TRY(mem.alloc(&Bw, (size_t)a_items * N * sizeof(cplx)));
  // device scale table: [a_0 .. a_{ns-1} | (step, norm*sqrt(a)) per scale | (lo, hi) per scale]
  // (ScaleIn); (lo, hi) = the e^-60 band in signed bins, or the whole spectrum
  std::vector<double> hsc(5 * (size_t)ns);
  for (int i = 0; i < ns; ++i) {
    const double a = scales_host[i];
    hsc[i] = a;
    hsc[ns + 2 * i] = wavelet == JW_CWT_MEXHAT ? 2.0 * kPi * a * fs / (double)N : a * fs / (double)N;
    hsc[ns + 2 * i + 1] = w.norm * std::sqrt(a);
    long b0;
    int nb;
    double lo = -(double)N, hi = (double)N;
    if (!cwt_band(wavelet, w, a, fs, N, &b0, &nb, &lo, &hi)) {
      lo = -(double)N;
      hi = (double)N;
    }
    hsc[3 * ns + 2 * i] = lo;
    hsc[3 * ns + 2 * i + 1] = hi;
  }
  JW_HIP_TRY(mem.alloc(&dsc, hsc.size() * sizeof(double)));
  JW_HIP_TRY(upload_async(dsc, hsc.data(), hsc.size() * sizeof(double), s));
  BandScale* dcoarse = nullptr;
  if (nband > 0 || !coarse.empty()) {
    JW_HIP_TRY(mem.alloc(&Xn, (size_t)batch * N * sizeof(cplx)));
    JW_HIP_TRY(mem.alloc(&psi, (size_t)psi_total * sizeof(double)));
  }
  if (nband > 0) {
    JW_HIP_TRY(mem.alloc(&wN1, (size_t)N1b * sizeof(double4)));
    JW_HIP_TRY(mem.alloc(&dbands, bands.size() * sizeof(BandScale)));
    JW_HIP_TRY(upload_async(dbands, bands.data(), bands.size() * sizeof(BandScale), s));
  }
  // coarse-grid workspaces (allocated and filled here, on the caller's stream, before the band
  // stream forks): U ~128 MB of coarse rows (gchunk signals of a group at a time), the
  // interpolation weights of each group's P, the row roots of each group's M
  cplx* U = nullptr;
  double* dwt = nullptr;
  double4* wroots = nullptr;
  std::vector<long> gchunk(groups.size()), uoff(groups.size(), 0);
  std::vector<Tables> gT(groups.size());
  // JW_CWT_SPLIT=1: the coarse band kernels of every group and signal run first, on the side
  // stream beside the two-pass chain (they are latency-bound, the chain HBM-bound), into one U
  // per group; the interpolations (HBM-bound) follow the chain on the caller's stream.
  const char* gsp = knob("JW_CWT_SPLIT");
  bool split = gsp && gsp[0] == '1' && !coarse.empty() && pairs > 0;
  for (size_t g = 0; g < groups.size(); ++g)
    if ((st = fft::tables(groups[g].M, &gT[g])) != JW_OK) return st;
  if (!coarse.empty()) {
    JW_HIP_TRY(mem.alloc(&dcoarse, coarse.size() * sizeof(BandScale)));
    JW_HIP_TRY(upload_async(dcoarse, coarse.data(), coarse.size() * sizeof(BandScale), s));
    long ubytes = 0, rtot = 0, utotal = 0;
    for (size_t g = 0; g < groups.size(); ++g)
      utotal += (long)batch * groups[g].n * groups[g].M * (long)sizeof(cplx);
    if (split) {  // every group's whole U at once: within 16 GB and a quarter of free HBM
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) != hipSuccess || utotal > (16L << 30) || (size_t)utotal > fr / 4)
        split = false;
      (void)hipGetLastError();
    }
    std::vector<double> hwt;
    for (size_t g = 0; g < groups.size(); ++g) {
      const long per_sig = (long)groups[g].n * groups[g].M * (long)sizeof(cplx);
      gchunk[g] = split ? batch : std::max(1L, std::min<long>(batch, (128L << 20) / per_sig));
      if (split) {
        uoff[g] = ubytes / (long)sizeof(cplx);
        ubytes += batch * per_sig;
      } else {
        ubytes = std::max(ubytes, gchunk[g] * per_sig);
      }
      rtot += groups[g].M / 512;
      std::vector<double> wt;
      interp_weights(N / groups[g].M, N, wt);
      hwt.insert(hwt.end(), wt.begin(), wt.end());
    }
    JW_HIP_TRY(mem.alloc(&U, (size_t)ubytes));
    JW_HIP_TRY(mem.alloc(&dwt, hwt.size() * sizeof(double)));
    JW_HIP_TRY(mem.alloc(&wroots, (size_t)rtot * sizeof(double4)));
    JW_HIP_TRY(upload_async(dwt, hwt.data(), hwt.size() * sizeof(double), s));
  }
  if (nfull > 0 && nfull < ns) {
    JW_HIP_TRY(mem.alloc(&dsmap, full.size() * sizeof(int)));
    JW_HIP_TRY(upload_async(dsmap, full.data(), full.size() * sizeof(int), s));
  }
  const PairMap pmf{dsmap, nfull, ns}, pm_all{nullptr, ns, ns};
  // forward FFTs read the padded signals in natural order (split N1n); the spectra are stored
  // column-major for the inverse FFTs' split N1 x N/N1 (fft::split_n1), and in natural order
  // for the band pass
  const long N1n = fft::split_n1(N, true), N1 = fft::split_n1(N, false);
  // forward FFT of the padded signals, gsig at a time
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += gsig) {
    const long nb = std::min<long>(gsig, batch - b0);
    PadIn in{x + b0 * n, n, N / N1n, padding};
    const SpecOut so{X, N, N1n, N1, N / N1, b0};
    if (Xn) {
      st = run_fft<-1>(N, nb, in, SpecOut1{X, N, b0}, SpecOutBoth{so, Xn}, A, s, T, (ntm & 1) != 0,
                       true, Bw);
    } else {
      st = run_fft<-1>(N, nb, in, SpecOut1{X, N, b0}, so, A, s, T, (ntm & 1) != 0, true, Bw);
    }
  }
  // with two-pass pairs to follow, the band kernel (FP64-issue bound) runs on a side stream
  // beside them; the coarse-grid scales go there too.  Without band scales nothing overlaps
  // usefully: the coarse-grid kernels and the two-pass passes are all HBM-bound, and side by
  // side cfg3 ran 32.0 ms against 30.6 one after the other (profiles/r05/ab/cwt_env_h.txt).
  // env JW_CWT_OVERLAP (A/B runs): 0 = never, 1 = whenever there are pairs.
  hipStream_t bs = s;
  const char* gov = knob("JW_CWT_OVERLAP");
  const bool overlap = (gov ? gov[0] != '0' : nband > 0) || split;
  if (st == JW_OK && (nband > 0 || !coarse.empty()) && pairs > 0) {
    if (overlap) {
      SideStream* side = nullptr;
      if ((st = side_stream(&side)) != JW_OK) return st;
      JW_HIP_TRY(hipEventRecord(side->fork, s));
      bs = side->s;
      JW_HIP_TRY(hipStreamWaitEvent(bs, side->fork, 0));
      join.side = side;  // armed before the launches: any exit below joins
    }
  }
  // band scales: one pass per (signal, scale) pair
  if (nband > 0 && st == JW_OK) {
    const dim3 gp((unsigned)((nb_hi * 512L + 255) / 256), (unsigned)nband);
    // (on the band stream: it forked before these tables)
    if (wavelet == JW_CWT_MORLET) {
      hipLaunchKernelGGL(cwt_band_psi<JW_CWT_MORLET>, gp, dim3(256), 0, bs, dbands, psi, w, dsc,
                         dsc + ns, N, N1b, fs);
    } else {
      hipLaunchKernelGGL(cwt_band_psi<JW_CWT_MEXHAT>, gp, dim3(256), 0, bs, dbands, psi, w, dsc,
                         dsc + ns, N, N1b, fs);
    }
    JW_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(cwt_band_roots, dim3((unsigned)((N1b + 255) / 256)), dim3(256), 0, bs, wN1,
                       N, N1b, T);
    JW_HIP_TRY(hipGetLastError());
    const CoefOut ob{out, n, N1b, 0, 1.0 / (double)N, (ntm & 2) != 0, pm_all};
    const long items = (long)batch * nband;
    // A/B runs: JW_CWT_BAND_V = 2 x (three workgroups per CU, one row group each, instead of
    // two with R) + (load prefetch); JW_CWT_BAND_MFMA=0: VALU band sums.  Measured at cfg3
    // (profiles/r03/cwt_band_v.log): band kernel 15.5 (0) / 15.2 (1) / 14.4 (2) / 14.0 ms (3).
    const char* gbv = knob("JW_CWT_BAND_V");
    const int bv = gbv ? std::atoi(gbv) : 3;
    const char* grr = knob("JW_CWT_BAND_R");  // A/B runs: row groups per workgroup
    int R = grr ? std::atoi(grr) : 8;  // two workgroups per CU: 1 -> 44.6, 8 -> 41.7 ms (r02)
    if (bv >= 2) R = 1;
    while (R > 1 && (N1b / fft::kT) % R) R >>= 1;
    R = std::max(1, std::min<int>(R, (int)(N1b / fft::kT)));
    const long blocks = (items + 7) / 8 * 8 * (N1b / fft::kT / R);
    if (blocks > 0x7fffffffL) return fail(JW_ERR_UNSUPPORTED, "CWT band grid too large");
    const char* gmf = knob("JW_CWT_BAND_MFMA");
    auto band = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(512), 0, bs, Xn, psi, dbands, nband,
                         wN1, N, N1b, items, ob, T, R, N);
    };
    if (gmf && gmf[0] == '0') {
      band(cwt_band512<false, false, 4, CoefOut>);
    } else if (bv == 0) {
      band(cwt_band512<true, false, 4, CoefOut>);
    } else if (bv == 1) {
      band(cwt_band512<true, true, 4, CoefOut>);
    } else if (bv == 2) {
      band(cwt_band512<true, false, 6, CoefOut>);
    } else {
      band(cwt_band512<true, true, 6, CoefOut>);
    }
    JW_HIP_TRY(hipGetLastError());
  }
  const bool nt = (ntm & 2) != 0;
  // interpolation of `items` coarse rows of one group (U rows from 0, signals from sg0)
  auto interp_launch = [&](const InterpJob& j, hipStream_t is) -> int {
    auto one = [&](auto lp) -> int {
      constexpr int LP = decltype(lp)::value;
      constexpr long TC = interp_tc<LP>();
      const long chunks = (n + TC - 1) / TC, iblocks = j.items * chunks;
      if (iblocks > 0x7fffffffL) return fail(JW_ERR_UNSUPPORTED, "CWT coarse grid too large");
      hipLaunchKernelGGL(cwt_interp<LP>, dim3((unsigned)iblocks), dim3(256), 0, is, j.U, j.M,
                         j.gb, j.gn, j.gw, N, n, ns, j.sg0, out, nt, T, (int)chunks);
      return JW_OK;
    };
    int r;
    switch (j.P) {
      case 2: r = one(std::integral_constant<int, 1>{}); break;
      case 4: r = one(std::integral_constant<int, 2>{}); break;
      case 8: r = one(std::integral_constant<int, 3>{}); break;
      case 16: r = one(std::integral_constant<int, 4>{}); break;
      case 32: r = one(std::integral_constant<int, 5>{}); break;
      default: r = one(std::integral_constant<int, 6>{}); break;
    }
    if (r != JW_OK) return r;
    JW_HIP_TRY(hipGetLastError());
    return JW_OK;
  };
  std::vector<InterpJob> deferred;  // JW_CWT_SPLIT: launched after the two-pass chain
  // coarse-grid scales: per group of equal M, the band kernel on the M-point grid into U, then
  // the Kaiser-Bessel interpolation to the N-point coefficients, a few signals at a time so
  // that U stays ~128 MB
  if (!groups.empty() && st == JW_OK) {
    // grids of 16+ rows: two row groups per workgroup from one set of band sums
    // (cwt_band512_par); env JW_CWT_PAR=0 (A/B runs): one row group per workgroup
    const char* gpr = knob("JW_CWT_PAR");
    const bool use_par = !(gpr && gpr[0] == '0');
    long woff = 0, roff = 0;
    // JW_TEST_CWT_FAIL_GROUP=k (tests only): fail at coarse group k, after groups < k have
    // launched on the side stream -- the error path must still join them (JoinGuard)
    const char* gtf = knob("JW_TEST_CWT_FAIL_GROUP");
    const long fail_group = gtf ? std::atol(gtf) : -1;
    for (size_t g = 0; g < groups.size() && st == JW_OK; ++g) {
      if ((long)g == fail_group) return fail(JW_ERR_FAILURE, "CWT: injected failure at coarse group %ld", (long)g);
      const CoarseGroup& G = groups[g];
      const long M = G.M, N1c = M / 512, P = N / M;
      const Tables& TM = gT[g];
      const BandScale* gb = dcoarse + G.first;
      const dim3 gp((unsigned)((G.nb_hi * 512L + 255) / 256), (unsigned)G.n);
      if (wavelet == JW_CWT_MORLET) {
        hipLaunchKernelGGL(cwt_interp_psi<JW_CWT_MORLET>, gp, dim3(256), 0, bs, gb, psi, w, dsc,
                           dsc + ns, N, N1b, fs, M);
      } else {
        hipLaunchKernelGGL(cwt_interp_psi<JW_CWT_MEXHAT>, gp, dim3(256), 0, bs, gb, psi, w, dsc,
                           dsc + ns, N, N1b, fs, M);
      }
      JW_HIP_TRY(hipGetLastError());
      double4* wN1c = wroots + roff;
      hipLaunchKernelGGL(cwt_band_roots, dim3((unsigned)((N1c + 255) / 256)), dim3(256), 0, bs,
                         wN1c, M, N1c, TM);
      JW_HIP_TRY(hipGetLastError());
      const double* gw = dwt + woff;
      woff += P * kInterpStride;
      roff += N1c;
      cplx* const Ug = U + uoff[g];

      for (long sg0 = 0; sg0 < batch; sg0 += gchunk[g]) {
        const long cs = std::min<long>(gchunk[g], batch - sg0);
        const long items = cs * G.n;
        const bool par = use_par && N1c >= 2 * fft::kT;
        const long blocks = (items + 7) / 8 * 8 * (N1c / fft::kT / (par ? 2 : 1));
        if (blocks > 0x7fffffffL)
          return fail(JW_ERR_UNSUPPORTED, "CWT coarse grid too large");
        if (par) {
          hipLaunchKernelGGL(cwt_band512_par<CoarseOut>, dim3((unsigned)blocks), dim3(512), 0, bs,
                             Xn + sg0 * N, psi, gb, G.n, wN1c, M, N1c, items,
                             CoarseOut{(double*)Ug, M, N1c, 0}, TM, N);
        } else {
          hipLaunchKernelGGL((cwt_band512<true, true, 6, CoarseOut>), dim3((unsigned)blocks),
                             dim3(512), 0, bs, Xn + sg0 * N, psi, gb, G.n, wN1c, M, N1c, items,
                             CoarseOut{(double*)Ug, M, N1c, 0}, TM, 1, N);
        }
        JW_HIP_TRY(hipGetLastError());
        const InterpJob job{Ug, M, P, sg0, items, gb, G.n, gw};
        if (split) {
          deferred.push_back(job);
        } else if ((st = interp_launch(job, bs)) != JW_OK) {
          return st;
        }
      }
    }
  }
  // the other (signal, scale) pairs: IFFT(X * psi_hat) -> coefficients in two passes
  if (pipe && st == JW_OK) {
    auto go = [&](auto kind) {
      constexpr int K = decltype(kind)::value;
      auto mk_in = [&](long p0) {
        return ScaleIn<K>{X, dsc, w, N, N1, N / N1, p0, pmf, fs, dsc + ns, dsc + 3 * ns, early};
      };
      auto mk_out = [&](long p0) {
        return CoefOut{out, n, N1, p0, 1.0 / (double)N, (ntm & 2) != 0, pmf};
      };
      return fft::run_fft512_pipelined<1>(N, pairs, gpair, mk_in, mk_out, A, A + gpair * N, s, T,
                                          (ntm & 1) != 0);
    };
    switch (wavelet) {
      case JW_CWT_MORLET: st = go(std::integral_constant<int, JW_CWT_MORLET>{}); break;
      case JW_CWT_MEXHAT: st = go(std::integral_constant<int, JW_CWT_MEXHAT>{}); break;
      case JW_CWT_PAUL: st = go(std::integral_constant<int, JW_CWT_PAUL>{}); break;
      case JW_CWT_DOG: st = go(std::integral_constant<int, JW_CWT_DOG>{}); break;
      default: st = go(std::integral_constant<int, JW_CWT_MEYER>{}); break;
    }
  }
  for (long p0 = 0; p0 < pairs && st == JW_OK && !pipe; p0 += gpair) {
    const long np_ = std::min<long>(gpair, pairs - p0);
    CoefOut o{out, n, N <= 4096 ? 1 : N1, p0, 1.0 / (double)N, (ntm & 2) != 0, pmf};
    CoefOut o1{out, n, 1, p0, 1.0 / (double)N, (ntm & 2) != 0, pmf};
    auto go = [&](auto kind) {
      ScaleIn<decltype(kind)::value> in{X, dsc, w, N, N1, N <= 4096 ? 1 : N / N1, p0, pmf, fs,
                                        dsc + ns, dsc + 3 * ns, early};
      return run_fft<1>(N, np_, in, o1, o, A, s, T, (ntm & 1) != 0, true, Bw);
    };
    switch (wavelet) {
      case JW_CWT_MORLET: st = go(std::integral_constant<int, JW_CWT_MORLET>{}); break;
      case JW_CWT_MEXHAT: st = go(std::integral_constant<int, JW_CWT_MEXHAT>{}); break;
      case JW_CWT_PAUL: st = go(std::integral_constant<int, JW_CWT_PAUL>{}); break;
      case JW_CWT_DOG: st = go(std::integral_constant<int, JW_CWT_DOG>{}); break;
      default: st = go(std::integral_constant<int, JW_CWT_MEYER>{}); break;
    }
  }
  if (!deferred.empty() && st == JW_OK) {
    // the coarse band kernels (side stream) are done before their rows are interpolated here
    if (join.side) {
      JW_HIP_TRY(hipEventRecord(join.side->join, join.side->s));
      JW_HIP_TRY(hipStreamWaitEvent(s, join.side->join, 0));
    }
    for (const InterpJob& j : deferred)
      if ((st = interp_launch(j, s)) != JW_OK) return st;
  }
  return st;
}

int cwt_fft_paths(int wavelet, const double* params, long n, const double* scales, int ns,
                  double fs, int* two_pass, int* band, int* coarse_grid) {
  long N = 1;
  while (N < n) N <<= 1;
  CwtSplit sp;
  if (n > 0 && ns > 0) cwt_split(wavelet, params, N, scales, ns, fs, &sp);
  *two_pass = n > 0 ? (int)sp.full.size() : 0;
  *band = (int)sp.bands.size();
  *coarse_grid = (int)sp.coarse.size();
  return JW_OK;
}

}  // namespace jw
