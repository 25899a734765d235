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
template <int K>
struct ScaleIn {  // X[sig][k] * conj(psi_hat(omega_k, a_s)), k = N2 k1 + col; item = pair in group
  static constexpr bool kStrided = false;  // column-major spectra: contiguous columns
  const cplx* X;
  const double* scales;
  WaveletFT w;
  long N, N1, N2, pair0;
  int ns;
  double fs;
  const double* sc;  // per scale (MORLET, MEXHAT): {bin step, norm * sqrt(a)}, see cwt_fft_device
  __device__ cplx operator()(long item, long k1, long col) const {
    const long p = pair0 + item, sig = p / ns;
    const int s = (int)(p - sig * ns);
    const long k = N2 * k1 + col;
    cplx wv;
    if constexpr (K == JW_CWT_MORLET || K == JW_CWT_MEXHAT) {
      // The same spectra with the per-bin divisions hoisted into per-scale constants: the
      // bin's signed index kk = k or k - N (createFrequencyAxis :453-456) times
      //   Morlet:      f = a*omega/(2 pi) = kk * (a fs / N)            (MorletWavelet :114-124)
      //   Mexican hat: a*omega = kk * (2 pi a fs / N)                  (MexicanHatWavelet :107-119)
      // (a few ulps from the reference's operation order; the tests bound it at 1e-12).
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
      wv = make_double2(m * exp(e), 0.0);
    } else {
      double om = 2.0 * kPi * (double)k * fs / (double)N;  // createFrequencyAxis :453-456
      if (k > N / 2) om -= 2.0 * kPi * fs;
      const double a = scales[s];
      wv = psi_hat<K>(w, om, a, sqrt(a));
    }
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
  WaveletFT w{};
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
  const char* gnt = std::getenv("JW_CWT_NT");  // A/B runs: bit 1 = NT stores of A, 2 = of coeffs
  const int ntm = gnt ? std::atoi(gnt) : 2;  // measured best: NT coefficient stores only
  const char* gmb = std::getenv("JW_CWT_GROUP_MB");  // A/B runs: workspace size in MiB
  const long ws = (gmb ? std::atol(gmb) : 128L) << 20;
  const long per = std::max(1L, ws / (N * (long)sizeof(cplx)));
  const long gsig = std::min<long>(batch, per), gpair = std::min<long>((long)batch * ns, per);
  // N = 2^18 (512 x 512): the pairs' inverse FFTs are software-pipelined over two workspaces
  // (run_fft512_pipelined); env JW_CWT_PIPE=0 runs the groups one after the other (A/B runs).
  const char* gpp = std::getenv("JW_CWT_PIPE");
  const bool pipe = N == (1L << 18) && (long)batch * ns > gpair && !(gpp && gpp[0] == '0');
  StreamAllocs mem(s);
  cplx *X = nullptr, *A = nullptr;
  double* dsc = nullptr;
  const long a_items = std::max(gsig, pipe ? 2 * gpair : gpair);
  JW_HIP_TRY(mem.alloc(&X, (size_t)batch * N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&A, (size_t)a_items * N * sizeof(cplx)));
  // device scale table: [a_0 .. a_{ns-1} | (step, norm*sqrt(a)) per scale] (ScaleIn)
  std::vector<double> hsc(3 * (size_t)ns);
  for (int i = 0; i < ns; ++i) {
    const double a = scales_host[i];
    hsc[i] = a;
    hsc[ns + 2 * i] = wavelet == JW_CWT_MEXHAT ? 2.0 * kPi * a * fs / (double)N : a * fs / (double)N;
    hsc[ns + 2 * i + 1] = w.norm * std::sqrt(a);
  }
  w.p2 = wavelet == JW_CWT_MORLET ? -2.0 * kPi * kPi * w.p0 : -0.5 * w.p0 * w.p0;
  JW_HIP_TRY(mem.alloc(&dsc, hsc.size() * sizeof(double)));
  JW_HIP_TRY(upload_async(dsc, hsc.data(), hsc.size() * sizeof(double), s));
  // forward FFTs read the padded signals in natural order (split N1n); the spectra are stored
  // column-major for the inverse FFTs' split N1 x N/N1 (fft::split_n1)
  const long N1n = fft::split_n1(N, true), N1 = fft::split_n1(N, false);
  // forward FFT of the padded signals, gsig at a time
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += gsig) {
    const long nb = std::min<long>(gsig, batch - b0);
    PadIn in{x + b0 * n, n, N / N1n, padding};
    st = run_fft<-1>(N, nb, in, SpecOut1{X, N, b0}, SpecOut{X, N, N1n, N1, N / N1, b0}, A, s, T,
                     (ntm & 1) != 0);
  }
  // per (signal, scale) pair: IFFT(X * psi_hat) -> coefficients
  const long pairs = (long)batch * ns;
  if (pipe && st == JW_OK) {
    auto go = [&](auto kind) {
      constexpr int K = decltype(kind)::value;
      auto mk_in = [&](long p0) {
        return ScaleIn<K>{X, dsc, w, N, N1, N / N1, p0, ns, fs, dsc + ns};
      };
      auto mk_out = [&](long p0) { return CoefOut{out, n, N1, p0, 1.0 / (double)N, (ntm & 2) != 0}; };
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
    CoefOut o{out, n, N <= 4096 ? 1 : N1, p0, 1.0 / (double)N, (ntm & 2) != 0};
    CoefOut o1{out, n, 1, p0, 1.0 / (double)N, (ntm & 2) != 0};
    auto go = [&](auto kind) {
      ScaleIn<decltype(kind)::value> in{X, dsc, w, N, N1, N <= 4096 ? 1 : N / N1, p0, ns, fs,
                                        dsc + ns};
      return run_fft<1>(N, np_, in, o1, o, A, s, T, (ntm & 1) != 0);
    };
    switch (wavelet) {
      case JW_CWT_MORLET: st = go(std::integral_constant<int, JW_CWT_MORLET>{}); break;
      case JW_CWT_MEXHAT: st = go(std::integral_constant<int, JW_CWT_MEXHAT>{}); break;
      case JW_CWT_PAUL: st = go(std::integral_constant<int, JW_CWT_PAUL>{}); break;
      case JW_CWT_DOG: st = go(std::integral_constant<int, JW_CWT_DOG>{}); break;
      default: st = go(std::integral_constant<int, JW_CWT_MEYER>{}); break;
    }
  }
  return st;
}

}  // namespace jw
