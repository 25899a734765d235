// jw_cwt_direct.hip -- ContinuousWaveletTransform.transform on the GPU: the direct
// (time-domain) CWT (src/main/java/jwave/transforms/ContinuousWaveletTransform.java:153-172;
// transformParallel :470-500 and transformParallelCustom :577-680 compute the same values).
//
// computeCoefficient (:240-260), for scale a and time index t:
//   [lo, hi] = [(int)(support[0] * a * fs), (int)(support[1] * a * fs)]
//   c[a][t]  = dt * sum_{i = max(0, t + lo)}^{min(N - 1, t + hi)} conj(psi_{a,0}((i - t) dt)) x[i]
// with psi_{a,0}(s) = psi(s / a) / sqrt(a) (ContinuousWavelet.wavelet :90-102), the sum taken
// in ascending i from (0, 0) with Complex.add / Complex.mul(double).
//
// The wavelet values depend only on k = i - t, so the host evaluates one table per scale,
// conj(psi(k dt / a) (1/sqrt a)) for k in [lo, hi], in the reference's operation order (the
// oracle evaluates it the same way with the same libm: the tables agree bit for bit).  The
// kernel gives one output per thread; every lane of a wave walks k = lo .. hi in lockstep (the
// table read is wave-uniform, the signal read lane-consecutive) and adds only the terms with
// 0 <= t + k < N: the same additions in the same order as the reference (bit-identical in
// JW_ARITH_STRICT).  Work is O(N * support * a): the FFT path is the fast one for long
// signals; this is the reference's small-signal path.
#include <algorithm>
#include <cmath>
#include <vector>

#include "jw_internal.hpp"

namespace jw {
namespace {

constexpr double kPi = 3.14159265358979323846;  // Math.PI

// Java's (int) cast of a double: NaN -> 0, saturating, else truncation toward zero.
int java_d2i(double v) {
  if (std::isnan(v)) return 0;
  if (v >= 2147483647.0) return 2147483647;
  if (v <= -2147483648.0) return -2147483647 - 1;
  return (int)v;
}

struct TimeWavelet {
  int kind;
  double p0, p1;
  int ord;
  double norm;          // Morlet 1/sqrt(2 pi fb); Mexican hat / DOG / Paul normConstant
  double herm[12];      // DOG Hermite coefficients (computeHermiteCoefficients :289-335)
  int nherm;
  double ipm_re, ipm_im;  // Paul i^m (computeIPowerM)
  double sup0, sup1;      // getEffectiveSupport
};

TimeWavelet make_time_wavelet(int kind, const double* params) {
  TimeWavelet w{};
  w.kind = kind;
  if (kind == JW_CWT_MORLET) {  // MorletWavelet.java:66-100, :151-154
    w.p0 = params[0];
    w.p1 = params[1];
    w.norm = 1.0 / std::sqrt(2.0 * kPi * w.p0);
    const double r = 4.0 * std::sqrt(w.p0);
    w.sup0 = -r, w.sup1 = r;
  } else if (kind == JW_CWT_MEXHAT) {  // MexicanHatWavelet.java:65-95, :139-142
    w.p0 = params[0];
    w.norm = 2.0 / (std::sqrt(3.0 * w.p0) * std::pow(kPi, 0.25));
    w.sup0 = -5.0 * w.p0, w.sup1 = 5.0 * w.p0;
  } else if (kind == JW_CWT_PAUL) {  // PaulWavelet.java:76-99, :185-191
    w.ord = (int)params[0];
    double fm = 1.0, f2m = 1.0;  // factorial(m), factorial(2m) in double
    for (int i = 2; i <= w.ord; ++i) fm *= i;
    for (int i = 2; i <= 2 * w.ord; ++i) f2m *= i;
    w.norm = std::pow(2, w.ord) * fm / std::sqrt(kPi * f2m);
    const double re[4] = {1, 0, -1, 0}, im[4] = {0, 1, 0, -1};
    w.ipm_re = re[w.ord % 4], w.ipm_im = im[w.ord % 4];
    w.sup0 = -1.0, w.sup1 = 2.0 * (w.ord + 1);
  } else if (kind == JW_CWT_DOG) {  // DOGWavelet.java:129-180, :245-250, :289-366
    w.ord = (int)params[0];
    w.p0 = params[1];
    const int n = w.ord;
    std::vector<std::vector<double>> c(n + 1);
    c[0] = {1.0};
    if (n > 0) c[1] = {0.0, 2.0};
    for (int k = 2; k <= n; ++k) {
      c[k].assign(k + 1, 0.0);
      for (int i = 1; i <= k; ++i)
        if (i - 1 < (int)c[k - 1].size()) c[k][i] += 2.0 * c[k - 1][i - 1];
      for (int i = 0; i <= k - 2; ++i) c[k][i] -= 2.0 * (k - 1) * c[k - 2][i];
    }
    const double sign = ((n + 1) % 2 == 0) ? 1.0 : -1.0;
    w.nherm = (int)c[n].size();
    for (int i = 0; i < w.nherm; ++i) w.herm[i] = c[n][i] * sign;
    double df = 1.0;  // doubleFactorial(2n - 1) :376-382
    for (int i = 2 * n - 1; i > 0; i -= 2) df *= i;
    w.norm = std::sqrt(df / (std::pow(2, n) * std::sqrt(kPi) * std::pow(w.p0, 2 * n + 1)));
    const double r = (3.0 + n / 2.0) * w.p0;
    w.sup0 = -r, w.sup1 = r;
  } else {  // Meyer, MeyerWavelet.java:315-319
    w.sup0 = -15.0, w.sup1 = 15.0;
  }
  return w;
}

double meyer_sinc(double x) {  // MeyerWavelet.sinc
  if (std::fabs(x) < 1e-10) {
    const double x2 = x * x;
    return 1.0 - x2 / 6.0 + x2 * x2 / 120.0;
  }
  return std::sin(x) / x;
}

// psi(t), the mother wavelet, in each class's operation order (wavelet(double t)).  Where a
// class takes both Math.cos and Math.sin of one angle this takes glibc's sincos (the oracle
// too, so the tables agree bit for bit; any libm is within an ulp of Java's Math there).
void psi_t(const TimeWavelet& w, double t, double* re, double* im) {
  *re = 0.0, *im = 0.0;
  if (w.kind == JW_CWT_MORLET) {  // MorletWavelet.java:85-100
    const double envelope = std::exp(-t * t / (2.0 * w.p0));
    const double phase = 2.0 * kPi * w.p1 * t;
    double sn, cs;
    ::sincos(phase, &sn, &cs);  // explicit: compilers fuse sin + cos differently
    *re = w.norm * envelope * cs;
    *im = w.norm * envelope * sn;
  } else if (w.kind == JW_CWT_MEXHAT) {  // MexicanHatWavelet.java:85-95
    const double tn = t / w.p0, tn2 = tn * tn;
    *re = w.norm * (1.0 - tn2) * std::exp(-0.5 * tn2);
  } else if (w.kind == JW_CWT_PAUL) {  // PaulWavelet.wavelet + complexPower :262-271
    const double zr = 1.0, zi = -t;
    const double mag = std::sqrt(zr * zr + zi * zi);  // Complex.getMag
    const double arg = std::atan2(zi, zr);
    const double p = -(w.ord + 1);
    const double nm = std::pow(mag, p), na = p * arg;
    double sn, cs;
    ::sincos(na, &sn, &cs);
    const double pr = nm * cs, pi = nm * sn;
    const double ar = w.ipm_re * w.norm, ai = w.ipm_im * w.norm;  // _iPowerM.mul(norm)
    *re = ar * pr - ai * pi;  // .mul(power), Complex.mul :286-288
    *im = ar * pi + ai * pr;
  } else if (w.kind == JW_CWT_DOG) {  // DOGWavelet.java:166-180
    const double x = t / w.p0;
    const double gaussian = std::exp(-0.5 * x * x);
    double h = 0.0;
    for (int i = w.nherm - 1; i >= 0; --i) h = h * x + w.herm[i];
    *re = w.norm * h * gaussian;
  } else {  // MeyerWavelet.wavelet(double t)
    if (std::fabs(t) > 15.0) return;
    const double envelope = std::exp(-0.5 * t * t / 25.0);
    const double omega0 = 0.7;
    double value = omega0 * meyer_sinc(omega0 * t) * envelope;
    const double omega1 = 1.4 * omega0;
    value += 0.2 * omega1 * meyer_sinc(omega1 * t) * envelope;
    const double omega2 = 0.5 * omega0;
    value += -0.1 * omega2 * meyer_sinc(omega2 * t) * envelope;
    value *= std::sqrt(2.0 / kPi);
    *re = value;
  }
}

template <bool FMA>
__device__ __forceinline__ double mac(double acc, double w, double x) {
  if constexpr (FMA) return __builtin_fma(w, x, acc);
  else return acc + w * x;
}

// out[b][s][t] = (re, im); table[off[s] + k - lo[s]] = conj(psi_{a,0}(k dt)).
template <bool FMA>
__global__ __launch_bounds__(256) void cwt_direct_kernel(const double* __restrict__ x, long n,
                                                         const double2* __restrict__ table,
                                                         const long* __restrict__ off,
                                                         const int* __restrict__ lohi, int ns,
                                                         double dt, double* __restrict__ out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const long b = blockIdx.z;
  const int lo = lohi[2 * s], hi = lohi[2 * s + 1];
  const double2* w = table + off[s] - lo;
  const double* xs = x + b * n;
  double re = 0.0, im = 0.0;
  // wave-uniform k range: the union of the lanes' windows (lanes outside add nothing)
  const long t0 = (long)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
  const long kb = max((long)lo, -(t0 + 63)), ke = min((long)hi, n - 1 - t0);
  for (long k = kb; k <= ke; ++k) {
    const long i = t + k;
    const double2 v = w[k];
    const bool in = i >= 0 && i < n && t < n;
    const double xv = in ? xs[i] : 0.0;
    const double r2 = mac<FMA>(re, v.x, xv), i2 = mac<FMA>(im, v.y, xv);
    re = in ? r2 : re;  // skip, not "+ 0.0": the reference adds only in-range terms
    im = in ? i2 : im;
  }
  if (t < n) {
    double2* o = (double2*)(out + 2 * ((b * ns + s) * n + t));
    *o = make_double2(re * dt, im * dt);  // sum.mul(dt)
  }
}

}  // namespace

void cwt_direct_support(int wavelet, const double* params, double a, double fs, double* lo,
                        double* hi) {
  const TimeWavelet w = make_time_wavelet(wavelet, params);
  *lo = java_d2i(w.sup0 * a * fs);
  *hi = java_d2i(w.sup1 * a * fs);
}

// some t in [0, n) has max(0, t + lo) <= min(n - 1, t + hi)
bool cwt_direct_window_nonempty(double lo, double hi, long n) {
  return lo <= hi && lo <= (double)(n - 1) && hi >= -(double)(n - 1);
}

int cwt_direct_device(int wavelet, const double* params, const double* x, long n,
                      const double* scales, int ns, double fs, int arith, double* out, int batch,
                      hipStream_t s) {
  if (n == 0 || ns == 0 || batch == 0) return JW_OK;
  if (n > (1L << 31) / 2) return fail(JW_ERR_UNSUPPORTED, "direct CWT length %ld too large", n);
  const TimeWavelet w = make_time_wavelet(wavelet, params);
  const double dt = 1.0 / fs;
  std::vector<long> off(ns + 1, 0);
  std::vector<int> lohi(2 * ns);
  for (int i = 0; i < ns; ++i) {
    const double a = scales[i];
    int lo = java_d2i(w.sup0 * a * fs), hi = java_d2i(w.sup1 * a * fs);
    // only the k with some in-range i = t + k can contribute: |k| <= n - 1
    lo = (int)std::max<long>(lo, -(n - 1));
    hi = (int)std::min<long>(hi, n - 1);
    if (hi < lo) hi = lo - 1;  // empty window (e.g. a < 0): the coefficient is 0 * dt
    lohi[2 * i] = lo, lohi[2 * i + 1] = hi;
    off[i + 1] = off[i] + (hi - lo + 1);
  }
  if (off[ns] > (1L << 28)) return fail(JW_ERR_UNSUPPORTED, "direct CWT wavelet tables too large");
  std::vector<double2> tab((size_t)std::max<long>(off[ns], 1));
  for (int i = 0; i < ns; ++i) {
    const double a = scales[i];
    const double nf = 1.0 / std::sqrt(a);  // ContinuousWavelet.wavelet :99-100
    for (int k = lohi[2 * i]; k <= lohi[2 * i + 1]; ++k) {
      const double tt = k * dt;  // (i - timeIdx) * dt
      double re, im;
      psi_t(w, (tt - 0.0) / a, &re, &im);
      tab[off[i] + k - lohi[2 * i]] = make_double2(re * nf, -(im * nf));  // .mul(nf).conjugate()
    }
  }
  double2* dtab = nullptr;
  long* doff = nullptr;
  int* dlohi = nullptr;
  StreamAllocs mem(s);
  JW_HIP_TRY(mem.alloc(&dtab, tab.size() * sizeof(double2)));
  JW_HIP_TRY(mem.alloc(&doff, off.size() * sizeof(long)));
  JW_HIP_TRY(mem.alloc(&dlohi, lohi.size() * sizeof(int)));
  JW_HIP_TRY(upload_async(dtab, tab.data(), tab.size() * sizeof(double2), s));
  JW_HIP_TRY(upload_async(doff, off.data(), off.size() * sizeof(long), s));
  JW_HIP_TRY(upload_async(dlohi, lohi.data(), lohi.size() * sizeof(int), s));
  int st = JW_OK;
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = std::min(65535, batch - b0);
    const dim3 g((unsigned)((n + 255) / 256), (unsigned)ns, (unsigned)nb);
    if (arith == JW_ARITH_FMA)
      hipLaunchKernelGGL(cwt_direct_kernel<true>, g, dim3(256), 0, s, x + (long)b0 * n, n, dtab,
                         doff, dlohi, ns, dt, out + (long)b0 * ns * n * 2);
    else
      hipLaunchKernelGGL(cwt_direct_kernel<false>, g, dim3(256), 0, s, x + (long)b0 * n, n, dtab,
                         doff, dlohi, ns, dt, out + (long)b0 * ns * n * 2);
    if (hipGetLastError() != hipSuccess) st = fail(JW_ERR_DEVICE, "direct CWT launch failed");
  }
  return st;
}

}  // namespace jw
