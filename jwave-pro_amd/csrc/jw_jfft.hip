// jw_jfft.hip -- JW_ARITH_STRICT FFT paths: the reference's own FFT (jw_jfft.hpp) behind
//   * FastFourierTransform.forward/reverse(Complex[]) (FastFourierTransform.java:112-164), and
//   * MODWTTransform's FFT convolution, level by level as the reference runs it
//     (performConvolution :640-664, circularConvolveFFT :752-786, circularConvolveFFTAdjoint
//     :798-837, wrapFilterToSignalLength :729-741),
// so a default-constructed MODWTTransform (AUTO) gets the JVM's values bit for bit.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <type_traits>
#include <vector>

#include "jw_jfft_host.hpp"

namespace jw {
namespace jf {
namespace {

// ---------------------------------------------------------------------------------------
// Twiddles: Tw[half + k] = wn_k of the stage of size 2 half, by the reference's recurrence
// (:188-201; host code is built with -ffp-contract=off, like the JVM).  Device layout:
// [0, lc1) natural (pass 1; lc1 = n for a one-column transform), then the pass-2 table
// transposed, Tw2[l lc2 + m] = Tw[m lc1 + l] (l < lc1, m < lc2 = n / lc1).
// ---------------------------------------------------------------------------------------
using TwKey = std::tuple<int, long, int, int>;  // device, n, inverse, lc1
DevCache<TwKey> g_tw(kCacheBytes);

constexpr double kJavaPi = 3.141592653589793;  // Math.PI

// The reference's twiddles of the stages half = 2^t, t in [t0, t1) (:188-201): put(idx, wn_k) for
// idx = half + k, k < half, in recurrence order.
template <class Put>
void java_stages(int t0, int t1, bool inverse, const Put& put) {
  for (int t = t0; t < t1; ++t) {
    const long half = 1L << t, size = 2 * half;
    const double angle = 2 * kJavaPi / (double)size * (double)(inverse ? 1 : -1);
    double wr, wi;  // Math.cos(angle), Math.sin(angle), correctly rounded (jw_crmath.cc)
    cr_sincos(angle, &wi, &wr);
    double nr = 1.0, ni = 0.0;  // wn = new Complex(1, 0)
    for (long k = 0; k < half; ++k) {
      put(half + k, make_double2(nr, ni));
      const double tr = nr * wr - ni * wi, ti = nr * wi + ni * wr;  // wn = wn.mul(w)
      nr = tr;
      ni = ti;
    }
  }
}

// Tw[idx] (idx = 1 .. n - 1) of an n-point transform, scattered by put straight into a device
// layout (no n-entry staging table: 16 GB at 2^30).  Each stage is one sequential recurrence and
// the longest two are half and a quarter of the work, so they run on threads of their own.
template <class Put>
void java_twiddles(long n, bool inverse, const Put& put) {
  const int lg = ilog2(n);
  if (n < (1L << 22) || host_threads() < 3) {
    java_stages(0, lg, inverse, put);
    return;
  }
  // a thread that cannot be started (std::system_error) leaves its stage to this one: nothing
  // may throw across the C-ABI
  std::thread top, next;
  try {
    top = std::thread([&] { java_stages(lg - 1, lg, inverse, put); });
    next = std::thread([&] { java_stages(lg - 2, lg - 1, inverse, put); });
  } catch (...) {
  }
  java_stages(0, lg - 2, inverse, put);
  if (!next.joinable()) java_stages(lg - 2, lg - 1, inverse, put);
  if (!top.joinable()) java_stages(lg - 1, lg, inverse, put);
  if (top.joinable()) top.join();
  if (next.joinable()) next.join();
}

cplx* host_table(size_t entries) {
  return static_cast<cplx*>(std::malloc(entries * sizeof(cplx)));
}

}  // namespace

int twiddles(long n, bool inverse, int lc1, Tw* out, StreamAllocs& mem, hipStream_t s) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  const bool one = lc1 >= n;
  const size_t entries = one ? (size_t)n : (size_t)lc1 + (size_t)n;
  const void* p = nullptr;
  int st = cached_table(g_tw, TwKey(dev, n, inverse ? 1 : 0, lc1), entries * sizeof(cplx), mem,
                        s, &p, [&](void* d) -> int {
                          cplx* h = host_table(entries);
                          if (!h) return fail(JW_ERR_NO_MEMORY, "twiddle table: %zu entries", entries);
                          const cplx zero = make_double2(0.0, 0.0);
                          h[0] = zero;  // Tw[0] is never read
                          const long lc2 = one ? 1 : n / lc1;
                          const int lb = ilog2(one ? n : lc1);
                          cplx* h2 = h + lc1;  // h2[l lc2 + m] = Tw[m lc1 + l]
                          if (!one) h2[0] = zero;
                          java_twiddles(n, inverse, [&](long idx, cplx w) {
                            if (idx < lc1 || one) h[idx] = w;
                            if (!one) h2[(idx & (lc1 - 1)) * lc2 + (idx >> lb)] = w;
                          });
                          JW_HIP_TRY(upload_owned(d, h, entries * sizeof(cplx), s));
                          return JW_OK;
                        });
  if (st != JW_OK) return st;
  out->n = n;
  out->lc1 = one ? (int)n : lc1;
  out->p1 = (const cplx*)p;
  out->p2 = one ? nullptr : (const cplx*)p + lc1;
  return JW_OK;
}

long three_pass_min() {
  const char* e = knob("JW_JFFT_3PASS_MIN");  // tests: a power of two >= 2^18
  long m = e ? std::atol(e) : 0;
  if (m < (1L << 18) || (m & (m - 1))) m = 1L << 25;
  return m;
}

using Tw3Key = std::tuple<int, long, int>;  // device, n, inverse (the split is a function of n)
// The three-pass tables are (A + AB + n) x 16 bytes: 1.08 GB at 2^26, 4.3 GB at 2^28, 17.2 GB at
// 2^30 per direction.  Their own budget holds both directions at 2^30, so the longest transforms
// keep their tables instead of rebuilding multi-GB host tables on every call; a table
// is kept only while it also fits a quarter of the free device memory (cached_table), and
// jw_release_caches drops them.
DevCache<Tw3Key> g_tw3(36UL << 30);

int twiddles3(long n, bool inverse, Tw3* out, StreamAllocs& mem, hipStream_t s) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  int a, b, c;
  split3(ilog2(n), &a, &b, &c);
  const long A = 1L << a, B = 1L << b, C = 1L << c, AB = A * B;
  const size_t entries = (size_t)(A + AB + n);
  const void* p = nullptr;
  int st = cached_table(g_tw3, Tw3Key(dev, n, inverse ? 1 : 0), entries * sizeof(cplx), mem, s, &p,
                        [&](void* d) -> int {
                          cplx* h = host_table(entries);
                          if (!h) return fail(JW_ERR_NO_MEMORY, "twiddle table: %zu entries", entries);
                          cplx* pm = h + A;   // pm[l B + m] = Tw[m A + l]
                          cplx* p3 = pm + AB; // p3[l C + m] = Tw[m A B + l]
                          h[0] = pm[0] = p3[0] = make_double2(0.0, 0.0);  // Tw[0]: never read
                          java_twiddles(n, inverse, [&](long idx, cplx w) {
                            if (idx < A) h[idx] = w;
                            if (idx < AB) pm[(idx & (A - 1)) * B + (idx >> a)] = w;
                            p3[(idx & (AB - 1)) * C + (idx >> (a + b))] = w;
                          });
                          JW_HIP_TRY(upload_owned(d, h, entries * sizeof(cplx), s));
                          return JW_OK;
                        });
  if (st != JW_OK) return st;
  out->n = n;
  out->A = (int)A;
  out->B = (int)B;
  out->C = (int)C;
  out->p1 = (const cplx*)p;
  out->pm = out->p1 + A;
  out->p3 = out->pm + AB;
  return JW_OK;
}

namespace {

// ---------------------------------------------------------------------------------------
// MODWT filter spectra: FFT(wrapFilterToSignalLength(upsample(f, j), N)) (:729-741, :770-771),
// rows [j - 1][0 = h (wavelet), 1 = g (scaling)], natural order; cached per (device, taps, N, J).
// ---------------------------------------------------------------------------------------
using SpecKey = std::tuple<int, long, int, std::vector<double>>;
// 2 J N x 16 bytes: 4 GiB for db4 J = 8 at 2^24 -- past a 2 GiB budget every call rebuilt them
// (the host-wrapped filters and 2 J transforms: 1.23 s per call against ~22 ms, profiles/r06/ab/
// spectra_cache/), so the budget holds J = 13 at 2^24 (7 GiB); a table is still kept only while
// it fits a quarter of the free device memory (cached_table)
DevCache<SpecKey> g_spec(16UL << 30);

// the up-sampled filter of level j (upsample :618-630) wrapped in the reference's order,
// zero taps included: wrappedFilter[i % N] += filter[i], i ascending
void wrapped_filter(const double* base, int L, int j, long N, double* row) {
  std::fill(row, row + N, 0.0);
  const long d = 1L << (j - 1);
  const long M = (long)(L - 1) * d + 1;
  for (long i = 0; i < M; ++i) row[i % N] += (i % d == 0) ? base[i / d] : 0.0;
}

int filter_spectra(const ModwtPlan& p, long N, int J, const cplx** F, StreamAllocs& mem,
                   hipStream_t s) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  std::vector<double> taps(p.g, p.g + p.L);
  taps.insert(taps.end(), p.h, p.h + p.L);
  const size_t bytes = (size_t)2 * J * N * sizeof(cplx);
  const void* out = nullptr;
  const int st =
      cached_table(g_spec, SpecKey(dev, N, J, taps), bytes, mem, s, &out, [&](void* d) -> int {
        std::vector<double> rows((size_t)2 * J * N);
        for (int j = 1; j <= J; ++j) {
          wrapped_filter(p.h, p.L, j, N, rows.data() + (size_t)(2 * (j - 1)) * N);
          wrapped_filter(p.g, p.L, j, N, rows.data() + (size_t)(2 * (j - 1) + 1) * N);
        }
        double* drows = nullptr;
        JW_HIP_TRY(mem.alloc(&drows, rows.size() * sizeof(double)));
        JW_HIP_TRY(upload_async(drows, rows.data(), rows.size() * sizeof(double), s));
        if (N & (N - 1)) return bs_spectra_real(N, 2L * J, drows, (cplx*)d, mem, s);
        return fft_rows(N, false, 2L * J, RowsR{drows, N}, OutCS{(cplx*)d, N, 1.0, 0}, mem, s);
      });
  *F = (const cplx*)out;
  return st;
}

const cplx* spec_h(const cplx* F, long N, int j) { return F + (long)(2 * (j - 1)) * N; }
const cplx* spec_g(const cplx* F, long N, int j) { return F + (long)(2 * (j - 1) + 1) * N; }

// The spectra again, each row stored per column of the two-pass kp2p view: FT[q][l C + h] =
// F[q][h R + l] (R columns of C points), so that a column's products read consecutive entries.
// Cached beside F per (device, N, J, taps, R).  env JW_AUTO_SPECT=0: natural order (A/B runs).
using SpecTKey = std::tuple<int, long, int, long, std::vector<double>>;
DevCache<SpecTKey> g_spect(16UL << 30);  // the same spectra per kp2p column (two-pass N <= 2^24)

__global__ __launch_bounds__(256) void kspec_t(const cplx* __restrict__ F, cplx* __restrict__ FT,
                                               long N, int rbits, long C) {
  __shared__ cplx t[32][33];
  const long R = 1L << rbits;
  const long q = blockIdx.z;
  const long h0 = (long)blockIdx.y * 32, l0 = (long)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int k = ty; k < 32; k += 8) t[k][tx] = F[q * N + (h0 + k) * R + l0 + tx];
  __syncthreads();
  for (int k = ty; k < 32; k += 8) FT[q * N + (l0 + k) * C + h0 + tx] = t[tx][k];
}

bool spect_enabled() {
  const char* e = knob("JW_AUTO_SPECT");
  return !(e && e[0] == '0');
}

int spectra_t(const ModwtPlan& p, long N, int J, const cplx* F, long R, const cplx** FT,
              StreamAllocs& mem, hipStream_t s) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  std::vector<double> taps(p.g, p.g + p.L);
  taps.insert(taps.end(), p.h, p.h + p.L);
  const long C = N / R;
  const void* out = nullptr;
  const int st = cached_table(g_spect, SpecTKey(dev, N, J, R, taps),
                              (size_t)2 * J * N * sizeof(cplx), mem, s, &out, [&](void* d) -> int {
                                if (R < 32 || C < 32)
                                  return fail(JW_ERR_UNSUPPORTED, "spectra_t: %ld x %ld", R, C);
                                hipLaunchKernelGGL(kspec_t, dim3((unsigned)(R / 32), (unsigned)(C / 32),
                                                                 (unsigned)(2 * J)),
                                                   dim3(256), 0, s, F, (cplx*)d, N, ilog2(R), C);
                                JW_HIP_TRY(hipGetLastError());
                                return JW_OK;
                              });
  *FT = (const cplx*)out;
  return st;
}

// ---------------------------------------------------------------------------------------
// MODWT, one level per step as MODWTTransform.forwardMODWT / inverseMODWT run it (:290-304,
// :355-372): FFT levels here, DIRECT levels through the direct per-level kernels (jw_modwt.hip).
// Rows V_j between levels live in two scratch rows (ping-pong) or, across two FFT levels, only
// as the next level's pass-1 output Z (the pass 2 of V_j's inverse FFT feeds it directly).
// ---------------------------------------------------------------------------------------
struct Chunk {
  long nb, N;
  int J;
  double* tmp[2];  // scratch V rows, nb x N each
};

int forward_lines(const ModwtPlan& p, const bool* fft, const cplx* F, const Tw& twf,
                  const Tw& twi, const double* x, double* coeffs, const Chunk& c, hipStream_t s) {
  const long N = c.N, rs = (long)(c.J + 1) * N;
  const double* vin = x;
  long vs = N;
  for (int j = 1; j <= c.J; ++j) {
    double* vout = j == c.J ? coeffs + (long)c.J * N : c.tmp[j & 1];
    const long vos = j == c.J ? rs : N;
    double* w = coeffs + (long)(j - 1) * N;
    int st;
    if (fft[j]) {
      st = with_lc(N, [&](auto LCc) -> int {
        constexpr int LC = decltype(LCc)::value;
        return launch_grid<LC, kLineEPT<LC>>(kline_modwt<LC, 1, 2, LineIn, LineFwdMid, LineOut>,
                               (c.nb + LineGeo<LC>::T - 1) / LineGeo<LC>::T, s, LineIn{vin, vs, vin, vs},
                               LineFwdMid{spec_h(F, N, j), spec_g(F, N, j)},
                               LineOut{w, rs, vout, vos}, c.nb, twf.p1, twi.p1, 1.0 / (double)N);
      });
    } else {
      st = modwt_level_forward_device(p, j, vin, vs, w, rs, vout, vos, N, (int)c.nb, s);
    }
    if (st != JW_OK) return st;
    vin = vout;
    vs = vos;
  }
  return JW_OK;
}

int inverse_lines(const ModwtPlan& p, const bool* fft, const cplx* F, const Tw& twf,
                  const Tw& twi, const double* coeffs, double* x, const Chunk& c, hipStream_t s) {
  const long N = c.N, rs = (long)(c.J + 1) * N;
  const double* vin = coeffs + (long)c.J * N;  // Arrays.copyOf(coefficients[maxLevel]) :353
  long vs = rs;
  for (int j = c.J; j >= 1; --j) {
    double* vout = j == 1 ? x : c.tmp[j & 1];
    const double* w = coeffs + (long)(j - 1) * N;
    int st;
    if (fft[j]) {
      st = with_lc(N, [&](auto LCc) -> int {
        constexpr int LC = decltype(LCc)::value;
        return launch_grid<LC, kLineEPT<LC>>(kline_modwt<LC, 2, 1, LineIn, LineAdjMid, LineOut>,
                               (c.nb + LineGeo<LC>::T - 1) / LineGeo<LC>::T, s, LineIn{vin, vs, w, rs},
                               LineAdjMid{spec_g(F, N, j), spec_h(F, N, j)},
                               LineOut{vout, N, vout, N}, c.nb, twf.p1, twi.p1, 1.0 / (double)N);
      });
    } else {
      st = modwt_level_inverse_device(p, j, vin, vs, w, rs, vout, N, N, (int)c.nb, s);
    }
    if (st != JW_OK) return st;
    vin = vout;
    vs = N;
  }
  return JW_OK;
}

// A/B builds: points per thread of the fused levels' pass-1 kernels (kp1 over real rows) at
// 512 / 1024 points (0: Geo's rule, 8)
#ifndef JF_FUSED_P1_EPT
#define JF_FUSED_P1_EPT 0
#endif
template <int LC>
constexpr int kFusedP1EPT = LC <= 1024 ? JF_FUSED_P1_EPT : 0;

// Column geometry of the level transforms: forward FFTs split N = R x C (pass 1 over columns
// of length R), inverse FFTs C x R, so every forward pass 2 feeds an inverse pass 1 and every
// inverse pass 2 a forward pass 1 (jw_jfft.hpp).
struct ColGeo {
  long N, R, C;
  int rbits, cbits;
};

// Z (nb x [C][R], forward pass-1 rows of V_{j-1}) -> Zi_h, Zi_g (inverse pass-1 rows) -> W_j,
// and V_j either stored (last level, or a DIRECT level next) or run straight into the next
// level's pass 1 (Z).
int forward_cols(const ModwtPlan& p, const bool* fft, const cplx* F, const cplx* FT,
                 const Tw& twf, const Tw& twi, const ColGeo& g, const double* x, double* coeffs,
                 const Chunk& c, cplx* Z, cplx* Zi, hipStream_t s) {
  const long N = c.N, nb = c.nb, rs = (long)(c.J + 1) * N;
  const double* vin = x;
  long vs = N;
  bool haveZ = false;
  int st = JW_OK;
  for (int j = 1; j <= c.J && st == JW_OK; ++j) {
    double* w = coeffs + (long)(j - 1) * N;
    const bool last = j == c.J;
    double* vout = last ? coeffs + (long)c.J * N : c.tmp[j & 1];
    const long vos = last ? rs : N;
    if (!fft[j]) {
      st = modwt_level_forward_device(p, j, vin, vs, w, rs, vout, vos, N, (int)nb, s);
      vin = vout;
      vs = vos;
      haveZ = false;
      continue;
    }
    if (!haveZ) {  // forward pass 1 of V_{j-1}
      st = with_big_lc(g.R, [&](auto LCc) -> int {
        constexpr int LC = decltype(LCc)::value;
        constexpr int E = kFusedP1EPT<LC>;
        return launch_grid<LC, E>(kp1<LC, RowsR, OutC, E>, (g.C / Geo<LC, E>::T) * nb, s,
                                  RowsR{vin, vs}, OutC{Z, N}, g.cbits, nb, twf.p1);
      });
      if (st != JW_OK) break;
    }
    // forward pass 2, X . F_h / X . F_g, inverse pass 1 of each (one filter per item: a
    // workgroup holding both products, Z read once, needed 168 VGPRs even with the twiddle fix
    // and ran the forward 44.0 -> 48.5 ms)
    st = with_big_lc(g.C, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      if (LC == 1024 && FT && use_wcol())
        return launch_wcol(kp2p_w<ZPair, FwdMidT, OutPair>, (g.R / wcol::T) * 2 * nb, s,
                           ZPair{Z, N}, FwdMidT{spec_h(FT, N, j), spec_g(FT, N, j), g.rbits, g.C},
                           OutPair{Zi, N, nb * N}, g.rbits, 2 * nb, twf.p2, twi.p1);
      if (FT)
        return launch_grid<LC>(kp2p<LC, 1, ZPair, FwdMidT, OutPair>, (g.R / Geo<LC>::T) * 2 * nb,
                               s, ZPair{Z, N},
                               FwdMidT{spec_h(FT, N, j), spec_g(FT, N, j), g.rbits, g.C},
                               OutPair{Zi, N, nb * N}, g.rbits, 2 * nb, twf.p2, twi.p1);
      return launch_grid<LC>(kp2p<LC, 1, ZPair, FwdMid, OutPair>, (g.R / Geo<LC>::T) * 2 * nb, s,
                             ZPair{Z, N}, FwdMid{spec_h(F, N, j), spec_g(F, N, j)},
                             OutPair{Zi, N, nb * N}, g.rbits, 2 * nb, twf.p2, twi.p1);
    });
    if (st != JW_OK) break;
    const double inv_n = 1.0 / (double)N;
    const bool fuse = !last && fft[j + 1];
    st = with_big_lc(g.R, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      const long blocks = (g.C / Geo<LC>::T) * nb;
      int r = launch_grid<LC>(kp2r<LC, 1, false, InS, PowPost, OutR>, blocks, s, InS{Zi, N, 0},
                              PowPost{inv_n}, OutR{w, rs}, g.cbits, nb, twi.p2, twf.p1);
      if (r != JW_OK) return r;
      const InS vin_s{Zi + nb * N, N, 0};
      if (fuse)
        return launch_grid<LC>(kp2r<LC, 1, true, InS, PowPost, OutC>, blocks, s, vin_s,
                               PowPost{inv_n}, OutC{Z, N}, g.cbits, nb, twi.p2, twf.p1);
      return launch_grid<LC>(kp2r<LC, 1, false, InS, PowPost, OutR>, blocks, s, vin_s,
                             PowPost{inv_n}, OutR{vout, vos}, g.cbits, nb, twi.p2, twf.p1);
    });
    haveZ = fuse;
    vin = vout;
    vs = vos;
  }
  return st;
}

// Zs = [Z_V | Z_W] (forward pass-1 rows of V_j and W_j), Zi = [Zi_A | Zi_D]
int inverse_cols(const ModwtPlan& p, const bool* fft, const cplx* F, const cplx* FT,
                 const Tw& twf, const Tw& twi, const ColGeo& g, const double* coeffs, double* x,
                 const Chunk& c, cplx* Zs, cplx* Zi, hipStream_t s) {
  const long N = c.N, nb = c.nb, rs = (long)(c.J + 1) * N;
  const double* vin = coeffs + (long)c.J * N;
  long vs = rs;
  bool haveZ = false;
  int st = JW_OK;
  for (int j = c.J; j >= 1 && st == JW_OK; --j) {
    const double* w = coeffs + (long)(j - 1) * N;
    double* vout = j == 1 ? x : c.tmp[j & 1];
    if (!fft[j]) {
      st = modwt_level_inverse_device(p, j, vin, vs, w, rs, vout, N, N, (int)nb, s);
      vin = vout;
      vs = N;
      haveZ = false;
      continue;
    }
    st = with_big_lc(g.R, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      constexpr int E = kFusedP1EPT<LC>;
      const long blocks = (g.C / Geo<LC, E>::T) * nb;
      if (!haveZ) {
        const int r = launch_grid<LC, E>(kp1<LC, RowsR, OutC, E>, blocks, s, RowsR{vin, vs},
                                         OutC{Zs, N}, g.cbits, nb, twf.p1);
        if (r != JW_OK) return r;
      }
      return launch_grid<LC, E>(kp1<LC, RowsR, OutC, E>, blocks, s, RowsR{w, rs},
                                OutC{Zs + nb * N, N}, g.cbits, nb, twf.p1);
    });
    if (st != JW_OK) break;
    st = with_big_lc(g.C, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      if (LC == 1024 && FT && use_wcol())
        return launch_wcol(kp2p_w<RowsC, AdjMidT, OutF>, (g.R / wcol::T) * 2 * nb, s,
                           RowsC{Zs, N}, AdjMidT{spec_g(FT, N, j), spec_h(FT, N, j), nb, g.rbits, g.C},
                           OutF{Zi, N, 0}, g.rbits, 2 * nb, twf.p2, twi.p1);
      if (FT)
        return launch_grid<LC>(kp2p<LC, 1, RowsC, AdjMidT, OutF>, (g.R / Geo<LC>::T) * 2 * nb, s,
                               RowsC{Zs, N},
                               AdjMidT{spec_g(FT, N, j), spec_h(FT, N, j), nb, g.rbits, g.C},
                               OutF{Zi, N, 0}, g.rbits, 2 * nb, twf.p2, twi.p1);
      return launch_grid<LC>(kp2p<LC, 1, RowsC, AdjMid, OutF>, (g.R / Geo<LC>::T) * 2 * nb, s,
                             RowsC{Zs, N}, AdjMid{spec_g(F, N, j), spec_h(F, N, j), nb},
                             OutF{Zi, N, 0}, g.rbits, 2 * nb, twf.p2, twi.p1);
    });
    if (st != JW_OK) break;
    const double inv_n = 1.0 / (double)N;
    const bool fuse = j > 1 && fft[j - 1];
    st = with_big_lc(g.R, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      const long blocks = (g.C / Geo<LC>::T) * nb;
      const InS in{Zi, N, nb * N};
      if (fuse)
        return launch_grid<LC>(kp2r<LC, 2, true, InS, PowPost, OutC>, blocks, s, in,
                               PowPost{inv_n}, OutC{Zs, N}, g.cbits, nb, twi.p2, twf.p1);
      return launch_grid<LC>(kp2r<LC, 2, false, InS, PowPost, OutR>, blocks, s, in,
                             PowPost{inv_n}, OutR{vout, N}, g.cbits, nb, twi.p2, twf.p1);
    });
    haveZ = fuse;
    vin = vout;
    vs = N;
  }
  return st;
}

// P[i] = X[i].mul(F[i]) (circularConvolveFFT :775-778), or with F[i].conjugate() (:820-824)
template <bool CONJ>
__global__ __launch_bounds__(256) void kmul_spec(const cplx* __restrict__ X,
                                                 const cplx* __restrict__ F, cplx* __restrict__ P,
                                                 long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const cplx f = F[i];
    P[i] = jmul(X[i], CONJ ? make_double2(f.x, -f.y) : f);
  }
}

template <bool CONJ>
int mul_spec(const cplx* X, const cplx* F, cplx* P, long n, hipStream_t s) {
  const long blocks = std::min<long>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(kmul_spec<CONJ>, dim3((unsigned)blocks), dim3(256), 0, s, X, F, P, n);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

// Long lines (three-pass transforms): each FFT level exactly as the reference writes it, one
// signal and one transform at a time -- FFT(V) (Complex(v, 0)), the product with the level's
// filter spectrum, the reverse FFT with its 1/n, the real part (:752-837); DIRECT levels
// through the direct per-level kernels.  Unfused (these lengths are for parity, not speed).
int modwt_strict_long(bool inverse, const ModwtPlan& p, const double* in, double* out, long N,
                      int J, int batch, const bool* fft, const cplx* F, StreamAllocs& mem,
                      hipStream_t s) {
  const long rs = (long)(J + 1) * N;
  cplx *X = nullptr, *P = nullptr;
  double* tmp = nullptr;
  JW_HIP_TRY(mem.alloc(&X, (size_t)N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&P, (size_t)N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&tmp, (size_t)2 * N * sizeof(double)));
  const double inv_n = 1.0 / (double)N;
  int st = JW_OK;
  // Each transform takes its workspace (and, past the table cache's budget, its three-pass
  // twiddles) from an allocator scoped to that one call, freed stream-ordered when it returns:
  // with the call's own allocator they would pile up over batch x levels x transforms until
  // modwt_strict returns (~7.5 GB per signal at 2^25, db4 J=8).
  auto rows = [&](bool inv, auto in, auto out) {
    StreamAllocs scoped(s);
    return fft_rows(N, inv, 1, in, out, scoped, s);
  };
  auto fwd = [&](const double* v) {  // X = FFT(Complex(v, 0))
    return rows(false, RowsR{v, N}, OutCS{X, N, 1.0, 0});
  };
  for (long b = 0; b < batch && st == JW_OK; ++b) {
    if (!inverse) {
      const double* x = in + b * N;
      double* c = out + b * rs;
      const double* vin = x;
      for (int j = 1; j <= J && st == JW_OK; ++j) {
        double* w = c + (long)(j - 1) * N;
        double* vout = j == J ? c + (long)J * N : tmp + (long)(j & 1) * N;
        if (!fft[j]) {
          st = modwt_level_forward_device(p, j, vin, N, w, rs, vout, N, N, 1, s);
        } else if ((st = fwd(vin)) == JW_OK &&
                   (st = mul_spec<false>(X, spec_h(F, N, j), P, N, s)) == JW_OK &&
                   (st = rows(true, RowsC{P, N}, OutRe<false>{w, N, inv_n})) == JW_OK &&
                   (st = mul_spec<false>(X, spec_g(F, N, j), P, N, s)) == JW_OK) {
          st = rows(true, RowsC{P, N}, OutRe<false>{vout, N, inv_n});
        }
        vin = vout;
      }
    } else {
      const double* c = in + b * rs;
      double* x = out + b * N;
      const double* vin = c + (long)J * N;
      for (int j = J; j >= 1 && st == JW_OK; --j) {
        const double* w = c + (long)(j - 1) * N;
        double* vout = j == 1 ? x : tmp + (long)(j & 1) * N;
        if (!fft[j]) {
          st = modwt_level_inverse_device(p, j, vin, N, w, rs, vout, N, N, 1, s);
        } else if ((st = fwd(vin)) == JW_OK &&
                   (st = mul_spec<true>(X, spec_g(F, N, j), P, N, s)) == JW_OK &&
                   (st = rows(true, RowsC{P, N}, OutRe<false>{vout, N, inv_n})) == JW_OK &&
                   (st = fwd(w)) == JW_OK &&
                   (st = mul_spec<true>(X, spec_h(F, N, j), P, N, s)) == JW_OK) {
          // vFromApprox[i] + vFromDetail[i] (:366-369)
          st = rows(true, RowsC{P, N}, OutRe<true>{vout, N, inv_n});
        }
        vin = vout;
      }
    }
  }
  return st;
}

int modwt_strict(bool inverse, const ModwtPlan& p, const double* in, double* out, long N, int J,
                 int batch, const bool* fft, hipStream_t s) {
  StreamAllocs mem(s);
  const cplx* F = nullptr;
  int st = filter_spectra(p, N, J, &F, mem, s);
  if (st != JW_OK) return st;
  if (N & (N - 1)) return modwt_strict_bs(inverse, p, in, out, N, J, batch, fft, F, mem, s);
  if (N > kLineMax && N >= three_pass_min())
    return modwt_strict_long(inverse, p, in, out, N, J, batch, fft, F, mem, s);
  const long rs = (long)(J + 1) * N;
  if (N <= kLineMax) {
    Tw twf, twi;
    if ((st = twiddles(N, false, (int)N, &twf, mem, s)) != JW_OK) return st;
    if ((st = twiddles(N, true, (int)N, &twi, mem, s)) != JW_OK) return st;
    const long chunk = std::max(1L, std::min<long>(batch, (1L << 30) / (16 * N)));
    double* tmp = nullptr;
    JW_HIP_TRY(mem.alloc(&tmp, (size_t)2 * chunk * N * sizeof(double)));
    for (long b0 = 0; b0 < batch && st == JW_OK; b0 += chunk) {
      const Chunk c{std::min(chunk, batch - b0), N, J, {tmp, tmp + chunk * N}};
      st = inverse ? inverse_lines(p, fft, F, twf, twi, in + b0 * rs, out + b0 * N, c, s)
                   : forward_lines(p, fft, F, twf, twi, in + b0 * N, out + b0 * rs, c, s);
    }
    return st;
  }
  ColGeo g;
  g.N = N;
  g.R = split_lc1(N);
  // The inverse levels run faster with the shorter pass-1 columns (more columns per kp1 / kp2r
  // workgroup: 128-byte pieces) and longer kp2p columns: at N = 2^20, 512 x 2048 instead of
  // 1024 x 1024 took the db4 J=8 inverse 50.6 -> 49.5 ms and the sym8 J=6 one 38.1 -> 37.2 ms per
  // 128 signals, while the forward prefers the square split (profiles/r04/ab/auto_split_r.log).
  // Bit-identical either way (the split changes no operation, only the access shapes).
  if (inverse && g.R >= 1024 && N / (g.R / 2) <= 2048) g.R /= 2;
  {
    // A/B runs: JW_AUTO_R = the forward pass-1 column length (a power of two, 64 .. 4096,
    // with N / R in the same range)
    const char* e = knob("JW_AUTO_R");
    const long r = e ? std::atol(e) : 0;
    if (r >= 64 && r <= 4096 && (r & (r - 1)) == 0 && N % r == 0 && N / r >= 64 && N / r <= 4096)
      g.R = r;
  }
  g.C = N / g.R;
  g.rbits = ilog2(g.R);
  g.cbits = ilog2(g.C);
  Tw twf, twi;  // forward FFTs split R x C, inverse FFTs C x R
  if ((st = twiddles(N, false, (int)g.R, &twf, mem, s)) != JW_OK) return st;
  if ((st = twiddles(N, true, (int)g.C, &twi, mem, s)) != JW_OK) return st;
  const cplx* FT = nullptr;  // the spectra per kp2p column (kp2p's view is [C][R])
  if (spect_enabled() && (st = spectra_t(p, N, J, F, g.R, &FT, mem, s)) != JW_OK) return st;
  // per signal: 4 complex rows of workspace (forward uses 3) + 2 real scratch rows
  const long per_sig = 4 * N * (long)sizeof(cplx) + 2 * N * (long)sizeof(double);
  const long chunk = std::max(1L, std::min<long>(batch, (4L << 30) / per_sig));
  cplx* W = nullptr;
  double* tmp = nullptr;
  JW_HIP_TRY(mem.alloc(&W, (size_t)4 * chunk * N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&tmp, (size_t)2 * chunk * N * sizeof(double)));
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += chunk) {
    const long nb = std::min(chunk, batch - b0);
    const Chunk c{nb, N, J, {tmp, tmp + chunk * N}};
    st = inverse ? inverse_cols(p, fft, F, FT, twf, twi, g, in + b0 * rs, out + b0 * N, c, W,
                                W + 2 * nb * N, s)
                 : forward_cols(p, fft, F, FT, twf, twi, g, in + b0 * N, out + b0 * rs, c, W,
                                W + nb * N, s);
  }
  return st;
}

}  // namespace
}  // namespace jf

// ---------------------------------------------------------------------------------------
// entry points (jw_internal.hpp)
// ---------------------------------------------------------------------------------------
// every length the reference's FFT path takes: powers of two (radix 2) up to 2^30 and, through
// Bluestein with m <= 2^30, any other n <= 2^29 (jw_internal.hpp kStrictFft*)
bool modwt_strict_fft_supported(long n) {
  return n >= 2 && n <= ((n & (n - 1)) == 0 ? kStrictFftPow2Max : kStrictFftOtherMax);
}

int modwt_forward_strict_device(const ModwtPlan& p, const double* x, double* coeffs, long n,
                                int J, int batch, const bool* fft_level, hipStream_t s) {
  return jf::modwt_strict(false, p, x, coeffs, n, J, batch, fft_level, s);
}

int modwt_inverse_strict_device(const ModwtPlan& p, const double* coeffs, double* x, long n,
                                int J, int batch, const bool* fft_level, hipStream_t s) {
  return jf::modwt_strict(true, p, coeffs, x, n, J, batch, fft_level, s);
}

int fft_strict_device(int S, const double* in, double* out, long n, long batch, hipStream_t s) {
  if (n == 0 || batch == 0) return JW_OK;
  if (n == 1) {  // forward/reverse return a copy (:117-119, :146-148)
    if (in != out)
      JW_HIP_TRY(hipMemcpyAsync(out, in, (size_t)batch * 2 * sizeof(double),
                                hipMemcpyDeviceToDevice, s));
    return JW_OK;
  }
  if ((n & (n - 1)) != 0) {
    if (n > kStrictFftOtherMax)
      return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: length %ld > %ld", n, kStrictFftOtherMax);
    return jf::bs_fft_strict(S > 0, (const jf::cplx*)in, (jf::cplx*)out, n, batch, s);
  }
  if (n > jf::kStrictPow2Max)
    return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: length %ld > %ld", n, jf::kStrictPow2Max);
  // in == out is safe: a line is read whole before it is written, and the column path reads
  // the input in pass 1 and writes the output in pass 2 (from the workspace Z)
  StreamAllocs mem(s);
  const jf::cplx* xi = (const jf::cplx*)in;
  jf::cplx* xo = (jf::cplx*)out;
  return jf::fft_rows(n, S > 0, batch, jf::RowsC{xi, n},
                      jf::OutCS{xo, n, 1.0 / (double)n, S > 0 ? 1 : 0}, mem, s);
}

}  // namespace jw
