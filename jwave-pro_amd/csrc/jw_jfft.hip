// jw_jfft.hip -- JW_ARITH_STRICT FFT paths: the reference's own FFT (jw_jfft.hpp) behind
//   * FastFourierTransform.forward/reverse(Complex[]) (FastFourierTransform.java:112-164), and
//   * MODWTTransform's FFT convolution, level by level as the reference runs it
//     (performConvolution :640-664, circularConvolveFFT :752-786, circularConvolveFFTAdjoint
//     :798-837, wrapFilterToSignalLength :729-741),
// so a default-constructed MODWTTransform (AUTO) gets the JVM's values bit for bit.
#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <vector>

#include "jw_jfft.hpp"

namespace jw {
namespace jf {
namespace {

constexpr long kLineMax = 4096;  // whole transform in one column up to here

// ---------------------------------------------------------------------------------------
// Device caches: built on the caller's stream, synchronised once, then published.  No lock is
// held across device work.  At most kCacheBytes per cache: past that a call builds its own
// table (stream-ordered, freed after the call).  jw_release_caches() frees them.
// ---------------------------------------------------------------------------------------
constexpr size_t kCacheBytes = 2UL << 30;

template <class Key>
class DevCache {
 public:
  const void* find(const Key& k) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(k);
    return it == m_.end() ? nullptr : it->second.first;
  }
  bool fits(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    return bytes_ + bytes <= kCacheBytes;
  }
  // takes ownership of p (complete); returns the entry to use -- another thread's if it
  // raced us, in which case p is freed
  const void* insert(const Key& k, void* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = m_.find(k);
    if (it != m_.end()) {
      (void)hipFree(p);
      return it->second.first;
    }
    m_.emplace(k, std::make_pair(p, bytes));
    bytes_ += bytes;
    return p;
  }
  size_t clear() {
    std::lock_guard<std::mutex> lk(mu_);
    const size_t b = bytes_;
    for (auto& e : m_) (void)hipFree(e.second.first);
    m_.clear();
    bytes_ = 0;
    return b;
  }

 private:
  std::mutex mu_;
  std::map<Key, std::pair<void*, size_t>> m_;
  size_t bytes_ = 0;
};

template <class Key, class Fill>
int cached_table(DevCache<Key>& cache, const Key& key, size_t bytes, StreamAllocs& mem,
                 hipStream_t s, const void** out, Fill&& fill) {
  if ((*out = cache.find(key)) != nullptr) return JW_OK;
  if (!cache.fits(bytes)) {
    void* p = nullptr;
    JW_HIP_TRY(mem.alloc(&p, bytes));
    *out = p;
    return fill(p);
  }
  void* p = nullptr;
  JW_HIP_TRY(hipMalloc(&p, bytes));
  int st = fill(p);
  const hipError_t e = hipStreamSynchronize(s);  // complete before other threads may see it
  if (st != JW_OK || e != hipSuccess) {
    (void)hipFree(p);
    return st != JW_OK ? st : fail(JW_ERR_DEVICE, "table build: %s", hipGetErrorString(e));
  }
  *out = cache.insert(key, p, bytes);
  return JW_OK;
}

// ---------------------------------------------------------------------------------------
// Twiddles: Tw[half + k] = wn_k of the stage of size 2 half, by the reference's recurrence
// (:188-201; host code is built with -ffp-contract=off, like the JVM).  Device layout:
// [0, lc1) natural (pass 1; lc1 = n for a one-column transform), then the pass-2 table
// transposed, Tw2[l lc2 + m] = Tw[m lc1 + l] (l < lc1, m < lc2 = n / lc1).
// ---------------------------------------------------------------------------------------
using TwKey = std::tuple<int, long, int, int>;  // device, n, inverse, lc1
DevCache<TwKey> g_tw;

constexpr double kJavaPi = 3.141592653589793;  // Math.PI

void java_twiddles(long n, bool inverse, std::vector<cplx>& tw) {
  tw.assign(n, make_double2(0.0, 0.0));
  for (long half = 1; half < n; half <<= 1) {
    const long size = 2 * half;
    const double angle = 2 * kJavaPi / (double)size * (double)(inverse ? 1 : -1);
    const double wr = std::cos(angle), wi = std::sin(angle);
    double nr = 1.0, ni = 0.0;  // wn = new Complex(1, 0)
    for (long k = 0; k < half; ++k) {
      tw[half + k] = make_double2(nr, ni);
      const double tr = nr * wr - ni * wi, ti = nr * wi + ni * wr;  // wn = wn.mul(w)
      nr = tr;
      ni = ti;
    }
  }
}

struct Tw {
  long n = 0;
  int lc1 = 0;
  const cplx* p1 = nullptr;
  const cplx* p2 = nullptr;
};

// pass-1 length of an n-point transform (n itself when it runs in one column)
int split_lc1(long n) { return n <= kLineMax ? (int)n : 1 << (ilog2(n) / 2); }

int twiddles(long n, bool inverse, int lc1, Tw* out, StreamAllocs& mem, hipStream_t s) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  const bool one = lc1 >= n;
  const size_t entries = one ? (size_t)n : (size_t)lc1 + (size_t)n;
  const void* p = nullptr;
  int st = cached_table(g_tw, TwKey(dev, n, inverse ? 1 : 0, lc1), entries * sizeof(cplx), mem,
                        s, &p, [&](void* d) -> int {
                          std::vector<cplx> tw;
                          java_twiddles(n, inverse, tw);
                          std::vector<cplx> h(entries);
                          std::copy(tw.begin(), tw.begin() + (one ? n : lc1), h.begin());
                          if (!one) {
                            const long lc2 = n / lc1;
                            for (long l = 0; l < lc1; ++l)
                              for (long m = 0; m < lc2; ++m)
                                h[lc1 + l * lc2 + m] = tw[m * lc1 + l];
                          }
                          JW_HIP_TRY(upload_async(d, h.data(), entries * sizeof(cplx), s));
                          return JW_OK;
                        });
  if (st != JW_OK) return st;
  out->n = n;
  out->lc1 = one ? (int)n : lc1;
  out->p1 = (const cplx*)p;
  out->p2 = one ? nullptr : (const cplx*)p + lc1;
  return JW_OK;
}

// ---------------------------------------------------------------------------------------
// Launch helpers: runtime column length -> template instantiation
// ---------------------------------------------------------------------------------------
#define JF_CASE(V) \
  case V:          \
    return f(std::integral_constant<int, V>{});

template <class F>
int with_lc(long lc, F&& f) {
  switch (lc) {
    JF_CASE(2) JF_CASE(4) JF_CASE(8) JF_CASE(16) JF_CASE(32) JF_CASE(64) JF_CASE(128)
    JF_CASE(256) JF_CASE(512) JF_CASE(1024) JF_CASE(2048) JF_CASE(4096)
    default:
      return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: line length %ld unsupported", lc);
  }
}
template <class F>
int with_big_lc(long lc, F&& f) {
  switch (lc) {
    JF_CASE(64) JF_CASE(128) JF_CASE(256) JF_CASE(512) JF_CASE(1024) JF_CASE(2048) JF_CASE(4096)
    default:
      return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: column length %ld unsupported", lc);
  }
}
#undef JF_CASE

template <int LC, class K, class... A>
int launch_grid(K kern, long blocks, hipStream_t s, A... args) {
  const size_t lds = Geo<LC>::LDS_BYTES;
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  if (blocks <= 0) return JW_OK;
  if (blocks >= (1L << 24))
    return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: grid of %ld workgroups", blocks);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kNT), lds, s, args...);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
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
// forward level: signalFFT[i].mul(filterFFT[i]), f = 0 -> h_j (W_j), f = 1 -> g_j (V_j) (:775-778)
struct FwdMid {
  const cplx* fh;
  const cplx* fg;
  __device__ cplx operator()(int f, long, long i, cplx x) const { return jmul(x, (f ? fg : fh)[i]); }
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
template <class In>
int fft_rows(long n, bool inverse, long items, In in, OutCS out, StreamAllocs& mem,
             hipStream_t s) {
  const int lc1 = split_lc1(n);
  Tw tw;
  int st = twiddles(n, inverse, lc1, &tw, mem, s);
  if (st != JW_OK) return st;
  if (n <= kLineMax) {
    return with_lc(n, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC>(kline_fft<LC, In, OutCS>, (items + Geo<LC>::T - 1) / Geo<LC>::T, s,
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
    OutCS out_c = out;
    out_c.p += i0 * out.st;
    st = with_big_lc(lc1, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC>(kp1<LC, In, OutC>, (lc2 / Geo<LC>::T) * ni, s, in_c, OutC{Z, n},
                             ilog2(lc2), ni, tw.p1);
    });
    if (st != JW_OK) break;
    st = with_big_lc(lc2, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC>(kp2s<LC, RowsC, OutCS>, (lc1 / Geo<LC>::T) * ni, s, RowsC{Z, n},
                             out_c, ilog2(lc1), ni, tw.p2);
    });
  }
  return st;
}

// ---------------------------------------------------------------------------------------
// MODWT filter spectra: FFT(wrapFilterToSignalLength(upsample(f, j), N)) (:729-741, :770-771),
// rows [j - 1][0 = h (wavelet), 1 = g (scaling)], natural order; cached per (device, taps, N, J).
// ---------------------------------------------------------------------------------------
using SpecKey = std::tuple<int, long, int, std::vector<double>>;
DevCache<SpecKey> g_spec;

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
        return fft_rows(N, false, 2L * J, RowsR{drows, N}, OutCS{(cplx*)d, N, 1.0, 0}, mem, s);
      });
  *F = (const cplx*)out;
  return st;
}

const cplx* spec_h(const cplx* F, long N, int j) { return F + (long)(2 * (j - 1)) * N; }
const cplx* spec_g(const cplx* F, long N, int j) { return F + (long)(2 * (j - 1) + 1) * N; }

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
        return launch_grid<LC>(kline_modwt<LC, 1, 2, LineIn, LineFwdMid, LineOut>,
                               (c.nb + Geo<LC>::T - 1) / Geo<LC>::T, s, LineIn{vin, vs, vin, vs},
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
        return launch_grid<LC>(kline_modwt<LC, 2, 1, LineIn, LineAdjMid, LineOut>,
                               (c.nb + Geo<LC>::T - 1) / Geo<LC>::T, s, LineIn{vin, vs, w, rs},
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
int forward_cols(const ModwtPlan& p, const bool* fft, const cplx* F, const Tw& twf,
                 const Tw& twi, const ColGeo& g, const double* x, double* coeffs, const Chunk& c,
                 cplx* Z, cplx* Zi, hipStream_t s) {
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
        return launch_grid<LC>(kp1<LC, RowsR, OutC>, (g.C / Geo<LC>::T) * nb, s, RowsR{vin, vs},
                               OutC{Z, N}, g.cbits, nb, twf.p1);
      });
      if (st != JW_OK) break;
    }
    // forward pass 2, X . F_h / X . F_g, inverse pass 1 of both
    st = with_big_lc(g.C, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC>(kp2p<LC, 2, RowsC, FwdMid, OutF>, (g.R / Geo<LC>::T) * nb, s,
                             RowsC{Z, N}, FwdMid{spec_h(F, N, j), spec_g(F, N, j)},
                             OutF{Zi, N, nb * N}, g.rbits, nb, twf.p2, twi.p1);
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
int inverse_cols(const ModwtPlan& p, const bool* fft, const cplx* F, const Tw& twf,
                 const Tw& twi, const ColGeo& g, const double* coeffs, double* x, const Chunk& c,
                 cplx* Zs, cplx* Zi, hipStream_t s) {
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
      const long blocks = (g.C / Geo<LC>::T) * nb;
      if (!haveZ) {
        const int r = launch_grid<LC>(kp1<LC, RowsR, OutC>, blocks, s, RowsR{vin, vs},
                                      OutC{Zs, N}, g.cbits, nb, twf.p1);
        if (r != JW_OK) return r;
      }
      return launch_grid<LC>(kp1<LC, RowsR, OutC>, blocks, s, RowsR{w, rs}, OutC{Zs + nb * N, N},
                             g.cbits, nb, twf.p1);
    });
    if (st != JW_OK) break;
    st = with_big_lc(g.C, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
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

int modwt_strict(bool inverse, const ModwtPlan& p, const double* in, double* out, long N, int J,
                 int batch, const bool* fft, hipStream_t s) {
  StreamAllocs mem(s);
  const cplx* F = nullptr;
  int st = filter_spectra(p, N, J, &F, mem, s);
  if (st != JW_OK) return st;
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
  g.C = N / g.R;
  g.rbits = ilog2(g.R);
  g.cbits = ilog2(g.C);
  Tw twf, twi;  // forward FFTs split R x C, inverse FFTs C x R
  if ((st = twiddles(N, false, (int)g.R, &twf, mem, s)) != JW_OK) return st;
  if ((st = twiddles(N, true, (int)g.C, &twi, mem, s)) != JW_OK) return st;
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
    st = inverse ? inverse_cols(p, fft, F, twf, twi, g, in + b0 * rs, out + b0 * N, c, W,
                                W + 2 * nb * N, s)
                 : forward_cols(p, fft, F, twf, twi, g, in + b0 * N, out + b0 * rs, c, W,
                                W + nb * N, s);
  }
  return st;
}

}  // namespace
}  // namespace jf

// ---------------------------------------------------------------------------------------
// entry points (jw_internal.hpp)
// ---------------------------------------------------------------------------------------
bool modwt_strict_fft_supported(long n) {
  return n >= 2 && (n & (n - 1)) == 0 && n <= (1L << 23);
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
  if ((n & (n - 1)) != 0 || n > (1L << 24))
    return fail(JW_ERR_UNSUPPORTED, "Java-order FFT: length %ld", n);
  // in == out is safe: a line is read whole before it is written, and the column path reads
  // the input in pass 1 and writes the output in pass 2 (from the workspace Z)
  StreamAllocs mem(s);
  const jf::cplx* xi = (const jf::cplx*)in;
  jf::cplx* xo = (jf::cplx*)out;
  return jf::fft_rows(n, S > 0, batch, jf::RowsC{xi, n},
                      jf::OutCS{xo, n, 1.0 / (double)n, S > 0 ? 1 : 0}, mem, s);
}

size_t release_strict_caches() { return jf::g_tw.clear() + jf::g_spec.clear(); }

}  // namespace jw
