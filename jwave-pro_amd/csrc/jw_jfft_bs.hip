// jw_jfft_bs.hip -- JW_ARITH_STRICT FFT paths for lengths that are not powers of two: the
// reference's Bluestein transform (FastFourierTransform.fftBluestein, :259-324) operation for
// operation, and MODWTTransform's FFT convolution on it (:752-837) -- so MODWT at n = 100, 288,
// 1000, 70001 (MODWTInverseTest.java:75-91) matches the JVM bit for bit, like the
// power-of-two lengths in jw_jfft.hip.
//
//   m = smallest power of two >= 2n - 1;  chirp[i] = (cos t, sin t), t = Math.PI * i * i / n * (+-1)
//   a[i] = x[i].mul(chirp[i]) (i < n, else 0);  b[0] = conj chirp[0], b[i] = b[m - i] = conj chirp[i]
//   a = FFT_m(a); b = FFT_m(b) (no 1/m);  a[i] = a[i].mul(b[i]);  a = IFFT_m(a) (no 1/m)
//   a[i] = a[i].mul(1.0 / m);  result[i] = a[i].mul(chirp[i]) (.mul(1.0 / n) for the inverse)
// chirp and FFT_m(b) depend on (n, direction) only: built once (host cos / sin in the
// reference's expression, the m-point transform on the device) and cached.
#include <cmath>
#include <cstdlib>
#include <thread>
#include <tuple>
#include <vector>

#include "jw_jfft_host.hpp"

namespace jw {
namespace jf {
namespace {

constexpr double kJavaPi = 3.141592653589793;  // Math.PI

long bs_m(long n) {
  long m = 1;
  while (m < 2 * n - 1) m <<= 1;  // :261-265
  return m;
}

// [chirp (n) | B = FFT_m(b) (m)] per (device, n, inverse).  Its own budget holds the longest
// one (n = 2^29: 24 GiB), so repeated long transforms keep their tables: rebuilding means one
// correctly rounded sin/cos per index on the host (~3 s for n = 3 x 2^25 on 16 threads) -- a
// table is still kept only while it fits a quarter of the free device memory (cached_table).
using BsKey = std::tuple<int, long, int>;
DevCache<BsKey> g_bst(26UL << 30);

struct BsTab {
  long n = 0, m = 0;
  const cplx* chirp = nullptr;
  const cplx* B = nullptr;
};

int bs_tables(long n, bool inverse, BsTab* out, StreamAllocs& mem, hipStream_t s) {
  int dev = 0;
  JW_HIP_TRY(hipGetDevice(&dev));
  const long m = bs_m(n);
  const void* p = nullptr;
  const int st = cached_table(
      g_bst, BsKey(dev, n, inverse ? 1 : 0), (size_t)(n + m) * sizeof(cplx), mem, s, &p,
      [&](void* d) -> int {
        cplx* chirp = static_cast<cplx*>(std::malloc((size_t)n * sizeof(cplx)));
        cplx* b = static_cast<cplx*>(std::calloc((size_t)m, sizeof(cplx)));
        if (!chirp || !b) {
          std::free(chirp);
          std::free(b);
          return fail(JW_ERR_NO_MEMORY, "Bluestein tables: n = %ld, m = %ld", n, m);
        }
        // :268-272, one angle per index: ~0.5 us each past 2^20 (the correctly rounded
        // sin / cos of arguments up to pi n), so long chirps are split over host threads
        auto fill = [&](long lo, long hi) {
          for (long i = lo; i < hi; ++i) {
            const double angle = kJavaPi * (double)i * (double)i / (double)n * (inverse ? 1 : -1);
            double c, sn;  // Math.cos / Math.sin, correctly rounded (jw_crmath.cc)
            cr_sincos(angle, &sn, &c);
            chirp[i] = make_double2(c, sn);
          }
        };
        const int nt = n >= (1L << 16) ? host_threads() : 1;
        std::vector<std::thread> pool;
        try {  // slices whose thread cannot be started run here: nothing throws across the C-ABI
          pool.reserve(nt);
          for (int t = 1; t < nt; ++t) pool.emplace_back(fill, n * t / nt, n * (t + 1) / nt);
        } catch (...) {
        }
        fill(0, n / nt);
        for (int t = (int)pool.size() + 1; t < nt; ++t) fill(n * t / nt, n * (t + 1) / nt);
        for (auto& th : pool) th.join();
        b[0] = make_double2(chirp[0].x, -chirp[0].y);  // :285-290, conjugate() = (r, -j)
        for (long i = 1; i < n; ++i) {
          b[i] = make_double2(chirp[i].x, -chirp[i].y);
          b[m - i] = make_double2(chirp[i].x, -chirp[i].y);
        }
        cplx* dev_b = nullptr;
        hipError_t e = mem.alloc(&dev_b, (size_t)m * sizeof(cplx));
        if (e != hipSuccess) {
          std::free(chirp);
          std::free(b);
          JW_HIP_TRY(e);
        }
        JW_HIP_TRY(upload_owned(d, chirp, (size_t)n * sizeof(cplx), s));
        JW_HIP_TRY(upload_owned(dev_b, b, (size_t)m * sizeof(cplx), s));
        // fftCooleyTukeyInternal(b, false) (:294)
        return fft_rows(m, false, 1, RowsC{dev_b, m}, OutCS{(cplx*)d + n, m, 1.0, 0}, mem, s);
      });
  if (st != JW_OK) return st;
  out->n = n;
  out->m = m;
  out->chirp = (const cplx*)p;
  out->B = (const cplx*)p + n;
  return JW_OK;
}

// ---- functors (item it = it0 + the launch's item index) ----
// x[i] of a transform, then a[i] = x[i].mul(chirp[i]) for i < n, 0 past n (:280-283)
struct Pre {
  enum Mode { kReal = 0, kCplx = 1, kProd = 2 };
  int mode = kReal;
  long it0 = 0;
  const double* r0 = nullptr;  // kReal: rows it < nb from r0, the others from r1
  long rs0 = 0;
  const double* r1 = nullptr;
  long rs1 = 0;
  long nb = 1L << 62;
  const cplx* c = nullptr;  // kCplx: rows; kProd: spectra rows (row it % cmod)
  long cst = 0, cmod = 1L << 62;
  const cplx* F0 = nullptr;  // kProd: x = c[row].mul(F) with F = F0 (it < nb) or F1,
  const cplx* F1 = nullptr;  //        conjugated for the adjoint (:820-824)
  int conj = 0;
  const cplx* chirp = nullptr;
  long n = 0;
  __device__ cplx operator()(long item, long i) const {
    if (i >= n) return make_double2(0.0, 0.0);
    const long it = item + it0;
    cplx x;
    if (mode == kReal) {
      x = make_double2(it < nb ? r0[it * rs0 + i] : r1[(it - nb) * rs1 + i], 0.0);
    } else if (mode == kCplx) {
      x = c[it * cst + i];
    } else {
      cplx f = (it < nb ? F0 : F1)[i];
      if (conj) f.y = -f.y;
      x = jmul(c[(it % cmod) * cst + i], f);  // signalFFT[i].mul(filterFFT[i]) (:775-778)
    }
    return jmul(x, chirp[i]);
  }
};

// result[i] = a[i].mul(1.0 / m).mul(chirp[i]) (.mul(1.0 / n) when inverse) (:304-321), i < n,
// stored as a complex row (kCplx) or its real part (kRe: rows it < nb to r0, the others to r1;
// getReal(), MODWTTransform.java:781-783)
struct Post {
  enum Mode { kCplx = 0, kRe = 1 };
  int mode = kCplx;
  long it0 = 0;
  cplx* c = nullptr;
  long cst = 0;
  double* r0 = nullptr;
  long rs0 = 0;
  double* r1 = nullptr;
  long rs1 = 0;
  long nb = 1L << 62;
  const cplx* chirp = nullptr;
  long n = 0;
  double inv_m = 1.0, inv_n = 1.0;
  int inverse = 0;
  __device__ void operator()(long item, long i, cplx v) const {
    if (i >= n) return;
    const long it = item + it0;
    cplx r = jmul(jscale(v, inv_m), chirp[i]);
    if (inverse) r = jscale(r, inv_n);
    if (mode == kCplx) {
      c[it * cst + i] = r;
    } else if (it < nb) {
      r0[it * rs0 + i] = r.x;
    } else {
      r1[(it - nb) * rs1 + i] = r.x;
    }
  }
};

struct BMid {  // a[i].mul(b[i]) (:300-302)
  const cplx* B;
  __device__ cplx operator()(int, long, long i, cplx x) const { return jmul(x, B[i]); }
};

// A three-pass transform's output (pass 3) times B: a[i].mul(b[i]) (:300-302)
struct OutMulB {
  cplx* p;
  long st;
  const cplx* B;
  __device__ void operator()(long it, long i, cplx v) const { p[it * st + i] = jmul(v, B[i]); }
};

// The convolution of fftBluestein with three-pass m-point transforms (m >= three_pass_min(),
// up to 2^30): FFT_m(a) = passes 1..3 (the last one multiplying by B), IFFT_m of the product =
// passes 1..3 into Post.  Same operations in the same order as the two-pass chain below.
int bs_conv3(long m, long items, const Pre& pre, const Post& post, const cplx* B,
             StreamAllocs& mem, hipStream_t s) {
  Tw3 twf, twi;
  int st = twiddles3(m, false, &twf, mem, s);
  if (st == JW_OK) st = twiddles3(m, true, &twi, mem, s);
  if (st != JW_OK) return st;
  const int abits = ilog2(twf.A), cbits = ilog2(twf.C);
  const long ab = (long)twf.A * twf.B;
  const long chunk = std::max(1L, std::min<long>(items, (2L << 30) / (2 * m * (long)sizeof(cplx))));
  cplx *Z = nullptr, *Zi = nullptr;
  JW_HIP_TRY(mem.alloc(&Z, (size_t)chunk * m * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&Zi, (size_t)chunk * m * sizeof(cplx)));
  // the passes of fft_rows3, unfused, so with the plain transforms' column geometry (PlainGeo)
  auto three = [&](auto in, auto out, const Tw3& tw, cplx* work, long ni) -> int {
    int r = with_big_lc(tw.A, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value, E = kPlainEPT<LC>;
      return launch_grid<LC, E>(kp1<LC, decltype(in), OutC, E>, (m / tw.A / Geo<LC, E>::T) * ni,
                                s, in, OutC{work, m}, ilog2(m / tw.A), ni, tw.p1);
    });
    if (r == JW_OK)
      r = with_big_lc(tw.B, [&](auto LCc) -> int {
        constexpr int LC = decltype(LCc)::value, E = kPlainEPT<LC>;
        const Plane pl{work, m, ab, cbits};
        return launch_grid<LC, E>(kp2s<LC, Plane, Plane, E>, (tw.A / Geo<LC, E>::T) * ni * tw.C,
                                  s, pl, pl, abits, ni * tw.C, tw.pm);
      });
    if (r == JW_OK)
      r = with_big_lc(tw.C, [&](auto LCc) -> int {
        constexpr int LC = decltype(LCc)::value, E = kPlainEPT<LC>;
        return launch_grid<LC, E>(kp2s<LC, RowsC, decltype(out), E>, (ab / Geo<LC, E>::T) * ni, s,
                                  RowsC{work, m}, out, ilog2(ab), ni, tw.p3);
      });
    return r;
  };
  for (long i0 = 0; i0 < items && st == JW_OK; i0 += chunk) {
    const long ni = std::min(chunk, items - i0);
    Pre pc = pre;
    pc.it0 += i0;
    Post qc = post;
    qc.it0 += i0;
    st = three(pc, OutMulB{Zi, m, B}, twf, Z, ni);            // FFT_m(a), times B (:293-302)
    if (st == JW_OK) st = three(RowsC{Zi, m}, qc, twi, Z, ni);  // IFFT_m, post (:303-321)
  }
  return st;
}

// `items` Bluestein transforms of length n: pre supplies x (before the chirp), post receives
// the results (both get the tables filled in here).  Workspaces are this call's own
// (stream-ordered: released after the kernels queued here have used them).
int bs_rows(long n, bool inverse, long items, Pre pre, Post post, StreamAllocs& /*caller*/,
            hipStream_t s) {
  StreamAllocs mem(s);
  BsTab T;
  int st = bs_tables(n, inverse, &T, mem, s);
  if (st != JW_OK) return st;
  const long m = T.m;
  pre.chirp = post.chirp = T.chirp;
  pre.n = post.n = n;
  post.inv_m = 1.0 / (double)m;
  post.inv_n = 1.0 / (double)n;
  post.inverse = inverse ? 1 : 0;
  if (m > kLineMax && m >= three_pass_min()) return bs_conv3(m, items, pre, post, T.B, mem, s);
  const int lc1 = split_lc1(m);
  Tw twf, twi;
  if ((st = twiddles(m, false, lc1, &twf, mem, s)) != JW_OK) return st;
  if (m <= kLineMax) {
    if ((st = twiddles(m, true, (int)m, &twi, mem, s)) != JW_OK) return st;
    return with_lc(m, [&](auto LCc) -> int {
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC, kLineEPT<LC>>(kline_conv<LC, Pre, Post>,
                                           (items + LineGeo<LC>::T - 1) / LineGeo<LC>::T, s,
                             pre, post, items, T.B, twf.p1, twi.p1);
    });
  }
  const long R = lc1, C = m / lc1;  // forward m = R x C, inverse C x R (jw_jfft.hpp)
  if ((st = twiddles(m, true, (int)C, &twi, mem, s)) != JW_OK) return st;
  const long chunk = std::max(1L, std::min<long>(items, (2L << 30) / (2 * m * (long)sizeof(cplx))));
  cplx *Z = nullptr, *Zi = nullptr;
  JW_HIP_TRY(mem.alloc(&Z, (size_t)chunk * m * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&Zi, (size_t)chunk * m * sizeof(cplx)));
  for (long i0 = 0; i0 < items && st == JW_OK; i0 += chunk) {
    const long ni = std::min(chunk, items - i0);
    Pre pc = pre;
    pc.it0 += i0;
    Post qc = post;
    qc.it0 += i0;
    st = with_big_lc(R, [&](auto LCc) -> int {  // FFT_m(a) pass 1 (:293)
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC>(kp1<LC, Pre, OutC>, (C / Geo<LC>::T) * ni, s, pc, OutC{Z, m},
                             ilog2(C), ni, twf.p1);
    });
    if (st != JW_OK) break;
    st = with_big_lc(C, [&](auto LCc) -> int {  // pass 2, times B, IFFT_m pass 1 (:295-303)
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC>(kp2p<LC, 1, RowsC, BMid, OutF>, (R / Geo<LC>::T) * ni, s,
                             RowsC{Z, m}, BMid{T.B}, OutF{Zi, m, 0}, ilog2(R), ni, twf.p2, twi.p1);
    });
    if (st != JW_OK) break;
    st = with_big_lc(R, [&](auto LCc) -> int {  // IFFT_m pass 2, then the post-processing
      constexpr int LC = decltype(LCc)::value;
      return launch_grid<LC>(kp2s<LC, RowsC, Post>, (C / Geo<LC>::T) * ni, s, RowsC{Zi, m}, qc,
                             ilog2(C), ni, twi.p2);
    });
  }
  return st;
}

__global__ void add_rows(const double* __restrict__ a, const double* __restrict__ d,
                         double* __restrict__ out, long n, long nb, long os) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * nb) return;
  const long it = i / n, k = i - it * n;
  out[it * os + k] = a[i] + d[i];  // vFromApprox[i] + vFromDetail[i] (:366-369)
}

}  // namespace

// natural-order spectra of `items` real rows of length n (not a power of two)
int bs_spectra_real(long n, long items, const double* rows, cplx* out, StreamAllocs& mem,
                    hipStream_t s) {
  Pre pre;
  pre.mode = Pre::kReal;
  pre.r0 = rows;
  pre.rs0 = n;
  Post post;
  post.mode = Post::kCplx;
  post.c = out;
  post.cst = n;
  return bs_rows(n, false, items, pre, post, mem, s);
}

// jw_fft_* (JW_ARITH_STRICT) for lengths that are not powers of two
int bs_fft_strict(bool inverse, const cplx* in, cplx* out, long n, long batch, hipStream_t s) {
  StreamAllocs mem(s);
  // in == out: every transform reads all of its input before its last pass writes
  Pre pre;
  pre.mode = Pre::kCplx;
  pre.c = in;
  pre.cst = n;
  Post post;
  post.mode = Post::kCplx;
  post.c = out;
  post.cst = n;
  return bs_rows(n, inverse, batch, pre, post, mem, s);
}

// MODWT levels for lengths that are not powers of two: DIRECT levels on the direct kernels,
// FFT levels as circularConvolveFFT{,Adjoint} on Bluestein transforms.  F: filter spectra
// [j - 1][h, g] (jw_jfft.hip).
int modwt_strict_bs(bool inverse, const ModwtPlan& p, const double* in, double* out, long N,
                    int J, int batch, const bool* fft, const cplx* F, StreamAllocs& mem,
                    hipStream_t s) {
  const long rs = (long)(J + 1) * N;
  const long m = bs_m(N);
  // per signal: 2 spectra + 2 real rows (A, D) + 2 scratch V rows; the Bluestein workspaces
  // are bounded separately (bs_rows chunks them)
  const long per_sig = 2 * N * (long)sizeof(cplx) + 4 * N * (long)sizeof(double) +
                       4 * m * (long)sizeof(cplx);
  const long chunk = std::max(1L, std::min<long>(batch, (2L << 30) / per_sig));
  cplx* S = nullptr;
  double* tmp = nullptr;
  JW_HIP_TRY(mem.alloc(&S, (size_t)2 * chunk * N * sizeof(cplx)));
  JW_HIP_TRY(mem.alloc(&tmp, (size_t)4 * chunk * N * sizeof(double)));
  int st = JW_OK;
  for (long b0 = 0; b0 < batch && st == JW_OK; b0 += chunk) {
    const long nb = std::min(chunk, batch - b0);
    double* vt[2] = {tmp, tmp + chunk * N};  // ping-pong V rows
    double* AD = tmp + 2 * chunk * N;        // [A rows | D rows]
    if (!inverse) {
      const double* x = in + b0 * N;
      double* c = out + b0 * rs;
      const double* vin = x;
      long vs = N;
      for (int j = 1; j <= J && st == JW_OK; ++j) {
        double* w = c + (long)(j - 1) * N;
        double* vout = j == J ? c + (long)J * N : vt[j & 1];
        const long vos = j == J ? rs : N;
        if (!fft[j]) {
          st = modwt_level_forward_device(p, j, vin, vs, w, rs, vout, vos, N, (int)nb, s);
        } else {
          Pre a;  // X = fft.forward(V_{j-1}) (:770)
          a.mode = Pre::kReal;
          a.r0 = vin;
          a.rs0 = vs;
          Post xa;
          xa.mode = Post::kCplx;
          xa.c = S;
          xa.cst = N;
          st = bs_rows(N, false, nb, a, xa, mem, s);
          if (st != JW_OK) break;
          Pre b;  // fft.reverse(X . FFT(h_j)) -> W_j, fft.reverse(X . FFT(g_j)) -> V_j
          b.mode = Pre::kProd;
          b.c = S;
          b.cst = N;
          b.cmod = nb;
          b.F0 = F + (long)(2 * (j - 1)) * N;
          b.F1 = F + (long)(2 * (j - 1) + 1) * N;
          b.nb = nb;
          Post o;
          o.mode = Post::kRe;
          o.r0 = w;
          o.rs0 = rs;
          o.r1 = vout;
          o.rs1 = vos;
          o.nb = nb;
          st = bs_rows(N, true, 2 * nb, b, o, mem, s);
        }
        vin = vout;
        vs = vos;
      }
    } else {
      const double* c = in + b0 * rs;
      double* x = out + b0 * N;
      const double* vin = c + (long)J * N;
      long vs = rs;
      for (int j = J; j >= 1 && st == JW_OK; --j) {
        const double* w = c + (long)(j - 1) * N;
        double* vout = j == 1 ? x : vt[j & 1];
        if (!fft[j]) {
          st = modwt_level_inverse_device(p, j, vin, vs, w, rs, vout, N, N, (int)nb, s);
        } else {
          Pre a;  // fft.forward(V_j), fft.forward(W_j) (:815-816)
          a.mode = Pre::kReal;
          a.r0 = vin;
          a.rs0 = vs;
          a.r1 = w;
          a.rs1 = rs;
          a.nb = nb;
          Post sa;
          sa.mode = Post::kCplx;
          sa.c = S;
          sa.cst = N;
          st = bs_rows(N, false, 2 * nb, a, sa, mem, s);
          if (st != JW_OK) break;
          Pre b;  // reverse(S_V . conj FFT(g_j)) -> A, reverse(S_W . conj FFT(h_j)) -> D
          b.mode = Pre::kProd;
          b.c = S;
          b.cst = N;
          b.F0 = F + (long)(2 * (j - 1) + 1) * N;
          b.F1 = F + (long)(2 * (j - 1)) * N;
          b.nb = nb;
          b.conj = 1;
          Post o;
          o.mode = Post::kRe;
          o.r0 = AD;
          o.rs0 = N;
          o.r1 = AD + nb * N;
          o.rs1 = N;
          o.nb = nb;
          st = bs_rows(N, true, 2 * nb, b, o, mem, s);
          if (st != JW_OK) break;
          hipLaunchKernelGGL(add_rows, dim3((unsigned)((N * nb + 255) / 256)), dim3(256), 0, s,
                             AD, AD + nb * N, vout, N, nb, N);
          JW_HIP_TRY(hipGetLastError());
        }
        vin = vout;
        vs = N;
      }
    }
  }
  return st;
}

}  // namespace jf
}  // namespace jw
