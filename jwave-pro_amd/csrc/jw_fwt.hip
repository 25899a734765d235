// jw_fwt.hip -- Fast Wavelet Transform (filter-bank cascade), 1-D and 2-D, for gfx950.
//
// Reference semantics (src/main/java/jwave/):
//   transforms/wavelets/Wavelet.java:236-260  forward(arr, h): for i < h/2
//       out[i]     = sum_j arr[(2i+j) wrap h] * sD[j]      (j ascending, from +0.0)
//       out[i+h/2] = sum_j arr[(2i+j) wrap h] * wD[j]
//   transforms/wavelets/Wavelet.java:277-303  reverse(arr, h): a SCATTER, i outer, j inner
//       out[(2i+j) wrap h] += (arr[i]*sR[j]) + (arr[i+h/2]*wR[j])
//   haar/Haar1Orthogonal.java:175-207 reverse: out[k] += 0.5 * ((a*sR) + (d*wR))
//   transforms/FastWaveletTransform.java:71-153  the cascade over h = n, n/2, ... (forward)
//       and h = tw << (log2 n - level) ... n (reverse)
//   transforms/BasicTransform.java:361-474  2-D: rows (lvlN) then columns (lvlM); reverse
//       columns then rows.
//
// The reverse scatter is evaluated here as a gather that adds, for each output k, exactly
// the contributions the Java loop adds to out[k], in the Java loop's order (i ascending,
// then j): bit-identical in JW_ARITH_STRICT.  Derivation: for h >= M every (i,j) wraps at
// most once, the j with 2i+j == k (i = (k-j)/2) come first in descending j, then the
// wrapped ones (2i+j == k+h) in descending j.  For h < M (multi-wrap) the Java loop is
// replayed per output.
#include "jw_internal.hpp"

namespace jw {
namespace {

constexpr int kNT = 256;
constexpr int kLdsN = 4096;              // signals up to this length run one workgroup each
constexpr int kPer = kLdsN / kNT;        // outputs per thread per level (max)

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

// Wavelet.forward output pair (i, i + h/2) from in[0..h).
template <bool FMA>
__device__ __forceinline__ void fwd_pair(const double* in, int h, int i, int M, const Filters& f,
                                         double& lo, double& hi) {
  lo = 0.;
  hi = 0.;
  for (int j = 0; j < M; ++j) {
    int k = (i << 1) + j;
    while (k >= h) k -= h;
    const double x = in[k];
    lo = madd<FMA>(lo, f.sD[j], x);
    hi = madd<FMA>(hi, f.wD[j], x);
  }
}

// Wavelet.reverse output k from in[0..h) (gather in the scatter's order).
template <bool FMA>
__device__ __forceinline__ double rev_out(const double* in, int h, int k, int M, int kind,
                                          const Filters& f) {
  const int half = h >> 1;
  double acc = 0.;
  if (h >= M) {
    const int p = k & 1;
    int jn = k < M - 1 ? k : M - 1;
    if ((jn & 1) != p) --jn;
    for (int j = jn; j >= p; j -= 2) {
      const int i = (k - j) >> 1;
      acc += contrib<FMA>(in[i], in[i + half], f.sR[j], f.wR[j], kind);
    }
    int jw = M - 1;
    if ((jw & 1) != p) --jw;
    for (int j = jw; j > k; j -= 2) {
      const int i = (k + h - j) >> 1;
      acc += contrib<FMA>(in[i], in[i + half], f.sR[j], f.wR[j], kind);
    }
  } else {
    for (int i = 0; i < half; ++i)
      for (int j = 0; j < M; ++j) {
        int kk = (i << 1) + j;
        while (kk >= h) kk -= h;
        if (kk == k) acc += contrib<FMA>(in[i], in[i + half], f.sR[j], f.wR[j], kind);
      }
  }
  return acc;
}

// One workgroup per signal, whole cascade in LDS (n <= kLdsN).
template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_fwd_lds(const double* __restrict__ x,
                                                   double* __restrict__ y, int n, int level,
                                                   int M, int tw, Filters f) {
  __shared__ double buf[kLdsN];
  const int tid = threadIdx.x;
  const double* xs = x + (long)blockIdx.x * n;
  double* ys = y + (long)blockIdx.x * n;
  for (int i = tid; i < n; i += kNT) buf[i] = xs[i];
  __syncthreads();
  int l = 0;
  for (int h = n; h >= tw && l < level; h >>= 1, ++l) {
    const int half = h >> 1;
    double lo[kPer / 2], hi[kPer / 2];
#pragma unroll
    for (int r = 0; r < kPer / 2; ++r) {
      const int i = tid + r * kNT;
      if (i < half) fwd_pair<FMA>(buf, h, i, M, f, lo[r], hi[r]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPer / 2; ++r) {
      const int i = tid + r * kNT;
      if (i < half) {
        buf[i] = lo[r];
        buf[i + half] = hi[r];
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += kNT) ys[i] = buf[i];
}

template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_rev_lds(const double* __restrict__ y,
                                                   double* __restrict__ x, int n, int h0, int M,
                                                   int tw, int kind, Filters f) {
  __shared__ double buf[kLdsN];
  const int tid = threadIdx.x;
  const double* ys = y + (long)blockIdx.x * n;
  double* xs = x + (long)blockIdx.x * n;
  for (int i = tid; i < n; i += kNT) buf[i] = ys[i];
  __syncthreads();
  for (int h = h0; h <= n && h >= tw; h <<= 1) {
    double o[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int k = tid + r * kNT;
      if (k < h) o[r] = rev_out<FMA>(buf, h, k, M, kind, f);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int k = tid + r * kNT;
      if (k < h) buf[k] = o[r];
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += kNT) xs[i] = buf[i];
}

// One level on global memory (long signals): out[0..h) of every signal from in[0..h).
template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_fwd_level(const double* __restrict__ in,
                                                     double* __restrict__ out, long stride, int h,
                                                     int M, Filters f) {
  const int i = blockIdx.x * kNT + threadIdx.x;
  if (i >= (h >> 1)) return;
  const double* src = in + (long)blockIdx.y * stride;
  double* dst = out + (long)blockIdx.y * stride;
  double lo, hi;
  fwd_pair<FMA>(src, h, i, M, f, lo, hi);
  dst[i] = lo;
  dst[i + (h >> 1)] = hi;
}

template <bool FMA>
__global__ __launch_bounds__(kNT) void fwt_rev_level(const double* __restrict__ in,
                                                     double* __restrict__ out, long stride, int h,
                                                     int M, int kind, Filters f) {
  const int k = blockIdx.x * kNT + threadIdx.x;
  if (k >= h) return;
  out[(long)blockIdx.y * stride + k] = rev_out<FMA>(in + (long)blockIdx.y * stride, h, k, M, kind, f);
}

// Tiled out-of-place transpose of `batch` rows x cols matrices (the 2-D column pass runs as
// transpose -> row cascade -> transpose).
__global__ __launch_bounds__(kNT) void transpose_kernel(const double* __restrict__ in,
                                                        double* __restrict__ out, int rows,
                                                        int cols) {
  __shared__ double tile[32][33];
  const long mat = (long)blockIdx.z * rows * cols;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int rr = r0 + r, cc = c0 + tx;
    if (rr < rows && cc < cols) tile[r][tx] = in[mat + (long)rr * cols + cc];
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int cc = c0 + r, rr = r0 + tx;
    if (cc < cols && rr < rows) out[mat + (long)cc * rows + rr] = tile[tx][r];
  }
}

Filters make_filters(const FwtPlan& p) {
  Filters f{};
  for (int i = 0; i < p.M; ++i) {
    f.sD[i] = p.sD[i];
    f.wD[i] = p.wD[i];
    f.sR[i] = p.sR[i];
    f.wR[i] = p.wR[i];
  }
  return f;
}

int log2_exact(long n) {
  int e = 0;
  while ((1L << e) < n) ++e;
  return e;
}

template <bool FMA>
int forward_t(const FwtPlan& p, const double* x, double* y, long n, int level, long batch,
              hipStream_t s) {
  const Filters f = make_filters(p);
  if (n <= kLdsN) {
    for (long b0 = 0; b0 < batch; b0 += 1L << 30) {
      const long nb = batch - b0 < (1L << 30) ? batch - b0 : (1L << 30);
      hipLaunchKernelGGL(fwt_fwd_lds<FMA>, dim3((unsigned)nb), dim3(kNT), 0, s, x + b0 * n,
                         y + b0 * n, (int)n, level, p.M, p.tw, f);
    }
    JW_HIP_TRY(hipGetLastError());
    return JW_OK;
  }
  double* tmp = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&tmp, sizeof(double) * (size_t)(n * batch), s));
  if (y != x) JW_HIP_TRY(hipMemcpyAsync(y, x, sizeof(double) * n * batch, hipMemcpyDeviceToDevice, s));
  int l = 0;
  for (long h = n; h >= p.tw && l < level; h >>= 1, ++l) {
    for (long b0 = 0; b0 < batch; b0 += 65535) {
      const long nb = batch - b0 < 65535 ? batch - b0 : 65535;
      dim3 grid((unsigned)(((h >> 1) + kNT - 1) / kNT), (unsigned)nb);
      hipLaunchKernelGGL(fwt_fwd_level<FMA>, grid, dim3(kNT), 0, s, y + b0 * n, tmp + b0 * n, n,
                         (int)h, p.M, f);
    }
    JW_HIP_TRY(hipMemcpy2DAsync(y, sizeof(double) * n, tmp, sizeof(double) * n,
                                sizeof(double) * h, batch, hipMemcpyDeviceToDevice, s));
  }
  JW_HIP_TRY(hipGetLastError());
  JW_HIP_TRY(hipFreeAsync(tmp, s));
  return JW_OK;
}

template <bool FMA>
int reverse_t(const FwtPlan& p, const double* y, double* x, long n, int level, long batch,
              hipStream_t s) {
  const Filters f = make_filters(p);
  long h0 = p.tw;
  const int steps = log2_exact(n);
  for (int l = level; l < steps; ++l) h0 <<= 1;  // FastWaveletTransform.java:137-141
  if (n <= kLdsN) {
    for (long b0 = 0; b0 < batch; b0 += 1L << 30) {
      const long nb = batch - b0 < (1L << 30) ? batch - b0 : (1L << 30);
      hipLaunchKernelGGL(fwt_rev_lds<FMA>, dim3((unsigned)nb), dim3(kNT), 0, s, y + b0 * n,
                         x + b0 * n, (int)n, (int)h0, p.M, p.tw, p.kind, f);
    }
    JW_HIP_TRY(hipGetLastError());
    return JW_OK;
  }
  double* tmp = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&tmp, sizeof(double) * (size_t)(n * batch), s));
  if (x != y) JW_HIP_TRY(hipMemcpyAsync(x, y, sizeof(double) * n * batch, hipMemcpyDeviceToDevice, s));
  for (long h = h0; h <= n && h >= p.tw; h <<= 1) {
    for (long b0 = 0; b0 < batch; b0 += 65535) {
      const long nb = batch - b0 < 65535 ? batch - b0 : 65535;
      dim3 grid((unsigned)((h + kNT - 1) / kNT), (unsigned)nb);
      hipLaunchKernelGGL(fwt_rev_level<FMA>, grid, dim3(kNT), 0, s, x + b0 * n, tmp + b0 * n, n,
                         (int)h, p.M, p.kind, f);
    }
    JW_HIP_TRY(hipMemcpy2DAsync(x, sizeof(double) * n, tmp, sizeof(double) * n,
                                sizeof(double) * h, batch, hipMemcpyDeviceToDevice, s));
  }
  JW_HIP_TRY(hipGetLastError());
  JW_HIP_TRY(hipFreeAsync(tmp, s));
  return JW_OK;
}

int transpose(const double* in, double* out, int rows, int cols, int batch, hipStream_t s) {
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32), (unsigned)batch);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(kNT), 0, s, in, out, rows, cols);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace

int fwt_forward_device(const FwtPlan& p, const double* x, double* y, long n, int level, int batch,
                       hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? forward_t<true>(p, x, y, n, level, batch, s)
                                 : forward_t<false>(p, x, y, n, level, batch, s);
}

int fwt_reverse_device(const FwtPlan& p, const double* y, double* x, long n, int level, int batch,
                       hipStream_t s) {
  return p.arith == JW_ARITH_FMA ? reverse_t<true>(p, y, x, n, level, batch, s)
                                 : reverse_t<false>(p, y, x, n, level, batch, s);
}

// 2-D (BasicTransform.java:361-399): every row with lvlN, then every column with lvlM.
int fwt2d_forward_device(const FwtPlan& p, const double* x, double* y, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  const size_t elems = (size_t)rows * cols * batch;
  double* t = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&t, sizeof(double) * elems, s));
  int st = fwt_forward_device(p, x, y, cols, lvlN, rows * batch, s);
  if (st == JW_OK) st = transpose(y, t, rows, cols, batch, s);
  if (st == JW_OK) st = fwt_forward_device(p, t, t, rows, lvlM, cols * batch, s);
  if (st == JW_OK) st = transpose(t, y, cols, rows, batch, s);
  JW_HIP_TRY(hipFreeAsync(t, s));
  return st;
}

// 2-D reverse (BasicTransform.java:436-474): every column with lvlM, then every row with lvlN.
int fwt2d_reverse_device(const FwtPlan& p, const double* y, double* x, int rows, int cols,
                         int lvlM, int lvlN, int batch, hipStream_t s) {
  const size_t elems = (size_t)rows * cols * batch;
  double* t = nullptr;
  JW_HIP_TRY(hipMallocAsync((void**)&t, sizeof(double) * elems, s));
  int st = transpose(y, t, rows, cols, batch, s);
  if (st == JW_OK) st = fwt_reverse_device(p, t, t, rows, lvlM, cols * batch, s);
  if (st == JW_OK) st = transpose(t, x, cols, rows, batch, s);
  if (st == JW_OK) st = fwt_reverse_device(p, x, x, cols, lvlN, rows * batch, s);
  JW_HIP_TRY(hipFreeAsync(t, s));
  return st;
}

}  // namespace jw
