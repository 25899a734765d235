// jw_fft_passes.hpp -- the two FFT pass kernels and the four-step driver, shared by the
// CWT (jw_cwt.hip) and MODWT FFT-convolution (jw_modwt_fft.hip) paths.  See jw_fft.hpp.
#pragma once
#include <algorithm>
#include <type_traits>

#include "jw_fft.hpp"

namespace jw {
namespace fft {

typedef double nt2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void nt_store(cplx* p, cplx v) {
  nt2 w = {v.x, v.y};
  __builtin_nontemporal_store(w, (nt2*)p);
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

// Output staging slot of (output index n, line c): 8 lines per n, the line XOR-swizzled by
// bits 3..5 of n.  A 16-byte element e sits on banks 4 (e mod 16) .. +3, so both sides are
// bank-conflict free: the transposed write (8-lane groups: n = q + 8 k1 + 64 k2, k1 = lane & 7,
// c fixed -> c ^ k1 distinct) and the coalescing read (16-lane groups: n = 8 w + (lane >> 3),
// c = lane & 7 -> 8 (n & 1) + (c ^ w) distinct).  The padded [n][9] layout it replaces put 4
// lanes of every write group on one bank group (SQ_LDS_BANK_CONFLICT = 62 % of LDS cycles).
__device__ __forceinline__ int out_slot(int n, int c) { return 8 * n + (c ^ ((n >> 3) & 7)); }

constexpr int kTileD = kT * fft::kXbuf;  // doubles: the split passes' tile (36.9 KB)
static_assert(kTileD >= kT * 512, "split tile must hold the 8-line staging");

template <int S, bool TWID, class Out>
__device__ __forceinline__ void pass512_tail(cplx (&a)[8], const Out& out, long N, long N2,
                                             const Tables& T, long item, long line0, cplx* tile);

// An output functor with its item fixed before a line's stores.  A functor whose item -> row
// mapping reads memory (CoefOut's scale map) provides bind(item): the lookup then happens once,
// not after every store (the compiler cannot hoist a load past stores that may alias it, and on
// gfx9 the wait for that load also drains every store issued before it).
template <class Out>
struct BoundOut {
  const Out& out;
  long item;
  __device__ void operator()(long idx, long line, cplx v) const { out(item, idx, line, v); }
};
template <class Out>
__device__ __forceinline__ auto bind_out(const Out& out, long item) {
  if constexpr (requires { out.bind(item); }) {
    return out.bind(item);
  } else {
    return BoundOut<Out>{out, item};
  }
}

// The four-step twiddle W_N^(S n1 col) of pass 1 on wave c's outputs n1 = q + 8 k1 + 64 k2.
__device__ __forceinline__ void twiddle_cols(cplx (&a)[8], int S, long N, const Tables& T,
                                             long col, int q, int k1) {
  // one table lookup per lane, then the wave-uniform step W_N^(64 col) applied k2 times
  // (7 products: ~1e-15 relative)
  cplx w = fft::twiddle(T, ((long)(q + 8 * k1) * col) & (N - 1));
  const cplx step = fft::twiddle(T, (64 * col) & (N - 1));
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    a[k2] = S < 0 ? fft::cmul_tw<-1>(a[k2], w) : fft::cmul_tw<1>(a[k2], w);
    if (k2 < 7) w = fft::cmul(w, step);
  }
}

// pass512_tail with the re/im-split buffers (tile: kTileD doubles): same values, same output
// order, half the LDS.
template <int S, bool TWID, class Out>
__device__ __forceinline__ void pass512_tail_split(cplx (&a)[8], const Out& out, long N, long N2,
                                                   const Tables& T, long item, long line0,
                                                   double* tile) {
  const int tid = threadIdx.x, lane = tid & 63, c = tid >> 6;
  fft::fft512_wave_split<S>(a, tile + c * fft::kXbuf, T.w512, lane);
  const int q = lane >> 3, k1 = lane & 7;
  if (TWID && N2 > 1) twiddle_cols(a, S, N, T, line0 + c, q, k1);
  double re[8];
  __syncthreads();
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) tile[out_slot(q + 8 * k1 + 64 * k2, c)] = a[k2].x;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) re[i] = tile[out_slot((tid >> 3) + 64 * i, tid & 7)];
  __syncthreads();
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) tile[out_slot(q + 8 * k1 + 64 * k2, c)] = a[k2].y;
  __syncthreads();
  const auto o = bind_out(out, item);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = (tid >> 3) + 64 * i, cc = tid & 7;
    o(n, line0 + cc, make_double2(re[i], tile[out_slot(n, cc)]));
  }
}

template <int S, bool IN_TILE, bool TWID, class In, class Out>
__device__ __forceinline__ void pass512_body_split(const In& in, const Out& out, long N, long N2,
                                                   const Tables& T, long item, long line0,
                                                   double* tile) {
  const int tid = threadIdx.x, lane = tid & 63, c = tid >> 6;
  cplx a[8];
  if (IN_TILE) {
    // tile[k1][c] <- in(k1, line0 + c): 8 consecutive columns per row, coalesced
    cplx v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = in(item, (tid >> 3) + 64 * i, line0 + (tid & 7));
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[((tid >> 3) + 64 * i) * (kT + 1) + (tid & 7)] = v[i].x;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r].x = tile[(lane + 64 * r) * (kT + 1) + c];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[((tid >> 3) + 64 * i) * (kT + 1) + (tid & 7)] = v[i].y;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r].y = tile[(lane + 64 * r) * (kT + 1) + c];
    __syncthreads();
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r] = in(item, lane + 64 * r, line0 + c);
  }
  pass512_tail_split<S, TWID>(a, out, N, N2, T, item, line0, tile);
}

// IN_TILE: the line's inputs are strided (pass 1 over a natural-order array): stage 8 lines
// through the tile.  TWID: apply the four-step twiddle W_N^(S n1 col) (pass 1).
template <int S, bool IN_TILE, bool TWID, class In, class Out>
__device__ __forceinline__ void pass512_body(const In& in, const Out& out, long N, long N2,
                                             const Tables& T, long item, long line0, cplx* tile) {
  const int tid = threadIdx.x, lane = tid & 63, c = tid >> 6;
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
  pass512_tail<S, TWID>(a, out, N, N2, T, item, line0, tile);
}

// The rest of a 512-line pass once wave c holds line line0 + c as a[r] = x[lane + 64 r]: the
// wavefront FFT, the four-step twiddle (TWID), and the 8-line output staged through the tile
// (the tile must be free: callers barrier after their last read of it).
template <int S, bool TWID, class Out>
__device__ __forceinline__ void pass512_tail(cplx (&a)[8], const Out& out, long N, long N2,
                                             const Tables& T, long item, long line0, cplx* tile) {
  const int tid = threadIdx.x, lane = tid & 63, c = tid >> 6;
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
  for (int k2 = 0; k2 < 8; ++k2) tile[out_slot(q + 8 * k1 + 64 * k2, c)] = a[k2];
  __syncthreads();
  const auto o = bind_out(out, item);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = (tid >> 3) + 64 * i, cc = tid & 7;
    o(n, line0 + cc, tile[out_slot(n, cc)]);
  }
}

template <int S, bool IN_TILE, bool TWID, class In, class Out>
__global__ __launch_bounds__(512) void pass512(In in, Out out, long N, long N2, Tables T) {
  __shared__ double tile[kTileD];
  pass512_body_split<S, IN_TILE, TWID>(in, out, N, N2, T, blockIdx.y, (long)blockIdx.x * kT, tile);
}

// Two independent 512-line passes in one grid, for software pipelining of a batch of
// four-step transforms: role 0 = pass 2 (rows) of group g, role 1 = pass 1 (columns) of
// group g+1, each on its own workspace.  Pass 2 is HBM-bound and pass 1 mostly on-chip
// (spectra from L2, psi_hat arithmetic), so interleaving their blocks on every CU overlaps
// the two.  Blocks alternate roles while both have work left (so both spread over all CUs).
struct TwoRoles {
  long nb0, nb1;        // blocks of each role
  long lines0, lines1;  // lines per item / kT (blocks per item)
  __device__ void pick(long b, int& role, long& item, long& line0) const {
    const long m = nb0 < nb1 ? nb0 : nb1;
    long idx;
    if (b < 2 * m) {
      role = (int)(b & 1);
      idx = b >> 1;
    } else {
      role = nb0 > nb1 ? 0 : 1;
      idx = m + (b - 2 * m);
    }
    const long per = role == 0 ? lines0 : lines1;
    item = idx / per;
    line0 = (idx - item * per) * kT;
  }
};
template <int S, class In0, class Out0, bool IT1, class In1, class Out1>
__global__ __launch_bounds__(512) void pass512_two(In0 in0, Out0 out0, In1 in1, Out1 out1, long N,
                                                   long N2, TwoRoles R, Tables T) {
  __shared__ double tile[kTileD];
  int role;
  long item, line0;
  R.pick(blockIdx.x, role, item, line0);
  if (role == 0) {
    pass512_body_split<S, false, false>(in0, out0, N, N2, T, item, line0, tile);
  } else {
    pass512_body_split<S, IT1, true>(in1, out1, N, N2, T, item, line0, tile);
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
// Long-line pass: one line of M = 512 R points (R = 2, 4, 8) per workgroup of R waves, the
// line contiguous in memory on both sides.  Decimation in time over R: wave w takes the
// subsequence x[R j + w] (j < 512) through fft512_wave, twiddles it by W_M^(w k), and the
// workgroup finishes with R-point DFTs across the waves:
//   X[k + 512 m] = sum_w W_R^(w m) (W_M^(w k) Y_w[k]),   k < 512, m < R.
// The line is staged through LDS on the way in (coalesced global reads; the padded layout
// makes the stride-R gathers bank-conflict free) and between the two stages.  TWID: times the
// four-step twiddle W_N^(n line) of output n (pass 1).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int pad16(int j) { return j + (j >> 4); }
__device__ __forceinline__ int pad8(int k) { return k + (k >> 3); }

template <int S, int R>
__device__ __forceinline__ void dftR(cplx (&v)[R]) {  // v[m] <- sum_w v[w] e^{S 2 pi i w m / R}
  if constexpr (R == 2) {
    const cplx a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  } else if constexpr (R == 4) {
    const cplx t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    const cplx t2 = cadd(v[1], v[3]), d = csub(v[1], v[3]);
    const cplx t3 = make_double2(-S * d.y, S * d.x);  // d * e^{S i pi / 2}
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, t3);
    v[3] = csub(t1, t3);
  } else {
    static_assert(R == 8, "R = 2, 4 or 8");
    dft8<S>(v);
  }
}

template <int R>
constexpr int big_lds() {  // complex entries: the padded line, or the R exchange buffers
  return R * kXbuf > 512 * R + 32 * R ? R * kXbuf : 512 * R + 32 * R;
}

template <int S, int R, bool TWID, class In, class Out>
__global__ __launch_bounds__(64 * R) void passbig(In in, Out out, long N, Tables T) {
  constexpr int M = 512 * R, NT = 64 * R;
  __shared__ cplx buf[big_lds<R>()];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long item = blockIdx.y, line = blockIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int j = tid + NT * i;
    buf[pad16(j)] = in(item, j, line);
  }
  __syncthreads();
  cplx a[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) a[r] = buf[pad16(R * (lane + 64 * r) + w)];
  __syncthreads();  // buf becomes the waves' exchange buffers
  fft512_wave<S>(a, buf + w * kXbuf, T.w512, lane);  // a[k2] = Y_w[q + 8 k1 + 64 k2]
  const int q = lane >> 3, k1 = lane & 7;
  const long step = N / M;  // W_M^x = W_N^(x N / M)
  if (w > 0) {
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const long k = q + 8 * k1 + 64 * k2;
      a[k2] = cmul_tw<S>(a[k2], twiddle(T, w * k * step));
    }
  }
  __syncthreads();
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) buf[w * kXbuf + pad8(q + 8 * k1 + 64 * k2)] = a[k2];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8 / R; ++i) {
    const int k = tid + NT * i;
    cplx v[R];
#pragma unroll
    for (int ww = 0; ww < R; ++ww) v[ww] = buf[ww * kXbuf + pad8(k)];
    dftR<S, R>(v);
#pragma unroll
    for (int m = 0; m < R; ++m) {
      const long n = k + 512 * m;
      cplx o = v[m];
      if (TWID) o = cmul_tw<S>(o, twiddle(T, (n * line) & (N - 1)));
      out(item, n, line, o);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Shared functors
// ---------------------------------------------------------------------------------------
// Spectra are stored "column-major" for the inverse's four-step: element k at
// (k mod N2) * N1 + k / N2, so each pass-1 column is contiguous.
__device__ __forceinline__ long tpos(long k, long N1, long N2) { return (k % N2) * N1 + k / N2; }
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
struct ColOutT {  // column-major workspace: A[item][col * N1 + n1] (long pass 1)
  cplx* A;
  long N, N1;
  __device__ void operator()(long item, long n1, long col, cplx v) const {
    A[item * N + col * N1 + n1] = v;
  }
};
struct RowInT {  // row n1 of a column-major workspace: A[item][k2 * N1 + n1] (strided)
  const cplx* A;
  long N, N1;
  __device__ cplx operator()(long item, long k2, long n1) const {
    return A[item * N + k2 * N1 + n1];
  }
};
// X[item][k], k = n1 + Nf * n2 (the forward FFT's output index, Nf its pass-1 length), stored
// at its column-major position for the inverse's split (N1 x N2): contiguous pass-1 columns.
struct SpecOut {
  cplx* X;
  long N, Nf, N1, N2;
  long item0;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    X[(item0 + item) * N + tpos(line + Nf * idx, N1, N2)] = v;
  }
};
struct SpecOutBoth {  // SpecOut, and the same spectrum in natural order: Xn[item][k]
  SpecOut a;
  cplx* Xn;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    a(item, idx, line, v);
    Xn[(a.item0 + item) * a.N + line + a.Nf * idx] = v;
  }
};
struct SpecOut1 {  // single pass: X[item][idx]
  cplx* X;
  long N, item0;
  __device__ void operator()(long item, long idx, long, cplx v) const {
    X[(item0 + item) * N + idx] = v;
  }
};

// run_fft: one full FFT (S = -1 forward, +1 reverse without the 1/N) of `items` lines of
// length N.  in(item, k1, col) supplies element k = N2 k1 + col; out_single receives the
// result when N <= 4096 (one pass); otherwise pass 1 writes A and out_final receives
// (item, n2, n1, v) for output index n1 + N1 n2.
// One full FFT (forward or reverse) of `items` lines of length N: in(item, k) -> out.
// Lengths 2^19 .. 2^21 split as 512 x M (M = 1024 .. 4096): the 512-point side runs pass512 (8
// strided lines per workgroup), the long side passbig (one contiguous line per workgroup).
// Which side goes first depends on the input: a natural-order (strided) input is read by
// pass512 (N1 = 512, workspace row-major, pass 2 long rows); a column-major input (the
// spectra, contiguous columns) by passbig (N1 = M, workspace column-major, pass 2 = pass512
// over strided rows, so the natural-order output is written in 8-line pieces).
inline bool long_split(long N) { return N >= (1L << 19) && N <= (1L << 21); }

template <int S, class In1, class Out2>
int run_fft_long(long N, long items, In1 in1, Out2 out_final, cplx* A, hipStream_t s,
                 const Tables& T, bool a_nt) {
  const long M = N / 512;
  const int R = (int)(M / 512);
  auto big = [&](auto rc, auto twid, auto in, auto out, long lines) {
    constexpr int RR = decltype(rc)::value;
    constexpr bool TW = decltype(twid)::value;
    hipLaunchKernelGGL((passbig<S, RR, TW, decltype(in), decltype(out)>),
                       dim3((unsigned)lines, (unsigned)items), dim3(64 * RR), 0, s, in, out, N, T);
  };
  auto big_r = [&](auto twid, auto in, auto out, long lines) {
    if (R == 2) big(std::integral_constant<int, 2>{}, twid, in, out, lines);
    else if (R == 4) big(std::integral_constant<int, 4>{}, twid, in, out, lines);
    else big(std::integral_constant<int, 8>{}, twid, in, out, lines);
  };
  if constexpr (In1::kStrided) {  // N1 = 512, N2 = M
    hipLaunchKernelGGL((pass512<S, true, true, In1, ColOut>), dim3((unsigned)(M / kT), (unsigned)items),
                       dim3(512), 0, s, in1, ColOut{A, N, M, a_nt}, N, M, T);
    JW_HIP_TRY(hipGetLastError());
    big_r(std::false_type{}, RowIn{A, N, M}, out_final, 512L);
  } else {  // N1 = M, N2 = 512
    big_r(std::true_type{}, in1, ColOutT{A, N, M}, 512L);
    JW_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL((pass512<S, true, false, RowInT, Out2>), dim3((unsigned)(M / kT), (unsigned)items),
                       dim3(512), 0, s, RowInT{A, N, M}, out_final, N, 512L, T);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

// Three passes (N = 2^27, 2^28): pass 1 runs 8192-point columns as usual; the rows of N2 =
// N / 8192 > 8192 points (too long for one workgroup's LDS) are then FFTs of their own, run as a
// two-pass four-step (run_fft again, N2 = N1' x N2') over the items x 8192 rows, through a
// second workspace B of the same size as A.
constexpr int kMaxLog1 = 13;  // the longest pass-1 line: 8192 points in 128 KB of LDS
// The four-step split used for length N: N1 = N (one pass) for N <= 4096, else
// N1 = 2^min(ceil(log2 N / 2), 13), N2 = N / N1 (run_fft with long_ok = false).
inline long split_n1(long N) {
  if (N <= 4096) return N;
  int logN = 0;
  while ((1L << logN) < N) ++logN;
  return 1L << std::min((logN + 1) / 2, kMaxLog1);
}
struct NestIn {  // row n1 of pass 1's workspace A as a line of N2 points, element N2i k1 + col
  static constexpr bool kStrided = false;
  const cplx* A;
  long N, N1, N2, N2i;
  __device__ cplx operator()(long item, long k1, long col) const {
    const long it = item / N1, n1 = item - it * N1;
    return A[it * N + n1 * N2 + N2i * k1 + col];
  }
};
template <class Out>
struct NestOut {  // the row FFT's output m = line + N1i idx is the outer n2 of row n1
  Out out;
  long N1, N1i, it0;
  __device__ void operator()(long item, long idx, long line, cplx v) const {
    const long it = item / N1, n1 = item - it * N1;
    out(it0 + it, line + N1i * idx, n1, v);
  }
};

template <int S, class In1, class Out1, class Out2, bool NEST = true>
int run_fft(long N, long items, In1 in1, Out1 out_single, Out2 out_final, cplx* A, hipStream_t s,
            const Tables& T, bool a_nt, bool long_ok = true, cplx* B = nullptr) {
  int logN = 0;
  while ((1L << logN) < N) ++logN;
  if (long_ok && long_split(N)) return run_fft_long<S>(N, items, in1, out_final, A, s, T, a_nt);
  if (N <= 4096) {  // one pass, N2 = 1
    hipLaunchKernelGGL((pass_generic<S, true, In1, Out1>), dim3(1, (unsigned)items), dim3(256),
                       (size_t)N * sizeof(cplx), s, in1, out_single, N, 1L, logN, T);
    JW_HIP_TRY(hipGetLastError());
    return JW_OK;
  }
  const int log1 = std::min((logN + 1) / 2, kMaxLog1), log2 = logN - log1;
  const long N1 = 1L << log1, N2 = 1L << log2;
  if (N2 > 8192 && (!B || N2 > (1L << 26)))
    return fail(JW_ERR_UNSUPPORTED, "FFT length %ld: three passes need a second workspace", N);
  // lines of 8192 points (N = 2^25, 2^26) stage 128 KB of LDS: past the 64 KB default
  auto lds_ok = [](auto kern, long M) -> hipError_t {
    const size_t b = (size_t)M * sizeof(cplx);
    return b > 65536 ? hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)b)
                     : hipSuccess;
  };
  ColOut a_out{A, N, N2, a_nt};
  RowIn a_in{A, N, N2};
  if (N1 == 512) {
    hipLaunchKernelGGL((pass512<S, In1::kStrided, true, In1, ColOut>),
                       dim3((unsigned)(N2 / kT), (unsigned)items), dim3(512), 0, s, in1, a_out, N,
                       N2, T);
  } else {
    JW_HIP_TRY(lds_ok(pass_generic<S, true, In1, ColOut>, N1));
    hipLaunchKernelGGL((pass_generic<S, true, In1, ColOut>), dim3((unsigned)N2, (unsigned)items),
                       dim3(256), (size_t)N1 * sizeof(cplx), s, in1, a_out, N, N2, log1, T);
  }
  JW_HIP_TRY(hipGetLastError());
  if constexpr (NEST) {
    if (N2 > 8192) {
    Tables T2;
    if (int st = tables(N2, &T2); st != JW_OK) return st;
    const long chunk = std::max(1L, 65535 / N1);  // inner items (rows) on grid.y <= 65535
    const long N1i = split_n1(N2);
    for (long it0 = 0; it0 < items; it0 += chunk) {
      const long nit = std::min(chunk, items - it0);
      const NestIn nin{A + it0 * N, N, N1, N2, N2 / N1i};
      const NestOut<Out2> nout{out_final, N1, N1i, it0};
      if (int st = run_fft<S, NestIn, NestOut<Out2>, NestOut<Out2>, false>(
              N2, nit * N1, nin, nout, nout, B, s, T2, a_nt, false);
          st != JW_OK)
        return st;
    }
    return JW_OK;
    }
  }
  if (N2 == 512) {
    hipLaunchKernelGGL((pass512<S, false, false, RowIn, Out2>),
                       dim3((unsigned)(N1 / kT), (unsigned)items), dim3(512), 0, s, a_in, out_final,
                       N, N2, T);
  } else {
    JW_HIP_TRY(lds_ok(pass_generic<S, false, RowIn, Out2>, N2));
    hipLaunchKernelGGL((pass_generic<S, false, RowIn, Out2>), dim3((unsigned)N1, (unsigned)items),
                       dim3(256), (size_t)N2 * sizeof(cplx), s, a_in, out_final, N, N2, log2, T);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

// A batch of `items` four-step FFTs of N = 512 x 512 points, in groups of `gsize` items,
// software-pipelined: one launch runs pass 2 of group g (workspace A[g % 2]) beside pass 1
// of group g+1 (workspace A[(g+1) % 2]).  mk_in(p0) / mk_out(p0) build the input / final
// output functors of the group whose first item is p0 (item indices inside a group are
// relative to p0, as in run_fft).
template <int S, class MkIn, class MkOut>
int run_fft512_pipelined(long N, long items, long gsize, MkIn mk_in, MkOut mk_out, cplx* A0,
                         cplx* A1, hipStream_t s, const Tables& T, bool a_nt) {
  constexpr long N1 = 512, N2 = 512;
  if (N != N1 * N2) return fail(JW_ERR_UNSUPPORTED, "pipelined FFT needs N = 2^18");
  using In1 = decltype(mk_in(0L));
  using Out2 = decltype(mk_out(0L));
  cplx* A[2] = {A0, A1};
  const long G = (items + gsize - 1) / gsize;
  auto cnt = [&](long g) { return items - g * gsize < gsize ? items - g * gsize : gsize; };
  hipLaunchKernelGGL((pass512<S, In1::kStrided, true, In1, ColOut>),
                     dim3((unsigned)(N2 / kT), (unsigned)cnt(0)), dim3(512), 0, s, mk_in(0L),
                     ColOut{A[0], N, N2, a_nt}, N, N2, T);
  JW_HIP_TRY(hipGetLastError());
  for (long g = 1; g <= G; ++g) {
    const RowIn rin{A[(g - 1) & 1], N, N2};
    if (g == G) {
      hipLaunchKernelGGL((pass512<S, false, false, RowIn, Out2>),
                         dim3((unsigned)(N1 / kT), (unsigned)cnt(g - 1)), dim3(512), 0, s, rin,
                         mk_out((g - 1) * gsize), N, N2, T);
    } else {
      const TwoRoles R{(N1 / kT) * cnt(g - 1), (N2 / kT) * cnt(g), N1 / kT, N2 / kT};
      hipLaunchKernelGGL((pass512_two<S, RowIn, Out2, In1::kStrided, In1, ColOut>),
                         dim3((unsigned)(R.nb0 + R.nb1)), dim3(512), 0, s, rin,
                         mk_out((g - 1) * gsize), mk_in(g * gsize), ColOut{A[g & 1], N, N2, a_nt},
                         N, N2, R, T);
    }
    JW_HIP_TRY(hipGetLastError());
  }
  return JW_OK;
}

// The split run_fft takes for an input functor of the given kind (run_fft_long).
inline long split_n1(long N, bool strided) {
  if (long_split(N)) return strided ? 512 : N / 512;
  return split_n1(N);
}

}  // namespace fft
}  // namespace jw
