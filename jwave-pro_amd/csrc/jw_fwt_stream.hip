// jw_fwt_stream.hip -- one-pass column kernels of the 2-D FWT for tall matrices (4096 rows:
// four column levels streamed, the rest in the LDS tail of jw_fwt.hip).  See DESIGN.md §5.3.
#include <cstdlib>
#include <utility>

#include "jw_fwt_common.hpp"

namespace jw {
namespace fwtc {
namespace {

// ---------------------------------------------------------------------------------------
// Streaming column forward: levels 1..S of 64 columns per wavefront in ONE pass over HBM
// (the strip kernels above take one pass per level).  Lane l owns column c0 + l and walks it
// top to bottom; every row read is a 512-byte coalesced piece.  Level k keeps its last 16
// inputs in registers (a ring indexed by stream position mod 16); output pair i of level k is
// produced as soon as input 2i + M - 1 arrives, its detail goes straight to its final row
// h_k/2 + i, its approximation feeds level k+1 (level S: row i, the tail's input).
// Circularity without saving anything: the level-1 stream simply runs past the bottom of the
// column (row p mod rows) for E = sum of the levels' look-ahead (210 rows for M = 16, S = 4),
// so every level sees its first inputs again at the end and computes its wrapped outputs
// then; the few outputs computed twice are written twice with identical values.
// Reads T (the row pass's output), writes y: the column cannot be updated in place (detail
// row h/2 + i is written long before row h/2 + i is read).  Same sums, same order as
// Wavelet.forward per column (bit-identical in STRICT).
// Every ring slot is a compile-time register: positions advance by known amounts per
// macro-step of 2^S rows, and 2^(S-1) macro-steps are unrolled per loop trip.
// ---------------------------------------------------------------------------------------
constexpr int kStreamRing = 16;  // taps per level kept in registers (filters up to 16 taps)

struct StreamCtx {
  double* dst;   // y + matrix + column
  long cols;
  long p0;       // level-1 stream position of the current loop trip (multiple of 2^(2S-1))
  int rows;
};

constexpr int smod(int q) { return ((q % kStreamRing) + kStreamRing) % kStreamRing; }

template <bool FMA, int M, int S, int K, int Q>
__device__ __forceinline__ void stream_feed(double (&ring)[S][kStreamRing], double v,
                                            const StreamCtx& c, const Filters& f) {
  // level K input at stream position (p0 >> (K-1)) + Q
  ring[K - 1][smod(Q)] = v;
  if constexpr ((Q & 1) != 0 && (Q - M + 1) % 2 == 0) {
    constexpr int O = (Q - M + 1) / 2;  // output pair (p0 >> K) + O is complete
    double lo = 0., hi = 0.;
#pragma unroll
    for (int t = 0; t < M; ++t) {
      const double x = ring[K - 1][smod(2 * O + t)];
      lo = madd<FMA>(lo, f.sD[t], x);
      hi = madd<FMA>(hi, f.wD[t], x);
    }
    const long i = (c.p0 >> K) + O;
    const int hk = c.rows >> (K - 1), halfk = hk >> 1;
    if (i >= 0) c.dst[(long)(halfk + (i & (halfk - 1))) * c.cols] = hi;
    if constexpr (K < S) {
      stream_feed<FMA, M, S, K + 1, O>(ring, lo, c, f);
    } else {
      if (i >= 0) c.dst[(long)(i & (halfk - 1)) * c.cols] = lo;
    }
  }
}

template <bool FMA, int M, int S, int U0, int... Js>
__device__ __forceinline__ void stream_macro(double (&ring)[S][kStreamRing],
                                             const double (&in)[1 << S], const StreamCtx& c,
                                             const Filters& f, std::integer_sequence<int, Js...>) {
  (stream_feed<FMA, M, S, 1, U0 * (1 << S) + Js>(ring, in[Js], c, f), ...);
}

template <bool FMA, int M, int S, int... Us>
__device__ __forceinline__ void stream_trip(double (&ring)[S][kStreamRing], double (&in)[1 << S],
                                            const double* src, long cols, int rows, StreamCtx& c,
                                            const Filters& f, std::integer_sequence<int, Us...>) {
  constexpr int MS = 1 << S;
  auto one = [&](auto uc) {
    constexpr int U = decltype(uc)::value;
    double nx[MS];  // the next macro-step's rows, in flight behind this one
    const long nb = c.p0 + (long)(U + 1) * MS;
#pragma unroll
    for (int j = 0; j < MS; ++j) nx[j] = src[((nb + j) & (rows - 1)) * cols];
    stream_macro<FMA, M, S, U>(ring, in, c, f, std::make_integer_sequence<int, MS>{});
#pragma unroll
    for (int j = 0; j < MS; ++j) in[j] = nx[j];
    // one macro-step of loads in flight: the scheduler may not hoist later steps' loads
    // (they would all be live at once and double the registers)
    __builtin_amdgcn_sched_barrier(0);
  };
  (one(std::integral_constant<int, Us>{}), ...);
}

// 8 macro-steps per trip: the trip start p0 is then a multiple of 2^(S+3), so every level's
// stream position (p0 >> (K-1)) is a multiple of the ring size.
constexpr int kStreamUnroll = 8;

template <bool FMA, int M, int S>
__global__ __launch_bounds__(64) void fwt_cols_stream_fwd(const double* __restrict__ T,
                                                          double* __restrict__ y, int rows,
                                                          int cols, long mstride, long trips,
                                                          Filters f) {
  static_assert(M <= kStreamRing && M % 2 == 0, "streamed filters: even, <= 16 taps");
  constexpr int MS = 1 << S, UN = kStreamUnroll;
  const long col = (long)blockIdx.x * 64 + threadIdx.x;
  const double* src = T + (long)blockIdx.y * mstride + col;
  StreamCtx c{y + (long)blockIdx.y * mstride + col, (long)cols, 0L, rows};
  double ring[S][kStreamRing];
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int q = 0; q < kStreamRing; ++q) ring[k][q] = 0.;
  double in[MS];
#pragma unroll
  for (int j = 0; j < MS; ++j) in[j] = src[(long)(j & (rows - 1)) * cols];
  for (long t = 0; t < trips; ++t) {
    stream_trip<FMA, M, S>(ring, in, src, (long)cols, rows, c, f,
                           std::make_integer_sequence<int, UN>{});
    c.p0 += (long)UN * MS;
  }
}

// ---------------------------------------------------------------------------------------
// Streaming column reverse: levels S..1 of 64 columns per wavefront in ONE pass (the strip
// kernels take one pass per level).  Level k (1 = finest, h_k = rows >> (k-1)) turns its
// approximations a_k (h_k/2: from the tail's output for k = S, else from level k+1) and
// details d_k (rows [h_k/2, h_k) of y) into h_k outputs; the output pair (2u, 2u+1) gathers
// a_k[u - t], d_k[u - t], t < M/2, in Wavelet.reverse's scatter order (strip_rev above).
// Per macro-step m, level k handles pairs [c_k m, c_k (m+1)), c_k = 2^(S-k), depth first
// from the coarsest pair, so each level's inputs are ready when it runs; its last M/2
// approximations and details sit in registers (ring slot = index mod 8).  Circularity: the
// first pairs of a level look back past index 0 to the end of the level (a_k[h_k/2 - 1] ...),
// so the stream starts 16 macro-steps early (m = -16) -- the coarser levels' pre-roll produces
// exactly those wrapped values (computed again at the end of the stream); finest-level
// outputs with u < 0 are not stored.  (A CPU model of this schedule checked it against the
// level-by-level gather for M = 2, 4, 16 before the kernel was written.)
// The pairs u < M/2 - 1 add their taps in the wrapped order; they all fall in the trip that
// starts at m = 0, which is compiled separately with every pair index static.
// ---------------------------------------------------------------------------------------
constexpr int kRevRing = 8;  // approximations / details kept per level (M/2 <= 8)
// Macro-steps run before m = 0.  Level S reads its inputs from memory and is valid once its
// ring is full (pair u >= 7 - Q); each finer level needs 7 more of its coarser neighbour's
// outputs, so the finest level is valid from u >= 105 - 8Q (S = 4, M = 16): Q = 16 (two
// trips) covers every u >= 0 with room to spare.
constexpr int kRevPreroll = 16;
constexpr int rmod(int q) { return ((q % kRevRing) + kRevRing) % kRevRing; }

struct RevCtx {
  double* T;     // output column
  long cols;
  long m0;       // macro-step of the current trip's first macro-step (multiple of 8)
};

// Level K, pair with static part J (absolute u = c_K m0 + J), inputs already in the rings.
template <bool FMA, int M, int KIND, int S, int K, int J, bool FIRST>
__device__ __forceinline__ void rev_pair(double (&ra)[S][kRevRing], double (&rd)[S][kRevRing],
                                         const RevCtx& c, const Filters& f, double& o0,
                                         double& o1) {
  constexpr int T2 = M / 2, CK = 1 << (S - K);
  double e0 = 0., e1 = 0.;
  auto tap = [&](auto tc) {
    constexpr int t = decltype(tc)::value;
    const double a = ra[K - 1][rmod(J - t)], d = rd[K - 1][rmod(J - t)];
    e0 = rev_acc<FMA, KIND>(e0, a, d, f.sR[2 * t], f.wR[2 * t]);
    e1 = rev_acc<FMA, KIND>(e1, a, d, f.sR[2 * t + 1], f.wR[2 * t + 1]);
  };
  // u = J in the trip starting at m = 0: taps that wrap (u < M/2 - 1) come in the scatter's
  // order t = u .. 0, then M/2 - 1 .. u + 1
  constexpr bool kWrapped = FIRST && J >= 0 && J < T2 - 1;
  [&]<int... Ts>(std::integer_sequence<int, Ts...>) {
    if constexpr (kWrapped) {
      constexpr int st0 = kWrapped ? J : T2 - 1;
      (tap(std::integral_constant<int, (st0 - Ts >= 0 ? st0 - Ts : st0 - Ts + T2)>{}), ...);
    } else {
      (tap(std::integral_constant<int, T2 - 1 - Ts>{}), ...);
    }
  }(std::make_integer_sequence<int, T2>{});
  o0 = e0;  // a_{K-1}[2u], a_{K-1}[2u + 1]: rev_node writes each just before its finer pair
  o1 = e1;
  if constexpr (K == 1) {
    const long u = (long)CK * c.m0 + J;
    if (u >= 0) {
      c.T[(2 * u) * c.cols] = e0;
      c.T[(2 * u + 1) * c.cols] = e1;
    }
  }
}

// One level-K pair (local index JJ of macro-step MM; in[0] = a_S, in[c_K + JJ] = d_K), then,
// depth first, the two finer pairs its approximations complete: every ring entry is consumed
// right after it is written, so 8 entries (the 7 of look-back + the new one) suffice.
template <bool FMA, int M, int KIND, int S, int K, int MM, int JJ, bool FIRST>
__device__ __forceinline__ void rev_node(double (&ra)[S][kRevRing], double (&rd)[S][kRevRing],
                                         const double (&in)[1 << S], const RevCtx& c,
                                         const Filters& f) {
  constexpr int CK = 1 << (S - K), J = CK * MM + JJ;
  rd[K - 1][rmod(J)] = in[CK + JJ];
  if constexpr (K == S) ra[S - 1][rmod(J)] = in[0];
  double e0, e1;
  rev_pair<FMA, M, KIND, S, K, J, FIRST>(ra, rd, c, f, e0, e1);
  if constexpr (K > 1) {
    // a_{K-1}[2J] overwrites a_{K-1}[2J - 8], which pair 2J no longer needs; a_{K-1}[2J + 1]
    // must wait until pair 2J has read a_{K-1}[2J - 7] from the same slot
    ra[K - 2][rmod(2 * J)] = e0;
    rev_node<FMA, M, KIND, S, K - 1, MM, 2 * JJ, FIRST>(ra, rd, in, c, f);
    ra[K - 2][rmod(2 * J + 1)] = e1;
    rev_node<FMA, M, KIND, S, K - 1, MM, 2 * JJ + 1, FIRST>(ra, rd, in, c, f);
  }
}

template <bool FMA, int M, int KIND, int S, bool FIRST>
__device__ __forceinline__ void rev_trip(double (&ra)[S][kRevRing], double (&rd)[S][kRevRing],
                                         double (&in)[1 << S], const double* A, const double* y,
                                         long cols, int rows, RevCtx& c, const Filters& f) {
  constexpr int NL = 1 << S;
  auto load = [&](double (&dst)[NL], long m) {
    const long hs2 = (long)(rows >> (S - 1)) >> 1;  // a_S length
    dst[0] = A[(m & (hs2 - 1)) * cols];
#pragma unroll
    for (int idx = 1; idx < NL; ++idx) {
      const int lg = 31 - __builtin_clz(idx), ck = 1 << lg, k = S - lg;  // d_k, pair idx - ck
      const long half = (long)(rows >> (k - 1)) >> 1;
      dst[idx] = y[(half + ((ck * m + idx - ck) & (half - 1))) * cols];
    }
  };
  [&]<int... MMs>(std::integer_sequence<int, MMs...>) {
    auto one = [&](auto mc) {
      constexpr int MM = decltype(mc)::value;
      double nx[NL];
      load(nx, c.m0 + MM + 1);  // the next macro-step's rows, in flight behind this one
      rev_node<FMA, M, KIND, S, S, MM, 0, FIRST>(ra, rd, in, c, f);
#pragma unroll
      for (int j = 0; j < NL; ++j) in[j] = nx[j];
      __builtin_amdgcn_sched_barrier(0);  // as in stream_trip
    };
    (one(std::integral_constant<int, MMs>{}), ...);
  }(std::make_integer_sequence<int, kStreamUnroll>{});
}

template <bool FMA, int M, int KIND, int S>
__global__ __launch_bounds__(64) void fwt_cols_stream_rev(const double* __restrict__ A, long ms_a,
                                                          const double* __restrict__ y,
                                                          double* __restrict__ T, int rows,
                                                          int cols, long mat, long trips,
                                                          Filters f) {
  static_assert(M % 2 == 0 && M / 2 <= kRevRing, "streamed filters: even, <= 16 taps");
  constexpr int NL = 1 << S;
  const long col = (long)blockIdx.x * 64 + threadIdx.x;
  const double* a = A + (long)blockIdx.y * ms_a + col;
  const double* ys = y + (long)blockIdx.y * mat + col;
  RevCtx c{T + (long)blockIdx.y * mat + col, (long)cols, -(long)kRevPreroll};
  double ra[S][kRevRing], rd[S][kRevRing];
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int q = 0; q < kRevRing; ++q) ra[k][q] = rd[k][q] = 0.;
  double in[NL];
  {
    const long m = c.m0;
    const long hs2 = (long)(rows >> (S - 1)) >> 1;
    in[0] = a[(m & (hs2 - 1)) * cols];
#pragma unroll
    for (int idx = 1; idx < NL; ++idx) {
      const int lg = 31 - __builtin_clz(idx), ck = 1 << lg, k = S - lg;
      const long half = (long)(rows >> (k - 1)) >> 1;
      in[idx] = ys[(half + ((ck * m + idx - ck) & (half - 1))) * cols];
    }
  }
  // the pre-roll trips (m = -16 .. -1); then m = 0 .. 7, the wrapped pairs (peeled, so its
  // static-order code never shares a loop body with the steady state's)
  constexpr int kPre = kRevPreroll / kStreamUnroll;
  for (int t = 0; t < kPre; ++t) {
    rev_trip<FMA, M, KIND, S, false>(ra, rd, in, a, ys, (long)cols, rows, c, f);
    c.m0 += kStreamUnroll;
  }
  rev_trip<FMA, M, KIND, S, true>(ra, rd, in, a, ys, (long)cols, rows, c, f);
  c.m0 += kStreamUnroll;
  for (long t = kPre + 1; t < trips; ++t) {
    rev_trip<FMA, M, KIND, S, false>(ra, rd, in, a, ys, (long)cols, rows, c, f);
    c.m0 += kStreamUnroll;
  }
}

}  // namespace

// Streaming forward column pass (S = 4 levels, filters of up to 16 taps): T -> y.
template <bool FMA>
bool launch_stream_fwd(int M, int S, hipStream_t s, const double* T, double* y, int rows,
                       int cols, long mat, int batch, const Filters& f) {
  const char* e = knob("JW_FWT_STREAM");
  if ((e && e[0] == '0') || S != 4 || M > kStreamRing || M % 2 || cols % 64) return false;
  const long E = ((1L << S) - 1) * (M - 2);           // look-ahead of the S levels, in rows
  const long trip = (long)kStreamUnroll << S;         // rows per loop trip
  const long trips = (rows + E + trip - 1) / trip;
  const dim3 g((unsigned)(cols / 64), (unsigned)batch), b(64);
  switch (M) {
#define JW_C(MM)                                                                            \
  case MM:                                                                                  \
    hipLaunchKernelGGL((fwt_cols_stream_fwd<FMA, MM, 4>), g, b, 0, s, T, y, rows, cols, mat, \
                       trips, f);                                                           \
    return true;
    JW_C(2) JW_C(4) JW_C(8) JW_C(16)
#undef JW_C
    default:
      return false;
  }
}

// Streaming reverse column pass (S = 4 levels): A (the tail's output, rows [0, rows >> S)) and
// the details of y -> T rows [0, rows).
template <bool FMA>
bool launch_stream_rev(int M, int kind, int S, hipStream_t s, const double* A, long ms_a,
                       const double* y, double* T, int rows, int cols, long mat, int batch,
                       const Filters& f) {
  const char* e = knob("JW_FWT_STREAM");
  if ((e && e[0] == '0') || S != 4 || M > 2 * kRevRing || M % 2 || cols % 64) return false;
  if (!(M == 2 || M == 4 || M == 8 || M == 16) || (kind == JW_WAVELET_HAAR_ORTH && M != 2))
    return false;
  const long steps = (long)rows / (2L << (S - 1)) + kRevPreroll;  // from m = -16
  if (steps % kStreamUnroll) return false;
  if (A == nullptr) return true;  // dry run: would the streaming pass run?
  const long trips = steps / kStreamUnroll;
  const dim3 g((unsigned)(cols / 64), (unsigned)batch), b(64);
  if (kind == JW_WAVELET_HAAR_ORTH) {
    if (M != 2) return false;
    hipLaunchKernelGGL((fwt_cols_stream_rev<FMA, 2, JW_WAVELET_HAAR_ORTH, 4>), g, b, 0, s, A, ms_a,
                       y, T, rows, cols, mat, trips, f);
    return true;
  }
  switch (M) {
#define JW_C(MM)                                                                               \
  case MM:                                                                                     \
    hipLaunchKernelGGL((fwt_cols_stream_rev<FMA, MM, JW_WAVELET_GENERIC, 4>), g, b, 0, s, A,   \
                       ms_a, y, T, rows, cols, mat, trips, f);                                 \
    return true;
    JW_C(2) JW_C(4) JW_C(8) JW_C(16)
#undef JW_C
    default:
      return false;
  }
}

template bool launch_stream_fwd<true>(int, int, hipStream_t, const double*, double*, int, int, long,
                                      int, const Filters&);
template bool launch_stream_fwd<false>(int, int, hipStream_t, const double*, double*, int, int,
                                       long, int, const Filters&);
template bool launch_stream_rev<true>(int, int, int, hipStream_t, const double*, long,
                                      const double*, double*, int, int, long, int, const Filters&);
template bool launch_stream_rev<false>(int, int, int, hipStream_t, const double*, long,
                                       const double*, double*, int, int, long, int,
                                       const Filters&);

}  // namespace fwtc
}  // namespace jw
