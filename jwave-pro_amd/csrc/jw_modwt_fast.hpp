// jw_modwt_fast.hpp -- the steady-state MODWT kernels (filter length L and level count J
// compile-time).  Same arithmetic, tap order and results as the generic kernels in
// jw_modwt.hip (and as MODWTTransform.java:256-375 DIRECT); see that file for the reference
// mapping and DESIGN.md "MODWT kernels" for the design.
//
// What makes these the fast path on gfx950:
//  * every step is straight-line code with a fixed number of vector-memory instructions, so
//    the compiler waits for a prefetched chunk with a counted s_waitcnt vmcnt(N) instead of
//    draining the step's coefficient stores (vmcnt counts loads and stores in issue order);
//  * inputs are prefetched two steps ahead into two register sets (no register moves);
//  * stores are raw buffer stores whose offset is pushed out of range for samples outside the
//    workgroup's segment -- the hardware range check drops them, no branch;
//  * lane-consecutive LDS addressing (bank-conflict free) with immediate offsets (the
//    dilation is compile-time per level);
//  * the inverse keeps V_j and W_j interleaved as (V, W) pairs in LDS, so one ds_read_b128
//    feeds both adjoint sums of a tap and every coefficient is read from HBM once.
#pragma once
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "jw_internal.hpp"

namespace jw {
namespace fast {

#ifndef JW_INV_SYNC
#define JW_INV_SYNC() __syncthreads()  // (microbenchmarks redefine it to time the barriers)
#endif
constexpr int kC = 512;           // samples per level per step (both directions)
constexpr int kOOB = 0x7ffff000;  // byte offset beyond any row (N < 2^27): store dropped
#ifndef JW_NT_ROWS
#define JW_NT_ROWS 1
#endif
constexpr bool kNtRows = JW_NT_ROWS;
#ifndef JW_INV_NT
#define JW_INV_NT 0
#endif
constexpr bool kInvNt = JW_INV_NT;  // A/B builds: non-temporal coefficient loads (LDS-top inverse)

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef double d2 __attribute__((ext_vector_type(2)));
using rsrc_t = __amdgpu_buffer_rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const double* p, long n) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)(n * 8), 0x00020000);
}
__device__ __forceinline__ double bload(rsrc_t r, int off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
// Cache-policy bits of the streamed HBM accesses of the fused MODWT kernels (A/B builds only:
// gfx950 aux bits sc0 = 1, nt = 2, sc1 = 16; 0 = the default policy, the product's choice).
#ifndef JW_FWD_SCP
#define JW_FWD_SCP 0  // forward: coefficient stores
#endif
#ifndef JW_FWD_LCP
#define JW_FWD_LCP 0  // forward: signal loads
#endif
#ifndef JW_INV_LCP
#define JW_INV_LCP 0  // inverse: coefficient loads
#endif
template <int CP>
__device__ __forceinline__ double bload_cp(rsrc_t r, int off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, CP));
}
// non-temporal (streamed once): gives the line up early so rows that are re-read stay in L2
__device__ __forceinline__ double bload_nt(rsrc_t r, int off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 2));
}
__device__ __forceinline__ void bstore(rsrc_t r, int off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
}

template <bool FMA>
__device__ __forceinline__ double madd(double acc, double f, double v) {
  if constexpr (FMA) {
    return __builtin_fma(f, v, acc);
  } else {
    return acc + f * v;  // -ffp-contract=off: Java's rounded product + rounded sum
  }
}

// Non-finite detection for JWave's zero-tap semantics (jw_modwt_nf.hip): a kernel that writes
// a final row (V_J forward, x inverse) ORs !isfinite over every value it computes there and, at
// its end, sets the signal's flag.  A non-finite sample anywhere in the cascade reaches that
// row at its own position (tap m = 0 of every level carries it, and a sum with a non-finite
// term is non-finite), so a clear flag proves the zero taps the kernels skip were all finite.
// Lanes store the constant 1 (vector stores; every writer writes the same value).
__device__ __forceinline__ void nonfinite_flag(int* nf, bool bad) {
  if (nf != nullptr && bad) nf[blockIdx.y] = 1;
}

template <int L, int J>
struct Geo {
  static constexpr int H = (L - 1) * ((1 << J) - 1);  // total history samples
  static constexpr int hist(int j) { return (L - 1) << (j - 1); }
  static constexpr int hoff(int j) { return (L - 1) * ((1 << (j - 1)) - 1); }  // flat history offset
  // forward: B_{j-1} = [hist_j | C] holds V_{j-1}
  static constexpr int fwd_off(int j) { return hoff(j) + (j - 1) * kC; }
  static constexpr int fwd_total = H + J * kC;  // doubles
};

// Inverse layout: VW_j = [C | hist_j] of (V_j, W_j) pairs, C samples per step.  With TOPG
// the top level J is not staged in LDS at all (its taps are read from global memory, see
// inv_step), so only levels 1..J-1 take space.
template <int L, int J, int C, bool TOPG = false>
struct GeoI {
  static constexpr int H = Geo<L, J>::H;
  static constexpr int inv_off(int j) { return Geo<L, J>::hoff(j) + (j - 1) * C; }  // pairs
  static constexpr int inv_total =
      TOPG ? 2 * (Geo<L, J>::hoff(J) + (J - 1) * C) : 2 * (H + J * C);  // doubles
};

// Flat history index e in [0, H) -> level j (1-based).
template <int L>
__device__ __forceinline__ int level_of(int e) {
  const unsigned q = (unsigned)e / (unsigned)(L - 1) + 1u;
  return 32 - __builtin_clz(q);
}

// ---------------------------------------------------------------------------------------
// Forward: left -> right.  Thread t owns the adjacent output pair (2t, 2t+1) of every level
// (C = 2*NT), so every LDS read, LDS write, global load and global store moves 16 bytes per
// lane.  For d = 2^(j-1) >= 2 the pair's taps are adjacent pairs (x[i-md], x[i+1-md]); for
// d = 1 the L+1 distinct samples x[i+1-k] come from L/2+1 aligned pairs.  B_{j-1} keeps its
// chunk 16-byte aligned: logical position p of level j's input lives at cs(j) + p with
// cs(j) = hoff(j+1) + (j-1)*C + 1 (L even).  Needs N even (pairs never straddle a wrap).
// ---------------------------------------------------------------------------------------
template <int L, int J, int C>
struct GeoF {
  static constexpr int H = Geo<L, J>::H;
  static constexpr int cs(int j) { return Geo<L, J>::hoff(j + 1) + (j - 1) * C + 1; }
  static constexpr int total = H + J * C + 2;  // doubles
};

template <int CP = 0>
__device__ __forceinline__ d2 bload2(rsrc_t r, int off) {
  return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, CP));
}
template <int CP = 0>
__device__ __forceinline__ void bstore2(rsrc_t r, int off, d2 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, CP);
}

template <int L, int J, bool FMA, int NT, int SCP, bool ONE, class Fetch>
__device__ __forceinline__ void fwd_step(double* lds, d2& cur, Fetch&& fetch, int a, int P,
                                         int seg_end, const rsrc_t (&rw)[ONE ? 1 : J + 1],
                                         int n8, const Taps& taps, bool& nf) {
  constexpr int C = 2 * NT;
  using G = GeoF<L, J, C>;
  const int t = threadIdx.x;
  const int i = 2 * t;
  *(d2*)&lds[G::cs(1) + i] = cur;
  fetch(cur);  // the chunk two steps ahead: in flight behind this step and the next
  __syncthreads();
  const int pos = a + i;  // may be negative in the warm-up (then out of range)
  const bool in = pos >= P && pos < seg_end;  // P, seg_end even
  const int off = in ? pos * 8 : kOOB;
  // row r's store offset: its own resource (off), or the one all-rows resource (r N 8 further)
  auto roff = [&](int r) -> int { return ONE ? (in ? off + r * n8 : kOOB) : off; };
#pragma unroll
  for (int j = 1; j <= J; ++j) {
    const int d = 1 << (j - 1);
    const double* src = lds + G::cs(j);
    double w0 = 0.0, v0 = 0.0, w1 = 0.0, v1 = 0.0;  // outputs i and i+1
    if (d == 1) {
      d2 pr[L / 2 + 1];
#pragma unroll
      for (int q = 0; q <= L / 2; ++q) pr[q] = *(const d2*)&src[i - 2 * q];
#pragma unroll
      for (int m = 0; m < L; ++m) {
        // x[i - m] = v[m+1], x[i + 1 - m] = v[m], v[k] = k even ? pr[k/2].y : pr[(k-1)/2].x
        const double lo = ((m + 1) & 1) ? pr[m / 2].x : pr[(m + 1) / 2].y;
        const double hi = (m & 1) ? pr[(m - 1) / 2].x : pr[m / 2].y;
        w0 = madd<FMA>(w0, taps.b[m], lo);
        v0 = madd<FMA>(v0, taps.a[m], lo);
        w1 = madd<FMA>(w1, taps.b[m], hi);
        v1 = madd<FMA>(v1, taps.a[m], hi);
      }
    } else {
#pragma unroll
      for (int m = 0; m < L; ++m) {
        const d2 pr = *(const d2*)&src[i - m * d];
        w0 = madd<FMA>(w0, taps.b[m], pr.x);
        v0 = madd<FMA>(v0, taps.a[m], pr.x);
        w1 = madd<FMA>(w1, taps.b[m], pr.y);
        v1 = madd<FMA>(v1, taps.a[m], pr.y);
      }
    }
    bstore2<SCP>(rw[ONE ? 0 : j - 1], roff(j - 1), d2{w0, w1});
    if (j < J) {
      *(d2*)&lds[G::cs(j + 1) + i] = d2{v0, v1};
    } else {
      bstore2<SCP>(rw[ONE ? 0 : J], roff(J), d2{v0, v1});
      nf |= !__builtin_isfinite(v0) | !__builtin_isfinite(v1);  // see nonfinite_flag
    }
    __syncthreads();
  }
  // History shift: level j's last hist_j samples [C - hist_j, C) move to [-hist_j, 0).  Flat
  // e over H: src e + j*C + 1, dst e + (j-1)*C + 1 (see GeoF).
  constexpr int kPer = (G::H + NT - 1) / NT;
  if constexpr (kPer > 0) {
    double hv[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int e = t + r * NT;
      if (e < G::H) hv[r] = lds[e + level_of<L>(e) * C + 1];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int e = t + r * NT;
      if (e < G::H) lds[e + (level_of<L>(e) - 1) * C + 1] = hv[r];
    }
  }
}

// SCP: cache-policy bits of the coefficient stores (A/B microbenchmarks; 0 in the product).
// ONE: the J + 1 coefficient rows through one buffer resource (the launch picks it when
// (J + 1) N 8 < kOOB): 4 SGPRs instead of 4 (J + 1); sym8 J=6 spilled 44 SGPRs with a resource
// per row.
template <int L, int J, bool FMA, int NT, int SCP = 0, bool ONE = false>
__global__ __launch_bounds__(NT) void modwt_fwd_fast(const double* __restrict__ x,
                                                     double* __restrict__ coeffs, long N,
                                                     long seg_len, long warm, long npairs,
                                                     Taps taps, int* __restrict__ nf = nullptr) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int C = 2 * NT;
  using G = GeoF<L, J, C>;
  const int t = threadIdx.x;
  // stream positions in 32 bits (N < 2^27, see kOOB; the warm-up starts at most one segment
  // plus warm before 0)
  const int Ni = (int)N;
  const int P = (int)(blockIdx.x * seg_len);
  const int seg_end = min(P + (int)seg_len, Ni);
  const double* xs = x + (long)blockIdx.y * N;
  double* cs = coeffs + (long)blockIdx.y * (long)(J + 1) * N;
  const rsrc_t rx = make_rsrc(xs, N);
  rsrc_t rw[ONE ? 1 : J + 1];
  if constexpr (ONE) {
    rw[0] = make_rsrc(cs, (long)(J + 1) * N);
  } else {
#pragma unroll
    for (int j = 0; j <= J; ++j) rw[j] = make_rsrc(cs + (long)j * N, N);
  }
  const int n8 = (int)(N * 8);  // row stride in bytes (used when ONE)
  for (int i = t; i < G::total; i += NT) lds[i] = 0.0;

  int a = P - (int)warm;
  int lb = a % Ni;  // load cursor: stream position of the next chunk to fetch, mod N (even)
  if (lb < 0) lb += Ni;
  auto fetch = [&](d2& dst) {
    int p = lb + 2 * t;
    p = p >= Ni ? p - Ni : p;
    dst = bload2<JW_FWD_LCP>(rx, p * 8);
    lb += C;
    if (lb >= Ni) lb -= Ni;
  };
  d2 A, B;
  fetch(A);
  __builtin_amdgcn_sched_barrier(0);  // keep A's loads strictly older than B's (counted waits)
  fetch(B);
  __builtin_amdgcn_sched_barrier(0);
  // Range-dropped dummy stores give the loop entry the same vector-memory queue depth as the
  // loop back-edge (two steps of stores + one fetch behind A), so the compiler's merged wait
  // at the first step is the steady-state counted vmcnt, not a near-drain.
#pragma unroll
  for (int k = 0; k < 2 * (J + 1); ++k) bstore(rx, kOOB - 8 * k, 0.0);  // distinct: not merged
  __syncthreads();
  bool bad = false;
  for (int k = 0; k < (int)npairs; ++k) {
    fwd_step<L, J, FMA, NT, SCP, ONE>(lds, A, fetch, a, P, seg_end, rw, n8, taps, bad);
    a += C;
    fwd_step<L, J, FMA, NT, SCP, ONE>(lds, B, fetch, a, P, seg_end, rw, n8, taps, bad);
    a += C;
  }
  nonfinite_flag(nf, bad);
}

// ---------------------------------------------------------------------------------------
// Inverse: right -> left.  VW_j holds (V_j, W_j) pairs at positions [a, a + C + hist_j);
// thread t owns samples t + r*NT.  cur[(J+1)*r + (j-1)] = W_j, cur[(J+1)*r + J] = V_J.
// Levels j >= RF (dilation >= 64) are ring buffers of S_j = C + hist_j pairs (position a + u
// lives at (rb[j] + u) mod S_j, rb[j] steps back by C per chunk): no history shift.  Levels
// below RF keep [chunk | history] linear and shift the history.
// ---------------------------------------------------------------------------------------
template <int L, int J, int C, int RF>
struct Ring {
  static_assert(RF > J || ((1 << (RF - 1)) >= 64 && C % 64 == 0), "ring levels need d >= 64");
  static constexpr bool on(int j) { return j >= RF; }
  static constexpr int S(int j) { return C + Geo<L, J>::hist(j); }
  static constexpr int shifted() {  // pairs of flat history that still shift (levels < RF)
    return RF > J ? Geo<L, J>::H : Geo<L, J>::hoff(RF);
  }
  // Every shifted level's history fits beside its chunk (hist_j <= C): level j's shift
  // [0, hist_j) -> [C, C + hist_j) then runs inside level j-1's phase (level 1's at the next
  // step's first phase) instead of a separate two-barrier phase.
  static constexpr bool inline_shift() {
    return J >= 2 && Geo<L, J>::hist(RF > J ? J : RF - 1 < 1 ? 1 : RF - 1) <= C;
  }
};

// Ring index of window position u = ub + lane, with ub wave-uniform.  Ring levels have a
// dilation >= 64 and C, NT are multiples of 64, so S_j, rb_j and ub are all multiples of 64
// and a wave's 64 lanes never straddle the ring's end: the wrap is decided once per wave on
// the scalar unit and costs one vector add per access.
template <int L, int J, int C, int RF>
__device__ __forceinline__ int ring_idx(int j, const int (&rb)[J + 1], int ub, int lane) {
  using Rg = Ring<L, J, C, RF>;
  int x = rb[j] + ub;  // uniform, multiple of 64, < 2 S_j
  x = x >= Rg::S(j) ? x - Rg::S(j) : x;
  return x + lane;
}

template <int L, int J, bool FMA, int C, int NT, int RF, bool TOPG, class Fetch, class TapLoad>
__device__ __forceinline__ void inv_step(d2* vw, double (&cur)[(C / NT) * (J + 1)],
                                         Fetch&& fetch, long a, long P, long seg_end,
                                         const rsrc_t& rx, const Taps& taps, int (&rb)[J + 1],
                                         double (&tv)[(C / NT) * 2 * L], TapLoad&& load_taps,
                                         bool& nf) {
  using G = GeoI<L, J, C, TOPG>;
  using Rg = Ring<L, J, C, RF>;
  constexpr int R = C / NT;
  const int t = threadIdx.x;
  // W_j samples of this step stay in registers until V_j is known (level j+1), so every
  // (V_j, W_j) pair reaches LDS as one 16-byte store (8-byte stores at a 16-byte stride
  // would conflict 2-way).
  double wj[R][J];
  const int lane = t & 63;
  const int w64 = __builtin_amdgcn_readfirstlane(t & ~63);  // wave-uniform part of t
  auto ridx = [&](int j, int ubase, int u) {  // u = ubase + lane; non-ring levels use u as is
    return Rg::on(j) ? ring_idx<L, J, C, RF>(j, rb, ubase, lane) : u;
  };
  // Inline history shift of linear level jj (see Ring::inline_shift).
  auto shift_level = [&](int jj) {
    if (jj < 1 || jj > J || Rg::on(jj) || (TOPG && jj == J)) return;
    const int hj = Geo<L, J>::hist(jj);
#pragma unroll
    for (int e0 = 0; e0 < C; e0 += NT) {
      const int e = e0 + t;
      if (e < hj) vw[G::inv_off(jj) + C + e] = vw[G::inv_off(jj) + e];
    }
  };
  constexpr bool kInline = Rg::inline_shift();
  // Level 1's chunk of the previous step becomes history first: with TOPG and J = 2 the
  // write below replaces that chunk (each lane shifts only slots it then rewrites itself).
  if constexpr (kInline) shift_level(1);
  if constexpr (TOPG) {
    // Level J straight from registers: tap m = 0 is this lane's own sample of the chunk,
    // taps m >= 1 were loaded from global memory (L2) one step ago by load_taps.  Same
    // sums in the same order as the LDS path.
    static_assert(J >= 2, "TOPG: at least two levels");
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double* c = cur + (J + 1) * r;
      const double* v = tv + 2 * L * r;
#pragma unroll
      for (int j = 1; j < J; ++j) wj[r][j] = c[j - 1];
      double ap = madd<FMA>(0.0, taps.a[0], c[J]);
      double dp = madd<FMA>(0.0, taps.b[0], c[J - 1]);
#pragma unroll
      for (int m = 1; m < L; ++m) {
        ap = madd<FMA>(ap, taps.a[m], v[m]);
        dp = madd<FMA>(dp, taps.b[m], v[L + m]);
      }
      vw[G::inv_off(J - 1) + ridx(J - 1, w64 + r * NT, t + r * NT)] = d2{ap + dp, wj[r][J - 1]};
    }
    load_taps();  // the next step's level-J taps: issued before this step's chunk fetch
    // keep every tap load strictly older than the fetch (vmcnt counts in issue order: a tap
    // load scheduled behind the fetch would make the next step wait for the fetch too)
    __builtin_amdgcn_sched_barrier(0);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      vw[G::inv_off(J) + ridx(J, w64 + r * NT, t + r * NT)] =
          d2{cur[(J + 1) * r + J], cur[(J + 1) * r + J - 1]};
#pragma unroll
      for (int j = 1; j < J; ++j) wj[r][j] = cur[(J + 1) * r + j - 1];
    }
  }
  fetch(cur);  // the chunk two steps ahead
  JW_INV_SYNC();
#pragma unroll
  for (int j = TOPG ? J - 1 : J; j >= 1; --j) {
    const int d = 1 << (j - 1);
    const d2* src = vw + G::inv_off(j);
    if constexpr (kInline) shift_level(j + 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = t + r * NT;
      double ap = 0.0, dp = 0.0;
#pragma unroll
      for (int m = 0; m < L; ++m) {
        const d2 p = src[ridx(j, w64 + r * NT + m * d, i + m * d)];
        ap = madd<FMA>(ap, taps.a[m], p.x);
        dp = madd<FMA>(dp, taps.b[m], p.y);
      }
      const double v = ap + dp;  // inverseMODWT :366-369, vFromApprox + vFromDetail
      if (j > 1) {
        vw[G::inv_off(j - 1) + ridx(j - 1, w64 + r * NT, i)] = d2{v, wj[r][j - 1]};
      } else {
        const long pos = a + i;
        bstore(rx, (pos >= P && pos < seg_end) ? (int)(pos * 8) : kOOB, v);
        nf |= !__builtin_isfinite(v);
      }
    }
    JW_INV_SYNC();
  }
  // History shift of the linear levels: [0 .. hist_j) -> [C .. C + hist_j) (flat e over
  // their pairs: src e + (j-1)*C, dst e + j*C).
  constexpr int HS = kInline ? 0
                     : TOPG && Rg::shifted() > Geo<L, J>::hoff(J) ? Geo<L, J>::hoff(J)
                                                                   : Rg::shifted();
  constexpr int kPer = (HS + NT - 1) / NT;
  if constexpr (kPer > 0) {
    d2 hv[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int e = t + r * NT;
      if (e < HS) hv[r] = vw[e + (level_of<L>(e) - 1) * C];
    }
    JW_INV_SYNC();
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int e = t + r * NT;
      if (e < HS) vw[e + level_of<L>(e) * C] = hv[r];
    }
  }
#pragma unroll
  for (int j = 1; j <= J; ++j) {
    if (Rg::on(j)) {
      rb[j] -= C;
      if (rb[j] < 0) rb[j] += Rg::S(j);
    }
  }
}

// TOPG: level J's taps come from global memory (they were streamed through L2 a step or
// more before; the other rows load non-temporal so these stay), so VW_J leaves LDS: 43 KB
// instead of 61 KB for db4 J=8 (three workgroups per CU instead of two) and one barrier
// phase fewer per step.  MINW = minimum waves per SIMD the register allocation must allow
// (3 workgroups of 256 threads -> 3).
template <int L, int J, bool FMA, int C, int NT, int D, int RF, bool TOPG, int MINW>
__global__ __launch_bounds__(NT, MINW) void modwt_inv_fast(const double* __restrict__ coeffs,
                                                           double* __restrict__ x, long N,
                                                           long seg_len, long a_start,
                                                           long npairs, Taps taps,
                                                           int* __restrict__ nf = nullptr) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = GeoI<L, J, C, TOPG>;
  constexpr int R = C / NT;
  const int t = threadIdx.x;
  const long P = (long)blockIdx.x * seg_len;
  const long seg_end = min(P + seg_len, N);
  const double* cs = coeffs + (long)blockIdx.y * (long)(J + 1) * N;
  const rsrc_t rx = make_rsrc(x + (long)blockIdx.y * N, N);
  rsrc_t rc[J + 1];
#pragma unroll
  for (int j = 0; j <= J; ++j) rc[j] = make_rsrc(cs + (long)j * N, N);
  for (int i = t; i < G::inv_total; i += NT) lds[i] = 0.0;

  long a = P + a_start;  // rightmost chunk start (segment end + warm-up, chunk aligned)
  long lb = a % N;
  long lt = lb;  // TOPG: chunk start (mod N) of the step whose level-J taps load next
  auto fetch = [&](double (&dst)[R * (J + 1)]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      long p = lb + t + r * NT;
      p = p >= N ? p - N : p;
      const int off = (int)(p * 8);
#pragma unroll
      for (int j = 0; j <= J; ++j) {
        // TOPG re-reads rows J-1 (W_J) and J (V_J) from L2 for the taps: stream the others
        const bool nt = TOPG ? kNtRows && j < J - 1 : kInvNt;
        dst[(J + 1) * r + j] = nt ? bload_nt(rc[j], off) : bload(rc[j], off);
      }
    }
    lb -= C;
    if (lb < 0) lb += N;
  };
  // Level-J taps m = 1..L-1 of one step: positions lt + t + m*2^(J-1) mod N.  Byte offsets
  // stay below 2N*8 < 2^31, so the wrap is one unsigned min (o - N*8 wraps high when o < N*8);
  // the dilation 2^(J-1) <= 512 <= N keeps every step below 2N.
  double tv[R * 2 * L];
  auto load_taps = [&]() {
    if constexpr (TOPG) {
      const unsigned n8 = (unsigned)(N * 8), d8 = 8u << (J - 1);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        unsigned o = (unsigned)((lt + t + r * NT) * 8);  // lt < N, t + r*NT < C <= N
        o = min(o, o - n8);
#pragma unroll
        for (int m = 1; m < L; ++m) {
          o += d8;
          o = min(o, o - n8);
          tv[2 * L * r + m] = bload(rc[J], (int)o);
          tv[2 * L * r + L + m] = bload(rc[J - 1], (int)o);
        }
      }
      lt -= C;
      if (lt < 0) lt += N;
    }
  };
  // D register sets: the chunk of step s is fetched at the top of step s - D + ... so D-1
  // whole steps of work hide each load.  With TOPG the prologue issues, like the steady
  // state, [set 0][stores][taps of step 0][set 1][stores], so the first step's counted wait
  // matches the loop's.
  double S[D][R * (J + 1)];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    if (TOPG && q == D - 1) {
      load_taps();
      __builtin_amdgcn_sched_barrier(0);
    }
    fetch(S[q]);
    __builtin_amdgcn_sched_barrier(0);  // set q's loads strictly older than set q+1's
    if constexpr (TOPG) {
#pragma unroll
      for (int i = 0; i < R; ++i) bstore(rx, kOOB - 8 * (q * R + i), 0.0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (!TOPG) {
#pragma unroll
    for (int i = 0; i < D * R; ++i) bstore(rx, kOOB - 8 * i, 0.0);  // queue-depth padding
  }
  int rb[J + 1];
#pragma unroll
  for (int j = 0; j <= J; ++j) rb[j] = 0;
  __syncthreads();
  bool bad = false;
  for (long k = 0; k < npairs; ++k) {  // npairs counts groups of D steps
#pragma unroll
    for (int q = 0; q < D; ++q) {
      inv_step<L, J, FMA, C, NT, RF, TOPG>((d2*)lds, S[q], fetch, a, P, seg_end, rx, taps, rb,
                                           tv, load_taps, bad);
      a -= C;
    }
  }
  nonfinite_flag(nf, bad);
}

// ---------------------------------------------------------------------------------------
// Host launchers (instantiated per filter length in jw_modwt_fast_l*.hip)
// ---------------------------------------------------------------------------------------
template <int L, int J>
constexpr bool fwd_ok() {
  return (size_t)GeoF<L, J, 512>::total * 8 <= 80 * 1024 && Geo<L, J>::H <= 16 * 256 &&
         L % 2 == 0;
}
template <int L, int J, int C>
constexpr bool inv_fits() {
  return (size_t)GeoI<L, J, C>::inv_total * 8 <= 160 * 1024 && Geo<L, J>::H <= 16 * C;
}
template <int L, int J>
constexpr bool inv_ok() {
  return inv_fits<L, J, 256>();
}

// Threads per workgroup (C = 512 samples per step either way): env JW_FWD_NT / JW_INV_NT
// (256 or 512) for A/B runs; defaults are the measured best.
inline int pick_nt(const char* env, int dflt) {
  const char* e = knob(env);
  if (e && e[0] == '2') return 256;
  if (e && e[0] == '5') return 512;
  return dflt;
}

// Segment of a signal per workgroup: whole chunks, at least 8x the warm-up, and enough
// segments that the grid holds several waves of workgroups.
inline long pick_seg(long N, int batch, long warm, int C = kC, long min_wgs = 8192) {
  const long nchunks = (N + C - 1) / C;
  long min_chunks = (8 * warm) / C;
  if (min_chunks < 1) min_chunks = 1;
  long seg_chunks = nchunks;
  while (seg_chunks > min_chunks &&
         (long)batch * ((nchunks + seg_chunks - 1) / seg_chunks) < min_wgs)
    seg_chunks = (seg_chunks + 1) / 2;
  if (seg_chunks < min_chunks) seg_chunks = min_chunks < nchunks ? min_chunks : nchunks;
  return seg_chunks * C;
}

template <class K>
int launch(K kern, size_t lds, long nseg, int batch, int nt, hipStream_t s, const double* in,
           long in_stride, double* out, long out_stride, long N, long seg, long p4, long npairs,
           const Taps& t, int* nf) {
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    hipLaunchKernelGGL(kern, dim3((unsigned)nseg, (unsigned)nb), dim3(nt), lds, s,
                       in + (long)b0 * in_stride, out + (long)b0 * out_stride, N, seg, p4, npairs,
                       t, nf ? nf + b0 : nullptr);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

template <int L, int J, bool FMA>
int launch_fwd(const Taps& t, const double* x, double* c, long N, int batch, hipStream_t s,
               int* nf) {
  constexpr int NT = 256, C = 2 * NT;
  using G = GeoF<L, J, C>;
  const long warm = ((long)(G::H + C - 1) / C) * C;
  const long seg = pick_seg(N, batch, warm, C);
  const long nseg = (N + seg - 1) / seg;
  const long npairs = ((seg + warm) / C + 1) / 2;  // an odd extra step runs right of the segment
  const size_t lds = (size_t)G::total * sizeof(double);
  const long cs = (long)(J + 1) * N;
  const char* g1 = knob("JW_FWD_ONE_RSRC");  // A/B runs: 0 = one resource per row
  if (cs * 8 < (long)kOOB && !(g1 && g1[0] == '0'))
    return launch(modwt_fwd_fast<L, J, FMA, NT, JW_FWD_SCP, true>, lds, nseg, batch, NT, s, x, N, c, cs, N,
                  seg, warm, npairs, t, nf);
  return launch(modwt_fwd_fast<L, J, FMA, NT, JW_FWD_SCP>, lds, nseg, batch, NT, s, x, N, c, cs, N, seg, warm,
                npairs, t, nf);
}

template <int L, int J, bool FMA, int C, int NT, int D, int RF, bool TOPG = false>
int launch_inv_c(const Taps& t, const double* c, double* x, long N, int batch, hipStream_t s,
                 int* nf) {
  using G = GeoI<L, J, C, TOPG>;
  const long warm = ((long)(G::H + C - 1) / C) * C;
  const long seg = pick_seg(N, batch, warm, C);
  const long nseg = (N + seg - 1) / seg;
  const long steps = seg / C + warm / C;
  const long ngroups = (steps + D - 1) / D;
  const long a_start = (steps - 1) * C;  // surplus steps (to a multiple of D) run left of the segment
  const size_t lds = (size_t)G::inv_total * sizeof(double);
  const long cs = (long)(J + 1) * N;
  // workgroups of NT threads that fit a CU's 160 KB of LDS (at most 4: 16 waves of 256)
  constexpr int kFit = (int)((160 * 1024) / ((size_t)G::inv_total * sizeof(double)));
  constexpr int kMinW = (kFit < 1 ? 1 : kFit > 4 ? 4 : kFit) * NT / 256;
  return launch(modwt_inv_fast<L, J, FMA, C, NT, D, RF, TOPG, (kMinW < 1 ? 1 : kMinW)>, lds, nseg,
                batch, NT, s, c, cs, x, N, N, seg, a_start, ngroups, t, nf);
}

template <int L, int J, int C>
constexpr bool inv_fits_topg() {
  return J >= 2 && (size_t)GeoI<L, J, C, true>::inv_total * 8 <= 160 * 1024 &&
         Geo<L, J>::H <= 16 * C;
}

// Inverse: two register sets; the levels with dilation >= 64 (j >= 7) are ring buffers by
// default (env JW_INV_RING=off shifts every level, A/B runs).  Chunk C = 256 samples, one per
// thread of 256.  A/B variants (measured equal on MI355X): env
// JW_INV_TOP=global reads level J's taps from global memory (TOPG: 43 KB of LDS, three
// workgroups per CU for db4 J=8) and JW_INV_C=512 then takes two samples per thread.
}  // namespace fast
}  // namespace jw
#include "jw_modwt_wave.hpp"
#include "jw_modwt_wave2.hpp"
namespace jw {
namespace fast {

template <int L, int J, bool FMA>
int launch_inv(const Taps& t, const double* c, double* x, long N, int batch, hipStream_t s,
               int* nf) {
  // The barrier-free kernels are the default wherever they fit: two outputs per lane on the LDS
  // levels (wave2, N even: 16-byte pairs) where inv_prefer2 says so, else one (wave).
  // JW_INV_KERNEL = wave2 / wave / wg forces one of them (A/B runs and the parity tests).
  const char* w = knob("JW_INV_KERNEL");
  const bool force_wg = w && !std::strcmp(w, "wg");
  const bool force_w1 = w && (!std::strcmp(w, "wave") || !std::strcmp(w, "wave1"));
  const bool force_w2 = w && !std::strcmp(w, "wave2");
  if constexpr (wave2::inv_ok<L, J>()) {
    if ((N % 2) == 0 && (force_w2 || (!force_wg && !(force_w1 && wave::inv_wave_ok<L, J>()) &&
                     (wave2::inv_prefer2<L, J, FMA>() || !wave::inv_wave_ok<L, J>()))))
      return wave2::launch_inv<L, J, FMA>(t, c, x, N, batch, s, nf);
  }
  if constexpr (wave::inv_wave_ok<L, J>()) {
    if (!force_wg) return wave::launch_inv_wave<L, J, FMA>(t, c, x, N, batch, s, nf);
  }
  constexpr int RF = J >= 7 ? 7 : J + 1;
  const char* e = knob("JW_INV_RING");
  const char* top = knob("JW_INV_TOP");
  const char* ce = knob("JW_INV_C");
  const bool lds_top = !(top && top[0] == 'g');
  const bool c512 = ce && ce[0] == '5';
  if (e && e[0] == 'o') {
    if (lds_top || J < 2) return launch_inv_c<L, J, FMA, 256, 256, 2, J + 1>(t, c, x, N, batch, s, nf);
    return launch_inv_c<L, J, FMA, 256, 256, 2, J + 1, (J >= 2)>(t, c, x, N, batch, s, nf);
  }
  if (lds_top || J < 2) return launch_inv_c<L, J, FMA, 256, 256, 2, RF>(t, c, x, N, batch, s, nf);
  if constexpr (inv_fits_topg<L, J, 512>()) {
    if (c512) return launch_inv_c<L, J, FMA, 512, 256, 2, RF, true>(t, c, x, N, batch, s, nf);
  }
  return launch_inv_c<L, J, FMA, 256, 256, 2, RF, (J >= 2)>(t, c, x, N, batch, s, nf);
}

// Returned when (L, J, N) has no fast kernel (the caller falls back to the generic ones).
constexpr int kNotHandled = -100;

template <int L>
int forward(const Taps& t, bool fma, const double* x, double* c, long N, int J, int batch,
            hipStream_t s, int* nf) {
  if (N < kC || (N & 1) || N >= (1L << 27)) return kNotHandled;
  int st = kNotHandled;
  auto one = [&](auto jc) {
    constexpr int JJ = decltype(jc)::value;
    if constexpr (fwd_ok<L, JJ>()) {
      st = fma ? launch_fwd<L, JJ, true>(t, x, c, N, batch, s, nf)
               : launch_fwd<L, JJ, false>(t, x, c, N, batch, s, nf);
    }
  };
  switch (J) {
#define JW_J(JJ)                            \
  case JJ:                                  \
    one(std::integral_constant<int, JJ>{}); \
    break;
    JW_J(1) JW_J(2) JW_J(3) JW_J(4) JW_J(5) JW_J(6) JW_J(7) JW_J(8) JW_J(9) JW_J(10)
#undef JW_J
    default:
      break;
  }
  return st;
}

template <int L>
int inverse(const Taps& t, bool fma, const double* c, double* x, long N, int J, int batch,
            hipStream_t s, int* nf) {
  if (N < kC || N >= (1L << 27)) return kNotHandled;
  int st = kNotHandled;
  auto one = [&](auto jc) {
    constexpr int JJ = decltype(jc)::value;
    if constexpr (inv_ok<L, JJ>()) {
      st = fma ? launch_inv<L, JJ, true>(t, c, x, N, batch, s, nf)
               : launch_inv<L, JJ, false>(t, c, x, N, batch, s, nf);
    }
  };
  switch (J) {
#define JW_J(JJ)                            \
  case JJ:                                  \
    one(std::integral_constant<int, JJ>{}); \
    break;
    JW_J(1) JW_J(2) JW_J(3) JW_J(4) JW_J(5) JW_J(6) JW_J(7) JW_J(8) JW_J(9) JW_J(10)
#undef JW_J
    default:
      break;
  }
  return st;
}

#define JW_FAST_EXTERN(LL)                                                                     \
  extern template int forward<LL>(const Taps&, bool, const double*, double*, long, int, int,   \
                                  hipStream_t, int*);                                          \
  extern template int inverse<LL>(const Taps&, bool, const double*, double*, long, int, int,   \
                                  hipStream_t, int*);
#define JW_FAST_INSTANTIATE(LL)                                                                \
  template int forward<LL>(const Taps&, bool, const double*, double*, long, int, int,          \
                           hipStream_t, int*);                                                 \
  template int inverse<LL>(const Taps&, bool, const double*, double*, long, int, int,          \
                           hipStream_t, int*);
#define JW_FAST_LENGTHS(X) X(2) X(4) X(6) X(8) X(12) X(16) X(20)

JW_FAST_LENGTHS(JW_FAST_EXTERN)

}  // namespace fast
}  // namespace jw
