// jw_modwt_wave2.hpp -- barrier-free inverse MODWT with two outputs per lane on the LDS levels.
// Same sums in the same order as modwt_inv_wave (jw_modwt_wave.hpp), modwt_inv_fast and
// MODWTTransform.java:355-372 DIRECT (vFromApprox + vFromDetail, taps m = 0..L-1), so the
// results are bit-identical to both in both arithmetic contracts.
//
// Why: on a level with dilation d, the output at p needs taps p + m*d (m < L).  Outputs p and
// p + d share L - 1 of them, so a lane that owns both reads L + 1 taps for two outputs instead
// of 2L.  The wave kernel reads 15 16-byte (V, W) taps per output per LDS level for Symlet8;
// this one reads 17 per TWO outputs.  The sym8 J=6 inverse was LDS-bound (LDS array busy 84 %
// of CU cycles); here its LDS cycles drop 37 % (PMC SQ_LDS_IDX_ACTIVE) and the kernel 17 %.
//
// Layout (one step = 128 positions [a, a + 128), right -> left; one wave per segment):
//  * LDS level j (dilation d = 2^(j-1) <= 16) keeps (V_j, W_j) pairs for logical positions
//    k in [0, 128 + hist(j)) ([chunk | history], k = position - a).  Position k = r + d*u
//    (block u, r < d) lives at pair (u & 1) * HALF + (u >> 1) * d + r: even blocks in the first
//    half, odd blocks in the second (HALF padded so chunk writes are bank-conflict free).
//  * Lane l owns the outputs of blocks u = 2g + e (e = 0, 1) at offset r, with g = l / d,
//    r = l % d.  Tap t = e + m (t = 0..L) of the lane is block 2g + t, at pair
//    l + (t & 1) * HALF + (t >> 1) * d: lane-linear plus an immediate, so each of the L + 1
//    tap reads is one conflict-free ds_read_b128.
//  * A lane writes V_j where it computed it (level j + 1's outputs) and loads W_j from HBM at
//    those same positions, so every LDS write is one full 16-byte pair.
//  * The history shift by 128 positions is +64 pairs in that layout, so the lane that wrote a
//    pair writes it again 64 (and 128, ...) pairs further on in the next steps, from registers;
//    nothing is read back to shift it.
//  * Levels >= 6 are the wave kernel's register levels (jw_modwt_wave.hpp), run as two 64-lane
//    sub-steps per step (positions a + 64 + l, then a + l).  The output x leaves as 16-byte
//    pairs (a + 2l, a + 2l + 1).
#pragma once
#include <utility>

namespace jw {
namespace wave2 {

using fast::bload;
using fast::bload2;
using fast::bstore2;
using fast::d2;
using fast::kOOB;
using fast::madd;
using fast::make_rsrc;
using fast::rsrc_t;
using wave::partner32;
using wave::wave_lds_sync;

constexpr int kS = 128;  // positions per step (two per lane)

template <int L, int J>
struct G2 {
  using W1 = wave::WGeo<L, J>;                // register levels (>= 6): the wave kernel's layout
  static constexpr int JL = J < 5 ? J : 5;    // LDS levels 1..JL
  static constexpr bool TOPREG = J >= 6;      // V_J enters through the register levels
  static constexpr int lg(int j) { return j - 1; }
  static constexpr int dil(int j) { return 1 << (j - 1); }
  static constexpr int hist(int j) { return (L - 1) << (j - 1); }
  static constexpr int nblk(int j) { return (kS + hist(j)) / dil(j); }
  // (V, W) pairs per half.  The odd half starts d pairs past a multiple of 8 for d < 8, so the
  // chunk writes of levels 1..3 (8 lanes per ds_write_b128 group split between the two halves)
  // land on disjoint banks.
  static constexpr int half(int j) {
    return ((((nblk(j) + 1) / 2) * dil(j) + 7) & ~7) + (dil(j) < 8 ? dil(j) : 0);
  }
  // level j's pair array at vo(j)
  static constexpr int vo(int j) {
    int o = 0;
    for (int i = 1; i < j; ++i) o += 2 * half(i);
    return o;
  }
  static constexpr int lds_doubles = 2 * vo(JL + 1);
  static constexpr int nh(int j) { return (hist(j) + kS - 1) / kS; }  // history generations
  static constexpr int H = (L - 1) * ((1 << J) - 1);
};

// logical position k of LDS level j -> its double index in the level's array
template <int L, int J, int j>
__device__ __forceinline__ int phys(int k) {
  using G = G2<L, J>;
  constexpr int d = G::dil(j), lgd = G::lg(j);
  const int u = k >> lgd;
  return (u & 1) * G::half(j) + (u >> 1) * d + (k & (d - 1));
}

// One LDS level j: writes this step's (V_j, W_j) pairs at logical kv[0..1] (the lane loaded W_j
// at the positions where it holds V_j), reads the L + 1 taps, forms the two outputs and writes
// the history generations.  hp keeps this lane's pairs of the last nh(j) steps.  Each tap is one
// ds_read_b128 (lane-linear, conflict free); each write one ds_write_b128.
template <int L, int J, bool FMA, int j>
__device__ __forceinline__ void lds_level(d2* lds, int lane, const Taps& taps, const d2 (&in)[2],
                                          const int (&kv)[2], d2 (&hp)[G2<L, J>::nh(j)][2],
                                          double (&out)[2]) {
  using G = G2<L, J>;
  constexpr int d = G::dil(j), HALF = G::half(j), NH = G::nh(j), HI = G::hist(j);
  d2* const P = lds + G::vo(j);
  const int p0 = phys<L, J, j>(kv[0]), p1 = phys<L, J, j>(kv[1]);
  P[p0] = in[0];
  P[p1] = in[1];
  wave_lds_sync();
  double ap0 = 0.0, dp0 = 0.0, ap1 = 0.0, dp1 = 0.0;
#pragma unroll
  for (int t = 0; t <= L; ++t) {
    const d2 p = P[lane + (t & 1) * HALF + (t >> 1) * d];
    if (t < L) {
      ap0 = t == 0 ? madd<FMA>(0.0, taps.a[0], p.x) : madd<FMA>(ap0, taps.a[t], p.x);
      dp0 = t == 0 ? madd<FMA>(0.0, taps.b[0], p.y) : madd<FMA>(dp0, taps.b[t], p.y);
    }
    if (t >= 1) {
      ap1 = t == 1 ? madd<FMA>(0.0, taps.a[0], p.x) : madd<FMA>(ap1, taps.a[t - 1], p.x);
      dp1 = t == 1 ? madd<FMA>(0.0, taps.b[0], p.y) : madd<FMA>(dp1, taps.b[t - 1], p.y);
    }
  }
  out[0] = ap0 + dp0;
  out[1] = ap1 + dp1;
  wave_lds_sync();  // every tap read issued before the history below overwrites it
  // history: the pair written s steps ago at logical k moves to k + 128 (s + 1), i.e. +64 (s + 1)
#pragma unroll
  for (int s = NH - 1; s >= 1; --s) {
    hp[s][0] = hp[s - 1][0];
    hp[s][1] = hp[s - 1][1];
  }
  hp[0][0] = in[0];
  hp[0][1] = in[1];
#pragma unroll
  for (int s = 0; s < NH; ++s) {
    if (kv[0] + kS * s < HI) P[p0 + 64 * (s + 1)] = hp[s][0];
    if (kv[1] + kS * s < HI) P[p1 + 64 * (s + 1)] = hp[s][1];
  }
}

// logical positions where level j's V_j values sit in this lane: the outputs of level j + 1
// (2l - r + d' e, d' = 2d, r = l mod d'), of the register level 6 (l + 64 e), or the pair 2l + e
// of V_J loaded from HBM (J <= 5)
template <int L, int J, int j>
__device__ __forceinline__ void v_positions(int lane, int (&kv)[2]) {
  using G = G2<L, J>;
  if constexpr (j == G::JL && G::TOPREG) {
    kv[0] = lane;
    kv[1] = lane + 64;
  } else if constexpr (j == J) {
    kv[0] = 2 * lane;
    kv[1] = 2 * lane + 1;
  } else {
    constexpr int dn = G::dil(j + 1);
    const int r = lane & (dn - 1);
    kv[0] = 2 * lane - r;
    kv[1] = 2 * lane - r + dn;
  }
}

// Levels JL .. 1 in compile-time recursion.
template <int L, int J, bool FMA, int j>
struct LdsLevels {
  template <class HP>
  __device__ __forceinline__ static void run(d2* lds, int lane, const Taps& taps, double (&v)[2],
                                             const double (&w)[G2<L, J>::JL][2], HP& hp) {
    int kv[2];
    v_positions<L, J, j>(lane, kv);
    const d2 in[2] = {d2{v[0], w[j - 1][0]}, d2{v[1], w[j - 1][1]}};
    lds_level<L, J, FMA, j>(lds, lane, taps, in, kv, hp.template get<j>(), v);
    if constexpr (j > 1) LdsLevels<L, J, FMA, j - 1>::run(lds, lane, taps, v, w, hp);
  }
};

// per-level history registers, indexed by level at compile time
template <int L, int J, int j>
struct HistP : HistP<L, J, j - 1> {
  d2 h[G2<L, J>::nh(j)][2] = {};
};
template <int L, int J>
struct HistP<L, J, 0> {};
template <int L, int J, int JL>
struct HP : HistP<L, J, JL> {
  template <int j>
  __device__ __forceinline__ auto& get() { return static_cast<HistP<L, J, j>&>(*this).h; }
};

// D register sets of prefetched coefficients (step s uses set s % D), U steps unrolled per
// loop trip (a multiple of D).  MEM = 0 (microbenchmarks only): no HBM traffic.
// ONE: every coefficient row through one buffer resource (row r at byte (r N + p) 8; the
// launch picks it when (J + 1) N 8 < 2^31) instead of one resource per row: 4 SGPRs instead of
// 4 (J + 1), which for sym8 J=6 cuts the SGPR spills (to VGPR lanes, read back per tap use)
// from 92 to 18.
// ROT: the register rings whose length divides a trip's sub-steps rotate by index instead of
// shifting (sym8 J=6: no ring moves, 4 steps per trip; db4 J=8: the compiler renamed them
// already).  cfg5 inverse 15.86-15.91 -> 15.69-15.71 ms, cfg2 unchanged, on one box
// (profiles/r04/ab/inv_rot_q.log); JW_INV2_ROT=0 builds the shifting form.
#ifndef JW_INV2_ROT
#define JW_INV2_ROT 1
#endif
template <int L, int J, bool FMA, int D, int U, int MEM = 1, bool ONE = false,
          bool ROT = JW_INV2_ROT != 0>
__global__ __launch_bounds__(64) void modwt_inv_wave2(const double* __restrict__ coeffs,
                                                      double* __restrict__ x, long N, long seg_len,
                                                      long a_start, long ngroups, Taps taps,
                                                      int* __restrict__ nf = nullptr) {
  static_assert(U % D == 0, "U must be a multiple of D");
  using G = G2<L, J>;
  using GW = typename G::W1;
  constexpr int JL = G::JL;
  constexpr int NR = G::TOPREG ? J - 4 : 0;  // rows in 64-lane sub-step form: W_6..W_J, V_J
  extern __shared__ __attribute__((aligned(16))) d2 lds[];
  const int lane = threadIdx.x;
  // positions in 32 bits (N < 2^28: the byte offsets below are 32-bit already), fewer SGPRs
  const int Ni = (int)N;
  const int P = (int)(blockIdx.x * seg_len);
  const int seg_end = min(P + (int)seg_len, Ni);
  const double* cs = coeffs + (long)blockIdx.y * (long)(J + 1) * N;
  const rsrc_t rx = make_rsrc(x + (long)blockIdx.y * N, N);
  rsrc_t rc[ONE ? 1 : J + 1];
  if constexpr (ONE) {
    rc[0] = make_rsrc(cs, (long)(J + 1) * N);
  } else {
#pragma unroll
    for (int j = 0; j <= J; ++j) rc[j] = make_rsrc(cs + (long)j * N, N);
  }
  // byte offset of position p (< N) of coefficient row `row`
  auto roff = [&](int row, int p) -> int { return (ONE ? p + row * Ni : p) * 8; };
  auto rrs = [&](int row) -> rsrc_t { return rc[ONE ? 0 : row]; };
  for (int i = lane; i < G::lds_doubles / 2; i += 64) lds[i] = d2{0.0, 0.0};
  d2 rg[GW::rtot];
#pragma unroll
  for (int i = 0; i < GW::rtot; ++i) rg[i] = d2{0.0, 0.0};
  d2 xr[GW::NX], zr[GW::NZ];  // level 6
#pragma unroll
  for (int i = 0; i < GW::NX; ++i) xr[i] = zr[i] = d2{0.0, 0.0};
  HP<L, J, JL> hp;

  int a = P + (int)a_start;  // chunk start of the current step (may exceed N: taken mod N)
  int lb = a % Ni;           // load cursor: chunk start (mod N) of the next fetch
  struct Set {
    double w[JL][2];                // W_j at the lane's V_j positions (v_positions), j = 1..JL
    d2 vtop;                        // V_J pair at a + 2l when J <= 5
    double r[NR > 0 ? NR : 1][2];   // rows 5..J at positions a + l (e = 0), a + 64 + l (e = 1)
  };
  auto fetch = [&](Set& dst) {
    auto ld = [&](int row, int k) -> double {
      int p = lb + k;
      p = p >= Ni ? p - Ni : p;
      return MEM ? fast::bload_cp<JW_INV_LCP>(rrs(row), roff(row, p)) : (double)(p + row);
    };
    [&]<int... js>(std::integer_sequence<int, js...>) {
      (([&] {
         constexpr int j = js + 1;
         int kv[2];
         v_positions<L, J, j>(lane, kv);
         dst.w[j - 1][0] = ld(j - 1, kv[0]);
         dst.w[j - 1][1] = ld(j - 1, kv[1]);
       }()),
       ...);
    }(std::make_integer_sequence<int, JL>{});
    if constexpr (!G::TOPREG) {
      int p2 = lb + 2 * lane;
      p2 = p2 >= Ni ? p2 - Ni : p2;
      dst.vtop = MEM ? bload2(rrs(J), roff(J, p2)) : d2{(double)p2, (double)(p2 + 1)};
    }
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < NR; ++i) dst.r[i][e] = ld(5 + i, 64 * e + lane);
    lb -= kS;
    if (lb < 0) lb += Ni;
  };
  Set S[D];
#pragma unroll
  for (int q = 0; q < D - 1; ++q) {
    fetch(S[q]);
    __builtin_amdgcn_sched_barrier(0);
  }
  wave_lds_sync();

  bool bad = false;
  for (int gi = 0; gi < (int)ngroups; ++gi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      fetch(S[(u + D - 1) % D]);
      __builtin_amdgcn_sched_barrier(0);
      Set& cur = S[u % D];
      double v[2] = {0.0, 0.0};
      if constexpr (G::TOPREG) {
        // register levels J .. 7 and level 6 for sub-steps e = 1 (a + 64 + l), then e = 0
#pragma unroll
        for (int e = 1; e >= 0; --e) {
          // ROT: a ring whose length divides the trip's 2U sub-steps is rotated by index (its
          // newest entry at (k - c) mod length in sub-step c of the trip) instead of shifted
          const int c = 2 * u + (1 - e);
          double vv = cur.r[J - 5][e];  // V_J
#pragma unroll
          for (int j = J; j > 6; --j) {
            const int ro = GW::roff(j), q = GW::q(j), R = GW::ring(j);
            const bool rot = ROT && (2 * U) % R == 0;
            auto ri = [&](int k) { return ro + (rot ? ((k - c) % R + R) % R : k); };
            if (!rot) {
#pragma unroll
              for (int k = R - 1; k >= 1; --k) rg[ro + k] = rg[ro + k - 1];
            }
            rg[ri(0)] = d2{vv, cur.r[j - 6][e]};
            double ap = 0.0, dp = 0.0;
#pragma unroll
            for (int m = 0; m < L; ++m) {
              ap = madd<FMA>(ap, taps.a[m], rg[ri(m * q)].x);
              dp = madd<FMA>(dp, taps.b[m], rg[ri(m * q)].y);
            }
            vv = ap + dp;  // V_{j-1}
          }
          constexpr bool RX = ROT && (2 * U) % GW::NX == 0 && (2 * U) % GW::NZ == 0;
          auto xi = [&](int k) { return RX ? ((k - c) % GW::NX + GW::NX) % GW::NX : k; };
          auto zi = [&](int k) { return RX ? ((k - c) % GW::NZ + GW::NZ) % GW::NZ : k; };
          if (!RX) {
#pragma unroll
            for (int k = GW::NX - 1; k >= 1; --k) xr[k] = xr[k - 1];
          }
          xr[xi(0)] = d2{vv, cur.r[0][e]};
          const d2 z = partner32(xr[xi(0)], xr[xi(1)], lane);
          if (!RX) {
#pragma unroll
            for (int k = GW::NZ - 1; k >= 1; --k) zr[k] = zr[k - 1];
          }
          zr[zi(0)] = z;
          double ap = 0.0, dp = 0.0;
#pragma unroll
          for (int m = 0; m < L; ++m) {
            const d2 t = (m & 1) ? zr[zi(m >> 1)] : xr[xi(m >> 1)];
            ap = madd<FMA>(ap, taps.a[m], t.x);
            dp = madd<FMA>(dp, taps.b[m], t.y);
          }
          v[e] = ap + dp;  // V_5 at a + 64 e + l
        }
      } else {
        v[0] = cur.vtop.x;  // V_J pair
        v[1] = cur.vtop.y;
      }
      LdsLevels<L, J, FMA, JL>::run(lds, lane, taps, v, cur.w, hp);
      const int pos = a + 2 * lane;
      bstore2(rx, (MEM && pos >= P && pos < seg_end) ? (int)(pos * 8) : kOOB, d2{v[0], v[1]});
      bad |= !__builtin_isfinite(v[0]) | !__builtin_isfinite(v[1]);
      a -= kS;
    }
  }
  fast::nonfinite_flag(nf, bad);
}

template <int L, int J>
constexpr bool inv_ok() {
  using G = G2<L, J>;
  return L % 2 == 0 && (size_t)G::lds_doubles * 8 <= 20 * 1024 &&
         (J >= 7 ? G::W1::rtot : 0) + (J >= 6 ? G::W1::NX + G::W1::NZ : 0) <= 31;
}

// Default choice over the one-output wave kernel (jw_modwt_wave.hpp), from the A/B runs at
// N = 2^20 x 1024 on random data (tools/micro/invwave2.hip, profiles/r03/invwave2_*.log):
// sym8 J6 19.5 -> 16.3 ms (FMA) and 23.5 -> 21.0 ms (STRICT), sym8 J7 24.0 -> 21.7 ms, db4 J6
// and J4 1-2 % faster; db4 J8 tied in FMA (16.8 vs 16.9 ms) and lost in STRICT (19.0 vs 17.4 ms)
// while the two register levels of J >= 8 needed 262 VGPRs, one wave per SIMD.  With 32-bit
// stream positions it fits 246 VGPRs, two waves per SIMD, and db4 J8 STRICT wins too: 17.5 vs
// 17.9-18.1 ms (profiles/r03/inv_kernel_choice.log).
template <int L, int J, bool FMA>
constexpr bool inv_prefer2() {
  return J <= 7 || L <= 8;
}

// steps per loop trip: 2, or 4 for 16 taps with ROT (the level-6 rings of 8 entries then rotate
// once per trip; at 8 taps they are 4 long and U = 2 suffices)
template <int L, int J, bool FMA, int D = 2, int U = (JW_INV2_ROT && L == 16) ? 4 : 2>
int launch_inv(const Taps& t, const double* c, double* x, long N, int batch, hipStream_t s,
               int* nf) {
  using G = G2<L, J>;
  const long warm = ((long)(G::H + kS - 1) / kS) * kS;
  const long seg = fast::pick_seg(N, batch, warm, kS, 8192);
  const long nseg = (N + seg - 1) / seg;
  long steps = seg / kS + warm / kS;
  steps = ((steps + U - 1) / U) * U;  // surplus steps extend the warm-up to the right
  const long ngroups = steps / U;
  const long a_start = (steps - 1) * kS;
  const size_t lds = (size_t)G::lds_doubles * sizeof(double);
  const char* g1 = knob("JW_INV_ONE_RSRC");  // A/B runs: 0 = one resource per row
  const bool one = (long)(J + 1) * N * 8 < 0x7fffffffL && !(g1 && g1[0] == '0');
  auto kern = one ? modwt_inv_wave2<L, J, FMA, D, U, 1, true> : modwt_inv_wave2<L, J, FMA, D, U>;
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  const long cstride = (long)(J + 1) * N;
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    hipLaunchKernelGGL(kern, dim3((unsigned)nseg, (unsigned)nb), dim3(64), lds, s,
                       c + (long)b0 * cstride, x + (long)b0 * N, N, seg, a_start, ngroups, t,
                       nf ? nf + b0 : nullptr);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace wave2
}  // namespace jw
