// jw_jfft.hpp -- the reference's own FFT, operation for operation, on gfx950 (JW_ARITH_STRICT).
//
// FastFourierTransform.fftCooleyTukey (src/main/java/jwave/transforms/FastFourierTransform.java
// :172-212) is a radix-2 decimation-in-time FFT: bit reversal (Integer.reverse, :176-184), then
// for size = 2, 4, .., n every block's butterflies
//     t = wn.mul(x[k + half]);  x[k] = u.add(t);  x[k + half] = u.sub(t);  wn = wn.mul(w)
// with w = (Math.cos(a), Math.sin(a)), a = 2 pi / size * (inverse ? 1 : -1), and wn restarting at
// (1, 0) in every block (:188-202).  Every block of one stage therefore uses the same twiddle
// sequence wn_k, k < half, built by the recurrence: the host tabulates it once per n in that
// order (Tw[half + k] = wn_k), so each butterfly here is the JVM's exact IEEE sequence
// (Complex.mul = (ac - bd, ad + bc), Complex.java:286-288; no FMA: -ffp-contract=off).  Grouping
// the butterflies of several stages in registers changes no operation, so the result is the
// reference's bit for bit.
//
// Geometry.  A transform of n = R x C (R, C powers of two) runs as two "column" passes:
//   pass 1: column c of the natural-order input viewed as [R][C] (x[r C + c]) is the block of
//           positions rev(c) R .. rev(c) R + R - 1 after the global bit reversal, placed at
//           rev_R(r): stages 1..log R on it, stored as row rev_C(c) of Z ([C][R], contiguous);
//   pass 2: column l of Z (Z[h R + l], h < C): stages log R + 1..log n pair h with h + 2^t and
//           take the twiddle Tw[(2^t + h mod 2^t) R + l]; the result is X[h R + l] in natural
//           order -- which is column l of the next transform's pass-1 view when that one splits
//           n as C x R (so a pass 2 can feed the next transform's pass 1 without HBM).
// The pass-2 twiddles are stored transposed (Tw2[l][m] = Tw[m R + l]) so that the lanes of one
// column read consecutive entries.  Short transforms (n <= 4096) run whole in one "column".
//
// A column of LC points is held by LC/EPT threads with EPT = min(8, LC) points each; a
// workgroup of 512 threads holds T = 512 EPT / LC columns in LDS (padded: one slot per 8
// points, one per column).  Stages run in register groups of up to 3 (radix 8): at <= 128
// VGPRs four waves per SIMD stay resident (16 points per thread needed ~200).
#pragma once
#include "jw_internal.hpp"

namespace jw {
namespace jf {

using cplx = double2;
constexpr int kNT = 512;
constexpr int kEPT = 8;  // points per thread (radix-8 register groups)

__host__ __device__ constexpr int ilog2(long v) {
  int r = 0;
  while ((1L << r) < v) ++r;
  return r;
}

// A/B builds (tools/build_variant.sh): points per thread of the 1024-point columns.  16 makes
// a 1024-point column one wavefront (wave-level syncs, radix-16 register groups, 8 columns =
// 128-byte pieces per workgroup) at 139 KB of LDS, one workgroup per CU.
#ifndef JF_EPT1024
#define JF_EPT1024 8
#endif
// Points per thread of the 2048- and 4096-point COLUMNS (kp1 / kp2s / kp2p / kp2r).  16: 4 and 2
// columns per workgroup (64- and 32-byte pieces) at 131 KB of LDS, one workgroup per CU; 8 (the
// whole-line kernels keep it, LineGeo): 2 and 1 columns (32- and 16-byte pieces), two per CU.
// JWave's FFT at 2^21 / 2^22: 2.89 -> 2.43 / 3.91 -> 2.97 ms per 128 Mi points; AUTO db4 J=8
// 1,516 -> 1,535 Msamples/s (profiles/r06/ab/ept_big/).  A/B builds: JF_EPT_BIG=8.
#ifndef JF_EPT_BIG
#define JF_EPT_BIG 16
#endif
#ifndef JF_SWZ  // LDS layout of a column (A/B builds: 0 = one pad slot per 8 points)
#define JF_SWZ 1
#endif
#ifndef JF_SWZ_MIN  // shortest column that takes the swizzle (A/B builds)
#define JF_SWZ_MIN 1024
#endif
// EPTO: the points per thread when given (the whole-line kernels' LineGeo), else the column rule
template <int LC, int EPTO = 0>
struct Geo {
  static constexpr int LOG = ilog2(LC);
  static constexpr int EPT = EPTO       ? EPTO
                             : LC == 1024 ? JF_EPT1024
                             : LC >= 2048 ? JF_EPT_BIG
                                          : (LC < kEPT ? LC : kEPT);
  static constexpr int GMAX = ilog2(EPT);
  static constexpr int TPC = LC / EPT;  // threads per column (divides 64 when <= 64)
  static constexpr int T = kNT / TPC;   // columns per workgroup
  // column stride: the XOR-swizzled layout (pidx) needs no padding inside a column, 6 slots
  // between columns; the padded one (columns under 1024 points, JF_SWZ=0) one slot per 8 points.
  // 512-point columns keep the padding: swizzled, the AUTO inverse's kp2r<512, 2> ran slower
  // (profiles/r04/ab/auto_swz_min1024_z.log: db4 J=8 1,491 -> 1,519 Msamples/s with the padding)
  static constexpr bool SWZ = JF_SWZ && LC >= JF_SWZ_MIN;
  static constexpr int CS = SWZ ? LC + 6 : LC + LC / 8 + (LC == 1024 ? 3 : LC == 2048 ? 5 : 1);
  static constexpr size_t LDS_BYTES = (size_t)T * CS * sizeof(cplx);
};
// the whole-line kernels (kline_*): 8 points per thread at every length (16 at 2048 / 4096 points
// would spill their NIN / NOUT streams)
template <int LC>
constexpr int kLineEPT = LC >= 2048 ? 8 : 0;
template <int LC>
using LineGeo = Geo<LC, kLineEPT<LC>>;
// the plain transforms' column passes (fft_rows / fft_rows3: kp1 and kp2s alone) take 16 points
// per thread at 1024 points too (8 columns, 128-byte pieces, one workgroup per CU): JWave's FFT
// at 2^20 2.30 -> 2.14 ms per 128 Mi points (profiles/r06/ab/ept_big/fft_ept1024_16.txt); the
// fused MODWT kernels keep 8 there (AUTO's forward kp2p<1024> wants two workgroups per CU)
#ifndef JF_PLAIN_EPT1024
#define JF_PLAIN_EPT1024 16
#endif
template <int LC>
constexpr int kPlainEPT = LC == 1024 ? JF_PLAIN_EPT1024 : 0;
template <int LC>
using PlainGeo = Geo<LC, kPlainEPT<LC>>;

// LDS slot of column position pos.  Columns of >= 1024 points: the low three bits XORed with bits
// 3-5, 6-8 and 9-11 (a permutation inside each group of 8 slots), which spreads the strided
// and bit-reversed accesses of the stage groups, the staging and the kp2p / kp2r transitions
// over the banks (a bank model of those phases: 9,984 vs 18,944 conflict-weighted group
// cycles for 1024 points with the 8-point padding; the bit-reversed transition writes were
// 8-way conflicts); shorter columns keep one pad slot per 8 points.
template <int LC>
__device__ __forceinline__ int pidx(int pos) {
  if constexpr (Geo<LC>::SWZ) {
    return pos ^ ((pos >> 3) & 7) ^ ((pos >> 6) & 7) ^ ((pos >> 9) & 7);
  } else {
    return pos + (pos >> 3);
  }
}
__device__ __forceinline__ int brev(int v, int bits) {
  return bits == 0 ? 0 : (int)(__builtin_bitreverse32((unsigned)v) >> (32 - bits));
}

// Complex.mul(Complex) :286-288 and mul(double) :299-301
__device__ __forceinline__ cplx jmul(cplx a, cplx b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ cplx jscale(cplx a, double s) { return make_double2(a.x * s, a.y * s); }
// one butterfly of fftCooleyTukey :196-199 (t = wn.mul(x[k + half]))
__device__ __forceinline__ void bfly(cplx& u, cplx& v, cplx w) {
  const cplx t = jmul(w, v);
  const cplx a = u;
  u = make_double2(a.x + t.x, a.y + t.y);
  v = make_double2(a.x - t.x, a.y - t.y);
}

template <int LC, int EO = 0>
__device__ __forceinline__ void col_sync() {
  if constexpr (Geo<LC, EO>::TPC <= 64) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  } else {
    __syncthreads();
  }
}

// The butterflies of stages t0 .. t0+G-1 on a thread's NSET = EPT / 2^G sets held in v (set i:
// positions base[i] + (m << t0), m < 2^G, at v[i 2^G + m]); stage t pairs j, j + 2^t with bit t
// clear and uses tw[2^t + (j mod 2^t)].
template <int LC, int G, int EO = 0>
__device__ __forceinline__ void stage_math(cplx (&v)[(Geo<LC, EO>::EPT)],
                                           const int (&base)[(Geo<LC, EO>::EPT >> G)], int t0,
                                           const cplx* __restrict__ tw) {
  using Gm = Geo<LC, EO>;
  constexpr int E = 1 << G, NSET = Gm::EPT / E;
  const int lowmask = (1 << t0) - 1;
#pragma unroll
  for (int u = 0; u < G; ++u) {
#pragma unroll
    for (int i = 0; i < NSET; ++i) {
      const int low = base[i] & lowmask;
#pragma unroll
      for (int r = 0; r < (1 << u); ++r) {
        const cplx w = tw[(1 << (t0 + u)) + low + (r << t0)];
#pragma unroll
        for (int q = 0; q < (E >> (u + 1)); ++q) {
          const int m = r + (q << (u + 1));
          bfly(v[i * E + m], v[i * E + m + (1 << u)], w);
        }
      }
    }
  }
}

// set -> its first position for a group starting at stage t0 of G stages
__device__ __forceinline__ int set_base(int set, int t0, int G) {
  return (set & ((1 << t0) - 1)) + ((set >> t0) << (t0 + G));
}

// Stages t0 .. t0+G-1 of one column (positions j; stage t pairs j, j + 2^t with bit t clear and
// uses tw[2^t + (j mod 2^t)]).  Thread tl owns EPT/2^G sets {base + m 2^t0 : m < 2^G}.
template <int LC, int G, int EO = 0>
__device__ __forceinline__ void stage_group(cplx* __restrict__ col, int tl, int t0,
                                            const cplx* __restrict__ tw) {
  using Gm = Geo<LC, EO>;
  constexpr int E = 1 << G, NSET = Gm::EPT / E;
  cplx v[Gm::EPT];
  int base[NSET];
#pragma unroll
  for (int i = 0; i < NSET; ++i) {
    base[i] = set_base(tl + Gm::TPC * i, t0, G);
#pragma unroll
    for (int m = 0; m < E; ++m) v[i * E + m] = col[pidx<LC>(base[i] + (m << t0))];
  }
  stage_math<LC, G, EO>(v, base, t0, tw);
#pragma unroll
  for (int i = 0; i < NSET; ++i) {
#pragma unroll
    for (int m = 0; m < E; ++m) col[pidx<LC>(base[i] + (m << t0))] = v[i * E + m];
  }
}

// all LOG stages of one column, in groups of GMAX (the column's points must be in place);
// stages T0 .. TEND - 1 only when TEND is given (a multiple of GMAX past T0)
template <int LC, int T0 = 0, int TEND = Geo<LC>::LOG, int EO = 0>
__device__ __forceinline__ void run_stages(cplx* __restrict__ col, int tl,
                                           const cplx* __restrict__ tw) {
  using Gm = Geo<LC, EO>;
  if constexpr (T0 < TEND) {
    constexpr int G = (TEND - T0) < Gm::GMAX ? (TEND - T0) : Gm::GMAX;
    if constexpr (T0 > 0) col_sync<LC, EO>();
    stage_group<LC, G, EO>(col, tl, T0, tw);
    run_stages<LC, T0 + G, TEND, EO>(col, tl, tw);
  }
}

// the thread's own points of its column: positions tl + TPC k
template <int LC, int EO = 0>
__device__ __forceinline__ int own_pos(int tl, int k) {
  return tl + Geo<LC, EO>::TPC * k;
}

// Workgroup -> (column tile, item).  When the tiles split evenly over the 8 XCDs, every XCD
// takes its own contiguous eighth of the tiles, and consecutive workgroups of an XCD take
// ADJACENT tiles of one item: a tile's column pieces are 64 bytes (4 columns of 16 B, 32 B for
// real input), so the neighbouring tile uses the other half of every 128-byte line while it is
// in L2; items go in pairs per tile, so the tile's twiddles and filter-spectrum columns serve
// two items per fetch.  (Running all items of one tile back to back instead keeps those hot,
// but fetches each data line twice: db4 J=8 AUTO 1,117 vs 1,295 Msamples/s, sym8 J=6 1,480 vs
// 1,695; items one at a time 1,258 / 1,652, in fours 1,258 / 1,653: profiles/r03/ab_tile*.)
__device__ __forceinline__ void tile_item(int ntiles, long nitems, int* tile, long* item) {
  const long b = (long)blockIdx.x + (long)blockIdx.y * gridDim.x;
  if ((ntiles & 7) == 0) {
    const int xcd = (int)(b & 7), per = ntiles >> 3;
    const long q = b >> 3;
    if ((nitems & 1) == 0) {
      *tile = xcd * per + (int)((q >> 1) % per);
      *item = (q >> 1) / per * 2 + (q & 1);
    } else {
      *tile = xcd * per + (int)(q % per);
      *item = q / per;
    }
  } else {
    *tile = (int)(b % ntiles);
    *item = b / ntiles;
  }
}

// ---------------------------------------------------------------------------------------
// Column passes.  Every functor addresses an item's points by natural index: In is
// cplx operator()(long item, long i) with i = r W + c for point (r, c) of the [LC][W] view
// (W = 2^wbits columns); outputs are operator()(long item, long i, cplx v), where a row store
// (Z, the pass-1 result) writes i = row LC + pos, row = rev(column).
// ---------------------------------------------------------------------------------------
template <int LC, bool REV, class In, int EO = 0>
__device__ __forceinline__ void load_cols(cplx* lds, const In& in, long item, int c0, int wbits) {
  using G = Geo<LC, EO>;
  cplx v[G::EPT];
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) {
    const int f = threadIdx.x + kNT * k;
    v[k] = in(item, ((long)(f / G::T) << wbits) + c0 + f % G::T);
  }
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) {
    const int f = threadIdx.x + kNT * k;
    const int r = f / G::T;
    lds[(f % G::T) * G::CS + pidx<LC>(REV ? brev(r, G::LOG) : r)] = v[k];
  }
}

template <int LC, class Out, int EO = 0>
__device__ __forceinline__ void store_rows(const cplx* lds, const Out& out, long item, int c0,
                                           int wbits) {
  using G = Geo<LC, EO>;
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) {
    const int f = threadIdx.x + kNT * k;
    const int cc = f / LC, pos = f % LC;
    out(item, (long)brev(c0 + cc, wbits) * LC + pos, lds[cc * G::CS + pidx<LC>(pos)]);
  }
}

template <int LC, class Out, int EO = 0>
__device__ __forceinline__ void store_cols(const cplx* lds, const Out& out, long item, int c0,
                                           int wbits) {
  using G = Geo<LC, EO>;
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) {
    const int f = threadIdx.x + kNT * k;
    const int cc = f % G::T, r = f / G::T;
    out(item, ((long)r << wbits) + c0 + cc, lds[cc * G::CS + pidx<LC>(r)]);
  }
}

// EO: points per thread when given (kPlainEPT: the plain transforms' kp1 / kp2s), else Geo's rule
// pass 1: columns of [LC][W] (bit-reversed into LDS), stages with the natural table, rows of Z
template <int LC, class In, class Out, int EO = 0>
__global__ __launch_bounds__(kNT) void kp1(In in, Out out, int wbits, long nitems,
                                           const cplx* __restrict__ tw1) {
  using G = Geo<LC, EO>;
  extern __shared__ cplx lds[];
  int tile;
  long item;
  tile_item((1 << wbits) / G::T, nitems, &tile, &item);
  const int c0 = tile * G::T;
  load_cols<LC, true, In, EO>(lds, in, item, c0, wbits);
  __syncthreads();
  const int cc = threadIdx.x / G::TPC, tl = threadIdx.x % G::TPC;
  run_stages<LC, 0, G::LOG, EO>(lds + cc * G::CS, tl, tw1);
  __syncthreads();
  store_rows<LC, Out, EO>(lds, out, item, c0, wbits);
}

// pass 2, natural-order output through Out (the spectrum, or a real row)
template <int LC, class In, class Out, int EO = 0>
__global__ __launch_bounds__(kNT) void kp2s(In in, Out out, int wbits, long nitems,
                                            const cplx* __restrict__ tw2) {
  using G = Geo<LC, EO>;
  extern __shared__ cplx lds[];
  int tile;
  long item;
  tile_item((1 << wbits) / G::T, nitems, &tile, &item);
  const int c0 = tile * G::T;
  load_cols<LC, false, In, EO>(lds, in, item, c0, wbits);
  __syncthreads();
  const int cc = threadIdx.x / G::TPC, tl = threadIdx.x % G::TPC;
  run_stages<LC, 0, G::LOG, EO>(lds + cc * G::CS, tl, tw2 + (long)(c0 + cc) * LC);
  __syncthreads();
  store_cols<LC, Out, EO>(lds, out, item, c0, wbits);
}

#ifndef JF_KP2R_SCHED
#define JF_KP2R_SCHED 0
#endif
#ifndef JF_KP2R_WPE
#define JF_KP2R_WPE 4
#endif
// pass 2, then NF pointwise products (Mid: cplx operator()(int f, long item, long i, cplx X),
// i = the natural index h W + l), each run through pass 1 of the next transform (table tw1)
// and stored as rows (Out: operator()(int f, long item, long j, cplx v), j = row LC + pos).
// (a workgroup of more than 80 KB of LDS is alone on its CU: two waves per SIMD, registers to match)
template <int LC>
constexpr int kColWPE = Geo<LC>::LDS_BYTES > 80 * 1024 ? 2 : JF_KP2R_WPE;
template <int LC, int NF, class In, class Mid, class Out>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(NF == 1 ? kColWPE<LC>
                                                                             : 1))) void kp2p(
    In in, Mid mid, Out out, int wbits, long nitems,
                                            const cplx* __restrict__ tw2,
                                            const cplx* __restrict__ tw1) {
  using G = Geo<LC>;
  extern __shared__ cplx lds[];
  int tile;
  long item;
  tile_item((1 << wbits) / G::T, nitems, &tile, &item);
  const int c0 = tile * G::T;
  load_cols<LC, false>(lds, in, item, c0, wbits);
  __syncthreads();
  const int cc = threadIdx.x / G::TPC, tl = threadIdx.x % G::TPC;
  cplx* col = lds + cc * G::CS;
  run_stages<LC>(col, tl, tw2 + (long)(c0 + cc) * LC);
  col_sync<LC>();
  cplx X[G::EPT];
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) X[k] = col[pidx<LC>(own_pos<LC>(tl, k))];
  const long l = c0 + cc;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    if (f == 0) {
      col_sync<LC>();
    } else {
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < G::EPT; ++k) {
      const int h = own_pos<LC>(tl, k);
      col[pidx<LC>(brev(h, G::LOG))] = mid(f, item, ((long)h << wbits) + l, X[k]);
    }
    col_sync<LC>();
    // every product runs the same pass-1 twiddles: opaque per product, or the compiler holds
    // the first product's twiddle values for the next (NF = 2: 208 VGPRs)
    const cplx* tw1f = tw1;
    if (NF > 1) asm volatile("" : "+v"(tw1f));
    run_stages<LC>(col, tl, tw1f);
    __syncthreads();
    store_rows<LC>(lds, [&](long it, long j, cplx v) { out(f, it, j, v); }, item, c0, wbits);
  }
}

// pass 2 of NIN inverse transforms of one item (In: cplx operator()(int s, long item, long i)),
// each reduced to a real value by Post (double operator()(int s, long item, long i, cplx v)),
// summed in stream order (the
// reference's vFromApprox[i] + vFromDetail[i], MODWTTransform.java:366-369).  FUSE: the sum
// (as Complex(v, 0)) runs through pass 1 of the next forward transform (table tw1f) and is
// stored as rows (Out: operator()(long item, long j, cplx v)); otherwise Out
// (operator()(long item, long i, double v)) stores it at natural index i.
// waves_per_eu(4): the LDS allows four waves per SIMD; the fused two-input form fits 128 VGPRs
// with no spill (the unfused one spilled 20, so it keeps its own allocation)
template <int LC, int NIN, bool FUSE, class In, class Post, class Out>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(
    NIN == 1 || FUSE ? kColWPE<LC> : 1))) void kp2r(
    In in, Post post, Out out, int wbits, long nitems,
                                            const cplx* __restrict__ tw2,
                                            const cplx* __restrict__ tw1f) {
  using G = Geo<LC>;
  extern __shared__ cplx lds[];
  int tile;
  long item;
  tile_item((1 << wbits) / G::T, nitems, &tile, &item);
  const int c0 = tile * G::T;
  const int cc = threadIdx.x / G::TPC, tl = threadIdx.x % G::TPC;
  cplx* col = lds + cc * G::CS;
  const long l = c0 + cc;
  double acc[G::EPT];
#pragma unroll
  for (int s = 0; s < NIN; ++s) {
    if (s > 0) __syncthreads();
    load_cols<LC, false>(lds, [&](long it, long i) { return in(s, it, i); }, item, c0, wbits);
    __syncthreads();
    // both inputs use the same twiddles: an opaque pointer per input keeps the compiler from
    // holding the first input's twiddle values for the second (NIN = 2 took 210 VGPRs, two
    // waves per SIMD, instead of ~120)
    const cplx* tws = tw2 + l * LC;
    if (NIN > 1) asm volatile("" : "+v"(tws));
    run_stages<LC>(col, tl, tws);
    col_sync<LC>();
#pragma unroll
    for (int k = 0; k < G::EPT; ++k) {
      const int h = own_pos<LC>(tl, k);
      const double v = post(s, item, ((long)h << wbits) + l, col[pidx<LC>(h)]);
      acc[k] = s == 0 ? v : acc[k] + v;
    }
    // keep the next input's loads behind this one's stages (register pressure, A/B builds)
    if (JF_KP2R_SCHED) __builtin_amdgcn_sched_barrier(0);
  }
  col_sync<LC>();
  if constexpr (FUSE) {
#pragma unroll
    for (int k = 0; k < G::EPT; ++k)
      col[pidx<LC>(brev(own_pos<LC>(tl, k), G::LOG))] = make_double2(acc[k], 0.0);
    col_sync<LC>();
    run_stages<LC>(col, tl, tw1f);
    __syncthreads();
    store_rows<LC>(lds, out, item, c0, wbits);
  } else {
#pragma unroll
    for (int k = 0; k < G::EPT; ++k) col[pidx<LC>(own_pos<LC>(tl, k))] = make_double2(acc[k], 0.0);
    __syncthreads();
    store_cols<LC>(lds, [&](long it, long i, cplx v) { out(it, i, v.x); }, item, c0, wbits);
  }
}

// ---------------------------------------------------------------------------------------
// Whole transforms in one column (n = LC <= 4096): T lines per workgroup, the line's points
// loaded by its own threads (positions tl + TPC k: coalesced), so only column syncs.
// ---------------------------------------------------------------------------------------
// load line `line` (In: cplx operator()(long line, int r)) bit-reversed into col
template <int LC, class In>
__device__ __forceinline__ void line_load_rev(cplx* col, int tl, const In& in, long line) {
  using G = LineGeo<LC>;
  constexpr int E = kLineEPT<LC>;
  cplx v[G::EPT];
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) v[k] = in(line, own_pos<LC, E>(tl, k));
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) col[pidx<LC>(brev(own_pos<LC, E>(tl, k), G::LOG))] = v[k];
}

// jw_fft (JW_ARITH_STRICT): In (line, r) -> cplx; Out (line, r, cplx); scale applied to both
// parts when inverse (x[i].mul(1.0 / n), :207-211)
template <int LC, class In, class Out>
__global__ __launch_bounds__(kNT) void kline_fft(In in, Out out, long nlines,
                                                 const cplx* __restrict__ tw, double scale,
                                                 int do_scale) {
  using G = LineGeo<LC>;
  constexpr int E = kLineEPT<LC>;
  extern __shared__ cplx lds[];
  const int cc = threadIdx.x / G::TPC, tl = threadIdx.x % G::TPC;
  const long line = (long)blockIdx.x * G::T + cc;
  const bool valid = line < nlines;  // no early exit: columns of 2048+ points sync the group
  cplx* col = lds + cc * G::CS;
  line_load_rev<LC>(col, tl, [&](long ln, int r) { return valid ? in(ln, r) : cplx{0.0, 0.0}; },
                    line);
  col_sync<LC, E>();
  run_stages<LC, 0, G::LOG, E>(col, tl, tw);
  col_sync<LC, E>();
  if (!valid) return;
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) {
    const int p = own_pos<LC, E>(tl, k);
    cplx v = col[pidx<LC>(p)];
    if (do_scale) v = jscale(v, scale);
    out(line, p, v);
  }
}

// One MODWT level on whole lines (n = LC <= 4096), MODWTTransform.java:290-304 / :355-372 with
// circularConvolveFFT{,Adjoint} (:752-837): NIN input rows per line, each FFT'd (Complex(x, 0)),
// multiplied by a filter spectrum (Mid: cplx operator()(int s, int f, long i, cplx X)), inverse
// FFT'd and reduced to its real part times 1/n.
//   forward (NIN = 1, NOUT = 2): row V_{j-1} -> W_j = Re IFFT(X Fh_j)/n, V_j = Re IFFT(X Fg_j)/n
//   inverse (NIN = 2, NOUT = 1): V_{j-1} = Re IFFT(FFT(V_j) conj Fg_j)/n
//                                        + Re IFFT(FFT(W_j) conj Fh_j)/n
// In: double operator()(int s, long line, int r);  Out: operator()(int f, long line, int r, double)
template <int LC, int NIN, int NOUT, class In, class Mid, class Out>
__global__ __launch_bounds__(kNT) void kline_modwt(In in, Mid mid, Out out, long nlines,
                                                   const cplx* __restrict__ twf,
                                                   const cplx* __restrict__ twi, double inv_n) {
  static_assert(NIN == 1 || NOUT == 1, "forward: 1 in / 2 out; inverse: 2 in / 1 out");
  using G = LineGeo<LC>;
  constexpr int E = kLineEPT<LC>;
  extern __shared__ cplx lds[];
  const int cc = threadIdx.x / G::TPC, tl = threadIdx.x % G::TPC;
  const long line = (long)blockIdx.x * G::T + cc;
  const bool valid = line < nlines;
  cplx* col = lds + cc * G::CS;
  double acc[G::EPT];
#pragma unroll
  for (int s = 0; s < NIN; ++s) {
    if (s > 0) col_sync<LC, E>();
    line_load_rev<LC>(
        col, tl,
        [&](long ln, int r) { return make_double2(valid ? in(s, ln, r) : 0.0, 0.0); }, line);
    col_sync<LC, E>();
    run_stages<LC, 0, G::LOG, E>(col, tl, twf);
    col_sync<LC, E>();
    cplx X[G::EPT];
#pragma unroll
    for (int k = 0; k < G::EPT; ++k) X[k] = col[pidx<LC>(own_pos<LC, E>(tl, k))];
#pragma unroll
    for (int f = 0; f < NOUT; ++f) {
      col_sync<LC, E>();
#pragma unroll
      for (int k = 0; k < G::EPT; ++k) {
        const int p = own_pos<LC, E>(tl, k);
        col[pidx<LC>(brev(p, G::LOG))] = mid(s, f, p, X[k]);
      }
      col_sync<LC, E>();
      run_stages<LC, 0, G::LOG, E>(col, tl, twi);
      col_sync<LC, E>();
#pragma unroll
      for (int k = 0; k < G::EPT; ++k) {
        const int p = own_pos<LC, E>(tl, k);
        const double v = col[pidx<LC>(p)].x * inv_n;  // result[i].mul(1.0/n).getReal()
        if constexpr (NOUT == 2) {
          if (valid) out(f, line, p, v);
        } else {
          acc[k] = s == 0 ? v : acc[k] + v;
        }
      }
    }
  }
  if constexpr (NOUT == 1) {
    if (valid) {
#pragma unroll
      for (int k = 0; k < G::EPT; ++k) out(0, line, own_pos<LC, E>(tl, k), acc[k]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// kp2p for 1024-point columns, 128-byte pieces at two workgroups per CU (round 6, A/B setting
// JW_AUTO_WCOL).  The default kp2p<1024> holds 4 columns per workgroup in LDS (64-byte pieces,
// ~3.3 TB/s); 8 columns of complex doubles need 128 KB of LDS (one workgroup per CU, measured
// slower).  Here each column is one wavefront holding its 1024 points in registers, 16 per lane,
// and the LDS only carries the exchanges between register stage groups -- real parts first, then
// imaginary parts, through one double per point: 8 columns in 66 KB.  The butterflies, twiddles
// and their order are stage_math's, so the values are kp2p's bit for bit.
// ---------------------------------------------------------------------------------------
namespace wcol {
constexpr int LC = 1024, LOG = 10, EPT = 16, T = 8;
// LDS slot of a point: one pad slot per 8 points.  Every layout below is lane-dependent base +
// compile-time offset under it (so the exchanges address with immediates, no address registers),
// and its 16-lane groups of 8-byte accesses hit distinct bank pairs (the rev(h) write aside);
// columns start 4 doubles apart modulo the banks (the staging writes of 8 columns).
constexpr int CSD = LC + LC / 8 + 4;  // 1156 doubles per column
constexpr size_t LDS_BYTES = (size_t)T * CSD * sizeof(double);  // 74 KB: two workgroups per CU

__device__ __forceinline__ int slot(int pos) { return pos + (pos >> 3); }
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
// Register layouts of a column's points over its wave: register k of lane l holds position
// pos(l, k); in LDS that point sits at slot(pos) = base(l) + off(k), written out per layout so
// every exchange addresses with immediate offsets.
//   L04: stage group (t0 = 0, G = 4): pos = 16 l + k
//   L44: group (4, 4):                pos = (l & 15) + 256 (l >> 4) + 16 k
//   L82: group (8, 2):                pos = l + 64 (k >> 2) + 256 (k & 3)
//   LNat: natural order:               pos = l + 64 k
//   LRev: bit-reversed natural order:  pos = rev10(l + 64 k) = 16 rev6(l) + rev4(k)
struct L04 {
  static __device__ __forceinline__ int base(int l) { return 18 * l; }
  static constexpr int off(int k) { return k + (k >> 3); }
};
struct L44 {
  static __device__ __forceinline__ int base(int l) {
    return (l & 15) + ((l & 15) >> 3) + 288 * (l >> 4);
  }
  static constexpr int off(int k) { return 18 * k; }
};
struct L82 {
  static __device__ __forceinline__ int base(int l) { return l + (l >> 3); }
  static constexpr int off(int k) { return 72 * (k >> 2) + 288 * (k & 3); }
};
struct LNat {
  static __device__ __forceinline__ int base(int l) { return l + (l >> 3); }
  static constexpr int off(int k) { return 72 * k; }
};
struct LRev {
  static __device__ __forceinline__ int base(int l) { return 18 * brev(l, 6); }
  static constexpr int rev4(int k) { return ((k & 1) << 3) | ((k & 2) << 1) | ((k & 4) >> 1) | ((k & 8) >> 3); }
  static constexpr int off(int k) { return rev4(k) + (rev4(k) >> 3); }
};
// the stages t0 .. t0+G-1 on registers in layout (t0, G): stage_math with EPT = 16
template <int G>
__device__ __forceinline__ void stages(cplx (&v)[EPT], int lane, int t0, const cplx* __restrict__ tw) {
  constexpr int E = 1 << G, NSET = EPT / E;
  const int lowmask = (1 << t0) - 1;
  int base[NSET];
#pragma unroll
  for (int i = 0; i < NSET; ++i) base[i] = set_base(lane + 64 * i, t0, G);
#pragma unroll
  for (int u = 0; u < G; ++u) {
#pragma unroll
    for (int i = 0; i < NSET; ++i) {
      const int low = base[i] & lowmask;
#pragma unroll
      for (int r = 0; r < (1 << u); ++r) {
        const cplx w = tw[(1 << (t0 + u)) + low + (r << t0)];
#pragma unroll
        for (int q = 0; q < (E >> (u + 1)); ++q) {
          const int m = r + (q << (u + 1));
          bfly(v[i * E + m], v[i * E + m + (1 << u)], w);
        }
      }
    }
    // one stage's twiddles live at a time (hoisted, the radix-16 group's 15 spilled)
    __builtin_amdgcn_sched_barrier(0);
  }
}
// v moves from layout F to layout To in the wave's column (re, then im)
template <class F, class To>
__device__ __forceinline__ void xchg(cplx (&v)[EPT], double* col, int lane) {
  double t[EPT];
  double* const pf = col + F::base(lane);
  double* const pt = col + To::base(lane);
  wsync();
#pragma unroll
  for (int k = 0; k < EPT; ++k) pf[F::off(k)] = v[k].x;
  wsync();
#pragma unroll
  for (int k = 0; k < EPT; ++k) t[k] = pt[To::off(k)];
  wsync();
#pragma unroll
  for (int k = 0; k < EPT; ++k) pf[F::off(k)] = v[k].y;
  wsync();
#pragma unroll
  for (int k = 0; k < EPT; ++k) v[k] = make_double2(t[k], pt[To::off(k)]);
}
// all 10 stages (groups (0,4), (4,4), (8,2)); v enters in layout (0,4), leaves in (8,2)
__device__ __forceinline__ void run10(cplx (&v)[EPT], double* col, int lane,
                                      const cplx* __restrict__ tw) {
  stages<4>(v, lane, 0, tw);
  xchg<L04, L44>(v, col, lane);
  stages<4>(v, lane, 4, tw);
  xchg<L44, L82>(v, col, lane);
  stages<2>(v, lane, 8, tw);
}
}  // namespace wcol

// pass 2 of a 1024-point column, one product (Mid), pass 1 of the next transform, rows out --
// kp2p<1024, 1, ...> with 8 columns per workgroup (see wcol above)
template <class In, class Mid, class Out>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(4))) void kp2p_w(
    In in, Mid mid, Out out, int wbits, long nitems, const cplx* __restrict__ tw2,
    const cplx* __restrict__ tw1) {
  using namespace wcol;
  extern __shared__ double ldsd[];
  int tile;
  long item;
  tile_item((1 << wbits) / T, nitems, &tile, &item);
  const int c0 = tile * T;
  const int tid = threadIdx.x, lane = tid & 63, cc = tid >> 6;
  double* col = ldsd + cc * CSD;
  cplx v[EPT];
  {
    // rows r = f / 8 of the 8 columns (128 bytes each), f = tid + 512 k, to the column's wave in
    // layout L04 (position r): slot(r) = (tid >> 3) + (tid >> 6) + 72 k in column tid & 7
    cplx g[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int f = tid + kNT * k;
      g[k] = in(item, ((long)(f >> 3) << wbits) + c0 + (f & 7));
    }
    double t[EPT];
    double* const pw = ldsd + (tid & 7) * CSD + (tid >> 3) + (tid >> 6);
    double* const pr = col + L04::base(lane);
#pragma unroll
    for (int k = 0; k < EPT; ++k) pw[72 * k] = g[k].x;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EPT; ++k) t[k] = pr[L04::off(k)];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EPT; ++k) pw[72 * k] = g[k].y;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EPT; ++k) v[k] = make_double2(t[k], pr[L04::off(k)]);
  }
  run10(v, col, lane, tw2 + (long)(c0 + cc) * LC);
  // to the natural positions h = lane + 64 k, the product, back at rev(h) for the next pass 1
  xchg<L82, LNat>(v, col, lane);
  const long l = c0 + cc;
#pragma unroll
  for (int k = 0; k < EPT; ++k) v[k] = mid(0, item, ((long)(lane + 64 * k) << wbits) + l, v[k]);
  xchg<LRev, L04>(v, col, lane);
  run10(v, col, lane, tw1);
  // rows out: column k / 2, position tid + 512 (k & 1) (f = tid + 512 k): 4 KB row pieces
  double t[EPT];
  double* const pw = col + L82::base(lane);
  const double* const pr = ldsd + tid + (tid >> 3);
  wsync();
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EPT; ++k) pw[L82::off(k)] = v[k].x;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EPT; ++k) t[k] = pr[(k >> 1) * CSD + 576 * (k & 1)];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EPT; ++k) pw[L82::off(k)] = v[k].y;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int c = k >> 1, pos = tid + 512 * (k & 1);
    out(0, item, (long)brev(c0 + c, wbits) * LC + pos,
        make_double2(t[k], pr[(k >> 1) * CSD + 576 * (k & 1)]));
  }
}

}  // namespace jf
}  // namespace jw

namespace jw {
namespace jf {

// The convolution inside fftBluestein (FastFourierTransform.java:259-324) on whole lines
// (m = LC <= 4096): a (In, already chirped, zero past n) is FFT'd, multiplied by B = FFT(b)
// (a[i].mul(b[i]), :300-302), inverse FFT'd without the 1/m, and every point handed to Out
// (operator()(long line, int r, cplx v)), which applies the reference's post-processing.
template <int LC, class In, class Out>
__global__ __launch_bounds__(kNT) void kline_conv(In in, Out out, long nlines,
                                                  const cplx* __restrict__ B,
                                                  const cplx* __restrict__ twf,
                                                  const cplx* __restrict__ twi) {
  using G = LineGeo<LC>;
  constexpr int E = kLineEPT<LC>;
  extern __shared__ cplx lds[];
  const int cc = threadIdx.x / G::TPC, tl = threadIdx.x % G::TPC;
  const long line = (long)blockIdx.x * G::T + cc;
  const bool valid = line < nlines;
  cplx* col = lds + cc * G::CS;
  line_load_rev<LC>(col, tl, [&](long ln, int r) { return valid ? in(ln, r) : cplx{0.0, 0.0}; },
                    line);
  col_sync<LC, E>();
  run_stages<LC, 0, G::LOG, E>(col, tl, twf);
  col_sync<LC, E>();
  cplx X[G::EPT];
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) X[k] = col[pidx<LC>(own_pos<LC, E>(tl, k))];
  col_sync<LC, E>();
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) {
    const int p = own_pos<LC, E>(tl, k);
    col[pidx<LC>(brev(p, G::LOG))] = jmul(X[k], B[p]);
  }
  col_sync<LC, E>();
  run_stages<LC, 0, G::LOG, E>(col, tl, twi);
  col_sync<LC, E>();
  if (!valid) return;
#pragma unroll
  for (int k = 0; k < G::EPT; ++k) {
    const int p = own_pos<LC, E>(tl, k);
    out(line, p, col[pidx<LC>(p)]);
  }
}

}  // namespace jf
}  // namespace jw
