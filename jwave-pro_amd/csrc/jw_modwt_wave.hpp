// jw_modwt_wave.hpp -- the barrier-free inverse MODWT: one wavefront streams one segment of
// one signal right -> left on its own, so no step ever waits at a workgroup barrier.
// Same sums in the same order as modwt_inv_fast (jw_modwt_fast.hpp) and as
// MODWTTransform.java:355-372 DIRECT (vFromApprox + vFromDetail, taps m = 0..L-1), so the
// results are bit-identical to the workgroup kernel in both arithmetic contracts.
//
// Layout of one wave's state (chunk = 64 positions, lane l owns position a + l):
//  * levels with dilation d = 2^(j-1) >= 64 keep their (V_j, W_j) history in REGISTERS: the
//    tap at a + l + m*d is lane l's own pair from m*d/64 steps ago, so level j is a per-lane
//    shift register of (L-1)*d/64 + 1 pairs (no LDS, no cross-lane traffic);
//  * levels with d <= 32 keep [chunk | history] linearly in the wave's LDS slice; the chunk
//    is written by its lanes, the taps m >= 1 are 16-byte reads at immediate offsets
//    (lane-consecutive, bank-conflict free), tap m = 0 is the lane's own pair in registers,
//    and the next step's history is written from registers (each lane keeps its last
//    ceil(hist/64) pairs), never read back and shifted;
//  * LDS ordering inside a wave needs no s_barrier: DS instructions of one wave execute in
//    issue order, and a wavefront-scope fence keeps the compiler from reordering them.
#pragma once

namespace jw {
namespace wave {

using fast::bload;
using fast::bstore;
using fast::d2;
using fast::kOOB;
using fast::madd;
using fast::make_rsrc;
using fast::rsrc_t;

constexpr int kW = 64;  // positions per step = lanes of the wave

template <int L, int J>
struct WGeo {
  static constexpr int JL = J < 5 ? J : 5;  // LDS levels 1..JL (dilation <= 16)
  // level 6 (dilation 32): the tap at a + l + 32m is lane l's own pair (m even) or its partner
  // lane l ^ 32's (m odd), so it lives in registers too: own pairs X[s-k] and partner pairs
  // Z[s-k] = (l < 32 ? X_{l+32}[s-k] : X_{l-32}[s-k-1]), one permlane32 swap per word.
  static constexpr bool P6 = J >= 6;
  static constexpr int NX = L / 2 > 2 ? L / 2 : 2, NZ = L / 2;  // X[s-1] feeds the swap
  static constexpr int hist(int j) { return (L - 1) << (j - 1); }
  static constexpr int off(int j) {  // pair offset of LDS level j's [chunk | history]
    int o = 0;
    for (int i = 1; i < j; ++i) o += kW + hist(i);
    return o;
  }
  static constexpr int lds_pairs = off(JL + 1);
  // register levels j > JL: dilation / 64 and the shift-register length (pairs)
  static constexpr int q(int j) { return 1 << (j - 7); }
  static constexpr int ring(int j) { return (L - 1) * q(j) + 1; }
  static constexpr int roff(int j) {  // offset of level j's shift register in the flat array
    int o = 0;
    for (int i = 7; i < j; ++i) o += ring(i);
    return o;
  }
  static constexpr int rtot = roff(J + 1) > 0 ? roff(J + 1) : 1;
  // LDS levels: pairs a lane keeps for the history writes (current one included)
  static constexpr int nh(int j) { return (hist(j) + kW - 1) / kW; }
  static constexpr int hoff(int j) {
    int o = 0;
    for (int i = 1; i < j; ++i) o += nh(i);
    return o;
  }
  static constexpr int htot = hoff(JL + 1);
  static constexpr int H = (L - 1) * ((1 << J) - 1);
};

// Z = (lane < 32 ? cur of lane + 32 : prev of lane - 32): v_permlane32_swap exchanges lanes
// 32..63 of its first operand with lanes 0..31 of its second.
__device__ __forceinline__ d2 partner32(d2 cur, d2 prev, int lane) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 c = __builtin_bit_cast(u32x4, cur), p = __builtin_bit_cast(u32x4, prev);
  u32x4 z;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const auto r = __builtin_amdgcn_permlane32_swap(c[w], p[w], false, false);
    z[w] = lane < 32 ? r[1] : r[0];
  }
  return __builtin_bit_cast(d2, z);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// D register sets of prefetched coefficients (step s uses set s % D; its loads were issued at
// the top of step s - D + 1), U steps unrolled per loop trip (a multiple of D, so every set
// index and shift-register slot is a compile-time register).
// MEM = 0 (microbenchmarks only): the fetch makes register values and every store is dropped,
// so the kernel times its LDS / VALU work alone.
template <int L, int J, bool FMA, int D, int U, int MEM = 1, int CP = 0>
__global__ __launch_bounds__(kW) void modwt_inv_wave(const double* __restrict__ coeffs,
                                                     double* __restrict__ x, long N, long seg_len,
                                                     long a_start, long ngroups, Taps taps,
                                                     int* __restrict__ nf = nullptr) {
  static_assert(U % D == 0, "U must be a multiple of D");
  using G = WGeo<L, J>;
  constexpr int JL = G::JL;
  extern __shared__ __attribute__((aligned(16))) d2 lds2[];
  const int lane = threadIdx.x;
  // stream positions in 32 bits (N < 2^27 on this path, see kOOB)
  const int Ni = (int)N;
  const int P = (int)(blockIdx.x * seg_len);
  const int seg_end = min(P + (int)seg_len, Ni);
  const double* cs = coeffs + (long)blockIdx.y * (long)(J + 1) * N;
  const rsrc_t rx = make_rsrc(x + (long)blockIdx.y * N, N);
  rsrc_t rc[J + 1];
#pragma unroll
  for (int j = 0; j <= J; ++j) rc[j] = make_rsrc(cs + (long)j * N, N);
  d2* const base = lds2 + lane;
  for (int i = lane; i < G::lds_pairs; i += kW) lds2[i] = d2{0.0, 0.0};
  d2 rg[G::rtot];
#pragma unroll
  for (int i = 0; i < G::rtot; ++i) rg[i] = d2{0.0, 0.0};
  d2 xr[G::NX], zr[G::NZ];  // level 6
#pragma unroll
  for (int i = 0; i < G::NX; ++i) xr[i] = zr[i] = d2{0.0, 0.0};
  d2 hp[G::htot > 0 ? G::htot : 1];
#pragma unroll
  for (int i = 0; i < (G::htot > 0 ? G::htot : 1); ++i) hp[i] = d2{0.0, 0.0};

  int a = P + (int)a_start;  // chunk start of the current step (>= 0, may exceed N: mod N)
  int lb = a % Ni;           // load cursor: chunk start (mod N) of the next fetch
  auto fetch = [&](double (&dst)[J + 1]) {
    int p = lb + lane;
    p = p >= Ni ? p - Ni : p;
    const int off = p * 8;
#pragma unroll
    for (int j = 0; j <= J; ++j)
      dst[j] = MEM ? __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc[j], off, 0, CP))
                   : (double)(p + j);
    lb -= kW;
    if (lb < 0) lb += Ni;
  };
  double S[D][J + 1];
#pragma unroll
  for (int q = 0; q < D - 1; ++q) {
    fetch(S[q]);
    __builtin_amdgcn_sched_barrier(0);  // set q's loads strictly older than set q+1's
  }
  wave_lds_sync();

  bool bad = false;
  for (int g = 0; g < (int)ngroups; ++g) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      fetch(S[(u + D - 1) % D]);  // the set consumed at step u-1: refilled for step u+D-1
      __builtin_amdgcn_sched_barrier(0);
      double(&cur)[J + 1] = S[u % D];
      double v = cur[J];  // V_J
      // register levels J .. JL+1
#pragma unroll
      for (int j = J; j > 6; --j) {
        const int ro = G::roff(j), q = G::q(j);
#pragma unroll
        for (int k = G::ring(j) - 1; k >= 1; --k) rg[ro + k] = rg[ro + k - 1];
        rg[ro] = d2{v, cur[j - 1]};
        double ap = 0.0, dp = 0.0;
#pragma unroll
        for (int m = 0; m < L; ++m) {
          ap = madd<FMA>(ap, taps.a[m], rg[ro + m * q].x);
          dp = madd<FMA>(dp, taps.b[m], rg[ro + m * q].y);
        }
        v = ap + dp;  // V_{j-1}
      }
      if constexpr (G::P6) {  // level 6: own / partner shift registers
#pragma unroll
        for (int k = G::NX - 1; k >= 1; --k) xr[k] = xr[k - 1];
        xr[0] = d2{v, cur[5]};
        const d2 z = partner32(xr[0], xr[1], lane);
#pragma unroll
        for (int k = G::NZ - 1; k >= 1; --k) zr[k] = zr[k - 1];
        zr[0] = z;
        double ap = 0.0, dp = 0.0;
#pragma unroll
        for (int m = 0; m < L; ++m) {
          const d2 t = (m & 1) ? zr[m >> 1] : xr[m >> 1];
          ap = madd<FMA>(ap, taps.a[m], t.x);
          dp = madd<FMA>(dp, taps.b[m], t.y);
        }
        v = ap + dp;  // V_5
      }
      // LDS levels JL .. 1
#pragma unroll
      for (int j = JL; j >= 1; --j) {
        const int d = 1 << (j - 1), o = G::off(j), ho = G::hoff(j);
        const d2 pr = d2{v, cur[j - 1]};
        base[o] = pr;
        wave_lds_sync();
        double ap = madd<FMA>(0.0, taps.a[0], pr.x);
        double dp = madd<FMA>(0.0, taps.b[0], pr.y);
#pragma unroll
        for (int m = 1; m < L; ++m) {
          const d2 t = base[o + m * d];
          ap = madd<FMA>(ap, taps.a[m], t.x);
          dp = madd<FMA>(dp, taps.b[m], t.y);
        }
        v = ap + dp;  // V_{j-1}
        wave_lds_sync();  // every tap read issued before the history below overwrites it
#pragma unroll
        for (int k = G::nh(j) - 1; k >= 1; --k) hp[ho + k] = hp[ho + k - 1];
        hp[ho] = pr;
#pragma unroll
        for (int k = 0; k < G::nh(j); ++k) {
          if ((k + 1) * kW <= G::hist(j) || kW * k + lane < G::hist(j))
            base[o + kW * (k + 1)] = hp[ho + k];
        }
      }
      const int pos = a + lane;
      bstore(rx, (MEM && pos >= P && pos < seg_end) ? pos * 8 : kOOB, v);
      bad |= !__builtin_isfinite(v);
      a -= kW;
    }
  }
  fast::nonfinite_flag(nf, bad);
}

template <int L, int J>
constexpr bool inv_wave_ok() {
  using G = WGeo<L, J>;
  return L % 2 == 0 && J >= 6 && (size_t)G::lds_pairs * 16 <= 20 * 1024 &&
         (J >= 7 ? G::rtot : 0) + G::NX + G::NZ <= 31;
}

template <int L, int J, bool FMA>
int launch_inv_wave(const Taps& t, const double* c, double* x, long N, int batch,
                    hipStream_t s, int* nf) {
  using G = WGeo<L, J>;
  constexpr int D = 3, U = 6;
  const long warm = ((long)(G::H + kW - 1) / kW) * kW;
  const long seg = fast::pick_seg(N, batch, warm, kW, 8192);
  const long nseg = (N + seg - 1) / seg;
  long steps = seg / kW + warm / kW;
  steps = ((steps + U - 1) / U) * U;  // surplus steps extend the warm-up to the right
  const long ngroups = steps / U;
  const long a_start = (steps - 1) * kW;
  const size_t lds = (size_t)G::lds_pairs * sizeof(d2);
  auto kern = modwt_inv_wave<L, J, FMA, D, U>;
  JW_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
  const long cstride = (long)(J + 1) * N;
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    hipLaunchKernelGGL(kern, dim3((unsigned)nseg, (unsigned)nb), dim3(kW), lds, s,
                       c + (long)b0 * cstride, x + (long)b0 * N, N, seg, a_start, ngroups, t,
                       nf ? nf + b0 : nullptr);
  }
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

}  // namespace wave
}  // namespace jw
