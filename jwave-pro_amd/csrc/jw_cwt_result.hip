// jw_cwt_result.hip -- CWTResult's accessors on the device (src/main/java/jwave/transforms/
// CWTResult.java:94-126 getMagnitude / getPhase, :272-287 getScalogram), so a scalogram of a
// device-resident CWT never pulls the B x ns x n complex coefficients to the host.
//
// Built with -ffp-contract=off: |c| = sqrt(re*re + im*im) in Complex.getMag's order
// (Complex.java:202-204; the f64 sqrt is correctly rounded, as Math.sqrt), so the magnitude
// is bit-identical to Java.  The phase follows Complex.getPhi's quadrant rules (:213-226) with
// the device atan (within an ulp of StrictMath's).  The scalogram sums mag*mag per row in a
// tree rather than Java's left-to-right loop: equal to ~1e-15 relative, not bitwise.
#include <cmath>

#include "jw_internal.hpp"

namespace jw {
namespace {

constexpr double kPi = 3.14159265358979323846;

__device__ __forceinline__ double cmag(double2 c) { return sqrt(c.x * c.x + c.y * c.y); }

__global__ __launch_bounds__(256) void magnitude_kernel(const double2* __restrict__ c, long count,
                                                        double* __restrict__ out) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < count; i += (long)gridDim.x * 256)
    out[i] = cmag(c[i]);
}

// Complex.getPhi (degrees) * Math.PI / 180.0 (CWTResult.getPhase :121)
__device__ __forceinline__ double cphase(double2 c) {
  const double r = c.x, j = c.y;
  if (r == 0.0 && j == 0.0) return 0.0;
  const double phi = atan(fabs(j / r)) * (180.0 / kPi);  // Math.toDegrees
  double d;
  if (r >= 0.0 && j >= 0.0) {
    d = phi;
  } else if (r <= 0.0 && j >= 0.0) {
    d = 180.0 - phi;
  } else if (r <= 0.0 && j <= 0.0) {
    d = phi + 180.0;
  } else if (r >= 0.0 && j <= 0.0) {
    d = 360.0 - phi;
  } else {
    d = phi;  // NaN parts fall through, as in Java
  }
  return d * kPi / 180.0;
}

__global__ __launch_bounds__(256) void phase_kernel(const double2* __restrict__ c, long count,
                                                    double* __restrict__ out) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < count; i += (long)gridDim.x * 256)
    out[i] = cphase(c[i]);
}

// One workgroup per row: strided partial sums of mag*mag, then a wave reduction through DPP
// shuffles and one LDS word per wave.
__global__ __launch_bounds__(256) void scalogram_kernel(const double2* __restrict__ c, long n,
                                                        double* __restrict__ energy) {
  __shared__ double part[4];
  const double2* row = c + (long)blockIdx.x * n;
  double acc = 0.0;
  for (long t = threadIdx.x; t < n; t += 256) {
    const double m = cmag(row[t]);
    acc += m * m;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) energy[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

unsigned grid_for(long count) {
  const long g = (count + 255) / 256;
  return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace

int cwt_magnitude_device(const double* c, long count, double* out, hipStream_t s) {
  hipLaunchKernelGGL(magnitude_kernel, dim3(grid_for(count)), dim3(256), 0, s, (const double2*)c,
                     count, out);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

int cwt_phase_device(const double* c, long count, double* out, hipStream_t s) {
  hipLaunchKernelGGL(phase_kernel, dim3(grid_for(count)), dim3(256), 0, s, (const double2*)c,
                     count, out);
  JW_HIP_TRY(hipGetLastError());
  return JW_OK;
}

int cwt_scalogram_device(const double* c, long rows, long n, double* energy, hipStream_t s) {
  for (long r0 = 0; r0 < rows; r0 += 0x7fffffffL) {
    const long cnt = rows - r0 < 0x7fffffffL ? rows - r0 : 0x7fffffffL;
    hipLaunchKernelGGL(scalogram_kernel, dim3((unsigned)cnt), dim3(256), 0, s,
                       (const double2*)c + r0 * n, n, energy + r0);
    JW_HIP_TRY(hipGetLastError());
  }
  return JW_OK;
}

}  // namespace jw
