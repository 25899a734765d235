// jw_crmath.cc -- correctly rounded sin / cos of a double, for the tables of the JW_ARITH_STRICT
// FFT paths (host only; built with g++, which has libquadmath).
//
// The reference evaluates Math.cos(angle) and Math.sin(angle) separately for every FFT stage
// twiddle (FastFourierTransform.java:189-190) and Bluestein chirp (:269-271).  Java specifies
// those to within 1 ulp; its implementations (fdlibm, the HotSpot intrinsics) return the
// correctly rounded value for all but a vanishing fraction of arguments.  glibc's double
// sin / cos / sincos do not always (measured: of the 2049 chirp angles of n = 2049, separate
// sin() misrounds one, sincos() another), so the engine (and the oracle, independently)
// use the correctly rounded value: an x87 long-double evaluation, rounded to double unless it
// lies within its error bound of a rounding boundary, else the quad-precision value.
#include <cmath>
#include <quadmath.h>

namespace jw {
namespace {
double cr_round(long double v, __float128 (*slow)(__float128), double x) {
  const double d = (double)v;
  if (v == 0.0L || !std::isfinite(d)) return d;
  // glibc's sinl / cosl are within a couple of 64-bit ulps; 16 is a safe bound
  const long double err = std::ldexp(1.0L, std::ilogb(v) - 63 + 4);
  const long double ld = d;
  const long double hi = (ld + (long double)std::nextafter(d, INFINITY)) / 2;   // exact midpoints
  const long double lo = (ld + (long double)std::nextafter(d, -INFINITY)) / 2;
  if (std::fabs(v - hi) > err && std::fabs(v - lo) > err) return d;
  return (double)slow((__float128)x);
}
}  // namespace

void cr_sincos(double x, double* s, double* c) {
  const long double xl = x;
  *s = cr_round(sinl(xl), sinq, x);
  *c = cr_round(cosl(xl), cosq, x);
}
}  // namespace jw
