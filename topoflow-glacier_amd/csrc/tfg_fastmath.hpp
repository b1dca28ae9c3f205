// tfg_fastmath.hpp -- fp64 exp, log and division by a constant for the fp64
// ("exact") engine.  The fp64 step is issue-bound (HISTORY.md section 5: 1450
// VALU instructions per wave and cell-step at ~90 % of the vector pipe before
// this file); per step it evaluates eight exp, three log and about fifteen
// divisions by a model constant.
//
//   log_k(x)       an fp32 seed refined by one step on exp_k (round 5): within
//                  ~1e-15 absolute of numpy's log, ~27 VALU; fdlibm's log
//                  (log_fd: k ln2 + log1p(f), s = f/(2+f), degree-14
//                  polynomial, 1 ulp, ~40 VALU; the device libm's double-double
//                  log is ~100) for the rare arguments outside [2^-120, 2^120].
//   div_k(x, c, rc)  x / c for a constant c with rc = RN(1/c) known up front:
//                  q = RN(x rc), then one FMA correction step, which gives the
//                  correctly rounded quotient, IEEE division's result bit for
//                  bit (Markstein's theorem; tests/test_fastmath.py checks 1e6
//                  random pairs and the engine's divisors); 6 VALU instead of
//                  the 11 of the general sequence (v_div_scale x2, v_rcp, five
//                  FMAs, v_div_fmas, v_div_fixup).
//   exp_k(x)       the device libm's exp restated (Cody-Waite reduction, ldexp,
//                  the same overflow/underflow selects, here behind one test of
//                  |x|) with a degree-10 polynomial where the libm's is degree
//                  12: within 3 ulp of numpy's (round 5), and the host build
//                  below computes exactly what the device does.  Degree 9
//                  (1.7e-14, scripts/fit_exp.py) flips a melt gate of the fp64
//                  dark-test run against the oracle (round 5, not taken).
//   div_r(x, rc)   x / c as x * RN(1/c), within 1 ulp: every constant divisor
//                  whose last bit no melt-out gate reads (round 5).
//   fdiv(x, y)     x / y for a variable y: reciprocal, one Newton step, one
//                  correction of the quotient (within 1 ulp; round 5: one
//                  Newton step fewer than IEEE-exactness needs, +3.1 %).
//   atan_q(n, d)   atan(n / d) from the two operands: octant reduction, one
//                  fdiv, degree-9 polynomial in x^2 (within 2 ulp; round 5,
//                  the wet bulb's arctangent).
//
// Same-box A/B at 4096^2 (scripts/gpu_ab_f64.sh, profiles/r3f_ab_f64.log):
// 26.6 -> 31.2 G cell-updates/s (+17 %).  Holding exp's polynomial
// coefficients in SGPRs at every call site (the scalar operand of v_fma_f64
// instead of a v_mov pair feeding v_fmac_f64) saves ~60 more VALU instructions
// of the step but raises it from 118 to 144 VGPRs (3 instead of 4 waves per
// SIMD): 29.5 (profiles/r3e_ab_f64.log).  Round 5, with the rest of the step
// leaner, SGPR constants at every exp call site keep it at 128 VGPRs (4 waves)
// and gain 0.9 % (profiles/r5_ab_f64.json), so exp_k holds them in SGPRs
// everywhere (exp_kv, the VGPR form, stays for the device test that both give
// the same bits); log_k's constants are always scalar operands.  A table-driven exp (2^(j/64) from LDS or from a
// 1 KB global table, degree-5 expm1; within 1 ulp of numpy's) was measured and
// dropped: it raised the step to 152 VGPRs and its static VALU count
// (2430 -> 2450), and a global table load shares vmcnt with the step's forcing
// prefetch, so waiting for it waits for the prefetch too.
//
// The same functions compile for the host (g++), with std::fma in place of the
// scalar-operand FMA: tests/test_fastmath.py builds them and checks them
// against numpy's exp, log and division over the physics' ranges and the
// special values, and its GPU test checks that the device computes exactly
// what the host build does.  Every fp64 step (grid k_fused<double>, one-cell
// k_cell / k_cell_run / k_cell_many) calls these, so the one-cell kernels still
// equal the grid kernel bit for bit.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TFG_FM_HD __host__ __device__
#else
#define TFG_FM_HD
#endif
#include <cmath>
#include <cstdint>

// No FMA contraction inside these functions (HIP compiles with contraction on
// by default; the host build passes -ffp-contract=off): device and host then
// round every operation alike.
#if defined(__clang__)
#define TFG_FM_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define TFG_FM_NO_CONTRACT
#endif


namespace tfg_fm {

// A branch the compiler must keep (an empty volatile asm cannot be speculated
// into a select): for rare special-value fix-ups, which then cost one compare
// and a skipped branch instead of their selects on every call.
#if defined(__HIP_DEVICE_COMPILE__)
#define TFG_FM_RARE() asm volatile("")
#else
#define TFG_FM_RARE() ((void)0)
#endif

// d = a * b + c with b (fma_vsv) or c (fma_vvs) a wave-uniform constant held in
// an SGPR pair.  Host: std::fma.
TFG_FM_HD inline double fma_vsv(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
  return d;
#else
  return std::fma(a, b, c);
#endif
}
TFG_FM_HD inline double fma_vvs(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
#else
  return std::fma(a, b, c);
#endif
}
TFG_FM_HD inline double fma_vv(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(a, b, c);
#else
  return std::fma(a, b, c);
#endif
}

TFG_FM_HD inline double bits_to_double(uint64_t b) {
  union { uint64_t u; double d; } v{b};
  return v.d;
}

// ---------------------------------------------------------------------------
// exp: the device libm's exp (ROCm 7.2 device libs) as the compiler emits it
// for this engine (reduction constants read off its machine code), with a
// degree-10 polynomial fitted on [-ln2/2, ln2/2] (round 5) for its degree 12.
// ---------------------------------------------------------------------------
// SGPR = true: the polynomial coefficients and reduction constants as the
// scalar operand of v_fma_f64 (SALU moves beside the vector pipe, ~10 fewer
// VALU instructions), where the call site's register pressure allows it
// (exp_k; exp_kv holds them in VGPRs): the same results either way.
template <bool SGPR>
TFG_FM_HD inline double fk(double a, double b, double c) {  // b constant
  if constexpr (SGPR) return fma_vsv(a, b, c);
  else return fma_vv(a, b, c);
}
template <bool SGPR>
TFG_FM_HD inline double fp(double a, double b, double c) {  // c constant
  if constexpr (SGPR) return fma_vvs(a, b, c);
  else return fma_vv(a, b, c);
}
template <bool SGPR>
TFG_FM_HD inline double exp_impl(double x) {
  TFG_FM_NO_CONTRACT
  const double dn = std::rint(x * bits_to_double(0x3ff71547652b82feull));  // x / ln 2
  double t = fk<SGPR>(dn, bits_to_double(0xbfe62e42fefa39efull), x);              // - dn ln2_hi
  t = fk<SGPR>(dn, bits_to_double(0xbc7abc9e3b39803full), t);                     // - dn ln2_lo
  // degree 10 (round 5; the device libm's is 12): within 3 ulp of numpy's exp
  double p = fp<SGPR>(t, 0x1.2677102fbfba0p-22, 0x1.72ea1106c32a0p-19);
  p = fp<SGPR>(t, p, 0x1.a01c31bed4303p-16);
  p = fp<SGPR>(t, p, 0x1.a0198c587737fp-13);
  p = fp<SGPR>(t, p, 0x1.6c16c077e694ap-10);
  p = fp<SGPR>(t, p, 0x1.11111126084c0p-7);
  p = fp<SGPR>(t, p, 0x1.55555555a61c8p-5);
  p = fp<SGPR>(t, p, 0x1.555555555059ap-3);
  p = fp<SGPR>(t, p, 0x1.ffffffffffdf2p-2);
  p = fma_vv(t, p, 1.0);
  p = fma_vv(t, p, 1.0);
#if defined(__HIP_DEVICE_COMPILE__)
  const int k = (int)dn;  // v_cvt_i32_f64 saturates
#else
  const int k = (int)std::fmin(std::fmax(dn, -2147483648.0), 2147483647.0);
#endif
  double z = std::ldexp(p, k);
  // overflow, underflow, +-inf and NaN (rare): one test on the common path
  if (__builtin_expect(!(std::fabs(x) <= 708.0), 0)) {
    TFG_FM_RARE();
    z = (x > 1024.0) ? (double)INFINITY : z;
    z = (x < -1075.0) ? 0.0 : z;
  }
  return z;
}
TFG_FM_HD inline double exp_k(double x) { return exp_impl<true>(x); }
TFG_FM_HD inline double exp_kv(double x) { return exp_impl<false>(x); }

// ---------------------------------------------------------------------------
// exp sized for the fp32 engine's fp64-flux form (round 6): that form needs its
// flux terms within ~1e-9 (a per-step error of 2e-8 of the
// flux magnitudes is what the year-long run tolerates), not exp_k's 3 ulp.
// One-constant Cody-Waite reduction (|dn ln2_lo| < 1e-13 for |x| <= 708) and a
// degree-7 polynomial (scripts/fit_exp.py 7: 5.2e-11 relative): 4 VALU fewer.
// ---------------------------------------------------------------------------
TFG_FM_HD inline double exp_p(double x) {
  TFG_FM_NO_CONTRACT
  const double dn = std::rint(x * bits_to_double(0x3ff71547652b82feull));  // x / ln 2
  const double t = fma_vsv(dn, bits_to_double(0xbfe62e42fefa39efull), x);   // - dn ln2
  double p = fma_vvs(t, 0x1.9f08a47c8a105p-13, 0x1.6d8cf41dff604p-10);
  p = fma_vvs(t, p, 0x1.1112708f1c74dp-7);
  p = fma_vvs(t, p, 0x1.55548dd8721c5p-5);
  p = fma_vvs(t, p, 0x1.5555544365d72p-3);
  p = fma_vvs(t, p, 0x1.0000003a1adefp-1);
  p = fma_vv(t, p, 1.0);
  p = fma_vv(t, p, 1.0);
#if defined(__HIP_DEVICE_COMPILE__)
  const int k = (int)dn;
#else
  const int k = (int)std::fmin(std::fmax(dn, -2147483648.0), 2147483647.0);
#endif
  double z = std::ldexp(p, k);
  if (__builtin_expect(!(std::fabs(x) <= 708.0), 0)) {
    TFG_FM_RARE();
    z = (x > 1024.0) ? (double)INFINITY : z;
    z = (x < -1075.0) ? 0.0 : z;
  }
  return z;
}

// exp(c + s) / exp(c) for |s| <= 0.41 (the flux form's lhc / p0 factor,
// exp(-M g elev / (R T_K)) with its exponent y in [-0.755, 0.065] centred at
// c = kP0Center, so elevations up to ~5 km at any air temperature): a degree-8
// polynomial in s with no reduction (scripts/fit_exp.py 8 on [-0.41, 0.41]:
// 5.1e-12 relative), 8 VALU for exp_p's 12.  The caller folds exp(c) into its
// constant factor and takes exp_p for a wave with a lane outside the range.
constexpr double kP0Center = -0.345;
constexpr double kP0Half = 0.41;
TFG_FM_HD inline double exp_near(double s) {
  TFG_FM_NO_CONTRACT
  double p = fma_vvs(s, 0x1.9deba1dca22f8p-16, 0x1.a215e42a84b4ep-13);
  p = fma_vvs(s, p, 0x1.6c1acb31a393fp-10);
  p = fma_vvs(s, p, 0x1.1110390688b5dp-7);
  p = fma_vvs(s, p, 0x1.5555520449441p-5);
  p = fma_vvs(s, p, 0x1.555555c3933f1p-3);
  p = fma_vvs(s, p, 0x1.0000000166a91p-1);
  p = fma_vv(s, p, 1.0);
  return fma_vv(s, p, 1.0);
}

// ---------------------------------------------------------------------------
// log: fdlibm e_log.c's reduction and polynomial (Lg1..Lg7), one formula for
// every argument, FMA Horner, s = f / (2 + f) by a Newton reciprocal.
// ---------------------------------------------------------------------------
TFG_FM_HD inline double rcp_approx(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcp(d);  // v_rcp_f64
#else
  return (double)(1.0f / (float)d);  // a coarser seed than the device's: two Newton steps cover both
#endif
}

TFG_FM_HD inline double log_fd(double x) {
  TFG_FM_NO_CONTRACT
#if defined(__HIP_DEVICE_COMPILE__)
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1) for finite nonzero x
  int k = __builtin_amdgcn_frexp_exp(x);
#else
  int k = 0;
  double m = std::frexp(x, &k);
#endif
  const bool lo = m < bits_to_double(0x3fe6a09e667f3bcdull);  // sqrt(1/2)
  m = lo ? m + m : m;
  k = lo ? k - 1 : k;
  const double f = m - 1.0;  // [sqrt(1/2) - 1, sqrt(2) - 1), exact
  const double d = f + 2.0;
  double r = rcp_approx(d);
  r = fma_vv(fma_vv(-d, r, 1.0), r, r);
  r = fma_vv(fma_vv(-d, r, 1.0), r, r);
  const double s = f * r;
  const double dk = (double)k;
  const double z = s * s, w = z * z;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  const double t1 = w * fma_vvs(w, fma_vsv(w, Lg6, Lg4), Lg2);
  const double t2 = z * fma_vvs(w, fma_vvs(w, fma_vsv(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  double y = fma_vsv(dk, ln2_hi, -((hfsq - fma_vv(s, hfsq + R, dk * ln2_lo)) - f));
  // special values (rare: one test on the common path): log(+-0) = -inf, log(x < 0) = NaN,
  // log(+inf) = +inf; NaN propagates through the above
  if (__builtin_expect(!(x > 0.0 && x < (double)INFINITY), 0)) {
    TFG_FM_RARE();
    y = (x == 0.0) ? -(double)INFINITY : y;
    y = (x < 0.0) ? (double)NAN : y;
    y = (x == (double)INFINITY) ? x : y;
  }
  return y;
}

// ---------------------------------------------------------------------------
// x / c for a constant c, rc = RN(1/c) (a literal 1.0 / c, or a reciprocal the
// host computed in fp64): correctly rounded, like the IEEE division.  Where the
// residual is zero (q exact, including x = +-0) or NaN (x infinite or NaN) the
// first product is already the quotient (and keeps -0 and +-inf).
// ---------------------------------------------------------------------------
TFG_FM_HD inline double div_k(double x, double c, double rc) {
  TFG_FM_NO_CONTRACT
  const double q = x * rc;
  const double e = fma_vv(-q, c, x);
  const double q1 = fma_vv(e, rc, q);
  return (e < 0.0 || e > 0.0) ? q1 : q;
}

// ---------------------------------------------------------------------------
// log (round 5, sized for ~1e-15 absolute): an fp32 seed y0 (v_log_f32, ~1e-7)
// refined by one step on exp, y = y0 + log1p(x e^-y0 - 1) with log1p(d) = d -
// d^2/2 (|d| ~ 1e-6, so the cubic term is below 1e-18): one exp_k instead of
// fdlibm's reduction and degree-14 polynomial.  Its error is exp_k's, ~1e-15
// absolute; relative near log x = 0 that is looser than fdlibm's 1 ulp
// (tests/test_fastmath.py bounds it absolutely).  Outside [2^-120, 2^120]
// (0, denormals, huge, negative, inf, NaN: rare) fdlibm's log_fd.
// ---------------------------------------------------------------------------
TFG_FM_HD inline double log_k(double x) {
  TFG_FM_NO_CONTRACT
#if defined(__HIP_DEVICE_COMPILE__)
  const double y0 = (double)__builtin_amdgcn_logf((float)x) * 0.69314718055994531;
#else
  const double y0 = (double)std::log2((float)x) * 0.69314718055994531;
#endif
  const double d = fma_vv(x, exp_k(-y0), -1.0);
  double y = y0 + fma_vv(-0.5 * d, d, d);
  if (__builtin_expect(!(x >= 0x1p-120 && x < 0x1p120), 0)) {
    TFG_FM_RARE();
    y = log_fd(x);
  }
  return y;
}

// log_k's form on exp_p (the fp64-flux form's dew point, round 6): within
// ~6e-11 absolute (exp_p's error carried into the correction), 4 VALU fewer.
TFG_FM_HD inline double log_p(double x) {
  TFG_FM_NO_CONTRACT
#if defined(__HIP_DEVICE_COMPILE__)
  const double y0 = (double)__builtin_amdgcn_logf((float)x) * 0.69314718055994531;
#else
  const double y0 = (double)std::log2((float)x) * 0.69314718055994531;
#endif
  const double d = fma_vv(x, exp_p(-y0), -1.0);
  double y = y0 + fma_vv(-0.5 * d, d, d);
  if (__builtin_expect(!(x >= 0x1p-120 && x < 0x1p120), 0)) {
    TFG_FM_RARE();
    y = log_fd(x);
  }
  return y;
}

// x / c for a constant c as x * RN(1/c): within 1 ulp of the quotient, 1 VALU.
// For every division by a model constant whose last bit does not decide a
// melt-out gate (round 5: the fp64 engine is held to 1e-12 of the reference,
// not to its last bit); div_k keeps the correctly rounded quotient where the
// reference's h - (h/3600) dt 3600 residual is read by an exact-zero test.
TFG_FM_HD inline double div_r(double x, double rc) {
  TFG_FM_NO_CONTRACT
  return x * rc;
}

// ---------------------------------------------------------------------------
// x / y for a variable y: the reciprocal from rcp_approx and one Newton step
// (relative error ~2^-46 from either seed), q = RN(x r), and one correction
// q + (x - q y) r, whose error is that of r times |q - x/y| -- IEEE's quotient
// but for rare last-bit cases (tests/test_fastmath.py: within 1 ulp of numpy's,
// equal in > 99.9 %), 6 VALU instead of the 11 of the general sequence
// (v_div_scale x2, v_rcp, five FMAs, v_div_fmas, v_div_fixup).  For finite x and finite nonzero y (every
// quotient of the physics); NaN propagates.  A zero or infinite operand gives
// NaN, where IEEE gives inf or 0: fdiv_z below for a divisor that can be zero.
// ---------------------------------------------------------------------------
TFG_FM_HD inline double fdiv(double x, double y) {
  TFG_FM_NO_CONTRACT
  double r = rcp_approx(y);
  r = fma_vv(fma_vv(-y, r, 1.0), r, r);
  const double q = x * r;
  return fma_vv(fma_vv(-q, y, x), r, q);
}

// fdiv with IEEE's result for a zero or infinite operand (round 6): where the
// divisor can be zero in the physics -- kappa / log((z - h_snow)/z0) of :670 at
// h_snow = z - z0, where the reference's quotient is inf -- fdiv's NaN is
// replaced by the IEEE quotient behind one rare test (NaN operands stay NaN).
TFG_FM_HD inline double fdiv_z(double x, double y) {
  double q = fdiv(x, y);
  if (__builtin_expect(q != q, 0)) {
    TFG_FM_RARE();
    q = x / y;
  }
  return q;
}

// ---------------------------------------------------------------------------
// atan(n / d) from the two operands, with one quotient (round 5; the wet
// bulb's atan((T + 1.676331) / (1 + (T + RH)(RH - 1.676331)))): the octant of
// |n / d| picks x = a / b, (a - b) / (a + b) or -b / a (a = |n|, b = |d|), so
// |x| <= tan(pi/8) and atan(|n / d|) = off + atan(x), off = 0, pi/4 or pi/2
// (hi + lo); atan(x) = x + x z Q(z), z = x^2, Q of degree 9 fitted by
// scripts/fit_atan.py (6.8e-17 before rounding).  Within 2 ulp of the
// arctangent of the exact quotient (tests/test_fastmath.py); d = 0 gives
// +-pi/2, n = d = 0 NaN.
// The device libm's atan(u) takes an IEEE division 1 / |u| and a degree-19
// polynomial on top of the quotient u.
// ---------------------------------------------------------------------------
TFG_FM_HD inline double atan_q(double n, double d) {
  TFG_FM_NO_CONTRACT
  const double a = std::fabs(n), b = std::fabs(d);
  const bool lo = a <= 0x1.a827999fcef32p-2 * b;  // tan(pi/8)
  const bool hi = a > 0x1.3504f333f9de6p+1 * b;   // tan(3 pi/8)
  const double num = lo ? a : (hi ? -b : a - b);
  const double den = lo ? b : (hi ? a : a + b);
  const double x = fdiv(num, den);
  const double z = x * x;
  double q = fma_vvs(z, 0x1.624ab16a6dac3p-6, -0x1.67e25b96c8da4p-5);
  q = fma_vvs(z, q, 0x1.d370891418ab2p-5);
  q = fma_vvs(z, q, -0x1.10245f5158aa3p-4);
  q = fma_vvs(z, q, 0x1.3b005b34c39e4p-4);
  q = fma_vvs(z, q, -0x1.745c1a89d2fd5p-4);
  q = fma_vvs(z, q, 0x1.c71c6a2c4a0ecp-4);
  q = fma_vvs(z, q, -0x1.249249155d429p-3);
  q = fma_vvs(z, q, 0x1.999999998297dp-3);
  q = fma_vvs(z, q, -0x1.5555555555555p-2);
  const double r = fma_vv(x * z, q, x);
  const double off_hi = lo ? 0.0 : (hi ? 0x1.921fb54442d18p+0 : 0x1.921fb54442d18p-1);
  const double off_lo = lo ? 0.0 : (hi ? 0x1.1a62633145c07p-54 : 0x1.1a62633145c07p-55);
  const double t = off_hi + (r + off_lo);
  return (std::signbit(n) != std::signbit(d)) ? -t : t;
}

}  // namespace tfg_fm
