// Host build of the fp64 engine's exp / log / constant-divisor division
// (topoflow-glacier_amd/csrc/tfg_fastmath.hpp) for tests/test_fastmath.py:
// the same source the device compiles, with std::fma for the scalar-operand
// FMAs.  Built by the test with g++ -O2 -ffp-contract=off (test infrastructure).
#include "../../topoflow-glacier_amd/csrc/tfg_fastmath.hpp"

extern "C" void fm_eval(const double* x, double* y, long n, int which) {
  for (long i = 0; i < n; ++i) {
    const double v = x[i];
    switch (which) {
      case 3: y[i] = tfg_fm::exp_k(v); break;
      case 5: y[i] = tfg_fm::log_k(v); break;
      case 7: y[i] = tfg_fm::div_k(v, 6.1121, 1.0 / 6.1121); break;
      case 8: y[i] = tfg_fm::div_k(v, 3600.0, 1.0 / 3600.0); break;
      case 10: y[i] = tfg_fm::fdiv(v, 7.3); break;
      case 11: y[i] = tfg_fm::fdiv(7.3, v); break;
      case 12: y[i] = tfg_fm::atan_q(v, 7.3); break;
      case 13: y[i] = tfg_fm::atan_q(-7.3, v); break;
      case 14: y[i] = tfg_fm::exp_p(v); break;
      case 15: y[i] = tfg_fm::log_p(v); break;
      case 16: y[i] = tfg_fm::exp_near(v); break;
      default: y[i] = 0.0; break;
    }
  }
}

// div_k(x[i], c[i], RN(1/c[i])) for arbitrary divisors
extern "C" void fm_div(const double* x, const double* c, double* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = tfg_fm::div_k(x[i], c[i], 1.0 / c[i]);
}

// fdiv(x[i], c[i]): the variable-divisor quotient
extern "C" void fm_fdiv(const double* x, const double* c, double* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = tfg_fm::fdiv(x[i], c[i]);
}

// fdiv_z(x[i], c[i]): fdiv with IEEE's quotient for a zero or infinite operand
extern "C" void fm_fdiv_z(const double* x, const double* c, double* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = tfg_fm::fdiv_z(x[i], c[i]);
}

// atan_q(x[i], c[i]): atan(x / c) from the two operands
extern "C" void fm_atan_q(const double* x, const double* c, double* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = tfg_fm::atan_q(x[i], c[i]);
}
