// tfg_physics.hpp -- per-cell glacier energy balance, device side (gfx950).
//
// One call of cell_step_* advances ONE cell by ONE time step: the body of
// BmiTopoflowGlacier.update() (bmi_topoflow_glacier.py:413-465) after the
// per-step uniform scalars have been hoisted to the host (tfg_uniforms).
//
// Two variants share the state layout:
//   cell_step_exact  fp64 everywhere, the reference's operation order, FMA
//                    contraction off.  Used for single-catchment BMI runs
//                    (float64 BMI surface, golden parity ~1e-13).
//   cell_step_fast   fp32 forcing/static/outputs and fp32 flux arithmetic,
//                    fp64 state update (cold contents, SWE/IWE, integrals) and
//                    fp64 evaluation of the discontinuity predicates (rain/snow
//                    split, depth tests, dark mask near sunrise/sunset).
//
// Elementwise rules for the reference's scalar-only branches:
// bot==0 (:642), T_air==T_surf / Ri>0 (:672-726), dark (SF:939-941) are
// evaluated per cell.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "tfg_fastmath.hpp"

namespace tfg {

using tfg_fm::div_k;
using tfg_fm::div_r;
using tfg_fm::fdiv;
using tfg_fm::exp_k;
using tfg_fm::log_k;
using tfg_fm::atan_q;

// Earth_Angular_Velocity() (SF:252) [rad/h] and its correctly rounded
// reciprocal (the divisor of the sunrise/sunset offsets, SF:783-830).
constexpr double kOmega = (360.0 / 24.0) * (3.141592653589793 / 180.0);
constexpr double kInvOmega = 1.0 / kOmega;

// ---------------------------------------------------------------------------
// Constants derived on the host (fp64) from tfg_params, in the reference's
// association order where it matters.
// ---------------------------------------------------------------------------
struct DevParams {
  double dt, da_m2, T_rs, dust, F, one_minus_F_172, cloud_term;
  double rho_snow_Cp_snow;    // (rho_snow*Cp_snow)               :1533
  double rho_air_Cp_air;      // (rho_air*Cp_air)                 :745
  double rho_air_Lv;          // rho_air*Lv                        :932
  double rho_H2O_Lf;          // (rho_H2O*Lf)                      :1368
  double lhc_100_p0;          // lhc*100/sea_p0: lhc/p0 = lhc_100_p0*exp(-x_p0)   :551-556, :931
  double inv_6p11, negM_g, R; // RN(1/(0.611*10)): RH = e_air*exp(-x_es)*inv_6p11 (:788-802, :838); -M*g, R_star  :552
  double eps, one_minus_eps;  // :817
  double gz;                  // g*z (z = 10 m)                    :640
  double z, kappa, z0;        // :670
  double em_surf_sigma, sigma, one_minus_em_surf;
  double inv_rho_H2O_Lf;      // RN(1/(rho_H2O*Lf)): div_k of :1368, :1428
  double negM_g_R;            // -M*g/R_star: the pressure exponent's factor    :552
  double T0;                  // T0_cc                             :389
  double Ecci0;               // initial ice cold content          :394-395
  double inv_dt, inv_dt_rhoLf, inv_z0;  // reciprocals (fast variant; inv_dt, inv_z0 also div_k's)
  double ws, wi;              // rho_H2O/rho_snow, rho_H2O/rho_ice :385-386
  double days_per_dt;         // dt/86400                          :287
  double sin_lat, cos_lat;    // of lat*(pi/180)                   SF:730-733
  double omega;               // Earth_Angular_Velocity()          SF:252
  double pi_over_180, c180_over_pi, half_pi, twopi;
  double qscale;              // 2^36: snowfall-window fixed point
  int64_t thr_q;              // ceil(0.03 * 2^36)                 :1040
  int32_t satterlund;
  int32_t ring_len;
  // fast variant: fp64 folds
  double c_sm3600;            // 3600/(dt*rho_H2O*Lf): SM*3600 from E_rem     :1368, :1598
  double dt3600;              // dt*3600                                      :1599, :1615
  // fast variant: fp32 constants, folded on the host in fp64
  float f_T_rs_dn;            // largest float <= T_rain_snow (exact T > T_rs test)
  float f_eps100, f_ome100;   // 100*eps, 100*(1-eps)                        :817-826
  float f_gz, f_z;            // g*z, z                                       :640, :670
  float f_k2;                 // (kappa/ln 2)^2                               :670-672
  float f_rho_air_Cp_air;     // :744
  float f_qe;                 // rho_air*Lv*lhc*100/sea_p0: Qe = f_qe*Dh*de*exp(Mg elev/(R T))  :931-934, :551-556
  float f_dust, f_1pdust;     // dust_atten, 1 + dust_atten                  SF:610, SF:652
  float f_em_surf_sigma;      // em_surf*sigma: Qn_LW = em_s*sigma*(em_air*Ta^4 - Ts^4)  :1231-1248
  float f_qfac;               // dt*ws*2^36: snowfall-window slot scale
  float f_dt, f_T0;
  float f_c_eccs;             // rho_snow*Cp_snow*dt*ws                       :1527-1533
  // scaled logarithm arguments (v_log_f32's -0.44 ulp bias is of its RESULT, so
  // arguments scaled by a power of two to ~1 keep it off the energy terms)
  float f_inv_z0s;            // 2^-k / z0: roughness log log2((z - h)/z0) = log2((z - h) f_inv_z0s) + k   :670
  float f_l2k2, f_l2kk;       // 2k, k^2
  float f_l2min;              // 0.01 * 2^-k: the clamp of :670 on the scaled argument
  float f_em_sc;              // 0.1 * 2^10: em_air's (e/T)^(1/7) = (e f_em_sc / T)^(1/7) 2^(-10/7)  :1167
  float f_ccFs;               // (1-F)*1.72*(1+0.22C^2) * 2^(-10/7)            :1167-1175
  float f_Fm1;                // F - 1: em_air - 1 for the long-wave balance
  // fast variant's fp64 turbulent chain (round 6)
  double d_eps100, d_ome100;  // 100 eps, 100 (1 - eps): e_air [mbar] = Q P_air / (d_eps100 + d_ome100 Q)   :817-826
  double d_k2;                // (kappa / ln 2)^2: Dn = uz d_k2 / log2((z - h)/z0)^2                       :670-672
  double d_l2k, d_l2kk;       // k, k^2 of the scaled roughness log (f_inv_z0s)
  double d_qe;                // rho_air Lv lhc 100 / sea_p0 exp(kP0Center) (the flux form's exp_near)    :931-934
  double d_es_k, d_es_c;      // e_sat(T_s) / e_sat(T_a) = exp(-d_es_k dTs / ((T_s + c)(T_a + c))), c = d_es_c  :788-807
};

// Per-cell static quantities derived from elev/slope/aspect (set_aspect_angle
// :1082-1093, set_slope_angle :1095-1113, Equivalent_Latitude SF:741,
// Longitude_Offset SF:718, Noon_Offset_Slope SF:772).
struct CellStatic {
  double elev;
  double cos_leq, sin_leq;  // of lat_eq [rad]                      SF:866-868
  double dlon;              // Longitude_Offset [rad]                SF:864
  double tan_eq;            // tan(eq_lat_deg*(pi/180))             SF:325
  double cos_dlon, sin_dlon;  // of dlon: cos(omega*th + dlon) by the angle-sum identity
};
constexpr int kStaticPlanes = 7;  // k_prepare_static's fp64 planes, in CellStatic order

// Noon_Offset_Slope (SF:776) [h], in the reference's operation order; needed
// only where the dark test falls back to the reference's form.
__device__ __forceinline__ double noon_offset(const DevParams& p, double dlon) { return -1.0 * dlon / p.omega; }

// Per-cell model state carried between steps (fp64).
struct CellState {
  double h_swe, h_iwe, Eccs, Ecci, n, albedo;
  double h_snow, h_ice;     // previous-step depths
  int64_t tot_q;            // snowfall-window running total, fixed point
};

struct CellOut {
  double h_snow, SM, h_ice, IM, M_total, RH;
};

struct CellDiag {
  double P, PR, PS, SM, IM, Pmax;
};

// numpy np.maximum / np.minimum: NaN-propagating
template <class R> __device__ __forceinline__ R npmax(R a, R b) { return (a >= b || a != a) ? a : b; }
template <class R> __device__ __forceinline__ R npmin(R a, R b) { return (a <= b || a != a) ? a : b; }

// numpy float remainder (npy_divmod) for b > 0
__device__ __forceinline__ double pyremainder(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0.0) != (m < 0.0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}

// Snowfall-window slot value in fixed point (2^-36 quantum, saturating).
// The reference keeps a ring of int(72/dt) float64 values and re-sums it each
// step (:1027-1041); only the predicate sum >= 0.03 is used.  A fixed-point
// running total decides it exactly up to ring_len*2^-37 (< 2.2e-9 at 288
// slots), with no drift.
//
// Missing data: a NaN snowfall (NaN forcing P) makes the reference's window
// sum NaN for as long as the slot stays in the ring, and then neither
// np.where of :1040-1041 fires, so n freezes.  A NaN slot is stored as the
// sentinel kWindowNan (no finite value quantises to it) and counts
// kWindowNanTot in the running total: |sum of finite slots| < 288 * 2^31 <
// 2^40, so the total is >= 2^43 exactly while a NaN slot is in the window.
constexpr int32_t kWindowNan = (int32_t)0x80000000;
constexpr int64_t kWindowNanTot = (int64_t)1 << 44;
constexpr int64_t kWindowNanMin = (int64_t)1 << 43;
__device__ __forceinline__ int32_t window_q(double v, double qscale) {
  double s = v * qscale;
  if (!(s == s)) return kWindowNan;
  if (s > 2147483647.0) return 2147483647;
  if (s < -2147483647.0) return -2147483647;
  return (int32_t)__double2ll_rn(s);
}
// A slot's contribution to the running total.
__device__ __forceinline__ int64_t window_tot(int32_t q) { return q == kWindowNan ? kWindowNanTot : (int64_t)q; }
// Days since the last major snowfall (:1040-1041): reset where the window
// total reaches 0.03 m, advanced where it stays below, unchanged while the
// total is NaN (a NaN slot in the window).
__device__ __forceinline__ double window_days(double n, int64_t tot_q, int64_t thr_q, double days_per_dt) {
  return tot_q >= kWindowNanMin ? n : (tot_q >= thr_q ? 0.0 : n + days_per_dt);
}

// ---------------------------------------------------------------------------
// Static derivation (once per launch per cell).
// ---------------------------------------------------------------------------
__device__ inline CellStatic derive_static(const DevParams& p, double elev, double slope, double aspect) {
#pragma clang fp contract(off)
  CellStatic s;
  s.elev = elev;
  // set_aspect_angle (:1086-1091): aspect in DEGREES used as radians (quirk)
  double alpha = p.half_pi - aspect;
  alpha = pyremainder(p.twopi + alpha, p.twopi);
  if (!isfinite(alpha)) alpha = 0.0;
  // set_slope_angle (:1099-1104); out-of-range beta is rejected at upload
  double beta = atan(slope);
  beta = pyremainder(p.twopi + beta, p.twopi);
  if (!isfinite(beta)) beta = 0.0;
  const double sb = sin(beta), cb = cos(beta), sa = sin(alpha), ca = cos(alpha);
  // Equivalent_Latitude SF:753-757
  const double t1 = sb * ca * p.cos_lat;
  const double t2 = cb * p.sin_lat;
  const double lat_eq = asin(t1 + t2);
  // Longitude_Offset SF:730-734
  const double u1 = sb * sa;
  const double u2 = cb * p.cos_lat;
  const double u3 = sb * p.sin_lat * ca;
  const double dlon = atan(u1 / (u2 - u3));
  s.dlon = dlon;
  s.cos_dlon = cos(dlon);
  s.sin_dlon = sin(dlon);
  s.cos_leq = cos(lat_eq);
  s.sin_leq = sin(lat_eq);
  // Sunrise_Offset(eq_lat_deg, ...) SF:320-325: degrees and back
  const double eq_lat_deg = lat_eq * p.c180_over_pi;
  s.tan_eq = tan(eq_lat_deg * p.pi_over_180);
  return s;
}

// Sunrise/sunset offsets on the slope (SF:783-830), fp64.
__device__ __forceinline__ void slope_sun_offsets(const DevParams& p, const CellStatic& s, double tan_d,
                                                  double flat_sr, double flat_ss, double& T_sr,
                                                  double& T_ss) {
#pragma clang fp contract(off)
  double arg = -1.0 * s.tan_eq * tan_d;
  arg = npmin(npmax(-1.0, arg), 1.0);
  const double ac = acos(arg);
  const double t_sr = div_k(-1.0 * ac, p.omega, kInvOmega);
  const double t_ss = div_k(ac, p.omega, kInvOmega);
  const double t_noon = noon_offset(p, s.dlon);
  T_sr = npmax(t_sr + t_noon, flat_sr);
  T_ss = npmin(t_ss + t_noon, flat_ss);
}

// cos(omega*th + dlon) (SF:867) from the step's cos/sin(omega*th) and the
// cell's cos/sin(dlon): absolute error ~4e-16 against the reference's
// cos of the rounded sum, one multiply and one multiply-subtract instead of a
// libm cos.
__device__ __forceinline__ double cos_hour_angle(const CellStatic& s, const tfg_uniforms& u) {
#pragma clang fp contract(off)
  return u.cos_wth * s.cos_dlon - u.sin_wth * s.sin_dlon;
}

// The dark test of Clear_Sky_Radiation (SF:939-941): th <= T_sr or th >= T_ss
// with T_sr = max(-ac/omega + t_noon, flat_sr), T_ss = min(ac/omega + t_noon,
// flat_ss), ac = acos(clip(-tan(lat_eq) tan(d))), t_noon = -dlon/omega.  With
// x = omega*th + dlon = omega*(th - t_noon):
//   dark  <=>  flat_dark  or  |x| >= ac  <=>  flat_dark or |x| > pi or cos(x) <= cos(ac) = arg,
// flat_dark (th <= flat_sr or th >= flat_ss) being decided on the host.  The
// reference's own rounding moves the boundary by < 1e-15 in cos(x) (and |x|),
// so outside a 1e-12 margin the cosine form decides as the reference does;
// inside it (a cell-step within ~1e-12 of sunrise or sunset on its slope) the
// reference's form runs: acos and the offsets, as slope_sun_offsets.
__device__ __forceinline__ bool sun_down(const DevParams& p, const CellStatic& s, const tfg_uniforms& u,
                                         double cos_wl) {
#pragma clang fp contract(off)
  if (u.flat_dark) return true;
  const double arg = npmin(npmax(-1.0, -1.0 * s.tan_eq * u.tan_d), 1.0);
  const double dv = cos_wl - arg;
  const double dpi = fabs(u.omega_th + s.dlon) - 3.141592653589793;
  if (fabs(dv) > 1e-12 && fabs(dpi) > 1e-12) return dpi > 0.0 || dv < 0.0;
  double T_sr, T_ss;
  slope_sun_offsets(p, s, u.tan_d, u.flat_sr, u.flat_ss, T_sr, T_ss);
  return (u.th <= T_sr) || (u.th >= T_ss);
}

// ---------------------------------------------------------------------------
// State update after the net energy flux (fp64, reference order).
// :1566-1731 -- shared by both variants.
// ---------------------------------------------------------------------------
// RAW (the grid kernel, round 6): the diagnostics gather SM and IM unscaled;
// k_fused applies da dt 3600 to the launch's sums (diag_scale).
template <bool RAW = false>
__device__ __forceinline__ void melt_and_mass(const DevParams& p, double Q_sum, double P_snow,
                                              double P_rain, double RH, double T_wb,
                                              CellState& st, CellOut& o,
                                              CellDiag& d, bool valid) {
#pragma clang fp contract(off)
  const double dt = p.dt;
  const double previous_swe = st.h_swe;  // :1566-1571
  // update_snow_meltrate :1364-1373
  double E_in = Q_sum * dt;
  double E_rem = npmax(E_in - st.Eccs, 0.0);
  double SM = div_r(div_r(E_rem, p.inv_dt), p.inv_rho_H2O_Lf);
  // enforce_max_snow_meltrate :1447-1465 -- only max(SM,0) executes; the
  // min(SM, h_swe/dt) lines are inside the method's docstring.
  // an identity where 1/dt and 1/(rho_H2O Lf) are > 0 (E_rem >= 0 or NaN): skipped there (round 6)
  const bool scale_pos = p.inv_dt > 0.0 && p.inv_rho_H2O_Lf > 0.0;
  if (!scale_pos) SM = npmax(SM, 0.0);
  // update_SM_integral :1486
  if (valid) {
    if constexpr (RAW) d.SM += SM;
    else d.SM += SM * p.da_m2 * dt * 3600.0;
  }
  // update_swe :1594-1606
  double h_swe = st.h_swe + P_snow * dt;
  double t = npmin(SM * 3600.0, h_swe);
  SM = div_k(t, 3600.0, 1.0 / 3600.0);
  h_swe = h_swe - SM * dt * 3600.0;
  h_swe = npmax(h_swe, 0.0);
  // update_snowfall_cold_content :1507-1537
  double Eccs = st.Eccs;
  if (P_snow > 0.0) {
    const double new_h_snow = (P_snow * dt) * p.ws;
    const double del_T = p.T0 - T_wb;
    Eccs = npmax(Eccs + p.rho_snow_Cp_snow * new_h_snow * del_T - E_in, 0.0);
  }
  // update_ice_meltrate :1418-1434
  E_rem = npmax(E_in - st.Ecci, 0.0);
  double IM = div_r(div_r(E_rem, p.inv_dt), p.inv_rho_H2O_Lf);
  if (!scale_pos) IM = npmax(IM, 0.0);
  IM = (h_swe == 0.0 && previous_swe == 0.0) ? IM : 0.0;
  double Ecci = npmax(st.Ecci - E_in, 0.0);
  Ecci = (st.h_ice == 0.0) ? 0.0 : Ecci;  // previous-step h_ice
  // enforce_max_ice_meltrate :1473-1480
  IM = npmin(IM, div_k(st.h_iwe, dt, p.inv_dt));
  IM = npmax(IM, 0.0);
  // update_IM_integral :1493
  if (valid) {
    if constexpr (RAW) d.IM += IM;
    else d.IM += IM * p.da_m2 * dt * 3600.0;
  }
  // update_iwe :1612-1617
  t = npmin(IM * 3600.0, st.h_iwe);
  IM = div_k(t, 3600.0, 1.0 / 3600.0);
  double h_iwe = st.h_iwe - IM * dt * 3600.0;
  h_iwe = npmax(h_iwe, 0.0);
  // update_combined_meltrate :1441-1443
  const double M_total = IM + SM + div_r(P_rain, 1.0 / 3600.0);
  // update_snow_depth :1711 / update_ice_depth :1726
  const double h_snow = h_swe * p.ws;
  const double h_ice = h_iwe * p.wi;
  // update_snowpack_cold_content :1556-1558 (new h_snow)
  Eccs = (P_snow <= 0.0) ? npmax(Eccs - E_in, 0.0) : Eccs;
  Eccs = (h_snow == 0.0) ? 0.0 : Eccs;

  st.h_swe = h_swe;
  st.h_iwe = h_iwe;
  st.Eccs = Eccs;
  st.Ecci = Ecci;
  st.h_snow = h_snow;
  st.h_ice = h_ice;
  o.h_snow = h_snow;
  o.h_ice = h_ice;
  o.SM = SM;
  o.IM = IM;
  o.M_total = M_total;
  o.RH = RH;
}

// Albedo ageing (:1020-1059) given the window predicate (exact variant).
__device__ __forceinline__ double albedo_step(const DevParams& p, CellState& st, double T_air) {
#pragma clang fp contract(off)  // 0.4 + 0.44 * exp(...) rounds the product first, as numpy does
  // n: where(tot >= .03, 0, n); where(tot < .03, n + days_per_dt, n)
  st.n = window_days(st.n, st.tot_q, p.thr_q, p.days_per_dt);
  const double r = (T_air > 0.0) ? 0.12 : 0.05;
  const double snow_albedo = 0.4 + 0.44 * exp_k(-st.n * r);
  double albedo = (st.h_snow > 0.0) ? snow_albedo : st.albedo;
  if (st.h_snow == 0.0 && st.h_ice > 0.0) albedo = 0.3;
  if (st.h_snow == 0.0 && st.h_ice == 0.0) albedo = 0.15;
  st.albedo = albedo;
  return albedo;
}

// A value the compiler cannot see as a constant.  pow() calls with a constant
// base (Satterlund's 10^y) go through it, so that the compiler emits the
// general pow in every kernel: the library's call-simplification may otherwise
// rewrite such a call in one kernel and not in another, and the one-cell step
// (cell_step_exact_wave, whose pow arguments are per-lane values) would no
// longer equal the grid step bit for bit.
__device__ __forceinline__ double opaque(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

// x^4 and x^1.5 of the exact engine (T^4 in the long-wave terms, :1231-1233;
// RH^1.5 of the wet bulb, :1520) as (x*x)*(x*x) and x*sqrt(x) instead of the
// general pow: at most ~1.5 ulp from numpy's correctly rounded `** 4.0` /
// `** 1.5`, against ~130 VALU instructions per general fp64 pow.  Grid and
// one-cell steps both call these, so they stay equal bit for bit.
__device__ __forceinline__ double pow4(double x) {
#pragma clang fp contract(off)
  const double x2 = x * x;
  return x2 * x2;
}
// The square root from v_rsq_f64's seed y: s = x y, h = y / 2, one Goldschmidt
// step and one correction s + (x - s^2) h (round 5; the device libm's sqrt adds
// range scaling and a second correction): within 1 ulp for x in [2^-900,
// 2^900]; other x (0, denormals, negatives, inf, NaN) take the libm's.
__device__ __forceinline__ double sqrt_k(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double s = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-h, s, 0.5);
  s = __builtin_fma(s, r, s);
  h = __builtin_fma(h, r, h);
  s = __builtin_fma(__builtin_fma(-s, s, x), h, s);
  if (__builtin_expect(!(x >= 0x1p-900 && x <= 0x1p900), 0)) {
    TFG_FM_RARE();
    s = __builtin_sqrt(x);
  }
  return s;
}
__device__ __forceinline__ double pow1p5(double x) {
#pragma clang fp contract(off)
  return x * sqrt_k(x);
}
// 1 / d from v_rcp_f64 and two Newton steps (within 1 ulp), or one (rcp_nr1:
// relative error ~1e-14, for a quotient that only corrects a value).
__device__ __forceinline__ double rcp_nr1(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
}
__device__ __forceinline__ double rcp_nr(double d) {
  const double r = rcp_nr1(d);
  return __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
}

// The stability correction (:672-726) with one quotient (round 5): Ri = top /
// bot with bot > 0, so Ri > 0 exactly where top > 0, and Dn / (1 + 10 Ri) =
// Dn bot / (bot + 10 top), Dn (1 - 10 Ri) = Dn (bot - 10 top) / bot; Ri = 0
// keeps Dh = Dn exactly.  Within 2 ulp of the reference's two quotients.
__device__ __forceinline__ double stability_dh(double Dn, double top, double bot) {
#pragma clang fp contract(off)
  const bool stable = top > 0.0;
  const double num = Dn * (stable ? bot : bot - (10.0 * top));
  const double den = stable ? bot + (10.0 * top) : bot;
  return (top == 0.0) ? Dn : fdiv(num, den);
}

// em_air's (e/T)^(1/7) (:1167): an fp32 seed y0 = exp2(log2(x)/7) (relative
// error e ~ 2e-7) and one Halley step y0 - y0 (y0^7 - x) / (4 y0^7 + 3 x)
// (error ~e^3; y0^7 - x is exact, so the step adds only its own roundings):
// within 2 ulp of numpy's x ** (1/7) (tests/test_power_rewrites.py), at about
// a third of the cost of a log and an exp (round 5; before: exp(log(x)/7), then
// two Newton steps).  x = 0 gives 0, a negative or NaN x NaN and +inf +inf, as
// numpy's power.
__device__ __forceinline__ double root7(double x) {
#pragma clang fp contract(off)
  const double y0 = (double)__builtin_amdgcn_exp2f(__builtin_amdgcn_logf((float)x) * (1.0f / 7.0f));
  const double y2 = y0 * y0;
  const double y7 = (y2 * y2) * (y2 * y0);
  const double c = (y7 - x) * rcp_nr1(__builtin_fma(4.0, y7, 3.0 * x));  // a correction ~e: 1e-14 of it suffices
  const double y = __builtin_fma(-y0, c, y0);
  return (x > 0.0 && x < INFINITY) ? y : y0;
}

// root7 sized for the fp32 engine's fp64-flux form (round 6): the same fp32
// seed, one Newton step y0 (1 - rho / 7) with rho = (y0^7 - x) / x taken in
// fp32 (rho ~ 1e-7, so its fp32 rounding is ~1e-14 of y): relative error
// ~1e-13 (3 rho^2 from Newton), three fp64 operations fewer than root7's Halley
// step and its fp64 reciprocal.
__device__ __forceinline__ double root7_p(double x) {
#pragma clang fp contract(off)
  const float xf = (float)x;
  const double y0 = (double)__builtin_amdgcn_exp2f(__builtin_amdgcn_logf(xf) * (1.0f / 7.0f));
  const double y2 = y0 * y0;
  const double y7 = (y2 * y2) * (y2 * y0);
  const float rho7 = (float)(y7 - x) * (__builtin_amdgcn_rcpf(xf) * (1.0f / 7.0f));
  const double y = __builtin_fma(-y0, (double)rho7, y0);
  return (x > 0.0 && x < INFINITY) ? y : y0;
}

// Stull's wet bulb (:1514-1520, RH a fraction), fp64, with one arctangent for
// four (round 5; ~1e-14 from the reference's form, tests/test_gpu_parity.py):
//   atan(T + RH) - atan(RH - 1.676331) = atan((T + 1.676331) / (1 + (T + RH)(RH - 1.676331)))
//       (+ pi sign(T + RH) where the denominator is negative), by atan_q from
//       the two operands (one quotient),
//   atan(0.151977 sqrt(RH + 8.313659)) by stull_atan0_poly, and
//   atan(0.023101 RH) by its series to x^9 (relative error x^10/11 < 1e-10 for
//       RH <= 5, on a term below 1e-3 K);
// waves with a lane whose RH is outside [0, 5] take the arctangents there.
// wet_bulb_parts gives the first arctangent's argument (off the fit) and the
// second's two operands; wet_bulb_finish the rest from the arctangents (the
// one-cell step batches the off-fit ones).
constexpr double kPi = 3.141592653589793;
__device__ __forceinline__ void wet_bulb_parts(double T_air, double RH, double& u0, double& num, double& den) {
#pragma clang fp contract(off)
  u0 = 0.151977 * sqrt(RH + 8.313659);
  den = 1.0 + (T_air + RH) * (RH - 1.676331);
  num = T_air + 1.676331;
}
// atan(0.151977 sqrt(RH + 8.313659)) for RH in [0, 5] as a degree-13
// polynomial in t = 0.4 RH - 1 (a Chebyshev fit, relative error < 2e-14,
// tests/test_power_rewrites.py): 13 FMAs for a square root and an arctangent,
// the coefficients as scalar operands.
__device__ __forceinline__ double stull_atan0_poly(double RH) {
  const double t = __builtin_fma(0.4, RH, -1.0);
  double y = tfg_fm::fma_vvs(t, 0x1.b58d687bb4412p-36, -0x1.a2f6161678e01p-34);
  y = tfg_fm::fma_vvs(y, t, 0x1.acccbc15e0e7fp-32);
  y = tfg_fm::fma_vvs(y, t, -0x1.17d5b0c2a427ap-29);
  y = tfg_fm::fma_vvs(y, t, 0x1.686a49a337c49p-27);
  y = tfg_fm::fma_vvs(y, t, -0x1.d44af1ebe2f10p-25);
  y = tfg_fm::fma_vvs(y, t, 0x1.38df9b2403c64p-22);
  y = tfg_fm::fma_vvs(y, t, -0x1.b16bbee999fe5p-20);
  y = tfg_fm::fma_vvs(y, t, 0x1.3be2008d543e9p-17);
  y = tfg_fm::fma_vvs(y, t, -0x1.f1959460701e0p-15);
  y = tfg_fm::fma_vvs(y, t, 0x1.bc9c3023533e3p-12);
  y = tfg_fm::fma_vvs(y, t, -0x1.ea2542f0a20c4p-9);
  y = tfg_fm::fma_vvs(y, t, 0x1.7aac28df5f664p-5);
  return tfg_fm::fma_vvs(y, t, 0x1.da94c1a0c29f5p-2);
}
// RH outside the fits' range [0, 5] (NaN stays on the fits and gives NaN)
__device__ __forceinline__ bool stull_off_fit(double RH) { return (RH < 0.0) || (RH > 5.0); }
__device__ __forceinline__ double atan_small_series(double x) {
#pragma clang fp contract(off)
  const double x2 = x * x;
  return x * (1.0 + x2 * (-1.0 / 3.0 + x2 * (1.0 / 5.0 + x2 * (-1.0 / 7.0 + x2 * (1.0 / 9.0)))));
}
__device__ __forceinline__ double wet_bulb_finish(double T_air, double RH, double at0, double at1, double den,
                                                   double at_small) {
#pragma clang fp contract(off)
  const double d = den < 0.0 ? at1 + copysign(kPi, T_air + RH) : at1;
  return T_air * at0 + d + ((0.00391838 * pow1p5(RH)) * at_small) - 4.86035;
}

// ---------------------------------------------------------------------------
// EXACT variant (fp64, reference order)
// ---------------------------------------------------------------------------
// QC: add the cell's lateral conduction flux qc [W m-2] (tfg_conduction.hpp)
// in the reference's Qc position of Q_sum (:1314); without it Qc = 0.
// The model constants as the caller holds them (ParamsAsIs), or re-read at
// each phase of the step (the grid kernel's KernargParams, tfg_fused.hpp), so
// that a phase's constants are live only in that phase.
struct ParamsAsIs {
  const DevParams& p;
  __device__ const DevParams& operator()() const { return p; }
};

template <bool QC, class PS>
__device__ inline void cell_step_exact(const DevParams& p, const CellStatic& s, const tfg_uniforms& u,
                                       double P, double T_air, double Hum_sp, double P_air, double uz,
                                       int32_t q_old, int32_t& q_new, CellState& st, CellOut& o,
                                       CellDiag& d, bool valid, double qc, const PS& params) {
#pragma clang fp contract(off)
  const double dt = p.dt;
  const double h_snow = st.h_snow, h_ice = st.h_ice;  // previous step
  // update_atm_pressure_from_elevation(T_C=True, MBAR=True) :551-556, read only
  // as lhc / p0 (:931): (100 lhc / sea_p0) exp(-x), one exp and no quotient
  // (round 5; within 2 ulp of the reference's quotient); 1 / T_K serves the
  // exponent and em_air's argument (:1167)
  const double T_K = T_air + 273.15;
  const double r_TK = rcp_nr(T_K);
  const double lhc_p0 = p.lhc_100_p0 * exp_k(-((p.negM_g_R * s.elev) * r_TK));
  // :567, :576, :585, :604, :613, :623
  const double P_rain = P * ((T_air > p.T_rs) ? 1.0 : 0.0);
  const double P_snow = P * ((T_air <= p.T_rs) ? 1.0 : 0.0);
  if (valid) {  // unscaled: k_fused applies da dt to the launch's sums (diag_scale; round 6)
    d.P += P;
    d.Pmax = npmax(d.Pmax, P);
    d.PR += P_rain;
    d.PS += P_snow;
  }
  // :817-826
  double e = fdiv(Hum_sp * P_air, p.eps + (p.one_minus_eps * Hum_sp));
  e = div_r(e, 1.0 / 1000.0);
  const double e_air = e * 10.0;
  // saturation vapour pressure (air) :788-802, read only as RH = e_air / e_sat_air
  // (:838): Brutsaert's e_air exp(-x) / 6.11 without the quotient (round 5)
  double RH;
  if (!p.satterlund) {
    RH = (e_air * exp_k(-fdiv(17.3 * T_air, T_air + 237.3))) * p.inv_6p11;
  } else {
    const double e_sat_air = div_r(pow(opaque(10.0), 11.4 - fdiv(2353.0, T_air + 273.15)), 1.0 / 1000.0) * 10.0;
    RH = fdiv(e_air, e_sat_air);
  }
  // :888-893
  const double log_term = log_k(div_r(e_air, 1.0 / 6.1121));
  const double T_dew = fdiv(257.14 * log_term, 18.678 - log_term);
  // :906-910 (previous-step depths)
  const double T_surf = (h_snow > 0.0 || h_ice > 0.0) ? npmin(T_dew, 0.0) : T_dew;
  double e_sat_surf;
  if (!p.satterlund) {
    e_sat_surf = 0.611 * exp_k(fdiv(17.3 * T_surf, T_surf + 237.3));
  } else {
    e_sat_surf = div_r(pow(opaque(10.0), 11.4 - fdiv(2353.0, T_surf + 273.15)), 1.0 / 1000.0);
  }
  e_sat_surf = e_sat_surf * 10.0;
  // :640-644, per cell
  const double top = p.gz * (T_air - T_surf);
  double bot = (uz * uz) * (T_air + 273.15);
  if (bot == 0.0) bot = 0.01;
  // :670-726
  const double arg = tfg_fm::fdiv_z(p.kappa, log_k(npmax(div_r(p.z - h_snow, p.inv_z0), 0.01)));
  const double Dn = uz * (arg * arg);
  const double Dh = stability_dh(Dn, top, bot);
  // :744-745
  const double Qh = p.rho_air_Cp_air * Dh * (T_air - T_surf);
  // :853 (SURFACE uses the air RH)
  const double e_surf = RH * e_sat_surf;
  // :931-934
  const double Qe = p.rho_air_Lv * Dh * (e_air - e_surf) * lhc_p0;
  // albedo :1023-1059 with the fixed-point window
  q_new = window_q(P_snow * dt * p.ws, p.qscale);
  st.tot_q += window_tot(q_new) - window_tot(q_old);
  const double albedo = albedo_step(p, st, T_air);
  const DevParams& p2 = params();  // Clear_Sky_Radiation phase
  // Clear_Sky_Radiation SF:904-941 (uniform parts hoisted), only while the sun
  // is up on a flat surface this step: flat_dark (a step uniform) makes every
  // cell dark, K_cs = 0 in the reference too, so half the steps skip W_p
  // (:919-920), tau and gam_s
  double K_cs = 0.0;
  if (!u.flat_dark) {
    const double W_p = 1.12 * exp_k(0.0614 * T_dew);  // :919-920
    const double a_sa = -0.1240 - (0.0207 * W_p);
    const double b_sa = -0.0682 - (0.0248 * W_p);
    const double tau = npmin(npmax(exp_k(a_sa + (b_sa * u.m_opt)) - p2.dust, 0.0), 1.0);
    const double cos_wl = cos_hour_angle(s, u);  // SF:867
    double K_ET = u.isc_e0 * ((u.cos_d * s.cos_leq) * cos_wl + s.sin_leq * u.sin_d);
    K_ET = npmax(K_ET, 0.0);
    const double a_s = -0.0363 - (0.0084 * W_p);
    const double b_s = -0.0572 - (0.0173 * W_p);
    const double gam_s = (1.0 - exp_k(a_s + (b_s * u.m_opt))) + p2.dust;
    const double K_dif = 0.5 * gam_s * u.k_et_flat;
    const double K_global = tau * u.k_et_flat + K_dif;
    const double K_bs = 0.5 * gam_s * albedo * K_global;
    K_cs = (tau * K_ET) + K_dif + K_bs;
    if (sun_down(p2, s, u, cos_wl)) K_cs = 0.0;
  }
  const double Qn_SW = K_cs * (1.0 - albedo);  // :1139
  const DevParams& p3 = params();  // long-wave and net flux phase
  // update_em_air :1167-1192
  const double T_air_K = T_air + 273.15;
  double em_air;
  if (!p3.satterlund) {
    const double term1 = p3.one_minus_F_172 * root7(div_r(e_air, 1.0 / 10.0) * r_TK);
    em_air = (term1 * p3.cloud_term) + p3.F;
  } else {
    em_air = 1.08 * (1.0 - exp_k(-1.0 * pow(e_air, div_r(T_air_K, 1.0 / 2016.0))));
  }
  // :1231-1248
  const double T_surf_K = T_surf + 273.15;
  const double LW_in = em_air * p3.sigma * pow4(T_air_K);
  double LW_out = p3.em_surf_sigma * pow4(T_surf_K);
  LW_out = LW_out + p3.one_minus_em_surf * LW_in;
  const double Qn_LW = LW_in - LW_out;
  // :1314 (Qa = 0; Qc = 0 unless the optional conduction term is on)
  const double Q_sum = Qn_SW + Qn_LW + Qh + Qe + 0.0 + (QC ? qc : 0.0);
  // Stull wet bulb (:1514-1520), only needed where it snows
  double T_wb = 0.0;
  if (P_snow > 0.0) {
    double u0, num, den;
    wet_bulb_parts(T_air, RH, u0, num, den);
    const double x = 0.023101 * RH;
    double at0 = stull_atan0_poly(RH), at_small = atan_small_series(x);
    if (__any(stull_off_fit(RH))) {
      const bool off = stull_off_fit(RH);
      at0 = off ? atan(u0) : at0;
      at_small = off ? atan(x) : at_small;
    }
    T_wb = wet_bulb_finish(T_air, RH, at0, atan_q(num, den), den, at_small);
  }
  const DevParams& p4 = params();  // melt and mass phase
  melt_and_mass<true>(p4, Q_sum, P_snow, P_rain, RH, T_wb, st, o, d, valid);
#if defined(TFG_DEBUG_EXACT)  // diagnostic builds only: a flux term replaces RH in the output
  { const double dbg[8] = {Q_sum, Qn_SW, Qn_LW, Qh, Qe, K_cs, LW_in, albedo}; o.RH = dbg[TFG_DEBUG_EXACT]; }
#endif
}

// ---------------------------------------------------------------------------
// EXACT variant for ONE cell on a whole workgroup (the single-catchment BMI
// step, k_cell / k_cell_run).  Every lane of every wave computes the same
// scalar arithmetic as cell_step_exact, in the same order, but the
// transcendental calls are batched by dependency level: each level's calls of
// one function run once, lane i evaluating the i-th argument.  With W = 4
// waves (one per SIMD of the CU), the function classes of a level also run
// side by side, wave c taking class c (level 1: exp | log | cos, acos, and
// Satterlund's pow; level 2: exp | atan, and Satterlund's pow; level 3: exp), and their results meet in LDS
// behind one barrier per level; with W = 1 the classes run one after another
// in the wave and the results are read back from their lanes (v_readlane).
// The serial chain of fp64 libm calls falls from 14-18 (exp x8, log x3,
// cos, acos, the wet bulb's atan off its fits) to 3 levels.  The same
// functions on the same arguments give the same values, so the result equals
// cell_step_exact bit for bit (test_one_cell_kernels_equal_the_grid_kernel).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double lane_value(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Class slots of the level exchange: [slot][4 lanes] doubles in LDS.
enum { X_POW1 = 0, X_EXP1, X_LOG1, X_TRIG1, X_POW2, X_EXP2, X_ATAN2, X_EXP3, X_SLOTS };
constexpr int kCellWaves = 4;

// Results of one function class: computed by wave `owner` (all waves when
// W = 1), read by every wave.
template <int W>
struct LevelXchg {
  double* x;   // [X_SLOTS][4] in LDS (W > 1)
  int wave;    // this wave's index (wave-uniform)
  int lane;
  __device__ bool mine(int slot) const { return W == 1 || wave == slot % W; }
  __device__ void put(int slot, double v) const {
    if (W > 1 && wave == slot % W && lane < 4) x[slot * 4 + lane] = v;
  }
  __device__ double get(int slot, double v, int l) const { return W == 1 ? lane_value(v, l) : x[slot * 4 + l]; }
};

__device__ __forceinline__ void lds_level_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int W>
__device__ inline void cell_step_exact_wave(const DevParams& p, const CellStatic& s, const tfg_uniforms& u,
                                            double P, double T_air, double Hum_sp, double P_air, double uz,
                                            int32_t q_old, int32_t& q_new, CellState& st, CellOut& o,
                                            CellDiag& d, double qc, double* lds_x) {
#pragma clang fp contract(off)
  const int lane = (int)(threadIdx.x & 63);
  const LevelXchg<W> X{lds_x, W == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane};
  const double dt = p.dt;
  const double h_snow = st.h_snow, h_ice = st.h_ice;  // previous step
  const double T_K = T_air + 273.15;
  // :567, :576, :585, :604, :613, :623
  const double P_rain = P * ((T_air > p.T_rs) ? 1.0 : 0.0);
  const double P_snow = P * ((T_air <= p.T_rs) ? 1.0 : 0.0);
  d.P += P * p.da_m2 * dt;
  d.Pmax = npmax(d.Pmax, P);
  d.PR += P_rain * p.da_m2 * dt;
  d.PS += P_snow * p.da_m2 * dt;
  // :817-826
  double e = fdiv(Hum_sp * P_air, p.eps + (p.one_minus_eps * Hum_sp));
  e = div_r(e, 1.0 / 1000.0);
  const double e_air = e * 10.0;
  const double T_air_K = T_air + 273.15;
  // window and days since snowfall (:1023-1040), ahead of the albedo exp
  q_new = window_q(P_snow * dt * p.ws, p.qscale);
  st.tot_q += window_tot(q_new) - window_tot(q_old);
  st.n = window_days(st.n, st.tot_q, p.thr_q, p.days_per_dt);
  const double r_alb = (T_air > 0.0) ? 0.12 : 0.05;

  // ---- level 1: arguments from inputs, state, statics and uniforms
  double ex1 = 0.0, lg1 = 0.0, cos_wl = 0.0, ac = 0.0, pw1 = 0.0;
  if (X.mine(X_EXP1)) {
    const double x_p0 = (p.negM_g_R * s.elev) * rcp_nr(T_K);      // :551, as cell_step_exact
    const double x_es = fdiv(17.3 * T_air, T_air + 237.3);        // :788
    const double x_alb = -st.n * r_alb;                          // :1041
    ex1 = exp_k(lane == 1 ? -x_es : (lane == 2 ? x_alb : -x_p0));
  }
  if (X.mine(X_LOG1))  // :670, :888
    lg1 = log_k(lane == 1 ? npmax(div_r(p.z - h_snow, p.inv_z0), 0.01) : div_r(e_air, 1.0 / 6.1121));
  if (X.mine(X_TRIG1)) ac = acos(npmin(npmax(-1.0, -1.0 * s.tan_eq * u.tan_d), 1.0));  // SF:325 (one argument)
  cos_wl = cos_hour_angle(s, u);                                                          // SF:867
  if (X.mine(X_POW1) && p.satterlund)  // e_air^(T/2016) (:1190), 10^(...) of e_sat_air (:796)
    pw1 = pow(lane == 2 ? 10.0 : e_air, lane == 2 ? 11.4 - fdiv(2353.0, T_air + 273.15) : div_r(T_air_K, 1.0 / 2016.0));
  X.put(X_EXP1, ex1);
  X.put(X_LOG1, lg1);
  X.put(X_TRIG1, ac);
  X.put(X_POW1, pw1);
  if (W > 1) lds_level_barrier();
  const double e_p0 = X.get(X_EXP1, ex1, 0), e_es = X.get(X_EXP1, ex1, 1), e_alb = X.get(X_EXP1, ex1, 2);
  const double log_term = X.get(X_LOG1, lg1, 0), log_dn = X.get(X_LOG1, lg1, 1);
  const double pw_em = X.get(X_POW1, pw1, 0), pw_es = X.get(X_POW1, pw1, 2);
  const double pw_ta4 = pow4(T_air_K);  // :1231
  if (W > 1) ac = X.get(X_TRIG1, 0.0, 0);

  // :551-556, :931 (lhc / p0); :788-802, :838 (RH), as cell_step_exact
  const double lhc_p0 = p.lhc_100_p0 * e_p0;
  const double RH = !p.satterlund ? (e_air * e_es) * p.inv_6p11 : fdiv(e_air, div_r(pw_es, 1.0 / 1000.0) * 10.0);
  // :888-893, :906-910
  const double T_dew = fdiv(257.14 * log_term, 18.678 - log_term);
  const double T_surf = (h_snow > 0.0 || h_ice > 0.0) ? npmin(T_dew, 0.0) : T_dew;
  // :640-644, :670-726, :744-745
  const double top = p.gz * (T_air - T_surf);
  double bot = (uz * uz) * (T_air + 273.15);
  if (bot == 0.0) bot = 0.01;
  const double arg = tfg_fm::fdiv_z(p.kappa, log_dn);  // inf at h_snow = z - z0, as the reference
  const double Dn = uz * (arg * arg);
  const double Dh = stability_dh(Dn, top, bot);
  const double Qh = p.rho_air_Cp_air * Dh * (T_air - T_surf);
  // albedo (:1041-1059)
  const double snow_albedo = 0.4 + 0.44 * e_alb;
  double albedo = (st.h_snow > 0.0) ? snow_albedo : st.albedo;
  if (st.h_snow == 0.0 && st.h_ice > 0.0) albedo = 0.3;
  if (st.h_snow == 0.0 && st.h_ice == 0.0) albedo = 0.15;
  st.albedo = albedo;
  // sunrise / sunset on the slope (SF:783-830)
  const double t_noon = noon_offset(p, s.dlon);  // SF:776
  const double T_sr = npmax(div_k(-1.0 * ac, p.omega, kInvOmega) + t_noon, u.flat_sr);
  const double T_ss = npmin(div_k(ac, p.omega, kInvOmega) + t_noon, u.flat_ss);
  const double T_surf_K = T_surf + 273.15;

  // ---- level 2: after T_dew, T_surf and RH
  double ex2 = 0.0, pw2 = 0.0, at2 = 0.0;
  if (X.mine(X_EXP2)) {
    double ea2 = lane == 1 ? 0.0614 * T_dew : fdiv(17.3 * T_surf, T_surf + 237.3);  // :919, :788 (surface)
    if (p.satterlund && lane == 2) ea2 = -1.0 * pw_em;                             // :1190
    ex2 = exp_k(ea2);
  }
  if (X.mine(X_POW2) && p.satterlund) pw2 = pow(opaque(10.0), 11.4 - fdiv(2353.0, T_surf + 273.15));  // :796 (surface)
  // Stull wet bulb (:1514-1520), only where it snows: wet_bulb_parts' two arguments and, for RH
  // outside [0, 5] (stull_off_fit), the arctangents off the fits
  double wb_u0 = 0.0, wb_num = 0.0, wb_den = 1.0;
  if (P_snow > 0.0) wet_bulb_parts(T_air, RH, wb_u0, wb_num, wb_den);
  if (X.mine(X_ATAN2) && P_snow > 0.0) at2 = atan(lane == 2 ? 0.023101 * RH : wb_u0);
  X.put(X_EXP2, ex2);
  X.put(X_POW2, pw2);
  X.put(X_ATAN2, at2);
  if (W > 1) lds_level_barrier();
  double e_sat_surf = !p.satterlund ? 0.611 * X.get(X_EXP2, ex2, 0) : div_r(X.get(X_POW2, pw2, 0), 1.0 / 1000.0);
  e_sat_surf = e_sat_surf * 10.0;
  const double W_p = 1.12 * X.get(X_EXP2, ex2, 1);
  // :853, :931-934
  const double e_surf = RH * e_sat_surf;
  const double Qe = p.rho_air_Lv * Dh * (e_air - e_surf) * lhc_p0;
  const double a_sa = -0.1240 - (0.0207 * W_p);
  const double b_sa = -0.0682 - (0.0248 * W_p);
  const double a_s = -0.0363 - (0.0084 * W_p);
  const double b_s = -0.0572 - (0.0173 * W_p);

  // ---- level 3: after W_p
  double ex3 = 0.0;
  if (X.mine(X_EXP3)) ex3 = exp_k(lane == 1 ? a_s + (b_s * u.m_opt) : a_sa + (b_sa * u.m_opt));  // SF:610, SF:652
  X.put(X_EXP3, ex3);
  if (W > 1) lds_level_barrier();
  const double tau = npmin(npmax(X.get(X_EXP3, ex3, 0) - p.dust, 0.0), 1.0);
  double K_ET = u.isc_e0 * ((u.cos_d * s.cos_leq) * cos_wl + s.sin_leq * u.sin_d);
  K_ET = npmax(K_ET, 0.0);
  const double gam_s = (1.0 - X.get(X_EXP3, ex3, 1)) + p.dust;
  const double K_dif = 0.5 * gam_s * u.k_et_flat;
  const double K_global = tau * u.k_et_flat + K_dif;
  const double K_bs = 0.5 * gam_s * albedo * K_global;
  double K_cs = (tau * K_ET) + K_dif + K_bs;
  if ((u.th <= T_sr) || (u.th >= T_ss)) K_cs = 0.0;
  const double Qn_SW = K_cs * (1.0 - albedo);  // :1139
  // :1167-1192, :1231-1248
  double em_air;
  if (!p.satterlund) {
    const double term1 = p.one_minus_F_172 * root7(div_r(e_air, 1.0 / 10.0) * rcp_nr(T_air_K));
    em_air = (term1 * p.cloud_term) + p.F;
  } else {
    em_air = 1.08 * (1.0 - X.get(X_EXP2, ex2, 2));
  }
  const double LW_in = em_air * p.sigma * pw_ta4;
  double LW_out = p.em_surf_sigma * pow4(T_surf_K);  // :1233
  LW_out = LW_out + p.one_minus_em_surf * LW_in;
  const double Qn_LW = LW_in - LW_out;
  // :1314 (Qa = 0; qc = 0 unless the optional conduction term is on)
  const double Q_sum = Qn_SW + Qn_LW + Qh + Qe + 0.0 + qc;
  double T_wb = 0.0;
  if (P_snow > 0.0) {
    const bool off = stull_off_fit(RH);
    const double at0 = off ? X.get(X_ATAN2, at2, 0) : stull_atan0_poly(RH);
    const double at_small = off ? X.get(X_ATAN2, at2, 2) : atan_small_series(0.023101 * RH);
    T_wb = wet_bulb_finish(T_air, RH, at0, atan_q(wb_num, wb_den), wb_den, at_small);
  }
  melt_and_mass(p, Q_sum, P_snow, P_rain, RH, T_wb, st, o, d, true);
#if defined(TFG_DEBUG_EXACT)  // diagnostic builds only: a flux term replaces RH in the output
  { const double dbg[8] = {Q_sum, Qn_SW, Qn_LW, Qh, Qe, K_ET, LW_in, albedo}; o.RH = dbg[TFG_DEBUG_EXACT]; }
#endif
  // No barrier needed before the next step's writes: a slot is rewritten one
  // step later, after two more level barriers, which every wave reaches only
  // after reading this step's value of it.
}

// ---------------------------------------------------------------------------
// FAST variant: fp32 fluxes, fp64 state and predicates
// ---------------------------------------------------------------------------
// Per-cell solar geometry of the fast variant (k_prepare_geo, once per static
// raster change), five fp32 planes:
//   ek    = (M g / R) * elev * log2(e)        p0 exponent          :551-556
//   sl    = sin(lat_eq)                                            SF:753-757
//   cc    = cos(lat_eq) * cos(dlon)                                SF:730-734
//   cs    = cos(lat_eq) * sin(dlon)
//   dlon  = Longitude_Offset [rad]
// plus two fp64 planes tan(lat_eq), t_noon read only by the exact dark test.
constexpr int kGeoF = 5;
struct CellStaticF {
  float ek, sl, cc, cs, dlon;
};

__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float flog2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// log2 refined by one Newton step on exp2 (v_exp_f32 is unbiased; v_log_f32
// has a mean error of -0.44 ulp of its result): y += (x*2^-y - 1)*log2(e).
// The residual error is second order, so no bias reaches the state.
__device__ __forceinline__ float flog2_nr(float x) {
  const float y = flog2(x);
  return fmaf(fmaf(x, fexp2(-y), -1.0f), 1.4426950408889634f, y);
}
// 1/x: v_rcp_f32 (~1 ulp, biased) and one Newton step (correctly rounded but
// for a rare last-bit miss, no bias): for the divisors whose quotient feeds
// the dew point, which every flux term reads
__device__ __forceinline__ float frcp_nr(float x) {
  const float r = frcp(x);
  return fmaf(fmaf(-x, r, 1.0f), r, r);
}
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// fp64 derivation of the per-cell geometry (exact trig identities from
// sin/cos of the slope and aspect angles; derive_static is the reference-order
// form of the same quantities).
struct CellGeo {
  float f[kGeoF];
  double tan_eq, t_noon;
};
__device__ inline CellGeo derive_geo(const DevParams& p, double elev, double slope, double aspect) {
  double sa, ca;
  sincos(aspect, &ca, &sa);  // alpha = pi/2 - aspect: cos(alpha) = sin(aspect), sin(alpha) = cos(aspect)
  if (!isfinite(sa) || !isfinite(ca)) { sa = 1.0; ca = 0.0; }
  double sb, cb;
  if (!(slope == slope)) { sb = 0.0; cb = 1.0; }
  else if (isinf(slope)) { sb = 1.0; cb = 0.0; }
  else { const double r = 1.0 / sqrt(1.0 + slope * slope); sb = slope * r; cb = r; }
  const double sl = sb * ca * p.cos_lat + cb * p.sin_lat;
  const double cl = sqrt(fmax(1.0 - sl * sl, 0.0));
  const double t = (sb * sa) / (cb * p.cos_lat - sb * p.sin_lat * ca);
  const double rt = 1.0 / sqrt(1.0 + t * t);
  const double dlon = atan(t);
  CellGeo g;
  g.f[0] = (float)(-p.negM_g / p.R * elev * 1.4426950408889634);
  g.f[1] = (float)sl;
  g.f[2] = (float)(cl * rt);
  g.f[3] = (float)(cl * t * rt);
  g.f[4] = (float)dlon;
  g.tan_eq = sl / cl;
  g.t_noon = -1.0 * dlon / p.omega;
  return g;
}

// Dark test in fp64 (SF:939) for a cell whose fp32 test lies within its
// error margin: the reference's Sunrise/Sunset_Offset_Slope from the cell's
// fp64 tan(eq_lat) and noon offset (read here, on the rare path).
__device__ __noinline__ bool dark_exact(const DevParams& p, const double* __restrict__ geo_d, int64_t n_pad,
                                        int64_t i, const tfg_uniforms* __restrict__ up) {
#pragma clang fp contract(off)
  const double tan_eq = geo_d[i], t_noon = geo_d[n_pad + i];
  double arg = -1.0 * tan_eq * up->tan_d;
  arg = npmin(npmax(-1.0, arg), 1.0);
  const double ac = acos(arg);
  const double T_sr = npmax(-1.0 * ac / p.omega + t_noon, up->flat_sr);
  const double T_ss = npmin(ac / p.omega + t_noon, up->flat_ss);
  return (up->th <= T_sr) || (up->th >= T_ss);
}

// atan for the fp32 path: argument reduced to [0, 1] (atan(x) = pi/2 -
// atan(1/x) above 1), minimax polynomial in z^2 (max rel. error ~1.5e-7).
__device__ __forceinline__ float fast_atanf(float x) {
  const float ax = fabsf(x);
  const bool big = ax > 1.0f;
  const float z = big ? frcp(ax) : ax;
  const float t = z * z;
  float u = 0.00282363896258175373f;
  u = fmaf(u, t, -0.0159569028764963150f);
  u = fmaf(u, t, 0.0425049886107444763f);
  u = fmaf(u, t, -0.0748900920152664185f);
  u = fmaf(u, t, 0.106347933411598206f);
  u = fmaf(u, t, -0.142027363181114197f);
  u = fmaf(u, t, 0.199926957488059998f);
  u = fmaf(u, t, -0.333331018686294556f);
  float r = fmaf(z * t, u, z);
  r = big ? 1.57079632679489662f - r : r;
  return copysignf(r, x);
}

// h - a*b with the product rounded first, as numpy evaluates it.  At melt-out
// (a*b ~ h) the residual decides the exact-zero tests of the next step (the IM
// gate :1424); a fused multiply-add would leave a one-ulp residual of either
// sign where the reference's rounded product mostly cancels exactly.
__device__ __forceinline__ double sub_rounded(double h, double a, double b) {
#pragma clang fp contract(off)
  return h - a * b;
}
__device__ __forceinline__ double add_rounded(double h, double a, double b) {
#pragma clang fp contract(off)
  return h + a * b;
}

// Stull's wet-bulb temperature (:1514-1520) of the air temperature [degC] and
// RH as a fraction (the reference's quirk), fp32.  Three rewrites keep it cheap
// (every wave with a snowing lane evaluates it: 99 % of the bench's wave-steps
// for 12 % of its cell-steps):
//   atan(T + RH) - atan(RH - 1.676331) = atan((T + 1.676331) / (1 + (T + RH)(RH - 1.676331)))
//       (+ pi sign(T + RH) when the denominator is negative): one arctangent for two;
//   0.00391838 RH^1.5 atan(0.023101 RH), a term below 1e-3 K for RH < 5, with
//       atan(x) = x (1 - x^2/3 + x^4/5) (relative error x^6/7 < 3e-7 on [0, 5]);
//   atan(0.151977 sqrt(RH + 8.313659)) as a polynomial fit on [0, 5].
// Waves with a lane outside [0, 5] (or NaN) take fast_atanf for both.  The
// square roots are v_sqrt_f32 alone (within 1 ulp; round 6): the IEEE sqrtf's
// scaling and two correction steps cost 15 more VALU in every snowing wave for
// a term below 1e-3 K.
__device__ __forceinline__ float wet_bulb_f(float rh, float T_air) {
  const float a = T_air + rh, b = rh - 1.676331f;
  const float den = fmaf(a, b, 1.0f);
  float d = fast_atanf((T_air + 1.676331f) * frcp(den));
  if (den < 0.0f) d += copysignf(3.14159265358979f, a);
  const float x = 0.023101f * rh, x2 = x * x;
  float at = x * fmaf(fmaf(0.2f, x2, -0.333333333f), x2, 1.0f);
  // atan(0.151977 sqrt(rh + 8.313659)) on [0, 5]: degree-6 fit in t = 0.4 rh - 1 (relative error < 1e-7)
  const float t = fmaf(0.4f, rh, -1.0f);
  float a0 = fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(-1.7216859760083025e-06f, t, 9.90594708127901e-06f), t,
                                       -5.9253852668916807e-05f), t, 0.0004237863759044558f), t,
                             -0.003739525331184268f), t, 0.046224694699048996f), t, 0.4634580910205841f);
  if (__any((rh < 0.0f) || (rh > 5.0f))) {  // outside the fits (NaN stays on them)
    const bool off = (rh < 0.0f) || (rh > 5.0f);
    a0 = off ? fast_atanf(0.151977f * __builtin_amdgcn_sqrtf(rh + 8.313659f)) : a0;
    at = off ? fast_atanf(x) : at;
  }
  return T_air * a0 + d + (0.00391838f * (rh * __builtin_amdgcn_sqrtf(rh))) * at - 4.86035f;
}

// Cold content a snowfall brings (:1507-1537): rho_s Cp_s (P_snow dt ws)
// (T0 - T_wb), fp32 (melt_core's increment, for the diagnostic build).
__device__ __forceinline__ float snowfall_cold(const DevParams& p, float P_snow, float rh, float T_air) {
  return p.f_c_eccs * P_snow * (p.f_T0 - wet_bulb_f(rh, T_air));
}

// Per-cell partial sums of the fast variant over one launch's steps (fp32;
// scaled and added to the fp64 accumulators once per cell, padding excluded).
struct DiagF {
  float P, PR, PS, Erem_s, IM, Pmax;
};
struct CellOutF {
  float h_snow, SM, h_ice, IM, M_total, RH;
};

// Missing data.  The reference's np.maximum / np.minimum propagate NaN, its
// P * (T > T_rs) and P * (T <= T_rs) are both 0 for a NaN T_air, and a NaN in
// the snowfall window freezes n (:1035-1041).  The fast step comes in two
// forms: NANSAFE = true spells all of that out (npmax / npmin, both rain/snow
// tests, the window's NaN count), NANSAFE = false uses single-instruction IEEE
// max / min and plain window arithmetic, which give the same results wherever
// the step's forcing, statics, state and window hold only finite values.  The
// host picks the form per launch (tfg_engine.hip, launch_fused): the clean
// form only when it has verified that a launch reads no non-finite value.
template <bool NS> __device__ __forceinline__ float nmax(float a, float b) { if constexpr (NS) return npmax(a, b); else return fmaxf(a, b); }
template <bool NS> __device__ __forceinline__ float nmin(float a, float b) { if constexpr (NS) return npmin(a, b); else return fminf(a, b); }
template <bool NS> __device__ __forceinline__ double dmax(double a, double b) { if constexpr (NS) return npmax(a, b); else return fmax(a, b); }
template <bool NS> __device__ __forceinline__ double dmin(double a, double b) { if constexpr (NS) return npmin(a, b); else return fmin(a, b); }

// The fast step's state update (:1566-1731): fp64 where depths and cold
// contents accumulate.  NANSAFE: max / min as numpy's np.maximum / np.minimum,
// so missing forcing turns the same outputs NaN as in the reference.  Returns
// the new state, the clamped melt rates and the two diagnostic terms.
struct MeltF {
  double h_swe, h_iwe, Eccs, Ecci;
  float SM, IM, Erem_s, IM_int;  // outputs; terms of the SM and IM integrals (:1486, :1493)
};
template <bool NS, class QT>
__device__ __forceinline__ MeltF melt_core(const DevParams& p, QT Q_sum, float P_snow, float RH, float T_air,
                                           double h_swe0, double h_iwe0, double Eccs0, double Ecci0,
                                           double h_ice_prev) {
  MeltF m;
  const double previous_swe = h_swe0;
  // dt in hours, as the reference (:1364); an fp64 Q_sum (the PREC form) times the fp64 dt
  const double E_in = sizeof(QT) == 8 ? (double)Q_sum * p.dt : (double)(Q_sum * p.f_dt);
  // snow melt (:1364-1373; max(SM, 0) is implied by E_rem >= 0), integral (:1486)
  const double E_rem_s = dmax<NS>(E_in - Eccs0, 0.0);
  m.Erem_s = (float)E_rem_s;
  // update_swe (:1594-1606)
  double h_swe = add_rounded(h_swe0, (double)P_snow, p.dt);
  const double ts = dmin<NS>(E_rem_s * p.c_sm3600, h_swe);
  const double SM = ts * (1.0 / 3600.0);
  h_swe = dmax<NS>(sub_rounded(h_swe, SM, p.dt3600), 0.0);  // dt*3600 folded: exact for dt = 2^k
  // snowfall cold content (:1507-1537), Stull wet bulb with RH as a fraction
  double Eccs = Eccs0;
  if (P_snow > 0.0f) Eccs = dmax<NS>(Eccs + (double)snowfall_cold(p, P_snow, RH, T_air) - E_in, 0.0);
  // ice melt (:1418-1434), cap (:1473-1480), integral (:1493), update_iwe (:1612-1617)
  const double E_rem_i = dmax<NS>(E_in - Ecci0, 0.0);
  double IM = (h_swe == 0.0 && previous_swe == 0.0) ? E_rem_i * p.inv_dt_rhoLf : 0.0;
  double Ecci = dmax<NS>(Ecci0 - E_in, 0.0);
  Ecci = (h_ice_prev == 0.0) ? 0.0 : Ecci;
  IM = dmin<NS>(IM, h_iwe0 * p.inv_dt);  // max(IM, 0) is implied (IM, h_iwe >= 0 or NaN)
  m.IM_int = (float)IM;
  const double ti = dmin<NS>(IM * 3600.0, h_iwe0);
  IM = ti * (1.0 / 3600.0);
  const double h_iwe = dmax<NS>(sub_rounded(h_iwe0, IM, p.dt3600), 0.0);
  // snowpack cold content (:1556-1558) with the new h_snow = h_swe * ws (> 0
  // exactly where h_swe > 0); P_snow <= 0 written out in the NaN-safe form:
  // a NaN snowfall leaves Eccs alone, as np.where does
  if (NS ? (P_snow <= 0.0f) : !(P_snow > 0.0f)) Eccs = dmax<NS>(Eccs - E_in, 0.0);
  Eccs = (h_swe * p.ws == 0.0) ? 0.0 : Eccs;
  m.h_swe = h_swe;
  m.h_iwe = h_iwe;
  m.Eccs = Eccs;
  m.Ecci = Ecci;
  m.SM = (float)SM;
  m.IM = (float)IM;
  return m;
}
template <bool NS, class QT>
__device__ __forceinline__ void melt_fast(const DevParams& p, QT Q_sum, float P_snow, float P_rain, float RH,
                                          float T_air, CellState& st, CellOutF& o, DiagF& d) {
  const MeltF m = melt_core<NS, QT>(p, Q_sum, P_snow, RH, T_air, st.h_swe, st.h_iwe, st.Eccs, st.Ecci, st.h_ice);
  d.Erem_s += m.Erem_s;
  d.IM += m.IM_int;
  // depths (:1711, :1726)
  const double h_snow = m.h_swe * p.ws;
  const double h_ice = m.h_iwe * p.wi;
  st.h_swe = m.h_swe;
  st.h_iwe = m.h_iwe;
  st.Eccs = m.Eccs;
  st.Ecci = m.Ecci;
  st.h_snow = h_snow;
  st.h_ice = h_ice;
  o.h_snow = (float)h_snow;
  o.h_ice = (float)h_ice;
  o.SM = m.SM;
  o.IM = m.IM;
  o.M_total = m.IM + m.SM + P_rain * (1.0f / 3600.0f);  // :1441-1443
  o.RH = RH;
}

// PREC (round 6): the dew point, the turbulent fluxes and the long-wave balance
// in fp64 (tfg_set_flux(TFG_FLUX_F64)).  Eccs integrates E_in over a cold spell
// and SM reads E_in - Eccs at melt onset, where the fp32 rounding of those
// terms adds up; the fp32 form is the default.
template <bool QC, bool NANSAFE, bool PREC = false>
__device__ inline void cell_step_fast(const DevParams& p, const CellStaticF& g, const tfg_uniforms* __restrict__ up,
                                      const tfg_uniforms& u, const double* __restrict__ geo_d, int64_t n_pad,
                                      int64_t cell, float P, float T_air, float Hum_sp, float P_air, float uz,
                                      int32_t q_old, int32_t& q_new, CellState& st, CellOutF& o, DiagF& d, float qc) {
  constexpr bool NS = NANSAFE;
  const bool snow_pos = st.h_snow > 0.0, ice_pos = st.h_ice > 0.0;  // previous-step depths
  const float T_K = T_air + 273.15f;
  const float rT = frcp(T_K);
  // rain/snow split (:578-604): T_air > T_rs, exact via the rounded-down
  // threshold; NaN-safe: both tests written out, so a NaN T_air gives P * 0
  // for both, as the reference's P * (T > T_rs) and P * (T <= T_rs) do
  const bool is_rain = T_air > p.f_T_rs_dn;
  const float P_rain = is_rain ? P : P * 0.0f;
  const float P_snow = (NS ? (T_air <= p.f_T_rs_dn) : !is_rain) ? P : P * 0.0f;
  d.P += P;
  d.Pmax = npmax(d.Pmax, P);
  d.PR += P_rain;
  d.PS += P_snow;
  // vapour pressures [mbar] (:788-826); RH = e_air / e_sat_air (:838)
  // Brutsaert: e_sat = 6.11 exp(17.3 T/(T+237.3)); Satterlund: 10^(11.4-2353/T_K)/100
  const float rA = p.satterlund ? rT : frcp(T_air + 237.3f);
  float inv_esat;
  if (!p.satterlund) {
    inv_esat = (1.0f / 6.11f) * fexp2((-17.3f * kLog2e) * T_air * rA);
  } else {
    inv_esat = 100.0f * fexp2((2353.0f * rT - 11.4f) * 3.3219280948873626f);
  }
  // dew point (:888-893), surface temperature (:906-910), T_air - T_surf
  double Td = T_air, e64 = 0.0, Tsd = 0.0, dTd = 0.0;
  float e_air, T_dew, T_surf, dTs;
  if constexpr (PREC) {
    e64 = ((double)Hum_sp * (double)P_air) * rcp_nr1(fma((double)Hum_sp, p.d_ome100, p.d_eps100));
    const double Ld = tfg_fm::log_p(e64 * (1.0 / 6.1121));
    const double Tdew = (257.14 * Ld) * rcp_nr1(18.678 - Ld);
    Tsd = (snow_pos || ice_pos) ? dmin<NS>(Tdew, 0.0) : Tdew;
    dTd = Td - Tsd;
    e_air = (float)e64;
    T_dew = (float)Tdew;
    T_surf = (float)Tsd;
    dTs = (float)dTd;
  } else {
    e_air = Hum_sp * P_air * frcp_nr(p.f_eps100 + p.f_ome100 * Hum_sp);
    // ln(e_air / 6.1121) as the log of the ratio (~1) and Newton-refined: no
    // bias of v_log_f32 reaches T_dew, which every flux term reads
    const float log_term = flog2_nr(e_air * (1.0f / 6.1121f)) * kLn2;
    T_dew = 257.14f * log_term * frcp_nr(18.678f - log_term);
    T_surf = (snow_pos || ice_pos) ? nmin<NS>(T_dew, 0.0f) : T_dew;
    dTs = T_air - T_surf;
  }
  const float RH = e_air * inv_esat;
  // turbulent fluxes (:640-745, :919-934)
  // log2((z - h_snow)/z0) = ly + k with ly = log2((z - h_snow) 2^-k / z0) ~ 0
  // (k = round(log2(z/z0)), host side): squared as ly (ly + 2k) + k^2, so
  // v_log_f32's error is relative to ly, not to the whole log (~13)
  const float ly2 = flog2(nmax<NS>((p.f_z - (float)st.h_snow) * p.f_inv_z0s, p.f_l2min));
  std::conditional_t<PREC, double, float> Qh, Qe;
  if constexpr (PREC) {
    const double uzd = uz;
    double botd = (uzd * uzd) * (Td + 273.15);
    if (botd == 0.0) botd = 0.01;
    const double top = p.gz * dTd;
    const double L2 = fma((double)ly2, (double)ly2 + 2.0 * p.d_l2k, p.d_l2kk);
    // Dh = Dn / (1 + 10 Ri) or Dn (1 - 10 Ri), Ri = top / bot: one quotient (stability_dh)
    const bool stable = top > 0.0;
    const double num = stable ? botd : fma(-10.0, top, botd);
    const double den = stable ? fma(10.0, top, botd) : botd;
    const double Dhd = (uzd * p.d_k2) * num * rcp_nr1(L2 * den);
    Qh = (p.rho_air_Cp_air * Dhd) * dTd;
    // e_air - e_surf = e_air (1 - e_sat(T_s) / e_sat(T_a)), the exponent difference in one exp
    const double x_es = (-p.d_es_k * dTd) * rcp_nr1((Tsd + p.d_es_c) * (Td + p.d_es_c));
    const double ded = e64 * (1.0 - tfg_fm::exp_p(x_es));
    // lhc / p0 = exp(y), y = ek ln2 / T_K, as exp(c) exp(y - c) with exp(c) in d_qe
    const double s0 = fma((double)g.ek * 0.69314718055994531, rcp_nr1(Td + 273.15), -tfg_fm::kP0Center);
    double p0f;
    if (__builtin_expect(__any(!(fabs(s0) <= tfg_fm::kP0Half)), 0)) {
      TFG_FM_RARE();
      p0f = tfg_fm::exp_p(s0);
    } else {
      p0f = tfg_fm::exp_near(s0);
    }
    Qe = (p.d_qe * Dhd) * ded * p0f;
  } else {
    float bot = (uz * uz) * T_K;
    if (bot == 0.0f) bot = 0.01f;
    const float Ri = p.f_gz * dTs * frcp(bot);
    const float L2sq = fmaf(ly2, ly2 + p.f_l2k2, p.f_l2kk);
    const float Dn = uz * p.f_k2 * frcp(L2sq);
    const float Dh = (Ri > 0.0f) ? Dn * frcp(fmaf(10.0f, Ri, 1.0f)) : Dn * fmaf(-10.0f, Ri, 1.0f);
    // e_air - e_surf with e_surf = RH*e_sat_surf = e_air*e_sat(T_surf)/e_sat(T_air)
    // (:853), written without the cancellation of the two near-equal pressures:
    //   e_air - e_surf = e_air*(1 - 2^x2),  x2 = -k*log2(e)*dTs/((T_s+c)(T_a+c))
    // (Brutsaert k = 17.3*237.3, c = 237.3; Satterlund k = 2353 ln 10, c = 273.15):
    // one unbiased exp2 of the exponent difference, so the remaining error is
    // random (v_exp_f32 rounding), not a bias that would accumulate in Eccs
    const float rS = frcp(T_surf + (p.satterlund ? 273.15f : 237.3f));
    const float xs2 = (p.satterlund ? -7816.4968f : -5922.6815f) * dTs * rS * rA;
    const float de = fmaf(-e_air, fexp2(xs2), e_air);
    Qh = p.f_rho_air_Cp_air * Dh * dTs;
    Qe = p.f_qe * Dh * de * fexp2(g.ek * rT);  // lhc / p0 folded
  }
  // snowfall window + albedo ageing (:1006-1059)
  {
    const float sq = P_snow * p.f_qfac;  // P_snow*dt*ws*2^36
    const int32_t q = (int32_t)__float2int_rn(fminf(fmaxf(sq, -2147483520.0f), 2147483520.0f));
    q_new = NS ? ((sq == sq) ? q : kWindowNan) : q;
  }
  if constexpr (NS) {
    st.tot_q += window_tot(q_new) - window_tot(q_old);
    st.n = window_days(st.n, st.tot_q, p.thr_q, p.days_per_dt);
  } else {  // no NaN slot in the window (nan_forcing)
    st.tot_q += (int64_t)q_new - (int64_t)q_old;
    st.n = (st.tot_q >= p.thr_q) ? 0.0 : st.n + p.days_per_dt;
  }
  float albedo;
  {
    // selects in fp32: albedo is rebuilt every step from n and the depths
    // (the previous value survives only for a NaN snow depth)
    const float r = (T_air > 0.0f) ? (0.12f * kLog2e) : (0.05f * kLog2e);
    const float snow_albedo = 0.4f + 0.44f * fexp2(-(float)st.n * r);
    float a = snow_pos ? snow_albedo : (float)st.albedo;
    if (st.h_snow == 0.0 && ice_pos) a = 0.3f;
    if (st.h_snow == 0.0 && st.h_ice == 0.0) a = 0.15f;
    st.albedo = (double)a;
    albedo = a;
  }
  // clear-sky shortwave (SF:904-941), only while the sun is up on a flat
  // surface somewhere this step (flat_dark, a step uniform, makes every cell
  // dark: K_cs = 0 in the reference too): half the steps skip W_p, tau and
  // gam_s and the slope geometry
  float K_cs = 0.0f;
  if (!u.flat_dark) {
    const float w = fexp2((0.0614f * kLog2e) * T_dew);
    const float tau = nmin<NS>(nmax<NS>(fexp2(fmaf(u.tau_c1, w, u.tau_c0)) - p.f_dust, 0.0f), 1.0f);  // SF:614
    const float gam_s = p.f_1pdust - fexp2(fmaf(u.gam_c1, w, u.gam_c0));
    // cos(lat_eq)*cos(omega*th + dlon)
    const float cwl = u.cos_wth_f * g.cc - u.sin_wth_f * g.cs;
    // SF:887; the geometry planes are never NaN (derive_geo maps a NaN slope or
    // aspect to the reference's 0), so IEEE max is exact here in both forms
    const float K_ET = fmaxf(fmaf(u.kc_f, cwl, u.ks_f * g.sl), 0.0f);
    const float kf = u.k_et_flat_f;
    const float K_dif = 0.5f * gam_s * kf;
    const float K_bs = 0.5f * gam_s * albedo * fmaf(tau, kf, K_dif);
    K_cs = tau * K_ET + K_dif + K_bs;
    // dark (SF:939-941): with x = omega*th + dlon and ac = acos(clip(-tan(lat_eq) tan(d))),
    // th <= T_sr or th >= T_ss  <=>  flat_dark or |x| >= ac
    //                           <=>  flat_dark or |x| > pi or cos(lat_eq) cos(x) <= -sin(lat_eq) tan(d).
    // Within the fp32 error margins the fp64 reference form decides.
    {
      const float dv = fmaf(g.sl, u.tan_d_f, cwl);
      const float ax = fabsf(u.omega_th_f + g.dlon);
      const float mpi = ax - 3.14159265358979f;
      bool dark;
      if (!(fabsf(dv) >= 1e-5f) || !(fabsf(mpi) >= 1e-4f)) {
        dark = dark_exact(p, geo_d, n_pad, cell, up);
      } else {
        dark = (mpi > 0.0f) || (dv <= 0.0f);  // flat_dark: handled above
      }
      if (dark) K_cs = 0.0f;
    }
  }
  const float Qn_SW = K_cs * (1.0f - albedo);
  // longwave (:1167-1248): em_air - 1 (the balance below needs only that)
  float em_m1;
  if (!p.satterlund) {
    if constexpr (PREC) {
      em_m1 = 0.0f;  // fp64 below
    } else {
      // (e_air / (10 T_K))^(1/7) as (e_air 102.4 / T_K)^(1/7) 2^(-10/7): the
      // scaled argument is ~1, so v_log_f32's relative error stays off the root
      const float em_r = fexp2(flog2(e_air * p.f_em_sc * rT) * (1.0f / 7.0f));
      em_m1 = fmaf(p.f_ccFs, em_r, p.f_Fm1);  // (1-F) 1.72 (1+0.22C^2) root + F - 1
    }
  } else {
    em_m1 = 1.08f * (1.0f - fexp2(-kLog2e * fexp2(flog2(e_air) * (T_K * (1.0f / 2016.0f))))) - 1.0f;
  }
  // em Ta^4 - Ts^4 without its cancellation (LW_in ~ LW_out ~ 300 W m-2, net
  // ~100): (em - 1) Ta^4 + (Ta - Ts)(Ta + Ts)(Ta^2 + Ts^2), with Ta - Ts the
  // degC difference dTs (free of the rounding of the two +273.15 sums)
  std::conditional_t<PREC, double, float> Qn_LW;
  if constexpr (PREC) {
    // em_air's seventh root by one Halley step from an fp32 seed (root7, the
    // fp64 engine's; Satterlund's em_air stays fp32), the balance in fp64
    const double TaK = Td + 273.15, TsK = Tsd + 273.15;
    const double emd_m1 = p.satterlund ? (double)em_m1
                                       : fma(p.one_minus_F_172 * p.cloud_term, root7_p((e64 * 0.1) * rcp_nr1(TaK)), p.F - 1.0);
    const double ta2d = TaK * TaK;
    Qn_LW = p.em_surf_sigma * fma(emd_m1, ta2d * ta2d, dTd * (TaK + TsK) * fma(TsK, TsK, ta2d));
  } else {
    const float T_surf_K = T_surf + 273.15f;
    const float ta2 = T_K * T_K;
    const float d4 = dTs * (T_K + T_surf_K) * fmaf(T_surf_K, T_surf_K, ta2);
    Qn_LW = p.f_em_surf_sigma * fmaf(em_m1, ta2 * ta2, d4);
  }
  // :1314 (Qa = 0; Qc last): fp64 in the PREC form, E_in = Q_sum dt then in fp64
  std::conditional_t<PREC, double, float> Q_sum;
  if constexpr (PREC) Q_sum = (((double)Qn_SW + Qn_LW) + Qh) + Qe + (QC ? (double)qc : 0.0);
  else {
    Q_sum = Qn_SW + Qn_LW + Qh + Qe;
    if constexpr (QC) Q_sum = Q_sum + qc;
  }

  melt_fast<NS, decltype(Q_sum)>(p, Q_sum, P_snow, P_rain, RH, T_air, st, o, d);
#if defined(TFG_DEBUG_TERMS)  // diagnostic builds only (tests/diagnostics/term_bias.py): the step's
                              // energy terms replace the six outputs; the state evolves as usual
  o.h_snow = Qn_SW;
  o.SM = (float)Qn_LW;
  o.h_ice = (float)Qh;
  o.IM = (float)Qe;
  o.M_total = P_snow > 0.0f ? snowfall_cold(p, P_snow, RH, T_air) : 0.0f;
  o.RH = (float)Q_sum;
#endif
}

}  // namespace tfg
