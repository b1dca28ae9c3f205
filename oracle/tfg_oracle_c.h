/* ORACLE (C) -- TEST INFRASTRUCTURE ONLY (see tfg_oracle_c.c).  Not part of the
 * product ABI (include/tfg.h); loaded only by tests/, smoke() and bench.py's
 * cpu_baseline leg through oracle/tfg_oracle_c.py. */
#ifndef TFG_ORACLE_C_H
#define TFG_ORACLE_C_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_OK = 0, ORC_ERR_ARG = 1, ORC_ERR_SLOPE = 2 };

/* config.py:6-115 fields the hot path reads (plus dt, da, lat) */
typedef struct {
  double dt, da, lat, T_rain_snow, dust_atten, canopy_factor, cloud_factor;
  double rho_air, rho_snow, rho_ice, rho_H2O, h_active_layer, T0, Cp_air, Cp_ice, Cp_snow;
  double g, Lf, eps, kappa, latent_heat_constant, Lv, sigma, sea_level_p0, uni_gas_const, M_mass_air;
  double z0_air, em_surf;
  int32_t satterlund;
  int32_t pad_;
} orc_params;

/* Run nsteps update() steps over ncell independent cells.
 *   static rasters and initial depths: [ncell] each
 *   forcing[5] = P, T_air, Hum_sp, P_air, uz, each [n_frames][ncell]; step k reads
 *     frame[k] (frame == NULL: frame k)
 *   jd, tsn: [nsteps] julian day and TSN offset of each step (the clock)
 *   out_last: [8][ncell] outputs of the last step (h_snow, h_swe, SM, h_ice, h_iwe, IM, M_total, RH) or NULL
 *   out_hist: [nsteps][8][ncell] or NULL
 *   diag: [6] vol_P, vol_PR, vol_PS, vol_SM, vol_IM, P_max or NULL
 *   nthreads: OpenMP threads (<= 0: the OpenMP default)
 * Returns ORC_OK, ORC_ERR_ARG, or ORC_ERR_SLOPE (a slope angle out of range,
 * bmi_topoflow_glacier.py:1106-1111; nothing is run). */
int orc_run(const orc_params* c, int64_t ncell, int nsteps, const double* elev, const double* slope,
            const double* aspect, const double* h0_snow, const double* h0_ice, const double* h0_swe,
            const double* h0_iwe, const double* const* forcing, const int32_t* frame, const double* jd,
            const double* tsn, double* out_last, double* out_hist, double* diag, int nthreads);

/* orc_run from a mid-run state instead of the initialize() state (:274-411):
 *   state0: [8][ncell] h_snow, h_ice (previous-step depths), h_swe, h_iwe, Eccs,
 *     Ecci, albedo, n; or NULL for the initial state from h0_*
 *   ring0: [ncell][ring_len] snowfall window, oldest slot first (the numpy
 *     oracle's `ring` attribute); or NULL for an empty window */
int orc_run_from(const orc_params* c, int64_t ncell, int nsteps, const double* elev, const double* slope,
                 const double* aspect, const double* h0_snow, const double* h0_ice, const double* h0_swe,
                 const double* h0_iwe, const double* state0, const double* ring0, const double* const* forcing,
                 const int32_t* frame, const double* jd, const double* tsn, double* out_last, double* out_hist,
                 double* diag, int nthreads);

/* orc_run_from with the optional lateral conduction flux Qc [W m-2] added to
 * Q_sum (:1314): step k of cell i uses qc[(k / qc_every) * ncell + i] (one
 * [ncell] row per conduction interval of qc_every steps); qc == NULL: Qc = 0. */
int orc_run_from_qc(const orc_params* c, int64_t ncell, int nsteps, const double* elev, const double* slope,
                    const double* aspect, const double* h0_snow, const double* h0_ice, const double* h0_swe,
                    const double* h0_iwe, const double* state0, const double* ring0, const double* const* forcing,
                    const int32_t* frame, const double* jd, const double* tsn, const double* qc, int qc_every,
                    double* out_last, double* out_hist, double* diag, int nthreads);

int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
