/*
 * tfg.h -- C ABI of the MI355X glacier energy-balance engine (libtfg).
 *
 * The reference (NGWPC/topoflow-glacier v0.1.0) has no native code: its hot
 * path is the pure-NumPy method BmiTopoflowGlacier.update()
 * (src/topoflow_glacier/bmi/bmi_topoflow_glacier.py:413-465), one catchment
 * per Python call.  This header is the boundary that replaces it: the Python
 * BMI class (topoflow-glacier_amd/topoflow_glacier/bmi/bmi_topoflow_glacier.py)
 * binds these entry points through ctypes (topoflow_glacier/_native.py).
 * Each entry point names the reference interface it stands in for.
 *
 * Calling rules
 *   - Every function returns an int status: 0 = TFG_OK, nonzero = error; the
 *     message is then available from tfg_last_error(h) (or tfg_last_error(NULL)
 *     for failures before a handle exists).  No C++ exception crosses the ABI.
 *   - A handle owns all device buffers of one grid shard and one HIP stream.
 *     Host pointers are borrowed for the duration of the call only.
 *   - One thread per handle; calls on a handle are not re-entrant.
 *   - Plain C types only: no torch / HIP types appear in the signatures
 *     (streams are passed as void*).
 */
#ifndef TFG_H
#define TFG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFG_ABI_VERSION 8

/* status codes */
enum {
  TFG_OK = 0,
  TFG_ERR_ARG = 1,     /* invalid argument (bad field id, size mismatch, null) */
  TFG_ERR_HIP = 2,     /* a HIP runtime call failed                            */
  TFG_ERR_STATE = 3,   /* call not valid in the handle's current state          */
  TFG_ERR_DOMAIN = 4,  /* physically invalid input, e.g. slope angle out of
                          [0, pi/2] (reference: set_slope_angle :1106-1111)    */
};

/* arithmetic of an engine / element type of a host or device buffer */
enum {
  TFG_F32 = 0, /* fp32 forcing/static/outputs, fp32 flux arithmetic, fp64 state */
  TFG_F64 = 1, /* fp64 everywhere, reference operation order (bit-near parity)  */
  TFG_I32 = 2, /* catchment-id raster only                                      */
};

/* Field ids.  Inputs follow _dynamic_input_vars (bmi_topoflow_glacier.py:18-26)
 * and outputs _output_vars (:28-37) in the same order. */
enum {
  /* dynamic inputs (per forcing frame).  LW and SW are accepted for BMI
   * completeness but the reference physics never reads them (:1122, :1235). */
  TFG_IN_LW_IN = 0,  /* land_surface_radiation~incoming~longwave__energy_flux */
  TFG_IN_P_AIR = 1,  /* land_surface_air__pressure [Pa]                         */
  TFG_IN_HUM_SP = 2, /* atmosphere_air_water~vapor__relative_saturation (q)     */
  TFG_IN_P = 3,      /* atmosphere_water__liquid_equivalent_precipitation_rate  */
  TFG_IN_SW_IN = 4,  /* land_surface_radiation~incoming~shortwave__energy_flux  */
  TFG_IN_T_AIR = 5,  /* land_surface_air__temperature [degC]                    */
  TFG_IN_UZ = 6,     /* wind_speed_UV [m s-1]                                   */
  /* BMI outputs (history slot addressable) */
  TFG_OUT_H_SNOW = 7,  /* snowpack__depth                                       */
  TFG_OUT_H_SWE = 8,   /* snowpack__liquid-equivalent_depth  (fp64 state)        */
  TFG_OUT_SM = 9,      /* snowpack__melt_volume_flux                             */
  TFG_OUT_H_ICE = 10,  /* glacier_ice__thickness                                 */
  TFG_OUT_H_IWE = 11,  /* glacier__liquid_equivalent_depth    (fp64 state)        */
  TFG_OUT_IM = 12,     /* glacier_ice__melt_volume_flux                          */
  TFG_OUT_M_TOTAL = 13,/* land_surface_water__runoff_volume_flux                 */
  TFG_OUT_RH = 14,     /* atmosphere_bottom_air_water-vapor__relative_saturation */
  /* static rasters (config.py:19-28 scalars `elev`, `slope`, `aspect` become
   * per-cell rasters) and the optional catchment-id raster */
  TFG_ST_ELEV = 15,
  TFG_ST_SLOPE = 16,
  TFG_ST_ASPECT = 17,
  TFG_ST_CATCH_ID = 18,
  /* internal state (not BMI-visible in the reference, exposed for checkpoint) */
  TFG_ST_ECCS = 19,   /* snowpack cold content  (:392, :1496-1564)           */
  TFG_ST_ECCI = 20,   /* ice cold content       (:394, :1375-1434)           */
  TFG_ST_ALBEDO = 21, /* albedo                 (:369, :1006-1059)           */
  TFG_ST_NDAYS = 22,  /* days since major snowfall (:1040)                   */
  /* snowfall window (checkpoint / restart): slot `index` (0..ring_len-1) in
   * metres of snow, P_snow*dt*ws of one step (:1027-1033); step k writes slot
   * k mod ring_len.  Setting a slot rebuilds the running total before the
   * next tfg_step. */
  TFG_ST_WINDOW = 23,
  /* lateral conduction flux Qc [W m-2] added to Q_sum (:1314) while the
   * optional conduction term is on: written by tfg_conduction_update, or set
   * directly (which switches the term on); zero otherwise, as the reference's
   * Qc (:312, :936-948).  Engine element type. */
  TFG_ST_QC = 24,
  TFG_NUM_FIELDS = 25
};

/* Diagnostics per catchment, in this order (:558-624, :1482-1494). */
enum { TFG_DIAG_VOL_P = 0, TFG_DIAG_VOL_PR, TFG_DIAG_VOL_PS, TFG_DIAG_VOL_SM,
       TFG_DIAG_VOL_IM, TFG_DIAG_P_MAX, TFG_NUM_DIAG };

/* Model constants: TopoflowGlacierConfig (config.py:6-115) fields consumed by
 * update(), plus the grid geometry the reference keeps as scalars. */
typedef struct tfg_params {
  double dt;             /* config.py:15 (hours; used as-is in energy terms)  */
  double da_m2;          /* cell area [m2] (reference: da_km2*1e6, :293-294)   */
  double lat, lon;       /* config.py:21-22 (uniform over the grid)           */
  double sin_lat, cos_lat; /* sin/cos of lat*(pi/180), as the host computes them
                              (Equivalent_Latitude SF:753-755)                  */
  double T_rain_snow, dust_atten, canopy_factor, cloud_factor;
  double rho_air, rho_snow, rho_ice, rho_H2O, h_active_layer, T0;
  double Cp_air, Cp_ice, Cp_snow, g, Lf, eps, kappa, latent_heat_constant, Lv;
  double sigma, sea_level_p0, uni_gas_const, M_mass_air, z0_air, em_surf;
  int32_t satterlund;    /* config.py:101                                      */
  int32_t ring_len;      /* int(3*24/dt) snowfall-window slots (:296)          */
  double glens_A;        /* Glen's flow-law rate factor [Pa^-3 yr^-1] (config.py:65);
                            read only by the optional ice-flow term          */
} tfg_params;

/* Per-step uniform scalars, computed on the host in fp64 from the model clock
 * (update_julian_day :957-1004 and the uniform part of Clear_Sky_Radiation,
 * SF:894-953).  One record per time step. */
typedef struct tfg_uniforms {
  double th;         /* TSN_offset [h]                                (:1004) */
  double omega_th;   /* omega*th [rad]                                  SF:867 */
  double cos_wth;    /* cos(omega*th)                                           */
  double sin_wth;    /* sin(omega*th)                                           */
  double sin_d;      /* sin(declination)                                 SF:205 */
  double cos_d;      /* cos(declination)                                        */
  double tan_d;      /* tan(declination)                                 SF:325 */
  double isc_e0;     /* Solar_Constant()*Eccentricity_Correction()       SF:869 */
  double m_opt;      /* Optical_Air_Mass(lat, delta, th)                 SF:498 */
  double k_et_flat;  /* ET_Radiation_Flux(lat, JD, th), clamped >= 0     SF:376 */
  double flat_sr;    /* Sunrise_Offset(lat, delta)                       SF:305 */
  double flat_ss;    /* Sunset_Offset(lat, delta)                        SF:334 */
  /* fp32 engine: coefficients derived from the fields above in fp64 on the
   * host, then rounded (Clear_Sky_Radiation SF:904-941 regrouped per step) */
  float cos_wth_f;   /* cos(omega*th)                                           */
  float sin_wth_f;   /* sin(omega*th)                                           */
  float omega_th_f;  /* omega*th                                                */
  float tan_d_f;     /* tan(declination)                                        */
  float kc_f;        /* isc_e0*cos(d): K_ET = kc*cos(lat_eq)*cos(w*th+dlon)     */
  float ks_f;        /* isc_e0*sin(d):        + ks*sin(lat_eq)        SF:867-869 */
  float k_et_flat_f; /* k_et_flat                                               */
  float tau_c0, tau_c1; /* tau = exp2(c0 + c1*w) - dust, w = exp(0.0614*T_dew):
                           log2(e)*(a_sa + b_sa*m_opt) regrouped     SF:606-613 */
  float gam_c0, gam_c1; /* gam_s = 1 + dust - exp2(c0 + c1*w)        SF:648-655 */
  float pad_f;
  int32_t frame;     /* forcing frame index this step reads                     */
  int32_t hist;      /* output-history slot this step writes                    */
  int32_t slot;      /* snowfall-window ring slot (step mod ring_len)           */
  int32_t flat_dark; /* th <= flat_sr || th >= flat_ss (fp64): dark on the flat
                        centroid, hence on every slope                SF:939-941 */
} tfg_uniforms;

typedef struct tfg_handle tfg_handle;

/* Library / device info.  tfg_build_info() names the ABI, the target and
 * "tfg-src-sha256=<hex>", the hash of the sources and compile flags the
 * library was built from (__graft_entry__.build() rebuilds on a mismatch). */
int tfg_abi_version(void);
const char* tfg_build_info(void);
int tfg_device_count(int* count);

/* Create one grid shard of ny*nx cells on `device`.
 *   engine      TFG_F32 or TFG_F64
 *   n_frames    forcing frames resident on the device (>= 1)
 *   hist_depth  output-history slots (>= 1); step k writes slot u[k].hist
 *   n_catch     catchments for the mass-balance diagnostics (>= 1)
 * Replaces: BmiTopoflowGlacier.__init__ + initialize() array setup
 * (bmi_topoflow_glacier.py:118-122, :281-395). */
int tfg_create(const tfg_params* p, int64_t ny, int64_t nx, int engine, int device,
               int n_frames, int hist_depth, int n_catch, tfg_handle** out);

/* Release everything, after the handle's stream (a caller-set one too) has
 * drained.  Replaces: finalize() (:467-469). */
int tfg_destroy(tfg_handle* h);

/* Run the work on a caller-provided HIP stream (hipStream_t as void*), or
 * NULL to return to the handle's own stream. */
int tfg_set_stream(tfg_handle* h, void* stream);
int tfg_get_stream(tfg_handle* h, void** stream);

/* The process-wide HIP stream of `device` (created on first use, never
 * destroyed), for callers that run many small handles in turn: NextGen steps
 * one single-catchment model per catchment, and one stream for all of them
 * saves ~12 us per instance-step at 500 instances.  Pass it to tfg_set_stream.
 * No reference counterpart (the reference is single-threaded NumPy). */
int tfg_shared_stream(int device, void** stream);

/* Copy n cells into a field.  `index` is the forcing frame for TFG_IN_*,
 * ignored otherwise.  src_dtype is the element type of `src`; it is converted
 * on the device.  src_on_device != 0 means `src` is a device pointer.
 * Replaces: set_value / Context.set_value (:1800-1802, context.py:42-44). */
int tfg_set_field(tfg_handle* h, int field, int index, const void* src, int src_dtype,
                  int64_t n, int src_on_device);

/* The five inputs the physics reads, for one forcing frame, in one call:
 * src is [5][n] in _dynamic_input_vars order without the radiation terms
 * (bmi_topoflow_glacier.py:18-26): P_air, Hum_sp, P, T_air, uz.  Host data is
 * copied into a pinned staging ring, so the call returns without waiting for
 * the device.  Replaces: the per-step set_value() calls of a caller
 * (examples/run_topoflow_glacier.py:63-71). */
int tfg_set_inputs(tfg_handle* h, int frame, const void* src, int src_dtype, int64_t n, int src_on_device);

/* The eight BMI outputs in _output_vars order (:28-37): h_snow, h_swe, SM,
 * h_ice, h_iwe, IM, M_total, RH, as dst[8][n], from output-history slot
 * `hist` (h_swe/h_iwe: the current state).  One gather and one copy.
 * Replaces: the per-step get_value() calls (:1810-1822). */
int tfg_get_outputs(tfg_handle* h, int hist, void* dst, int dst_dtype, int64_t n, int dst_on_device);

/* One synchronous model step for callers that step from the host (the BMI's
 * update(), :413-465): the same as tfg_set_inputs(h, frame, src, ...) +
 * tfg_step(h, u, 1) + tfg_get_outputs(h, u->hist, dst, ...), with u->frame ==
 * frame, but the kernels read src and u and write dst through one pinned,
 * device-mapped block (no staging copies) and the call returns with dst
 * filled.  src[5][n] / dst[8][n] are host buffers in the orders of
 * tfg_set_inputs / tfg_get_outputs. */
int tfg_update(tfg_handle* h, int frame, const void* src, int src_dtype, const tfg_uniforms* u, void* dst,
               int dst_dtype, int64_t n);

/* One synchronous step of each of m single-cell TFG_F64 handles, in ONE
 * launch: for handle hs[i], the same as tfg_update(hs[i], u[i]->frame,
 * src[i], TFG_F64, u[i], dst[i], TFG_F64, 1), and the same results bit for
 * bit.  src[i] is that handle's 5 fp64 inputs in tfg_set_inputs order
 * (P_air, Hum_sp, P, T_air, uz), dst[i] its 8 fp64 outputs in
 * tfg_get_outputs order.  Every handle must be on one device and share one
 * stream (tfg_shared_stream), and may appear once.  Errors name the handle's
 * index and are read with tfg_last_error(NULL); no step runs then.
 * Replaces: update() (:413-465) of many single-catchment models, one Python
 * object per catchment as NextGen runs them, when a caller has advanced them
 * all before reading any (the BMI's `defer_update` mode). */
int tfg_update_many(tfg_handle* const* hs, int m, const double* const* src, const tfg_uniforms* const* u,
                    double* const* dst);

/* `index` value for TFG_OUT_H_SNOW / TFG_OUT_H_ICE: the fp64 previous-step
 * depth the next step reads (:895-911 uses the previous depths), rather than a
 * history slot -- exact checkpoint / restart. */
#define TFG_PREV_DEPTH (-1)

/* Copy n cells of a field out: n = ny*nx, or fewer for the first n cells in
 * row-major order (a leading block of rows, e.g. a sample of a large shard).
 * `index` is the history slot for TFG_OUT_* (except H_SWE/H_IWE, which are
 * state; TFG_PREV_DEPTH above), the frame for TFG_IN_*.
 * Replaces: get_value / get_value_ptr (:1810-1828). */
int tfg_get_field(tfg_handle* h, int field, int index, void* dst, int dst_dtype, int64_t n,
                  int dst_on_device);

/* (Re)initialise the internal state from the current depth fields: cold
 * contents Eccs/Ecci (:389-395), albedo 0.3 (:369), days-since-snowfall 0
 * (:288), empty snowfall window (:296), zero diagnostics (:314-317, :362-363).
 * Call after the initial h_snow/h_ice/h_swe/h_iwe rasters are set. */
int tfg_init_state(tfg_handle* h);

/* Advance nsteps time steps; u[k] are the uniforms of step k.
 * Replaces: update() (:413-465) when nsteps == 1 and update_until()
 * (:471-490) otherwise.  Steps are fused into multi-step launches that keep
 * the per-cell state in registers; every step still reads its forcing frame
 * and writes its six outputs to history slot u[k].hist. */
int tfg_step(tfg_handle* h, const tfg_uniforms* u, int64_t nsteps);

/* Maximum steps fused into one launch (default 24; 1 disables fusion). */
int tfg_set_fuse(tfg_handle* h, int max_steps_per_launch);

/* Mass-balance diagnostics, out[n_catch][TFG_NUM_DIAG] (fp64, blocking).
 * Replaces: the vol_P/vol_PR/vol_PS/vol_SM/vol_IM integrals and P_max
 * (:558-624, :1482-1494). */
int tfg_get_diag(tfg_handle* h, double* out, int n_catch);
int tfg_reset_diag(tfg_handle* h);

/* Wait for all work queued on the handle's stream. */
int tfg_sync(tfg_handle* h);

/* Missing data (fp32 engine).  The reference's numpy arithmetic propagates NaN
 * (np.maximum / np.minimum, the NaN window sum freezing n; :1035-1041,
 * :1364-1434).  Each launch of the fp32 engine runs its clean step form when
 * everything the launch reads (its forcing frames or tfg_update's inputs, the
 * elevation raster, the Qc plane in use, the state and the snowfall window) is
 * known to be finite, and its NaN-safe form otherwise; the results agree
 * wherever the data is finite.  Finiteness is checked where data enters from
 * host memory (tfg_set_field, tfg_set_inputs and tfg_update; fp64 values as
 * the fp32 values they become).  Data set from device memory stays
 * stream-ordered (no host wait) and of unknown status; before a launch of 8
 * or more steps unknown data is checked (a synchronous device check), and a
 * shorter launch runs the NaN-safe form.  *count = launches that ran the
 * NaN-safe form. */
int tfg_nan_safe_launches(tfg_handle* h, int64_t* count);

/* The fp32 engine's step form: TFG_FORM_AUTO (the default: chosen per launch
 * as above) or TFG_FORM_NAN_SAFE (every launch; the same results wherever the
 * data is finite -- tests and measurements of the two forms).  No reference
 * counterpart. */
#define TFG_FORM_AUTO 0
#define TFG_FORM_NAN_SAFE 1
int tfg_set_step_form(tfg_handle* h, int form);

/* The fp32 engine's energy-flux precision (ABI 7, round 6): TFG_FLUX_F32 (the
 * default) computes the step's flux terms in fp32; TFG_FLUX_F64 computes the
 * dew point (:888-910), the turbulent fluxes (:640-745, :919-934) and the
 * long-wave balance (:1146-1257) in fp64, so that the cold content Eccs, which
 * integrates E_in = Q_sum dt over a cold spell (:1496-1564), carries no fp32
 * rounding into the snow melt at melt onset (:1321-1373).  Forcing, state
 * layout and outputs are the same; the fp64 engine ignores it.  Replaces no
 * reference interface (the reference is fp64 numpy throughout). */
#define TFG_FLUX_F32 0
#define TFG_FLUX_F64 1
int tfg_set_flux(tfg_handle* h, int flux);

/* Split launches (ABI 8, round 6).  A grid of at most 2^24 cells fills the
 * chip's resident workgroups only a few times per launch, and the end of every
 * launch drains with most slots idle.  The fp32 engine then steps it as two
 * parts of about half the cells each, the second on a second stream of its own
 * with its own copy of the step uniforms: one part's next launch fills the other
 * part's drain (+4-5 % at 1024^2 and 4096^2; none at 8192^2, which runs one part).
 * Results are the same bit for bit (the update is pointwise; each part's
 * workgroups fold their diagnostics into the slab rows of their own cells).
 *   TFG_SPLIT_AUTO  (default) split fp32-engine grids of 2^18 (one round of the
 *                   resident workgroups) to 2^24 cells
 *   TFG_SPLIT_OFF   one launch over the whole grid
 *   TFG_SPLIT_ON    split every fp32-engine grid of at least 512 cells (tests)
 * While split, tfg_step returns with the second part's launches queued on the
 * second stream only: every other call of this API orders the handle's stream
 * after them first, and tfg_join does just that (without waiting on the host),
 * for a caller that queues its own work on the handle's stream (tfg_get_stream)
 * after tfg_step, e.g. an event marking the steps' end.  No reference
 * counterpart (the reference is single-threaded NumPy). */
#define TFG_SPLIT_AUTO 0
#define TFG_SPLIT_OFF 1
#define TFG_SPLIT_ON 2
int tfg_set_split(tfg_handle* h, int mode);
int tfg_join(tfg_handle* h);
/* 1 if the handle's next tfg_step runs split, else 0. */
int tfg_get_split(tfg_handle* h, int* split);

/* Self-test of the fp64 engine's power rewrites on the device (tests only):
 * out[i] = pow4(x[i]) (which = 0: T^4, :1231-1233), pow1p5(x[i]) (1: RH^1.5,
 * :1520) or root7(x[i]) (2: em_air's 1/7 power, :1167), computed by the
 * same device functions the engine's steps call; and the fp64 engine's exp,
 * log and constant-divisor division (csrc/tfg_fastmath.hpp): exp_k (3), the
 * device libm's exp (4), log_k (5), the device libm's log (6), x / 6.1121 (7)
 * and x / 3600 (8) by div_k, exp_kv (9: exp_k with its constants in
 * vector registers), fdiv(x, 7.3) (10), fdiv(7.3, x) (11), and the wet bulb's
 * arctangent atan_q: atan(x / 7.3) (12) and atan(-7.3 / x) (13).  Host arrays
 * of n values, synchronous. */
int tfg_selftest_powers(int device, const double* x, int64_t n, int which, double* out);

/* Device-side synthetic workload generator (bench / tests): fills the forcing
 * frames, static rasters and initial depths from a counter-based hash of
 * (seed, field, frame, global cell index).  `row0` is this shard's first row in
 * the global grid so shards of one grid agree with an unsharded run.
 * `diurnal` holds n_frames fp32 diurnal-cycle factors.  The host mirror is
 * topoflow_glacier/synthetic.py (bit-identical fp32 values). */
int tfg_fill_synthetic(tfg_handle* h, uint64_t seed, int64_t row0, int64_t nx_global,
                       const float* diurnal, int n_frames);

/* Terrain from a DEM (extension): slope (tan beta) and
 * aspect rasters from the handle's elevation raster by Horn's 3x3 finite
 * differences, fp64.  The reference takes both as YAML scalars (config.py:19,
 * :28) and uses them through set_slope_angle / set_aspect_angle (:1082-1113);
 * aspect here is the downslope direction in radians counter-clockwise from
 * east, the quantity those functions turn into alpha = pi/2 - aspect.
 *   dx, dy      cell size [m]; rows run north to south, columns west to east
 *   halo_north  elevation row just north of this shard's first row (nx values),
 *   halo_south  ... just south of its last row; NULL at the domain edge (the
 *               edge row is replicated, as are the first/last columns)
 *   halo_dtype  TFG_F32 / TFG_F64; halo_on_device != 0: device pointers
 * Row-block shards exchange these one-row halos (topoflow_glacier/sharding.py,
 * RCCL over xGMI); the sharded result equals the unsharded one. */
int tfg_terrain_from_dem(tfg_handle* h, double dx, double dy, const void* halo_north, const void* halo_south,
                         int halo_dtype, int halo_on_device);

/* Optional lateral ice flow (extension): the
 * shallow-ice approximation with Glen's law (n = 3) moves ice thickness
 * H = h_iwe * rho_H2O/rho_ice between neighbouring cells over the bed
 * `elev`.  The reference declares the flow parameters (glens_A, in
 * Pa^-3 yr^-1, config.py:64-65) but never moves ice (Qc = Qa = 0, :936-955),
 * so the term is off unless a caller invokes it and results then depart from
 * the reference by design.  Explicit, flux form on cell faces, fp64:
 *   q_face = -Gamma * Hf^5 * |grad s|^2 * ds/dn,  Gamma = 2A/5 (rho_ice g)^3,
 *   Hf the face-mean thickness, each face flux limited to a quarter of the
 *   donor cell's ice per sub-step (H never goes negative), zero flux across
 *   the domain edge.  Ice volume is conserved to rounding.
 * Halo rows are [2][nx] fp64: row 0 the surface elevation s = elev + H, row 1
 * the ice thickness H, of the neighbour shard's row adjacent to this shard;
 * NULL at the domain edge.  Row-block shards exchange them before every
 * sub-step (topoflow_glacier/sharding.py, RCCL over xGMI); the sharded result
 * equals the unsharded one bit for bit.
 *
 * This shard's first and last rows as halo rows for its neighbours
 * (first[2][nx], last[2][nx], fp64; blocking). */
int tfg_ice_flow_edges(tfg_handle* h, double* first, double* last, int on_device);
/* Largest face diffusivity Gamma*Hf^5*|grad s|^2 [m2 yr-1] (blocking); it
 * sets the stable sub-step dt <= min(dx, dy)^2 / (4 D). */
int tfg_ice_flow_dmax(tfg_handle* h, double dx, double dy, const double* halo_north, const double* halo_south,
                      int halo_on_device, double* dmax);
/* One explicit sub-step of dt_years.  `part` splits it so a sharded caller
 * can overlap its halo exchange with the interior rows:
 *   TFG_FLOW_ALL       the whole sub-step (blocking);
 *   TFG_FLOW_INTERIOR  the rows that read no halo row, queued asynchronously
 *                      (pass no halos); it must be followed by
 *   TFG_FLOW_EDGES     the rows next to the halos, then the commit (blocking).
 * The sub-step reads the pre-step h_iwe throughout, so ALL == INTERIOR + EDGES
 * bit for bit.  The new h_iwe lands in the state at the commit; h_ice, which
 * the sub-step does not read, is written as each part runs. */
enum { TFG_FLOW_ALL = 0, TFG_FLOW_INTERIOR = 1, TFG_FLOW_EDGES = 2 };
int tfg_ice_flow_step(tfg_handle* h, double dt_years, double dx, double dy, const double* halo_north,
                      const double* halo_south, int halo_on_device, int part);
/* n_sub sub-steps of dt_years / n_sub on an unsharded grid (no halos), in one
 * blocking call: the sub-steps alternate between the state plane and a
 * scratch plane, so no per-sub-step commit pass is needed.  Equals n_sub
 * tfg_ice_flow_step calls bit for bit. */
int tfg_ice_flow_run(tfg_handle* h, double dt_years, double dx, double dy, int n_sub);

/* Optional lateral heat conduction (extension): the
 * conduction term the reference reserves in the energy balance and leaves at
 * zero (update_conduction_heat_flux :936-948, Qc = 0 from :312; Q_sum adds Qc
 * last, :1314).  Fourier's law between neighbouring cells, fp64:
 *   T_snow = T0 - Eccs / (rho_snow Cp_snow h_snow),
 *   T_ice  = T0 - Ecci / (rho_ice Cp_ice h_active_layer)   (:389-395),
 *   Qc = sum over the 4 faces of k_snow min(h_snow, h_snow') (T_snow' - T_snow)
 *        / d^2  [both cells snow-covered] + k_ice h_active_layer
 *        (T_ice' - T_ice) / d^2  [both cells ice-covered],
 * d = dx (west/east) or dy (north/south); no flux across the domain edge.
 * The pair of cells of a face see exact negatives of one flux.  Qc is
 * evaluated from the current state and then held by every tfg_step until the
 * next update (operator splitting over a conduction interval; the step
 * fusion is unchanged).
 * Halo rows are [4][nx] fp64: T_snow, h_snow, T_ice, h_ice of the neighbour
 * shard's row adjacent to this shard; NULL at the domain edge.  Row-block
 * shards exchange them before each update (topoflow_glacier/sharding.py,
 * RCCL over xGMI); the sharded Qc equals the unsharded one bit for bit.
 *
 * This shard's first and last rows as halo rows (first[4][nx], last[4][nx];
 * blocking). */
int tfg_conduction_edges(tfg_handle* h, double* first, double* last, int on_device);
/* Evaluate Qc from the current state and switch the term on (k_snow, k_ice
 * [W m-1 K-1], dx, dy [m]; q_ground [W m-2] is added to every cell: the
 * ground heat flux, the reference's declared but unused geothermal flux Qg,
 * config.py:84 / :333, converted from J yr-1 m-2; 0 for none).  The halo rows
 * are read before the call returns. */
int tfg_conduction_update(tfg_handle* h, double k_snow, double k_ice, double dx, double dy, double q_ground,
                          const double* halo_north, const double* halo_south, int halo_on_device);
/* Switch the term off (Qc = 0: the reference's energy balance again). */
int tfg_conduction_off(tfg_handle* h);

/* Last error message of a handle (NULL: the last create/global error). */
const char* tfg_last_error(const tfg_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* TFG_H */
