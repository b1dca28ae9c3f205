// tfg_engine.hip -- MI355X (gfx950) glacier energy-balance engine: kernels and
// the C ABI declared in include/tfg.h.  The fused step kernel k_fused is in
// tfg_fused.hpp; its fp64 instantiations are compiled in tfg_fused_f64.hip.
//
// Hot path: k_fused<R, EXACT, READ_DEPTHS, CATCH> advances every cell of the
// shard by K consecutive time steps in ONE launch.  A thread owns C adjacent
// cells (C*sizeof(R) = 16 B: one dwordx4 per field per wave-lane); it loads the
// cells' static rasters and fp64 state once, keeps the state in registers for
// the K steps, and per step streams in the step's forcing frame and the
// expiring snowfall-window slot and streams out the new slot and the six BMI
// outputs.  There is no lateral coupling in the reference physics (Qc = Qa = 0,
// bmi_topoflow_glacier.py:936-955), so no LDS tile or halo is needed; LDS only
// holds the per-wave mass-balance bins.
//
// Mass-balance diagnostics (vol_P/PR/PS/SM/IM, P_max: :558-624, :1482-1494)
// are reduced without atomics: lane registers -> wave butterfly (__shfl_xor) ->
// per-wave LDS bins -> one slab row per workgroup (accumulated over launches)
// -> k_diag_reduce when the diagnostics are read, which folds
// the slab into the running fp64 totals in a fixed order (bitwise
// reproducible).
#include <hip/hip_runtime.h>
#include <mutex>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <atomic>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/tfg.h"
#include "tfg_physics.hpp"
#include "tfg_conduction.hpp"
#include "tfg_fused.hpp"

namespace {

using namespace tfg_kern;

// One step of a one-cell fp64 handle for tfg_update (the single-catchment BMI
// update(), :413-465, one model per catchment as NextGen runs it): the step's
// inputs and uniforms arrive as kernel arguments, one workgroup of four waves
// (one per SIMD) runs the step with its transcendental calls batched across
// lanes and function classes across waves (cell_step_exact_wave), and
// thread 0 writes the state, the window slot, the history slot, the frame, the
// eight outputs into the pinned host block, the diagnostic slab row and the
// release flag.  Same arithmetic as k_fused<double, true, ...> with K = 1, so
// the same results bit for bit; the per-launch fixed work (LDS bins, the
// read-back of the history slot, host-memory reads of inputs and uniforms) is
// gone from the critical path.
struct CellIo {
  tfg_uniforms u;
  double in[kNumForc];  // P, T_air, Hum_sp, P_air, uz (device frame order)
};

// The one cell's fp64 state (the depths read or re-derived as k_fused does)
// and its static geometry (k_prepare_static's planes).
__device__ __forceinline__ void load_one_cell(const DevParams& p, int64_t np, const double* __restrict__ st,
                                              const int64_t* __restrict__ tot, const double* __restrict__ geo,
                                              int read_depths, CellState& cs, CellStatic& sx) {
  cs.h_swe = st[S_HSWE * np];
  cs.h_iwe = st[S_HIWE * np];
  cs.Eccs = st[S_ECCS * np];
  cs.Ecci = st[S_ECCI * np];
  cs.n = st[S_N * np];
  cs.albedo = st[S_ALB * np];
  if (read_depths) {
    cs.h_snow = st[S_HSNOW * np];
    cs.h_ice = st[S_HICE * np];
  } else {
    cs.h_snow = cs.h_swe * p.ws;  // :1711, bit-identical to the last step
    cs.h_ice = cs.h_iwe * p.wi;   // :1726
  }
  cs.tot_q = tot[0];
  sx = {geo[0], geo[np], geo[2 * np], geo[3 * np], geo[4 * np], geo[5 * np], geo[6 * np]};
}

// Write the state back and add the step(s)' diagnostics to the slab row `srow`
// (whose values at kernel start were `sv`) as k_fused accumulates them: the
// wave and workgroup sums of one cell add zeros.
__device__ __forceinline__ void store_one_cell(int64_t np, const CellState& cs, const CellDiag& d, const double (&sv)[6],
                                               double* __restrict__ st, int64_t* __restrict__ tot,
                                               double* __restrict__ srow) {
  st[S_HSWE * np] = cs.h_swe;
  st[S_HIWE * np] = cs.h_iwe;
  st[S_ECCS * np] = cs.Eccs;
  st[S_ECCI * np] = cs.Ecci;
  st[S_N * np] = cs.n;
  st[S_ALB * np] = cs.albedo;
  tot[0] = cs.tot_q;
  srow[0] = sv[0] + d.P;
  srow[1] = sv[1] + d.PR;
  srow[2] = sv[2] + d.PS;
  srow[3] = sv[3] + d.SM;
  srow[4] = sv[4] + d.IM;
  srow[5] = tfg::npmax(sv[5], d.Pmax);
}

__global__ __launch_bounds__(64 * tfg::kCellWaves) void k_cell(const KArgs a, const CellIo io, const double* __restrict__ geo,
                                             const int32_t* __restrict__ catch_id, double* __restrict__ st,
                                             int64_t* __restrict__ tot, int32_t* __restrict__ ring,
                                             double* __restrict__ forc, double* __restrict__ hist,
                                             double* __restrict__ slab, const double* __restrict__ qcf,
                                             int read_depths) {
  __shared__ double lds_x[tfg::X_SLOTS * 4];
  const DevParams& p = a.p;
  const int64_t np = a.n_pad;
  const tfg_uniforms& u = io.u;
#ifdef TFG_CELL_TIMING  // diagnostic build: phase times [wall-clock ticks] replace the outputs
  const long long tt0 = wall_clock64();
#endif
  CellState cs;
  CellStatic sx;
  load_one_cell(p, np, st, tot, geo, read_depths, cs, sx);
  const int32_t q_old = ring[(int64_t)u.slot * np];
  double* srow = slab + (catch_id ? catch_id[0] : 0) * 6;
  double sv[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) sv[i] = srow[i];
  const double qc = qcf ? qcf[0] : 0.0;
  CellDiag d;
  diag_zero(d);
  CellOut o;
  int32_t q_new;
#ifdef TFG_CELL_TIMING
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  asm volatile("" ::"v"(cs.h_swe), "v"(sx.elev), "v"(sv[0]), "v"(q_old));
  const long long tt1 = wall_clock64();
#endif
  tfg::cell_step_exact_wave<tfg::kCellWaves>(p, sx, u, io.in[F_P], io.in[F_T], io.in[F_Q], io.in[F_PA], io.in[F_UZ],
                                              q_old, q_new, cs, o, d, qc, lds_x);
#ifdef TFG_CELL_TIMING
  asm volatile("" ::"v"(o.SM), "v"(o.RH), "v"(cs.Eccs), "v"(o.h_snow), "v"(d.SM));
  const long long tt2 = wall_clock64();
#endif
  if (threadIdx.x == 0) {
    ring[(int64_t)u.slot * np] = q_new;
    double* h = hist + (int64_t)u.hist * kNumHist * np;
    h[H_HSNOW * np] = o.h_snow;
    h[H_SM * np] = o.SM;
    h[H_HICE * np] = o.h_ice;
    h[H_IM * np] = o.IM;
    h[H_MTOT * np] = o.M_total;
    h[H_RH * np] = o.RH;
    double* fr = forc + (int64_t)u.frame * kNumForc * np;
#pragma unroll
    for (int f = 0; f < kNumForc; ++f) fr[f * np] = io.in[f];
    store_one_cell(np, cs, d, sv, st, tot, srow);
    double* out = a.io_out;  // [8][1]: h_snow, h_swe, SM, h_ice, h_iwe, IM, M_total, RH
    out[0] = o.h_snow;
    out[1] = cs.h_swe;
    out[2] = o.SM;
    out[3] = o.h_ice;
    out[4] = cs.h_iwe;
    out[5] = o.IM;
    out[6] = o.M_total;
    out[7] = o.RH;
#ifdef TFG_CELL_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long tt3 = wall_clock64();
    out[0] = (double)(tt1 - tt0);
    out[1] = (double)(tt2 - tt1);
    out[2] = (double)(tt3 - tt2);
#endif
    __threadfence_system();
    __hip_atomic_store(a.io_flag, a.io_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// K consecutive steps of a one-cell fp64 handle (tfg_step: update_until and
// bulk runs of one catchment): k_cell's lane-batched step in a loop, the state
// in registers, each step's frame values, window slot and uniforms requested
// one step ahead (a one-slot window runs one step per launch, tfg_step).
// Same arithmetic as k_fused<double, true, ...>, so the same results bit for
// bit.  Every thread stores the same values to the same addresses, so no
// store sits behind a branch and each wave reads back only window slots it
// wrote itself.
__global__ __launch_bounds__(64 * tfg::kCellWaves) void k_cell_run(const KArgs a, const tfg_uniforms* __restrict__ uni,
                                                 const double* __restrict__ geo, const int32_t* __restrict__ catch_id,
                                                 double* __restrict__ st, int64_t* __restrict__ tot,
                                                 int32_t* __restrict__ ring, const double* __restrict__ forc,
                                                 double* __restrict__ hist, double* __restrict__ slab,
                                                 const double* __restrict__ qcf, int read_depths) {
  __shared__ double lds_x[tfg::X_SLOTS * 4];
  const DevParams& p = a.p;
  const int64_t np = a.n_pad;
  CellState cs;
  CellStatic sx;
  load_one_cell(p, np, st, tot, geo, read_depths, cs, sx);
  double* srow = slab + (catch_id ? catch_id[0] : 0) * 6;
  double sv[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) sv[i] = srow[i];
  const double qc = qcf ? qcf[0] : 0.0;
  CellDiag d;
  diag_zero(d);
  struct In {
    double v[kNumForc];
    int32_t q;
  };
  auto fetch = [&](int k, In& x) {
    const tfg_uniforms* un = uni + (k < a.K ? k : a.K - 1);
    const double* fr = forc + (int64_t)un->frame * kNumForc * np;
#pragma unroll
    for (int f = 0; f < kNumForc; ++f) x.v[f] = fr[f * np];
    x.q = ring[(int64_t)un->slot * np];
  };
  In cur, nxt;
  fetch(0, cur);
  for (int k = 0; k < a.K; ++k) {
    TFG_STEP_PARAMS(p);  // per-step constants (-2.5 % per step, same-box A/B, scripts/gpu_ab_cellrun.sh)
    fetch(k + 1, nxt);
    const tfg_uniforms u = uni[k];
    CellOut o;
    int32_t q_new;
    tfg::cell_step_exact_wave<tfg::kCellWaves>(p, sx, u, cur.v[F_P], cur.v[F_T], cur.v[F_Q], cur.v[F_PA], cur.v[F_UZ],
                                                cur.q, q_new, cs, o, d, qc, lds_x);
    ring[(int64_t)u.slot * np] = q_new;
    double* h = hist + (int64_t)u.hist * kNumHist * np;
    h[H_HSNOW * np] = o.h_snow;
    h[H_SM * np] = o.SM;
    h[H_HICE * np] = o.h_ice;
    h[H_IM * np] = o.IM;
    h[H_MTOT * np] = o.M_total;
    h[H_RH * np] = o.RH;
    cur = nxt;
  }
  store_one_cell(np, cs, d, sv, st, tot, srow);
}

// One step of many one-cell fp64 handles in one launch (tfg_update_many: the
// per-catchment BMI models of a process that have each been asked for a step;
// NextGen-style ensembles stepped together).  Workgroup j runs job j exactly
// as k_cell runs its one handle: the job record (the handle's DevParams and
// buffers, the step's uniforms and inputs) sits in a pinned, device-mapped
// host block; the workgroup stages it into LDS with one coalesced read, so
// every later uniform read is an LDS broadcast instead of a PCIe round trip.
struct CellJob {
  DevParams p;
  tfg_uniforms u;
  double in[kNumForc];  // P, T_air, Hum_sp, P_air, uz (device frame order)
  const double* geo;
  const int32_t* catch_id;
  double* st;
  int64_t* tot;
  int32_t* ring;
  double* forc;
  double* hist;
  double* slab;
  const double* qc;  // null while the conduction term is off
  int64_t n_pad;
  int32_t read_depths;
  int32_t pad_;
};
static_assert(sizeof(CellJob) % 8 == 0, "CellJob is staged as 8-byte words");

__global__ __launch_bounds__(64 * tfg::kCellWaves) void k_cell_many(const CellJob* __restrict__ jobs,
                                                  double* __restrict__ out, uint32_t* __restrict__ flags,
                                                  uint32_t seq) {
  __shared__ double lds_x[tfg::X_SLOTS * 4];
  __shared__ CellJob job;
  {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(jobs + blockIdx.x);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&job);
    for (int i = threadIdx.x; i < (int)(sizeof(CellJob) / 8); i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const DevParams& p = job.p;
  const int64_t np = job.n_pad;
  double* const st = job.st;
  int64_t* const tot = job.tot;
  int32_t* const ring = job.ring;
  CellState cs;
  CellStatic sx;
  load_one_cell(p, np, st, tot, job.geo, job.read_depths, cs, sx);
  const int32_t q_old = ring[(int64_t)job.u.slot * np];
  double* srow = job.slab + (job.catch_id ? job.catch_id[0] : 0) * 6;
  double sv[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) sv[i] = srow[i];
  const double qc = job.qc ? job.qc[0] : 0.0;
  CellDiag d;
  diag_zero(d);
  CellOut o;
  int32_t q_new;
  tfg::cell_step_exact_wave<tfg::kCellWaves>(p, sx, job.u, job.in[F_P], job.in[F_T], job.in[F_Q], job.in[F_PA],
                                              job.in[F_UZ], q_old, q_new, cs, o, d, qc, lds_x);
  if (threadIdx.x == 0) {
    ring[(int64_t)job.u.slot * np] = q_new;
    double* h = job.hist + (int64_t)job.u.hist * kNumHist * np;
    h[H_HSNOW * np] = o.h_snow;
    h[H_SM * np] = o.SM;
    h[H_HICE * np] = o.h_ice;
    h[H_IM * np] = o.IM;
    h[H_MTOT * np] = o.M_total;
    h[H_RH * np] = o.RH;
    double* fr = job.forc + (int64_t)job.u.frame * kNumForc * np;
#pragma unroll
    for (int f = 0; f < kNumForc; ++f) fr[f * np] = job.in[f];
    store_one_cell(np, cs, d, sv, st, tot, srow);
    double* ob = out + (int64_t)blockIdx.x * 8;  // h_snow, h_swe, SM, h_ice, h_iwe, IM, M_total, RH
    ob[0] = o.h_snow;
    ob[1] = cs.h_swe;
    ob[2] = o.SM;
    ob[3] = o.h_ice;
    ob[4] = cs.h_iwe;
    ob[5] = o.IM;
    ob[6] = o.M_total;
    ob[7] = o.RH;
    __threadfence_system();
    __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Per-cell solar geometry of the fast engine, once per static-raster change:
// kGeoF fp32 planes then [tan(eq_lat), t_noon] fp64 (tfg::derive_geo).
template <class R>
__global__ void k_prepare_geo(const DevParams p, const R* __restrict__ stat, float* __restrict__ geo, int64_t n_pad) {
  double* gd = reinterpret_cast<double*>(geo + tfg::kGeoF * n_pad);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * blockDim.x) {
    const tfg::CellGeo g = tfg::derive_geo(p, (double)stat[i], (double)stat[n_pad + i], (double)stat[2 * n_pad + i]);
#pragma unroll
    for (int f = 0; f < tfg::kGeoF; ++f) geo[f * n_pad + i] = g.f[f];
    gd[i] = g.tan_eq;
    gd[n_pad + i] = g.t_noon;
  }
}

// Exact engine: CellStatic planes [kStaticPlanes][n_pad] fp64 (elev, cos_leq,
// sin_leq, dlon, tan_eq, cos_dlon, sin_dlon), derived once per static-raster
// change instead of once per launch.
template <class R>
__global__ void k_prepare_static(const DevParams p, const R* __restrict__ stat, double* __restrict__ gx, int64_t n_pad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * blockDim.x) {
    const CellStatic s = tfg::derive_static(p, (double)stat[i], (double)stat[n_pad + i], (double)stat[2 * n_pad + i]);
    gx[i] = s.elev;
    gx[n_pad + i] = s.cos_leq;
    gx[2 * n_pad + i] = s.sin_leq;
    gx[3 * n_pad + i] = s.dlon;
    gx[4 * n_pad + i] = s.tan_eq;
    gx[5 * n_pad + i] = s.cos_dlon;
    gx[6 * n_pad + i] = s.sin_dlon;
  }
}

// acc[i] = reduce over workgroups of slab[b][i]; one workgroup per diag entry.
__global__ __launch_bounds__(kBlock) void k_diag_reduce(const double* __restrict__ slab, int nblocks, int nb,
                                                        double* __restrict__ acc) {
  __shared__ double red[kBlock];
  const int i = blockIdx.x;
  const bool is_max = (i % 6) == 5;
  double v = is_max ? -INFINITY : 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock) {
    const double x = slab[(int64_t)b * nb + i];
    v = is_max ? tfg::npmax(v, x) : v + x;
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const double o = red[threadIdx.x + s];
      red[threadIdx.x] = is_max ? tfg::npmax(red[threadIdx.x], o) : red[threadIdx.x] + o;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) acc[i] = red[0];
}

template <class D, class S>
__global__ void k_convert(D* __restrict__ dst, const S* __restrict__ src, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (D)src[i];
}

// initialize() state (:389-395, :369, :288, :296) from the current depths
__global__ void k_init_state(double* __restrict__ st, int64_t n_pad, double rhoCp_snow, double del_T,
                             double Ecci0, int albedo_f32) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * blockDim.x) {
    const double e = rhoCp_snow * st[S_HSNOW * n_pad + i] * del_T;
    st[S_ECCS * n_pad + i] = tfg::npmax(e, 0.0);
    st[S_ECCI * n_pad + i] = Ecci0;
    st[S_N * n_pad + i] = 0.0;
    if (albedo_f32) reinterpret_cast<float*>(st + S_ALB * n_pad)[i] = 0.3f;  // the fp32 engine's albedo plane
    else st[S_ALB * n_pad + i] = 0.3;
  }
}

// materialise previous-step depths before a host overwrite of a depth field
__global__ void k_materialise_depths(double* __restrict__ st, int64_t n_pad, double ws, double wi) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * blockDim.x) {
    st[S_HSNOW * n_pad + i] = st[S_HSWE * n_pad + i] * ws;
    st[S_HICE * n_pad + i] = st[S_HIWE * n_pad + i] * wi;
  }
}

template <class R>
__global__ void k_check_slope(const R* __restrict__ slope, int64_t n, int32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (slope[i] < (R)0) atomicOr(flag, 1);
}

// --- synthetic workload (mirror: topoflow_glacier/synthetic.py) -----------
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float hash_u01(uint64_t seed, uint64_t field, uint64_t frame, uint64_t cell) {
  const uint64_t k = (field << 58) ^ (frame << 42) ^ cell;
  return (float)(splitmix64(seed ^ splitmix64(k)) >> 40) * 0x1p-24f;
}

template <class R>
__global__ void k_fill_synthetic(R* __restrict__ forc, R* __restrict__ stat, double* __restrict__ st,
                                 int64_t n, int64_t n_pad, int64_t nx, int64_t row0, int64_t nx_global,
                                 uint64_t seed, const float* __restrict__ diurnal, int n_frames) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nx, c = i % nx;
    const uint64_t cell = (uint64_t)((row0 + r) * nx_global + c);
    const float Tbar = -8.0f + 16.0f * hash_u01(seed, 6, 0, cell);
    stat[i] = (R)(1500.0f + 1500.0f * hash_u01(seed, 7, 0, cell));
    stat[n_pad + i] = (R)(0.5f + 99.5f * hash_u01(seed, 8, 0, cell));
    stat[2 * n_pad + i] = (R)(360.0f * hash_u01(seed, 9, 0, cell));
    const float h_swe = 0.25f * (0.8f + 0.4f * hash_u01(seed, 10, 0, cell));
    const float h_iwe = 1.834f * (0.8f + 0.4f * hash_u01(seed, 11, 0, cell));
    st[S_HSWE * n_pad + i] = (double)h_swe;
    st[S_HIWE * n_pad + i] = (double)h_iwe;
    st[S_HSNOW * n_pad + i] = (double)(h_swe * 20.0f);
    st[S_HICE * n_pad + i] = (double)(h_iwe * 1.0905125f);
    for (int f = 0; f < n_frames; ++f) {
      R* fr = forc + (int64_t)f * kNumForc * n_pad;
      const float T = (Tbar + 5.0f * diurnal[f]) + 2.0f * (hash_u01(seed, 0, f, cell) - 0.5f);
      const float q = 0.0019f + 0.0042f * hash_u01(seed, 1, f, cell);
      const float pa = 87100.0f + 2600.0f * hash_u01(seed, 2, f, cell);
      const float uz = 0.28f + 15.5f * hash_u01(seed, 3, f, cell);
      const float P = (hash_u01(seed, 4, f, cell) < 0.24f) ? 5.2e-7f * hash_u01(seed, 5, f, cell) : 0.0f;
      fr[F_P * n_pad + i] = (R)P;
      fr[F_T * n_pad + i] = (R)T;
      fr[F_Q * n_pad + i] = (R)q;
      fr[F_PA * n_pad + i] = (R)pa;
      fr[F_UZ * n_pad + i] = (R)uz;
    }
  }
}

thread_local std::string g_err;  // errors before a handle exists (per calling thread)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

}  // namespace

// ===========================================================================
// Handle
// ===========================================================================
// Horn's 3x3 slope/aspect (tfg_terrain_from_dem).  halo: [2][nx] fp64, the
// rows north of row 0 and south of row ny-1.  fp64, contraction off, so the
// numpy restatement in tests reproduces it up to libm rounding.
template <class R>
__global__ void k_terrain(const R* __restrict__ elev, const double* __restrict__ halo, R* __restrict__ slope,
                          R* __restrict__ aspect, int64_t ny, int64_t nx, double inv8dx, double inv8dy) {
#pragma clang fp contract(off)
  const int64_t n = ny * nx;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nx, c = i % nx;
    const int64_t cw = c > 0 ? c - 1 : c, ce = c < nx - 1 ? c + 1 : c;
    auto z = [&](int64_t rr, int64_t cc) -> double {
      if (rr < 0) return halo[cc];
      if (rr >= ny) return halo[nx + cc];
      return (double)elev[rr * nx + cc];
    };
    const double a = z(r - 1, cw), b = z(r - 1, c), cc_ = z(r - 1, ce);
    const double d = z(r, cw), f = z(r, ce);
    const double g = z(r + 1, cw), hh = z(r + 1, c), ii = z(r + 1, ce);
    const double dzdx = ((cc_ + 2.0 * f + ii) - (a + 2.0 * d + g)) * inv8dx;   // east
    const double dzds = ((g + 2.0 * hh + ii) - (a + 2.0 * b + cc_)) * inv8dy;  // south
    slope[i] = (R)sqrt(dzdx * dzdx + dzds * dzds);
    // downslope direction (-dz/dx, -dz/dnorth) = (-dzdx, +dzds), CCW from east
    aspect[i] = (R)((dzdx == 0.0 && dzds == 0.0) ? 0.0 : atan2(dzds, -dzdx));
  }
}


#include "tfg_flow.hpp"  // the optional ice-flow kernels (tfg_ice_flow_*)

// tfg_set_inputs / tfg_get_outputs: the per-step BMI traffic of one call each.
// src [5][n]: P_air, Hum_sp, P, T_air, uz (BMI order) -> frame planes.
template <class R, class S>
__global__ void k_scatter_inputs(R* __restrict__ fr, const S* __restrict__ src, int64_t n, int64_t n_pad) {
  const int map[5] = {F_PA, F_Q, F_P, F_T, F_UZ};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
#pragma unroll
    for (int f = 0; f < 5; ++f) fr[map[f] * n_pad + i] = (R)src[f * n + i];
}
// dst [8][n]: h_snow, h_swe, SM, h_ice, h_iwe, IM, M_total, RH.  Before the
// first step (depths not yet derived) the depths come from the fp64 state.
template <class R, class D>
__global__ void k_gather_outputs(D* __restrict__ dst, const R* __restrict__ hs, const double* __restrict__ st, int64_t n,
                                 int64_t n_pad, int depths_from_state) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    dst[0 * n + i] = depths_from_state ? (D)st[S_HSNOW * n_pad + i] : (D)hs[H_HSNOW * n_pad + i];
    dst[1 * n + i] = (D)st[S_HSWE * n_pad + i];
    dst[2 * n + i] = (D)hs[H_SM * n_pad + i];
    dst[3 * n + i] = depths_from_state ? (D)st[S_HICE * n_pad + i] : (D)hs[H_HICE * n_pad + i];
    dst[4 * n + i] = (D)st[S_HIWE * n_pad + i];
    dst[5 * n + i] = (D)hs[H_IM * n_pad + i];
    dst[6 * n + i] = (D)hs[H_MTOT * n_pad + i];
    dst[7 * n + i] = (D)hs[H_RH * n_pad + i];
  }
}

// Snowfall-window checkpoint I/O (TFG_ST_WINDOW): metres <-> fixed point, and
// the running total rebuilt from the slots.
__global__ void k_window_set(int32_t* __restrict__ slot, const double* __restrict__ v, int64_t n, double qscale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    slot[i] = tfg::window_q(v[i], qscale);
}
__global__ void k_window_get(double* __restrict__ v, const int32_t* __restrict__ slot, int64_t n, double inv_qscale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = slot[i] == tfg::kWindowNan ? (double)NAN : (double)slot[i] * inv_qscale;
}
__global__ void k_window_total(int64_t* __restrict__ tot, const int32_t* __restrict__ ring, int ring_len, int64_t n_pad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = 0;
    for (int s = 0; s < ring_len; ++s) t += tfg::window_tot(ring[(int64_t)s * n_pad + i]);
    tot[i] = t;
  }
}

// Non-finite checks behind the fp32 engine's choice of step form (see
// tfg_handle::plane_state): flag |= 1 where a value is NaN or infinite, or
// where a window total holds a NaN slot.
// Planes of n cells at a stride of `stride` elements (padding cells excluded:
// they are computed along, from zero inputs, and may hold anything).
template <class T>
__global__ void k_nonfinite(const T* __restrict__ p, int64_t n, int64_t stride, int planes, int32_t* __restrict__ flag) {
  bool bad = false;
  for (int k = 0; k < planes; ++k)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
      bad |= !isfinite(p[k * stride + i]);
  if (bad) atomicOr(flag, 1);
}
// the same check for each of a frame's planes at once (blockIdx.y = plane): flags[plane] |= 1
template <class T>
__global__ void k_nonfinite_planes(const T* __restrict__ p, int64_t n, int64_t stride, int32_t* __restrict__ flags) {
  const T* __restrict__ q = p + (int64_t)blockIdx.y * stride;
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(q[i]);
  if (bad) atomicOr(flags + blockIdx.y, 1);
}
__global__ void k_window_nan(const int64_t* __restrict__ tot, int64_t n, int32_t* __restrict__ flag) {
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= tot[i] >= tfg::kWindowNanMin;
  if (bad) atomicOr(flag, 1);
}

enum : uint8_t { kUnknown = 0, kOk = 1, kDirty = 2 };

// tfg_selftest_powers: the fp64 engine's power rewrites (tfg_physics.hpp) and
// its exp / log / constant-divisor division (tfg_fastmath.hpp) on device, with
// the device libm's exp and log beside them
__global__ void k_selftest_powers(const double* __restrict__ x, double* __restrict__ y, int64_t n, int which) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    double r;
    switch (which) {
      case 0: r = tfg::pow4(v); break;
      case 1: r = tfg::pow1p5(v); break;
      case 2: r = tfg::root7(v); break;
      case 3: r = tfg_fm::exp_k(v); break;
      case 4: r = exp(v); break;
      case 5: r = tfg_fm::log_k(v); break;
      case 6: r = log(v); break;
      case 7: r = tfg_fm::div_k(v, 6.1121, 1.0 / 6.1121); break;
      case 9: r = tfg_fm::exp_kv(v); break;
      case 10: r = tfg_fm::fdiv(v, 7.3); break;
      case 11: r = tfg_fm::fdiv(7.3, v); break;
      case 12: r = tfg_fm::atan_q(v, 7.3); break;
      case 13: r = tfg_fm::atan_q(-7.3, v); break;
      default: r = tfg_fm::div_k(v, 3600.0, 1.0 / 3600.0); break;
    }
    y[i] = r;
  }
}

struct tfg_handle {
  int device = 0, engine = TFG_F32;
  int64_t ny = 0, nx = 0, n = 0, n_pad = 0;
  int n_frames = 1, hist_depth = 1, n_catch = 1, ring_len = 72;
  size_t rsz = 4;
  DevParams dp{};
  hipStream_t own_stream = nullptr, stream = nullptr;
  void* forc = nullptr;
  void* stat = nullptr;
  void* lwsw = nullptr;          // [2][n_pad] R, not read by the physics
  float* geo = nullptr;          // fast engine: [5][n_pad] f32 + [2][n_pad] f64 solar geometry; exact: [kStaticPlanes][n_pad] f64 CellStatic
                                 // (elev, cos_leq, sin_leq, dlon, tan_eq, cos_dlon, sin_dlon)
  bool geo_dirty = true;
  int32_t* catch_id = nullptr;
  double* st = nullptr;
  int64_t* tot = nullptr;
  int32_t* ring = nullptr;
  void* hist = nullptr;
  double* diag = nullptr;        // [n_catch][6]
  double* slab = nullptr;        // [max_blocks][n_catch][6]
  float* d_diurnal = nullptr;
  int32_t* d_flag = nullptr;
  tfg_uniforms* d_u = nullptr;
  int64_t d_u_cap = 0;
  tfg_uniforms* h_u[2] = {nullptr, nullptr};
  hipEvent_t h_u_ev[2] = {nullptr, nullptr};
  int64_t h_u_cap[2] = {0, 0};
  int h_u_next = 0;
  void* staging = nullptr;
  size_t staging_bytes = 0;
  int max_blocks = 2048;
  int fuse = 24;
  bool depths_derived = false;
  bool slope_invalid = false;
  bool initialised = false;
  bool tot_dirty = false;        // window slots set through TFG_ST_WINDOW
  double* wtmp = nullptr;        // [n_pad] f64 scratch for window I/O
  double* halo = nullptr;        // [2][nx] f64 DEM halo rows (tfg_terrain_from_dem)
  double* flow_halo = nullptr;   // [2 sides][2][nx] f64 ice-flow halo rows (s, H)
  double* flow_edges = nullptr;  // [2 rows][2][nx] f64 this shard's edge rows
  double* flow_red = nullptr;    // f64 per-workgroup maxima of k_ice_flow<R, true>
  double flow_gamma = 0.0;       // 2A/(n+2) (rho_ice g)^n, n = 3 [m^-3 yr^-1]
  // optional lateral conduction: Qc plane (engine type) added to Q_sum while qc_on
  void* qc = nullptr;            // [n_pad] R
  bool qc_on = false;
  double* cond_halo = nullptr;   // [2 sides][4][nx] f64 halo rows (T_snow, h_snow, T_ice, h_ice)
  double* cond_edges = nullptr;  // [2 rows][4][nx] f64 this shard's edge rows
  double inv_cs = 0.0, inv_ci = 0.0, h_active = 0.0;  // 1/(rho_s Cp_s), 1/(rho_i Cp_i h_al), h_al
  // tfg_set_inputs: pinned host staging ring (2 slots) + device staging
  void* in_h[2] = {nullptr, nullptr};
  void* in_d[2] = {nullptr, nullptr};
  size_t in_cap[2] = {0, 0};
  hipEvent_t in_ev[2] = {nullptr, nullptr};
  int in_next = 0;
  // tfg_get_outputs: device gather buffer + pinned host buffer
  void* out_d = nullptr;
  void* out_h = nullptr;
  size_t out_cap = 0;
  // tfg_update: one pinned host block (inputs | uniforms | outputs) that the
  // kernels read and write directly through its device mapping
  char* io_h = nullptr;
  char* io_d = nullptr;
  size_t io_cap = 0;
  uint32_t io_seq = 0;
  int64_t last_hist = 0;
  // Finite-data tracking for the fp32 engine's two step forms (tfg_physics.hpp,
  // "Missing data"): a launch runs the clean form only when everything it reads
  // is known to be finite.  kUnknown: written by a path that did not check it;
  // kDirty: checked, holds a NaN or an infinity.
  std::vector<uint8_t> plane_state;  // [n_frames][kNumForc] forcing planes
  std::vector<int> chk_frames;       // choose_form's scratch list of frames to check
  uint8_t state_state = 1;           // fp64 state planes and the snowfall window
  uint8_t elev_state = 1;            // the elevation raster (the fp32 flux reads it unguarded)
  uint8_t qc_state = 1;              // the Qc plane while the conduction term is on
  int state_recheck = 0;             // launches before a dirty state is checked again
  int64_t ns_launches = 0;           // launches that ran the NaN-safe form (tfg_nan_safe_launches)
  bool force_ns = false;             // tfg_set_step_form(TFG_FORM_NAN_SAFE): every launch NaN-safe
  bool flux_f64 = false;             // tfg_set_flux(TFG_FLUX_F64): the fp32 engine's fp64-flux form
  // Split launches (tfg_set_split): the second part's stream, its copy of the
  // step uniforms, and the events that order it against the handle's stream
  int split_mode = TFG_SPLIT_AUTO;
  hipStream_t side = nullptr;
  hipEvent_t side_fork = nullptr, side_join = nullptr;
  tfg_uniforms* d_u2 = nullptr;
  int64_t d_u2_cap = 0;
  hipEvent_t h_u_ev2[2] = {nullptr, nullptr};
  bool side_busy = false;   // the side stream holds launches the handle's stream is not yet ordered after
  bool side_stale = true;   // the handle's stream holds work the side stream's next launch must follow
  std::string err;
};

namespace {

int fail(tfg_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg; else g_err = msg;
  return code;
}

#define HIPCHK(h, call)                                                                  \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail((h), TFG_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

size_t dtype_size(int dt) { return dt == TFG_F64 ? 8 : 4; }

// The Qc plane, allocated (zeroed) on first use.
int ensure_qc(tfg_handle* h) {
  if (h->qc) return TFG_OK;
  HIPCHK(h, hipMalloc(&h->qc, (size_t)h->n_pad * h->rsz));
  HIPCHK(h, hipMemsetAsync(h->qc, 0, (size_t)h->n_pad * h->rsz, h->stream));
  return TFG_OK;
}

// Split launches (include/tfg.h tfg_set_split).  The parts are whole 256-cell
// chunks; AUTO splits grids of one to 64 rounds of the resident workgroups.
bool split_active(const tfg_handle* h) {
  if (h->engine != TFG_F32 || h->split_mode == TFG_SPLIT_OFF) return false;
  if (h->split_mode == TFG_SPLIT_ON) return h->n_pad >= 2 * kBlock;
  return h->n >= ((int64_t)1 << 18) && h->n <= ((int64_t)1 << 24);
}
// The handle's stream after the side stream's launches so far (no host wait).
int join_side(tfg_handle* h) {
  if (!h->side_busy) return TFG_OK;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipEventRecord(h->side_join, h->side));
  HIPCHK(h, hipStreamWaitEvent(h->stream, h->side_join, 0));
  h->side_busy = false;
  return TFG_OK;
}
// The side stream after the handle's stream's work so far: only when that
// holds something other than the first parts' launches (a field set, the
// window totals, ...), so consecutive tfg_step calls leave the streams free.
int fork_side(tfg_handle* h) {
  if (!h->side_stale) return TFG_OK;
  HIPCHK(h, hipEventRecord(h->side_fork, h->stream));
  HIPCHK(h, hipStreamWaitEvent(h->side, h->side_fork, 0));
  h->side_stale = false;
  return TFG_OK;
}
// Every API call but tfg_step: order the handle's stream after the side's
// launches, and have the side's next launch follow what the call queues.
int api_sync(tfg_handle* h) {
  if (!h) return TFG_OK;
  h->side_stale = true;
  return join_side(h);
}
int ensure_side(tfg_handle* h) {
  if (h->side) return TFG_OK;
  HIPCHK(h, hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
  HIPCHK(h, hipEventCreateWithFlags(&h->side_fork, hipEventDisableTiming));
  HIPCHK(h, hipEventCreateWithFlags(&h->side_join, hipEventDisableTiming));
  h->side_stale = true;
  return TFG_OK;
}

int ensure_staging(tfg_handle* h, size_t bytes) {
  if (bytes <= h->staging_bytes) return TFG_OK;
  if (h->staging) HIPCHK(h, hipFree(h->staging));
  h->staging = nullptr;
  HIPCHK(h, hipMalloc(&h->staging, bytes));
  h->staging_bytes = bytes;
  return TFG_OK;
}

int grid_for(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 8192); }

// copy n elements of type st (host/device) into device buffer dst of type dt
int upload(tfg_handle* h, void* dst, int dt, const void* src, int st, int64_t n, int on_dev) {
  if (n <= 0) return TFG_OK;
  const size_t sbytes = (size_t)n * dtype_size(st);
  if (dt == st) {
    HIPCHK(h, hipMemcpyAsync(dst, src, sbytes, on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream));
    if (!on_dev) HIPCHK(h, hipStreamSynchronize(h->stream));
    return TFG_OK;
  }
  const void* dsrc = src;
  if (!on_dev) {
    int rc = ensure_staging(h, sbytes);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(h->staging, src, sbytes, hipMemcpyHostToDevice, h->stream));
    dsrc = h->staging;
  }
  const int gb = grid_for(n);
  if (dt == TFG_F32 && st == TFG_F64)
    hipLaunchKernelGGL((k_convert<float, double>), gb, 256, 0, h->stream, (float*)dst, (const double*)dsrc, n);
  else if (dt == TFG_F64 && st == TFG_F32)
    hipLaunchKernelGGL((k_convert<double, float>), gb, 256, 0, h->stream, (double*)dst, (const float*)dsrc, n);
  else
    return fail(h, TFG_ERR_ARG, "unsupported dtype conversion");
  HIPCHK(h, hipGetLastError());
  if (!on_dev) HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}

// kOk when every value of `planes` planes of n cells (stride `stride`
// elements) at device pointer p is finite, kDirty otherwise (synchronous).
int check_finite(tfg_handle* h, const void* p, int dtype, int64_t n, uint8_t* out, int planes = 1, int64_t stride = 0) {
  HIPCHK(h, hipMemsetAsync(h->d_flag, 0, 4, h->stream));
  if (dtype == TFG_F64)
    hipLaunchKernelGGL((k_nonfinite<double>), grid_for(n), 256, 0, h->stream, (const double*)p, n, stride, planes, h->d_flag);
  else
    hipLaunchKernelGGL((k_nonfinite<float>), grid_for(n), 256, 0, h->stream, (const float*)p, n, stride, planes, h->d_flag);
  HIPCHK(h, hipGetLastError());
  int32_t flag = 0;
  HIPCHK(h, hipMemcpyAsync(&flag, h->d_flag, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  *out = flag ? kDirty : kOk;
  return TFG_OK;
}

// The same check on host values (the BMI inputs of tfg_update / tfg_set_inputs).
template <class T>
uint8_t host_finite(const T* p, int64_t n) {
  bool bad = false;
  for (int64_t i = 0; i < n; ++i) bad |= !std::isfinite(p[i]);
  return bad ? kDirty : kOk;
}
// fp64 host values the fp32 engine will hold: finite after the conversion (a
// finite double beyond FLT_MAX becomes inf in the frame)
uint8_t host_finite_as_f32(const double* p, int64_t n) {
  bool bad = false;
  for (int64_t i = 0; i < n; ++i) bad |= !std::isfinite((float)p[i]);
  return bad ? kDirty : kOk;
}

int download(tfg_handle* h, void* dst, int dt, const void* src, int st, int64_t n, int on_dev) {
  if (n <= 0) return TFG_OK;
  const size_t dbytes = (size_t)n * dtype_size(dt);
  const void* dsrc = src;
  if (dt != st) {
    void* conv = dst;
    if (!on_dev) {
      int rc = ensure_staging(h, dbytes);
      if (rc) return rc;
      conv = h->staging;
    }
    const int gb = grid_for(n);
    if (dt == TFG_F32 && st == TFG_F64)
      hipLaunchKernelGGL((k_convert<float, double>), gb, 256, 0, h->stream, (float*)conv, (const double*)src, n);
    else if (dt == TFG_F64 && st == TFG_F32)
      hipLaunchKernelGGL((k_convert<double, float>), gb, 256, 0, h->stream, (double*)conv, (const float*)src, n);
    else
      return fail(h, TFG_ERR_ARG, "unsupported dtype conversion");
    HIPCHK(h, hipGetLastError());
    if (on_dev) return TFG_OK;
    dsrc = conv;
  }
  HIPCHK(h, hipMemcpyAsync(dst, dsrc, dbytes, on_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, h->stream));
  if (!on_dev) HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}

void derive_params(const tfg_params& q, DevParams& p) {
  std::memset(&p, 0, sizeof(p));
  const double pi = 3.141592653589793;
  p.dt = q.dt;
  p.da_m2 = q.da_m2;
  p.T_rs = q.T_rain_snow;
  p.dust = q.dust_atten;
  p.F = q.canopy_factor;
  p.one_minus_F_172 = (1.0 - q.canopy_factor) * 1.72;
  p.cloud_term = 1.0 + (0.22 * (q.cloud_factor * q.cloud_factor));
  p.rho_snow_Cp_snow = q.rho_snow * q.Cp_snow;
  p.rho_air_Cp_air = q.rho_air * q.Cp_air;
  p.rho_air_Lv = q.rho_air * q.Lv;
  p.rho_H2O_Lf = q.rho_H2O * q.Lf;
  p.inv_rho_H2O_Lf = 1.0 / p.rho_H2O_Lf;
  p.lhc_100_p0 = q.latent_heat_constant * 100.0 / q.sea_level_p0;
  p.inv_6p11 = 1.0 / (0.611 * 10.0);
  p.negM_g = -q.M_mass_air * q.g;
  p.R = q.uni_gas_const;
  p.eps = q.eps;
  p.one_minus_eps = 1.0 - q.eps;
  p.z = 10.0;
  p.gz = q.g * 10.0;
  p.kappa = q.kappa;
  p.z0 = q.z0_air;
  p.sigma = q.sigma;
  p.em_surf_sigma = q.em_surf * q.sigma;
  p.one_minus_em_surf = 1.0 - q.em_surf;
  p.negM_g_R = -q.M_mass_air * q.g / q.uni_gas_const;
  p.T0 = q.T0;
  p.ws = q.rho_H2O / q.rho_snow;
  p.wi = q.rho_H2O / q.rho_ice;
  p.days_per_dt = q.dt / 86400.0;
  p.pi_over_180 = pi / 180.0;
  p.c180_over_pi = 180.0 / pi;
  p.sin_lat = q.sin_lat;  // numpy values from the host (the reference computes them with numpy)
  p.cos_lat = q.cos_lat;
  {
    // Ecci = max(((rho_ice*Cp_ice)*h_active_layer)*del_T, 0), del_T = T0 - 0  (:394-395)
    const double e = (q.rho_ice * q.Cp_ice) * q.h_active_layer * (q.T0 - 0.0);
    p.Ecci0 = (e >= 0.0 || e != e) ? e : 0.0;
  }
  p.omega = tfg::kOmega;  // (360 / 24) * (pi / 180)
  p.half_pi = pi / 2.0;
  p.twopi = 2.0 * pi;
  p.qscale = 68719476736.0;  // 2^36
  p.thr_q = (int64_t)std::ceil(0.03 * 68719476736.0);
  p.satterlund = q.satterlund;
  p.ring_len = q.ring_len;
  p.inv_dt = 1.0 / q.dt;
  p.inv_dt_rhoLf = 1.0 / (q.dt * p.rho_H2O_Lf);
  p.c_sm3600 = 3600.0 / (q.dt * p.rho_H2O_Lf);
  p.dt3600 = q.dt * 3600.0;
  {
    float t = (float)q.T_rain_snow;  // largest float <= T_rain_snow
    if ((double)t > q.T_rain_snow) t = std::nextafter(t, -INFINITY);
    p.f_T_rs_dn = t;
  }
  p.f_eps100 = (float)(100.0 * q.eps);
  p.f_ome100 = (float)(100.0 * (1.0 - q.eps));
  p.f_gz = (float)p.gz;
  p.f_z = 10.0f;
  p.f_k2 = (float)((q.kappa / std::log(2.0)) * (q.kappa / std::log(2.0)));
  p.f_rho_air_Cp_air = (float)p.rho_air_Cp_air;
  p.f_qe = (float)(p.rho_air_Lv * q.latent_heat_constant * 100.0 / q.sea_level_p0);
  p.f_dust = (float)q.dust_atten;
  p.f_1pdust = (float)(1.0 + q.dust_atten);
  p.f_em_surf_sigma = (float)p.em_surf_sigma;
  p.f_qfac = (float)(q.dt * p.ws * p.qscale);
  p.f_dt = (float)q.dt;
  p.f_T0 = (float)q.T0;
  p.f_c_eccs = (float)(p.rho_snow_Cp_snow * q.dt * p.ws);
  p.inv_z0 = 1.0 / q.z0_air;
  {
    const int k = (int)std::lround(std::log2(0.7 * p.z / q.z0_air));  // (z - h)/z0 near 2^k for h ~ 0.3 z
    p.f_inv_z0s = (float)std::ldexp(1.0 / q.z0_air, -k);
    p.f_l2k2 = (float)(2 * k);
    p.f_l2kk = (float)(k * k);
    p.f_l2min = (float)std::ldexp(0.01, -k);
  }
  p.f_em_sc = 102.4f;  // 0.1 * 2^10
  p.f_ccFs = (float)(p.one_minus_F_172 * p.cloud_term * std::exp2(-10.0 / 7.0));
  p.f_Fm1 = (float)(q.canopy_factor - 1.0);
  p.d_eps100 = 100.0 * q.eps;
  p.d_ome100 = 100.0 * (1.0 - q.eps);
  p.d_k2 = (q.kappa / std::log(2.0)) * (q.kappa / std::log(2.0));
  p.d_l2k = (double)p.f_l2k2 * 0.5;
  p.d_l2kk = (double)p.f_l2kk;
  // exp(c) of the flux form's lhc / p0 = exp(c) exp(y - c) (tfg_fm::exp_near)
  p.d_qe = p.rho_air_Lv * q.latent_heat_constant * 100.0 / q.sea_level_p0 * std::exp(tfg_fm::kP0Center);
  p.d_es_k = q.satterlund ? 2353.0 * std::log(10.0) : 17.3 * 237.3;
  p.d_es_c = q.satterlund ? 273.15 : 237.3;
}

void* field_ptr(tfg_handle* h, int field, int index, int* dtype) {
  const int64_t np = h->n_pad;
  const size_t rs = h->rsz;
  char* f = static_cast<char*>(h->forc);
  char* hs = static_cast<char*>(h->hist);
  switch (field) {
    case TFG_IN_LW_IN: *dtype = h->engine; return static_cast<char*>(h->lwsw);
    case TFG_IN_SW_IN: *dtype = h->engine; return static_cast<char*>(h->lwsw) + np * rs;
    case TFG_IN_P: *dtype = h->engine; return f + ((int64_t)index * kNumForc + F_P) * np * rs;
    case TFG_IN_T_AIR: *dtype = h->engine; return f + ((int64_t)index * kNumForc + F_T) * np * rs;
    case TFG_IN_HUM_SP: *dtype = h->engine; return f + ((int64_t)index * kNumForc + F_Q) * np * rs;
    case TFG_IN_P_AIR: *dtype = h->engine; return f + ((int64_t)index * kNumForc + F_PA) * np * rs;
    case TFG_IN_UZ: *dtype = h->engine; return f + ((int64_t)index * kNumForc + F_UZ) * np * rs;
    case TFG_OUT_H_SNOW: *dtype = h->engine; return hs + ((int64_t)index * kNumHist + H_HSNOW) * np * rs;
    case TFG_OUT_SM: *dtype = h->engine; return hs + ((int64_t)index * kNumHist + H_SM) * np * rs;
    case TFG_OUT_H_ICE: *dtype = h->engine; return hs + ((int64_t)index * kNumHist + H_HICE) * np * rs;
    case TFG_OUT_IM: *dtype = h->engine; return hs + ((int64_t)index * kNumHist + H_IM) * np * rs;
    case TFG_OUT_M_TOTAL: *dtype = h->engine; return hs + ((int64_t)index * kNumHist + H_MTOT) * np * rs;
    case TFG_OUT_RH: *dtype = h->engine; return hs + ((int64_t)index * kNumHist + H_RH) * np * rs;
    case TFG_OUT_H_SWE: *dtype = TFG_F64; return h->st + S_HSWE * np;
    case TFG_OUT_H_IWE: *dtype = TFG_F64; return h->st + S_HIWE * np;
    case TFG_ST_ELEV: *dtype = h->engine; return static_cast<char*>(h->stat);
    case TFG_ST_SLOPE: *dtype = h->engine; return static_cast<char*>(h->stat) + np * rs;
    case TFG_ST_ASPECT: *dtype = h->engine; return static_cast<char*>(h->stat) + 2 * np * rs;
    case TFG_ST_CATCH_ID: *dtype = TFG_I32; return h->catch_id;
    case TFG_ST_ECCS: *dtype = TFG_F64; return h->st + S_ECCS * np;
    case TFG_ST_ECCI: *dtype = TFG_F64; return h->st + S_ECCI * np;
    case TFG_ST_ALBEDO: *dtype = h->engine == TFG_F32 ? TFG_F32 : TFG_F64; return h->st + S_ALB * np;  // fp32 engine: fp32
    case TFG_ST_NDAYS: *dtype = TFG_F64; return h->st + S_N * np;
    default: return nullptr;
  }
}

bool is_frame_field(int f) { return f == TFG_IN_P || f == TFG_IN_T_AIR || f == TFG_IN_HUM_SP || f == TFG_IN_P_AIR || f == TFG_IN_UZ; }
bool is_hist_field(int f) { return f == TFG_OUT_H_SNOW || f == TFG_OUT_SM || f == TFG_OUT_H_ICE || f == TFG_OUT_IM || f == TFG_OUT_M_TOTAL || f == TFG_OUT_RH; }

// tfg_update's single-step launch (KArgs::io_*); empty for every other launch
struct IoArgs {
  const void* in = nullptr;
  double* out = nullptr;
  uint32_t* flag = nullptr;
  uint32_t seq = 0;
  uint8_t in_state = kUnknown;  // the inputs' finite-data status (tfg_handle::plane_state)
};

// One part of a split launch (launch_steps): cells [c0, c0 + cells) of the
// plane stride, n_valid of them grid cells, on `stream` with its own uniforms;
// its workgroups fold into slab rows from slab_row0.
struct Part {
  int64_t c0, cells, n_valid, slab_row0;
  hipStream_t stream;
};

template <class R, bool EXACT>
int launch_fused(tfg_handle* h, const tfg_uniforms* d_u, int K, int blocks, size_t lds, const IoArgs& io, bool ns,
                 const Part* part = nullptr) {
  const hipStream_t stream = part ? part->stream : h->stream;
  KArgs a;
  a.p = h->dp;
  a.K = K;
  a.io_in = io.in;
  a.io_out = io.out;
  a.io_flag = io.flag;
  a.io_seq = io.seq;
  a.n_catch = h->n_catch;
  a.n = part ? part->n_valid : h->n;
  a.n_pad = h->n_pad;
  a.n_step = part ? part->cells : h->n_pad;
  // a part's buffers start at its first cell in every plane (the planes keep
  // their stride); the kernel corrects its two mixed-width views by c0
  const int64_t c0 = part ? part->c0 : 0;
  a.part_c0 = c0;
  const size_t rb = (size_t)c0 * h->rsz;
  const FusedBufs fb = {d_u, static_cast<const char*>(h->forc) + rb, static_cast<const char*>(h->stat) + rb, h->geo + c0,
                        h->catch_id ? h->catch_id + c0 : nullptr, h->st + c0, h->tot + c0, h->ring + c0,
                        static_cast<char*>(h->hist) + rb, h->slab + (part ? part->slab_row0 : 0) * h->n_catch * 6,
                        h->qc ? static_cast<const char*>(h->qc) + rb : nullptr};
  const bool rd = !h->depths_derived;
  const bool ct = h->catch_id != nullptr;
  if constexpr (EXACT) {  // the fp64 engine's instantiations live in tfg_fused_f64.hip
    HIPCHK(h, launch_fused_exact(a, fb, rd, ct, h->qc_on, blocks, lds, stream));
    return TFG_OK;
  } else {
  if (h->flux_f64) {  // the fp64-flux form's instantiations live in tfg_fused_prec.hip
    HIPCHK(h, launch_fused_prec(a, fb, rd, ct, h->qc_on, ns, blocks, lds, stream));
    return TFG_OK;
  }
  constexpr int C = kCellsPerThread;
#define TFG_ARGS a, d_u, (const R*)fb.forc, (const R*)fb.stat, fb.geo, fb.catch_id, fb.st, fb.tot, fb.ring, (R*)fb.hist, \
                 fb.slab, (const R*)fb.qc
#define TFG_LAUNCH(RD, CT, QC, NS) \
  hipLaunchKernelGGL((k_fused<R, EXACT, RD, CT, QC, C, NS>), blocks, kBlock, lds, stream, TFG_ARGS)
#define TFG_LAUNCH_NS(RD, CT, QC) \
  do { if (ns) TFG_LAUNCH(RD, CT, QC, true); else TFG_LAUNCH(RD, CT, QC, false); } while (0)
  if (h->qc_on) {  // the optional lateral conduction term (tfg_conduction_update / TFG_ST_QC)
    if (rd && ct) TFG_LAUNCH_NS(true, true, true);
    else if (rd) TFG_LAUNCH_NS(true, false, true);
    else if (ct) TFG_LAUNCH_NS(false, true, true);
    else TFG_LAUNCH_NS(false, false, true);
  } else {
    if (rd && ct) TFG_LAUNCH_NS(true, true, false);
    else if (rd) TFG_LAUNCH_NS(true, false, false);
    else if (ct) TFG_LAUNCH_NS(false, true, false);
    else TFG_LAUNCH_NS(false, false, false);
  }
#undef TFG_LAUNCH_NS
#undef TFG_LAUNCH
#undef TFG_ARGS
  HIPCHK(h, hipGetLastError());
  return TFG_OK;
  }
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int tfg_abi_version(void) { return TFG_ABI_VERSION; }

#ifndef TFG_SRC_HASH
#define TFG_SRC_HASH "unknown"
#endif
// build() (__graft_entry__.py) passes the sha256 of the sources and flags; it
// finds this string in the built library to decide whether to recompile.  Host
// side only: in the device code it would make the code objects (whose sha256
// keys the PMC provenance in bench.py) change with every source edit.
#define TFG_STR2(x) #x
#define TFG_STR(x) TFG_STR2(x)
#if !defined(__HIP_DEVICE_COMPILE__)
__attribute__((used)) static const char tfg_build_tag[] =
    "libtfg abi=" TFG_STR(TFG_ABI_VERSION) " arch=gfx950 (hipcc) tfg-src-sha256=" TFG_SRC_HASH
    "; kernels: k_fused<float|double,exact|fast,...>, k_cell, k_cell_run, k_cell_many, k_diag_reduce, k_fill_synthetic";

const char* tfg_build_info(void) { return tfg_build_tag; }
#else
const char* tfg_build_info(void);
#endif

int tfg_device_count(int* count) {
  if (!count) return fail(nullptr, TFG_ERR_ARG, "null count");
  HIPCHK(nullptr, hipGetDeviceCount(count));
  return TFG_OK;
}

// Plane-stride skew of large shards (tfg_create), a multiple of the 256-cell chunk.
constexpr int64_t kPlaneSkew = 512;

int tfg_create(const tfg_params* p, int64_t ny, int64_t nx, int engine, int device, int n_frames,
               int hist_depth, int n_catch, tfg_handle** out) {
  if (!p || !out) return fail(nullptr, TFG_ERR_ARG, "null params/out");
  *out = nullptr;
  if (ny <= 0 || nx <= 0) return fail(nullptr, TFG_ERR_ARG, "grid must have ny, nx >= 1");
  if (ny > (1ll << 31) || nx > (1ll << 31))  // before forming ny*nx
    return fail(nullptr, TFG_ERR_ARG, "shard too large: ny and nx must stay below 2^31");
  if (engine != TFG_F32 && engine != TFG_F64) return fail(nullptr, TFG_ERR_ARG, "engine must be TFG_F32 or TFG_F64");
  if (n_frames < 1 || hist_depth < 1 || n_catch < 1) return fail(nullptr, TFG_ERR_ARG, "n_frames, hist_depth, n_catch must be >= 1");
  if (n_catch > 512) return fail(nullptr, TFG_ERR_ARG, "n_catch > 512 not supported");
  if (p->ring_len < 1) return fail(nullptr, TFG_ERR_ARG, "ring_len must be >= 1");
  if (!(p->dt > 0)) return fail(nullptr, TFG_ERR_ARG, "dt must be > 0");
  // derive_params takes log2(z / z0_air) and squares its rounding (the roughness
  // log's scaling): a z0_air that is zero, negative, NaN or infinite has none
  if (!(p->z0_air > 0.0 && p->z0_air < INFINITY)) return fail(nullptr, TFG_ERR_ARG, "z0_air must be finite and > 0");
  tfg_handle* h = new (std::nothrow) tfg_handle();
  if (!h) return fail(nullptr, TFG_ERR_ARG, "out of host memory");
  auto bail = [&](int rc) {
    g_err = h->err;
    tfg_destroy(h);
    return rc;
  };
  h->device = device;
  h->engine = engine;
  h->rsz = dtype_size(engine);
  h->ny = ny;
  h->nx = nx;
  h->n = ny * nx;
  h->n_pad = round_up(h->n, 64);
  // Plane stride n_pad = round_up(n, 64) + kPlaneSkew cells for shards of 2^20
  // cells or more, so that the planes of a power-of-two shard do not sit at
  // power-of-two distances.  With the plain stride the streaming rate depended
  // on where the allocator put the buffers: 105-115 G cell-updates/s over fresh
  // allocations of one 4096^2 shard in one process, 113.8-116.0 with 512 cells
  // (2 KB) of skew; 1024 x 8192: 111.9-114.1 against 113.7-115.2; 8192^2:
  // 116.4-117.4 against 117.2-117.5 (tests/diagnostics/alloc_variance.py,
  // HISTORY.md section 5).
  h->n_pad += h->n_pad >= ((int64_t)1 << 20) ? kPlaneSkew : 0;
  if (h->n_pad * 8 >= (int64_t)1 << 32) {
    h->err = "shard too large: ny*nx must stay below 2^29 cells per device (32-bit field offsets)";
    g_err = h->err;
    delete h;
    return TFG_ERR_ARG;
  }
  h->n_frames = n_frames;
  h->hist_depth = hist_depth;
  h->n_catch = n_catch;
  h->ring_len = p->ring_len;
  derive_params(*p, h->dp);
  {
    const double rg = p->rho_ice * p->g;  // Glen's law n = 3: Gamma = 2A/5 (rho_ice g)^3
    h->flow_gamma = 2.0 * p->glens_A / 5.0 * (rg * rg * rg);
    h->inv_cs = 1.0 / (p->rho_snow * p->Cp_snow);
    h->inv_ci = 1.0 / ((p->rho_ice * p->Cp_ice) * p->h_active_layer);
    h->h_active = p->h_active_layer;
  }
  if (hipSetDevice(device) != hipSuccess) { h->err = "hipSetDevice failed"; return bail(TFG_ERR_HIP); }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { h->err = "hipGetDeviceProperties failed"; return bail(TFG_ERR_HIP); }
  // 512 workgroups per CU: each thread walks ~2 cells at 8192^2.  Freshly
  // dispatched workgroups start their per-cell state loads at staggered times,
  // which hides the latency bubble at the start of every cell; measured
  // +9 % for 128 per CU over 8 (round 1), and with the two-step prefetch
  // +0.6 % for 512 over 128 at 8192^2, +0.6 % on the 4096 x 8192 shard, even
  // at 4096^2 (where the chunk count caps it at 256 per CU; HISTORY.md
  // section 5).  The per-workgroup diagnostic slab is kept under 256 MiB for
  // large catchment counts: 65536 workgroups at config 5's 43 catchments
  // (135 MB), +1.2 % on its slab against the 16384 a 64 MiB cap gave.
  h->max_blocks = std::max(256, prop.multiProcessorCount * 512);
  h->max_blocks = (int)std::max<int64_t>(256, std::min<int64_t>(h->max_blocks, (256ll << 20) / ((int64_t)n_catch * 6 * 8)));
  // a power of two: with many catchments a slab-capped odd count (31775 at 44
  // catchments) measured 10 % slower than 32768 or 16384 (A/B, same box)
  while (h->max_blocks & (h->max_blocks - 1)) h->max_blocks &= h->max_blocks - 1;
  // no more workgroups (slab rows) than the grid has chunks: a one-cell BMI
  // handle keeps one row, not 32768 (NextGen may hold thousands of handles)
  h->max_blocks = (int)std::min<int64_t>(h->max_blocks, (h->n_pad / kCellsPerThread + kBlock - 1) / kBlock);
  if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) { h->err = "stream create failed"; return bail(TFG_ERR_HIP); }
  h->stream = h->own_stream;
  const int64_t np = h->n_pad;
  const size_t rs = h->rsz;
  struct A { void** p; size_t bytes; } allocs[] = {
      {&h->forc, (size_t)n_frames * kNumForc * np * rs},
      {&h->stat, 3 * (size_t)np * rs},
      {&h->lwsw, 2 * (size_t)np * rs},
      {(void**)&h->geo, engine == TFG_F32 ? (size_t)np * (tfg::kGeoF * 4 + 2 * 8) : (size_t)np * tfg::kStaticPlanes * 8},
      {(void**)&h->st, (size_t)kNumState * np * 8},
      {(void**)&h->tot, (size_t)np * 8},
      {(void**)&h->ring, (size_t)p->ring_len * np * 4},
      {&h->hist, (size_t)hist_depth * kNumHist * np * rs},
      {(void**)&h->diag, (size_t)n_catch * 6 * 8},
      {(void**)&h->slab, (size_t)h->max_blocks * n_catch * 6 * 8},
      {(void**)&h->d_flag, (size_t)n_frames * kNumForc * 4},  // a flag per forcing plane (choose_form)
  };
  for (auto& a : allocs) {
    hipError_t e = hipMalloc(a.p, a.bytes);
    if (e != hipSuccess) {
      h->err = std::string("hipMalloc(") + std::to_string(a.bytes) + " B) failed: " + hipGetErrorString(e);
      return bail(TFG_ERR_HIP);
    }
    if (hipMemsetAsync(*a.p, 0, a.bytes, h->stream) != hipSuccess) { h->err = "hipMemset failed"; return bail(TFG_ERR_HIP); }
  }
  if (hipStreamSynchronize(h->stream) != hipSuccess) { h->err = "sync failed"; return bail(TFG_ERR_HIP); }
  h->plane_state.assign((size_t)n_frames * kNumForc, kOk);  // zero-filled: finite
  *out = h;
  return TFG_OK;
}

int tfg_destroy(tfg_handle* h) {
  if (!h) return TFG_OK;
  (void)hipSetDevice(h->device);
  // work queued on a caller's stream (tfg_set_stream) may still use the buffers
  if (h->stream && h->stream != h->own_stream) (void)hipStreamSynchronize(h->stream);
  if (h->own_stream) (void)hipStreamSynchronize(h->own_stream);
  if (h->side) (void)hipStreamSynchronize(h->side);
  void* ptrs[] = {h->forc, h->stat, h->lwsw, h->geo, h->catch_id, h->st, h->tot, h->ring, h->hist, h->diag, h->wtmp, h->halo,
                  h->flow_halo, h->flow_edges, h->flow_red, h->qc, h->cond_halo, h->cond_edges,
                  h->slab, h->d_diurnal, h->d_flag, h->d_u, h->d_u2, h->staging};
  for (void* q : ptrs) if (q) (void)hipFree(q);
  for (int i = 0; i < 2; ++i) {
    if (h->h_u[i]) (void)hipHostFree(h->h_u[i]);
    if (h->h_u_ev[i]) (void)hipEventDestroy(h->h_u_ev[i]);
    if (h->h_u_ev2[i]) (void)hipEventDestroy(h->h_u_ev2[i]);
    if (h->in_h[i]) (void)hipHostFree(h->in_h[i]);
    if (h->in_d[i]) (void)hipFree(h->in_d[i]);
    if (h->in_ev[i]) (void)hipEventDestroy(h->in_ev[i]);
  }
  if (h->out_d) (void)hipFree(h->out_d);
  if (h->out_h) (void)hipHostFree(h->out_h);
  if (h->io_h) (void)hipHostFree(h->io_h);
  if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
  if (h->side_fork) (void)hipEventDestroy(h->side_fork);
  if (h->side_join) (void)hipEventDestroy(h->side_join);
  if (h->side) (void)hipStreamDestroy(h->side);
  delete h;
  return TFG_OK;
}

int tfg_set_stream(tfg_handle* h, void* stream) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  h->stream = stream ? static_cast<hipStream_t>(stream) : h->own_stream;
  return TFG_OK;
}

int tfg_shared_stream(int device, void** stream) {
  // One non-blocking stream per device for the whole process, created on first
  // use and never destroyed (handles that use it outlive no process).
  static std::mutex mu;
  static hipStream_t streams[64] = {};
  if (!stream) return fail(nullptr, TFG_ERR_ARG, "null stream");
  int count = 0;
  HIPCHK(nullptr, hipGetDeviceCount(&count));
  if (device < 0 || device >= count || device >= 64) return fail(nullptr, TFG_ERR_ARG, "device out of range");
  std::lock_guard<std::mutex> lock(mu);
  if (!streams[device]) {
    int prev = 0;
    HIPCHK(nullptr, hipGetDevice(&prev));
    HIPCHK(nullptr, hipSetDevice(device));
    const hipError_t e = hipStreamCreateWithFlags(&streams[device], hipStreamNonBlocking);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
      streams[device] = nullptr;
      return fail(nullptr, TFG_ERR_HIP, "shared stream create failed");
    }
  }
  *stream = streams[device];
  return TFG_OK;
}

int tfg_get_stream(tfg_handle* h, void** stream) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h || !stream) return fail(h, TFG_ERR_ARG, "null argument");
  *stream = h->stream;
  return TFG_OK;
}

int tfg_set_fuse(tfg_handle* h, int k) {
  if (!h || k < 1) return fail(h, TFG_ERR_ARG, "fuse must be >= 1");
  h->fuse = k;
  return TFG_OK;
}

int tfg_set_step_form(tfg_handle* h, int form) {
  if (!h || (form != TFG_FORM_AUTO && form != TFG_FORM_NAN_SAFE)) return fail(h, TFG_ERR_ARG, "form must be TFG_FORM_AUTO or TFG_FORM_NAN_SAFE");
  h->force_ns = form == TFG_FORM_NAN_SAFE;
  return TFG_OK;
}

int tfg_set_flux(tfg_handle* h, int flux) {
  if (!h || (flux != TFG_FLUX_F32 && flux != TFG_FLUX_F64)) return fail(h, TFG_ERR_ARG, "flux must be TFG_FLUX_F32 or TFG_FLUX_F64");
  h->flux_f64 = flux == TFG_FLUX_F64;  // the fp64 engine computes every flux in fp64 either way
  return TFG_OK;
}

int tfg_set_split(tfg_handle* h, int mode) {
  if (!h || (mode != TFG_SPLIT_AUTO && mode != TFG_SPLIT_OFF && mode != TFG_SPLIT_ON))
    return fail(h, TFG_ERR_ARG, "split must be TFG_SPLIT_AUTO, TFG_SPLIT_OFF or TFG_SPLIT_ON");
  if (int rc = api_sync(h)) return rc;
  h->split_mode = mode;
  return TFG_OK;
}

int tfg_join(tfg_handle* h) {
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  return join_side(h);
}

int tfg_get_split(tfg_handle* h, int* split) {
  if (!h || !split) return fail(h, TFG_ERR_ARG, "null argument");
  *split = split_active(h) ? 1 : 0;
  return TFG_OK;
}

int tfg_set_field(tfg_handle* h, int field, int index, const void* src, int src_dtype, int64_t n,
                  int src_on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!src) return fail(h, TFG_ERR_ARG, "null src");
  if (n != h->n) return fail(h, TFG_ERR_ARG, "n = " + std::to_string(n) + " != ny*nx = " + std::to_string(h->n));
  HIPCHK(h, hipSetDevice(h->device));
  // setting a depth writes the previous-step depth the next step reads, so TFG_PREV_DEPTH is slot 0
  if ((field == TFG_OUT_H_SNOW || field == TFG_OUT_H_ICE) && index == TFG_PREV_DEPTH) index = 0;  // same as a plain depth set
  if (is_frame_field(field) && (index < 0 || index >= h->n_frames)) return fail(h, TFG_ERR_ARG, "frame index out of range");
  if (is_hist_field(field) && (index < 0 || index >= h->hist_depth)) return fail(h, TFG_ERR_ARG, "history slot out of range");
  if (field == TFG_ST_CATCH_ID) {
    if (src_dtype != TFG_I32) return fail(h, TFG_ERR_ARG, "catchment ids must be TFG_I32");
    if (!h->catch_id) {
      HIPCHK(h, hipMalloc((void**)&h->catch_id, (size_t)h->n_pad * 4));
      HIPCHK(h, hipMemsetAsync(h->catch_id, 0, (size_t)h->n_pad * 4, h->stream));
    }
    HIPCHK(h, hipMemcpyAsync(h->catch_id, src, (size_t)n * 4, src_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream));
    std::vector<int32_t> tmp;
    const int32_t* hs = static_cast<const int32_t*>(src);
    if (src_on_device) {
      tmp.resize(n);
      HIPCHK(h, hipMemcpyAsync(tmp.data(), src, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
      hs = tmp.data();
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    for (int64_t i = 0; i < n; ++i)
      if (hs[i] < 0 || hs[i] >= h->n_catch) return fail(h, TFG_ERR_ARG, "catchment id out of [0, n_catch)");
    return TFG_OK;
  }
  if (src_dtype != TFG_F32 && src_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "src dtype must be TFG_F32/TFG_F64");
  const bool track = h->engine == TFG_F32;  // finite-data tracking (tfg_handle::plane_state)
  if (field == TFG_ST_QC) {  // a caller-supplied conduction flux: on until tfg_conduction_off
    if (int rc = ensure_qc(h)) return rc;
    if (int rc = upload(h, h->qc, h->engine, src, src_dtype, n, src_on_device)) return rc;
    h->qc_on = true;
    // device sources stay stream-ordered: their status is checked lazily before a launch (choose_form)
    if (track && src_on_device) h->qc_state = kUnknown;
    else if (track) return check_finite(h, h->qc, h->engine, n, &h->qc_state);
    return TFG_OK;
  }
  if (field == TFG_ST_WINDOW) {
    if (index < 0 || index >= h->ring_len) return fail(h, TFG_ERR_ARG, "window slot out of range");
    if (!h->wtmp) HIPCHK(h, hipMalloc((void**)&h->wtmp, (size_t)h->n_pad * 8));
    int rc = upload(h, h->wtmp, TFG_F64, src, src_dtype, n, src_on_device);
    if (rc) return rc;
    hipLaunchKernelGGL(k_window_set, grid_for(n), 256, 0, h->stream, h->ring + (int64_t)index * h->n_pad, h->wtmp, n,
                       h->dp.qscale);
    HIPCHK(h, hipGetLastError());
    h->tot_dirty = true;
    if (track && src_on_device) {
      h->state_state = kUnknown;  // checked lazily (choose_form -> check_state reads the rebuilt totals)
    } else if (track) {  // a NaN slot makes the window dirty; a finite one leaves the state's status as it was
      uint8_t st = kOk;
      if (int rc = check_finite(h, h->wtmp, TFG_F64, n, &st)) return rc;
      if (st != kOk) h->state_state = kDirty;
    }
    return TFG_OK;
  }
  int fdt = 0;
  void* dst = field_ptr(h, field, index, &fdt);
  if (!dst) return fail(h, TFG_ERR_ARG, "unknown field id " + std::to_string(field));
  const bool depth = field == TFG_OUT_H_SNOW || field == TFG_OUT_H_ICE || field == TFG_OUT_H_SWE || field == TFG_OUT_H_IWE;
  if (depth && h->depths_derived) {
    // keep the previous-step depths the next update() must see (:895-911)
    hipLaunchKernelGGL(k_materialise_depths, grid_for(h->n_pad), 256, 0, h->stream, h->st, h->n_pad, h->dp.ws, h->dp.wi);
    HIPCHK(h, hipGetLastError());
    h->depths_derived = false;
  }
  if (field == TFG_OUT_H_SNOW || field == TFG_OUT_H_ICE) {
    // user-set depth: both the fp64 state and the visible output
    double* sd = h->st + (field == TFG_OUT_H_SNOW ? S_HSNOW : S_HICE) * h->n_pad;
    int rc = upload(h, sd, TFG_F64, src, src_dtype, n, src_on_device);
    if (rc) return rc;
    if (track && src_on_device) {
      h->state_state = kUnknown;
    } else if (track) {
      uint8_t st = kOk;
      if (int rc2 = check_finite(h, sd, TFG_F64, n, &st)) return rc2;
      if (st != kOk) h->state_state = kDirty;
    }
    return upload(h, dst, fdt, src, src_dtype, n, src_on_device);
  }
  int rc = upload(h, dst, fdt, src, src_dtype, n, src_on_device);
  if (rc) return rc;
  // Finite-data status of what was written (tfg_handle::plane_state).  A host
  // source is checked now (its upload is synchronous anyway); a device source
  // keeps the set stream-ordered and non-blocking: its plane is marked
  // unknown and checked lazily before a launch long enough to pay for it
  // (choose_form), or the launch runs the NaN-safe form.
  const bool state_field = field == TFG_OUT_H_SWE || field == TFG_OUT_H_IWE || field == TFG_ST_ECCS ||
                           field == TFG_ST_ECCI || field == TFG_ST_ALBEDO || field == TFG_ST_NDAYS;
  if (track && is_frame_field(field)) {
    const int plane = field == TFG_IN_P ? F_P : field == TFG_IN_T_AIR ? F_T : field == TFG_IN_HUM_SP ? F_Q
                    : field == TFG_IN_P_AIR ? F_PA : F_UZ;
    uint8_t* ps = &h->plane_state[(size_t)index * kNumForc + plane];
    if (src_on_device) *ps = kUnknown;
    else if (int rc2 = check_finite(h, dst, fdt, n, ps)) return rc2;
  } else if (track && field == TFG_ST_ELEV) {
    if (src_on_device) h->elev_state = kUnknown;
    else if (int rc2 = check_finite(h, dst, fdt, n, &h->elev_state)) return rc2;
  } else if (track && state_field && src_on_device) {
    h->state_state = kUnknown;
  } else if (track && state_field) {
    uint8_t st = kOk;
    if (int rc2 = check_finite(h, dst, fdt, n, &st)) return rc2;
    if (st != kOk) h->state_state = kDirty;
  }
  if (field == TFG_ST_ELEV || field == TFG_ST_SLOPE || field == TFG_ST_ASPECT) h->geo_dirty = true;
  if (field == TFG_ST_SLOPE) {
    HIPCHK(h, hipMemsetAsync(h->d_flag, 0, 4, h->stream));
    if (h->engine == TFG_F32)
      hipLaunchKernelGGL((k_check_slope<float>), grid_for(n), 256, 0, h->stream, (const float*)dst, n, h->d_flag);
    else
      hipLaunchKernelGGL((k_check_slope<double>), grid_for(n), 256, 0, h->stream, (const double*)dst, n, h->d_flag);
    int32_t flag = 0;
    HIPCHK(h, hipMemcpyAsync(&flag, h->d_flag, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->slope_invalid = flag != 0;
    if (flag) return fail(h, TFG_ERR_DOMAIN, "ERROR: some slope angles are out of range (beta not in [0, pi/2]; bmi_topoflow_glacier.py:1106-1111)");
  }
  return TFG_OK;
}

int tfg_get_field(tfg_handle* h, int field, int index, void* dst, int dst_dtype, int64_t n, int dst_on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!dst) return fail(h, TFG_ERR_ARG, "null dst");
  if (n <= 0 || n > h->n) return fail(h, TFG_ERR_ARG, "n outside 1..ny*nx");  // n < ny*nx: the first n cells
  HIPCHK(h, hipSetDevice(h->device));
  if ((field == TFG_OUT_H_SNOW || field == TFG_OUT_H_ICE) && index == TFG_PREV_DEPTH) {
    // the fp64 previous-step depth the next step reads (checkpoint / restart)
    if (dst_dtype != TFG_F32 && dst_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "dst dtype must be TFG_F32/TFG_F64");
    if (h->depths_derived) {
      hipLaunchKernelGGL(k_materialise_depths, grid_for(h->n_pad), 256, 0, h->stream, h->st, h->n_pad, h->dp.ws, h->dp.wi);
      HIPCHK(h, hipGetLastError());
    }
    return download(h, dst, dst_dtype, h->st + (field == TFG_OUT_H_SNOW ? S_HSNOW : S_HICE) * h->n_pad, TFG_F64, n,
                    dst_on_device);
  }
  if (is_frame_field(field) && (index < 0 || index >= h->n_frames)) return fail(h, TFG_ERR_ARG, "frame index out of range");
  if (is_hist_field(field) && (index < 0 || index >= h->hist_depth)) return fail(h, TFG_ERR_ARG, "history slot out of range");
  if (field == TFG_ST_CATCH_ID) {
    if (dst_dtype != TFG_I32) return fail(h, TFG_ERR_ARG, "catchment ids are TFG_I32");
    if (!h->catch_id) return fail(h, TFG_ERR_STATE, "no catchment-id raster set");
    HIPCHK(h, hipMemcpyAsync(dst, h->catch_id, (size_t)n * 4, dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return TFG_OK;
  }
  if (dst_dtype != TFG_F32 && dst_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "dst dtype must be TFG_F32/TFG_F64");
  if (field == TFG_ST_QC) {  // zero until a conduction pass or a set (the reference's Qc = 0, :312)
    if (int rc = ensure_qc(h)) return rc;
    return download(h, dst, dst_dtype, h->qc, h->engine, n, dst_on_device);
  }
  if (field == TFG_ST_WINDOW) {
    if (index < 0 || index >= h->ring_len) return fail(h, TFG_ERR_ARG, "window slot out of range");
    if (!h->wtmp) HIPCHK(h, hipMalloc((void**)&h->wtmp, (size_t)h->n_pad * 8));
    hipLaunchKernelGGL(k_window_get, grid_for(n), 256, 0, h->stream, h->wtmp, h->ring + (int64_t)index * h->n_pad, n,
                       1.0 / h->dp.qscale);
    HIPCHK(h, hipGetLastError());
    return download(h, dst, dst_dtype, h->wtmp, TFG_F64, n, dst_on_device);
  }
  int fdt = 0;
  const void* src = field_ptr(h, field, index, &fdt);
  if (!src) return fail(h, TFG_ERR_ARG, "unknown field id " + std::to_string(field));
  if ((field == TFG_OUT_H_SNOW || field == TFG_OUT_H_ICE) && !h->depths_derived) {
    // before any step (or right after a host set) the depths live in the fp64 state
    src = h->st + (field == TFG_OUT_H_SNOW ? S_HSNOW : S_HICE) * h->n_pad;
    fdt = TFG_F64;
  }
  return download(h, dst, dst_dtype, src, fdt, n, dst_on_device);
}

int tfg_init_state(tfg_handle* h) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  HIPCHK(h, hipSetDevice(h->device));
  const DevParams& p = h->dp;
  // Eccs = max((rho_snow*Cp_snow)*h_snow*del_T, 0); del_T = T0 - T_surf(=0)  (:389-395)
  const double del_T = p.T0 - 0.0;
  hipLaunchKernelGGL(k_init_state, grid_for(h->n_pad), 256, 0, h->stream, h->st, h->n_pad, p.rho_snow_Cp_snow, del_T, p.Ecci0,
                     h->engine == TFG_F32 ? 1 : 0);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipMemsetAsync(h->tot, 0, (size_t)h->n_pad * 8, h->stream));
  HIPCHK(h, hipMemsetAsync(h->ring, 0, (size_t)h->ring_len * h->n_pad * 4, h->stream));
  HIPCHK(h, hipMemsetAsync(h->hist, 0, (size_t)h->hist_depth * kNumHist * h->n_pad * h->rsz, h->stream));
  HIPCHK(h, hipMemsetAsync(h->slab, 0, (size_t)h->max_blocks * h->n_catch * 6 * 8, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->depths_derived = false;
  h->tot_dirty = false;
  h->initialised = true;
  return TFG_OK;
}

namespace {

int check_step(tfg_handle* h, const tfg_uniforms* u, int64_t nsteps) {
  if (!u) return fail(h, TFG_ERR_ARG, "null uniforms");
  if (!h->initialised) return fail(h, TFG_ERR_STATE, "tfg_init_state() has not been called");
  if (h->slope_invalid) return fail(h, TFG_ERR_DOMAIN, "slope raster invalid (bmi_topoflow_glacier.py:1106-1111)");
  for (int64_t k = 0; k < nsteps; ++k) {
    if (u[k].frame < 0 || u[k].frame >= h->n_frames) return fail(h, TFG_ERR_ARG, "uniforms: frame out of range");
    if (u[k].hist < 0 || u[k].hist >= h->hist_depth) return fail(h, TFG_ERR_ARG, "uniforms: hist slot out of range");
    if (u[k].slot < 0 || u[k].slot >= h->ring_len) return fail(h, TFG_ERR_ARG, "uniforms: ring slot out of range");
  }
  return TFG_OK;
}

// The launches of nsteps steps whose uniforms the device reads at d_u (u is
// the host copy of the same records).
int64_t chunks_of(int64_t cells) { return (cells / kCellsPerThread + kBlock - 1) / kBlock; }
int fused_blocks(const tfg_handle* h) {  // k_fused steps the whole plane stride
  return (int)std::min<int64_t>(std::max<int64_t>(chunks_of(h->n_pad), 1), h->max_blocks);
}

// Work a launch of the step kernels depends on: window totals after slots were
// set, and the per-cell geometry after the static rasters changed.
int prepare_steps(tfg_handle* h) {
  if (h->tot_dirty || h->geo_dirty)  // rewrites planes a split launch's second part may still read
    if (int rc = api_sync(h)) return rc;
  if (h->tot_dirty) {  // window slots were set: rebuild the running totals
    hipLaunchKernelGGL(k_window_total, grid_for(h->n_pad), 256, 0, h->stream, h->tot, h->ring, h->ring_len, h->n_pad);
    HIPCHK(h, hipGetLastError());
    h->tot_dirty = false;
  }
  if (h->geo_dirty) {
    if (h->engine == TFG_F32)
      hipLaunchKernelGGL((k_prepare_geo<float>), grid_for(h->n_pad), 256, 0, h->stream, h->dp, (const float*)h->stat,
                         h->geo, h->n_pad);
    else
      hipLaunchKernelGGL((k_prepare_static<double>), grid_for(h->n_pad), 256, 0, h->stream, h->dp,
                         (const double*)h->stat, reinterpret_cast<double*>(h->geo), h->n_pad);
    HIPCHK(h, hipGetLastError());
    h->geo_dirty = false;
  }
  return TFG_OK;
}

// Launches of at least this many steps check unknown data before choosing the
// fp32 step form (a synchronous device check); shorter ones run NaN-safe.
constexpr int kVerifySteps = 8;

// The state's finite-data status: the fp64 state planes and the window totals
// (after prepare_steps has rebuilt them).  Synchronous.
int check_state(tfg_handle* h) {
  uint8_t st = kOk;
  {  // the state planes, the albedo plane in the engine's type (fp32 for the fp32 engine)
    const int64_t np = h->n_pad;
    HIPCHK(h, hipMemsetAsync(h->d_flag, 0, 4, h->stream));
    hipLaunchKernelGGL((k_nonfinite<double>), grid_for(h->n), 256, 0, h->stream, (const double*)h->st, h->n, np, S_ALB, h->d_flag);
    if (h->engine == TFG_F32)
      hipLaunchKernelGGL((k_nonfinite<float>), grid_for(h->n), 256, 0, h->stream, (const float*)(h->st + S_ALB * np), h->n,
                         (int64_t)0, 1, h->d_flag);
    else
      hipLaunchKernelGGL((k_nonfinite<double>), grid_for(h->n), 256, 0, h->stream, (const double*)(h->st + S_ALB * np), h->n,
                         (int64_t)0, 1, h->d_flag);
    hipLaunchKernelGGL((k_nonfinite<double>), grid_for(h->n), 256, 0, h->stream, (const double*)(h->st + (S_ALB + 1) * np),
                       h->n, np, kNumState - S_ALB - 1, h->d_flag);
    HIPCHK(h, hipGetLastError());
    int32_t flag = 0;
    HIPCHK(h, hipMemcpyAsync(&flag, h->d_flag, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    st = flag ? kDirty : kOk;
  }
  if (st == kOk) {
    HIPCHK(h, hipMemsetAsync(h->d_flag, 0, 4, h->stream));
    hipLaunchKernelGGL(k_window_nan, grid_for(h->n), 256, 0, h->stream, h->tot, h->n, h->d_flag);
    HIPCHK(h, hipGetLastError());
    int32_t flag = 0;
    HIPCHK(h, hipMemcpyAsync(&flag, h->d_flag, 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    st = flag ? kDirty : kOk;
  }
  h->state_state = st;
  return TFG_OK;
}

// The fp32 engine's step form for one launch of K steps (tfg_physics.hpp,
// "Missing data"): the clean form when the launch's forcing frames (or the
// tfg_update inputs), the elevation raster, the Qc plane in use, the state and
// the window are known to hold only finite values; the NaN-safe form
// otherwise.  Unknown data is checked first when the launch is long enough to
// pay for a synchronous check.
int choose_form(tfg_handle* h, const tfg_uniforms* u, int K, const IoArgs& io, bool* ns) {
  const bool check = K >= kVerifySteps;
  bool inputs_ok = true;
  if (io.in) {
    inputs_ok = io.in_state == kOk;
  } else {
    if (check) {
      // every frame the launch reads that holds a plane of unknown status is
      // checked on the device, all of them before one host wait
      int nf = 0;
      for (int k = 0; k < K; ++k) {
        const int fr = u[k].frame;
        const uint8_t* ps = &h->plane_state[(size_t)fr * kNumForc];
        if (std::find(ps, ps + kNumForc, kUnknown) == ps + kNumForc) continue;
        if (std::find(h->chk_frames.begin(), h->chk_frames.begin() + nf, fr) != h->chk_frames.begin() + nf) continue;
        if ((int)h->chk_frames.size() <= nf) h->chk_frames.resize(nf + 1);
        h->chk_frames[nf++] = fr;
      }
      if (nf) {
        HIPCHK(h, hipMemsetAsync(h->d_flag, 0, (size_t)nf * kNumForc * 4, h->stream));
        const dim3 grid(std::max(1, std::min(grid_for(h->n), 2048)), kNumForc);
        for (int j = 0; j < nf; ++j) {
          const char* fp = static_cast<const char*>(h->forc) + (size_t)h->chk_frames[j] * kNumForc * h->n_pad * h->rsz;
          hipLaunchKernelGGL((k_nonfinite_planes<float>), grid, 256, 0, h->stream, (const float*)fp, h->n, h->n_pad,
                             h->d_flag + j * kNumForc);
        }
        HIPCHK(h, hipGetLastError());
        std::vector<int32_t> flags((size_t)nf * kNumForc);
        HIPCHK(h, hipMemcpyAsync(flags.data(), h->d_flag, flags.size() * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        for (int j = 0; j < nf; ++j) {
          uint8_t* ps = &h->plane_state[(size_t)h->chk_frames[j] * kNumForc];
          for (int f = 0; f < kNumForc; ++f)
            if (ps[f] == kUnknown) ps[f] = flags[(size_t)j * kNumForc + f] ? kDirty : kOk;
        }
      }
    }
    for (int k = 0; k < K; ++k) {
      const uint8_t* ps = &h->plane_state[(size_t)u[k].frame * kNumForc];
      for (int f = 0; f < kNumForc; ++f) inputs_ok &= ps[f] == kOk;
    }
  }
  if (check && (h->state_state == kUnknown || (h->state_state == kDirty && --h->state_recheck <= 0))) {
    if (int rc = api_sync(h)) return rc;  // the state a split launch's second part writes
    if (int rc = check_state(h)) return rc;
    if (h->state_state == kDirty) h->state_recheck = kVerifySteps;  // launches until the next look
  }
  if (h->qc_on && h->qc_state == kUnknown && check)
    if (int rc = check_finite(h, h->qc, h->engine, h->n, &h->qc_state)) return rc;
  if (h->elev_state == kUnknown && check)  // a device-sourced elevation raster (tfg_set_field)
    if (int rc = check_finite(h, h->stat, h->engine, h->n, &h->elev_state)) return rc;
  *ns = h->force_ns ||
        !(inputs_ok && h->state_state == kOk && h->elev_state == kOk && (!h->qc_on || h->qc_state == kOk));
  return TFG_OK;
}

int launch_steps(tfg_handle* h, const tfg_uniforms* d_u, const tfg_uniforms* u, int64_t nsteps,
                 const IoArgs& io = IoArgs(), bool split = false) {
  if (int rc = prepare_steps(h)) return rc;
  const int blocks = fused_blocks(h);
  const size_t lds = (size_t)kWaves * h->n_catch * 6 * sizeof(double);
  // a fused launch reads each step's expiring window slot 1 (fp64 engine) or
  // kPrefetchFast (fp32 engine) steps ahead: a shorter window runs unfused
  // (see the prefetch note in k_fused)
  const int fuse = h->ring_len > (h->engine == TFG_F32 ? kPrefetchFast : 1) ? h->fuse : 1;
  const bool one_cell = h->engine == TFG_F64 && h->n == 1 && !io.in;  // k_cell_run
  for (int64_t k0 = 0; k0 < nsteps; k0 += fuse) {
    const int K = (int)std::min<int64_t>(fuse, nsteps - k0);
    int rc = TFG_OK;
    if (one_cell) {
      KArgs a;
      a.p = h->dp;
      a.K = K;
      a.n_catch = h->n_catch;
      a.n = h->n;
      a.n_pad = h->n_pad;
      a.n_step = h->n_pad;
  a.n_step = h->n_pad;
      a.io_in = nullptr;
      a.io_out = nullptr;
      a.io_flag = nullptr;
      a.io_seq = 0;
      hipLaunchKernelGGL(k_cell_run, 1, 64 * tfg::kCellWaves, 0, h->stream, a, d_u + k0, reinterpret_cast<const double*>(h->geo),
                         h->catch_id, h->st, h->tot, h->ring, static_cast<const double*>(h->forc),
                         static_cast<double*>(h->hist), h->slab, h->qc_on ? static_cast<const double*>(h->qc) : nullptr,
                         h->depths_derived ? 0 : 1);
      HIPCHK(h, hipGetLastError());
    } else if (h->engine == TFG_F32 && split && !io.in) {
      // two parts on two streams: the first on the handle's stream, the second
      // on the side stream with its own uniforms (tfg_step copied them there)
      bool ns = true;
      if ((rc = choose_form(h, u + k0, K, io, &ns))) return rc;
      if ((rc = fork_side(h))) return rc;
      // an odd chunk count for the first part: the parts' planes then do not sit a
      // power of two apart (+0.3-0.5 % at 2048^2 against an even split, same box)
      const int64_t chA = (chunks_of(h->n_pad) / 2) | 1, chB = chunks_of(h->n_pad) - chA;
      const int64_t nA = chA * kBlock * kCellsPerThread;
      const bool fit = chA + chB <= h->max_blocks;  // one workgroup per chunk, as unsplit
      const int bA = (int)(fit ? chA : std::min<int64_t>(chA, h->max_blocks / 2));
      const int bB = (int)(fit ? chB : std::min<int64_t>(chB, h->max_blocks / 2));
      const Part pa = {0, nA, std::min(h->n, nA), 0, h->stream};
      const Part pb = {nA, h->n_pad - nA, std::max<int64_t>(h->n - nA, 0), bA, h->side};
      if ((rc = launch_fused<float, false>(h, d_u + k0, K, bA, lds, io, ns, &pa))) return rc;
      if ((rc = launch_fused<float, false>(h, h->d_u2 + k0, K, bB, lds, io, ns, &pb))) return rc;
      h->side_busy = true;
      if (ns) {
        ++h->ns_launches;
        if (h->state_state == kOk) h->state_state = kUnknown;
      }
    } else if (h->engine == TFG_F32) {
      bool ns = true;
      if ((rc = choose_form(h, u + k0, K, io, &ns))) return rc;
      rc = launch_fused<float, false>(h, d_u + k0, K, blocks, lds, io, ns);
      if (ns) {
        ++h->ns_launches;
        // the NaN-safe form may have carried missing data into the state
        if (h->state_state == kOk) h->state_state = kUnknown;
      }
    } else {
      rc = launch_fused<double, true>(h, d_u + k0, K, blocks, lds, io, false);
    }
    if (rc) return rc;
    h->depths_derived = true;
  }
  h->last_hist = u[nsteps - 1].hist;
  return TFG_OK;
}

}  // namespace

int tfg_step(tfg_handle* h, const tfg_uniforms* u, int64_t nsteps) {
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (nsteps <= 0) return TFG_OK;
  if (int rc = check_step(h, u, nsteps)) return rc;
  HIPCHK(h, hipSetDevice(h->device));
  const bool split = split_active(h);
  if (split) {
    if (int rc = ensure_side(h)) return rc;
  } else if (int rc = api_sync(h)) {  // a handle that stopped splitting (tfg_set_split)
    return rc;
  }
  // stage uniforms: pinned double buffer -> device array (and the side stream's copy)
  const int b = h->h_u_next;
  h->h_u_next ^= 1;
  if (h->h_u_ev[b]) HIPCHK(h, hipEventSynchronize(h->h_u_ev[b]));
  else HIPCHK(h, hipEventCreateWithFlags(&h->h_u_ev[b], hipEventDisableTiming));
  if (h->h_u_ev2[b]) HIPCHK(h, hipEventSynchronize(h->h_u_ev2[b]));
  if (h->h_u_cap[b] < nsteps) {
    if (h->h_u[b]) HIPCHK(h, hipHostFree(h->h_u[b]));
    h->h_u[b] = nullptr;
    HIPCHK(h, hipHostMalloc((void**)&h->h_u[b], (size_t)nsteps * sizeof(tfg_uniforms), hipHostMallocDefault));
    h->h_u_cap[b] = nsteps;
  }
  if (h->d_u_cap < nsteps) {
    // the previous launches may still read d_u: wait before reallocating
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->d_u) HIPCHK(h, hipFree(h->d_u));
    h->d_u = nullptr;
    HIPCHK(h, hipMalloc((void**)&h->d_u, (size_t)nsteps * sizeof(tfg_uniforms)));
    h->d_u_cap = nsteps;
  }
  std::memcpy(h->h_u[b], u, (size_t)nsteps * sizeof(tfg_uniforms));
  HIPCHK(h, hipMemcpyAsync(h->d_u, h->h_u[b], (size_t)nsteps * sizeof(tfg_uniforms), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipEventRecord(h->h_u_ev[b], h->stream));
  if (split) {
    if (h->d_u2_cap < nsteps) {
      HIPCHK(h, hipStreamSynchronize(h->side));  // its launches may still read d_u2
      if (h->d_u2) HIPCHK(h, hipFree(h->d_u2));
      h->d_u2 = nullptr;
      HIPCHK(h, hipMalloc((void**)&h->d_u2, (size_t)nsteps * sizeof(tfg_uniforms)));
      h->d_u2_cap = nsteps;
    }
    if (!h->h_u_ev2[b]) HIPCHK(h, hipEventCreateWithFlags(&h->h_u_ev2[b], hipEventDisableTiming));
    HIPCHK(h, hipMemcpyAsync(h->d_u2, h->h_u[b], (size_t)nsteps * sizeof(tfg_uniforms), hipMemcpyHostToDevice, h->side));
    HIPCHK(h, hipEventRecord(h->h_u_ev2[b], h->side));
  }
  return launch_steps(h, h->d_u, u, nsteps, IoArgs(), split);
}

int tfg_get_diag(tfg_handle* h, double* out, int n_catch) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h || !out) return fail(h, TFG_ERR_ARG, "null argument");
  if (n_catch != h->n_catch) return fail(h, TFG_ERR_ARG, "n_catch mismatch");
  HIPCHK(h, hipSetDevice(h->device));
  const int nb = n_catch * 6;
  hipLaunchKernelGGL(k_diag_reduce, nb, kBlock, 0, h->stream, h->slab, h->max_blocks, nb, h->diag);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipMemcpyAsync(out, h->diag, (size_t)n_catch * 6 * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  // P_max of an empty history is 0 like the reference's initial P_max (:314)
  for (int c = 0; c < n_catch; ++c) if (out[c * 6 + 5] == -INFINITY) out[c * 6 + 5] = 0.0;
  return TFG_OK;
}

int tfg_reset_diag(tfg_handle* h) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipMemsetAsync(h->slab, 0, (size_t)h->max_blocks * h->n_catch * 6 * 8, h->stream));
  return TFG_OK;
}

int tfg_selftest_powers(int device, const double* x, int64_t n, int which, double* out) {
  if (!x || !out || n < 0 || which < 0 || which > 13) return fail(nullptr, TFG_ERR_ARG, "bad arguments");
  if (n == 0) return TFG_OK;
  HIPCHK(nullptr, hipSetDevice(device));
  double* d = nullptr;
  HIPCHK(nullptr, hipMalloc((void**)&d, (size_t)n * 16));
  hipError_t e = hipMemcpy(d, x, (size_t)n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_selftest_powers, grid_for(n), 256, 0, nullptr, d, d + n, n, which);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, d + n, (size_t)n * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(nullptr, TFG_ERR_HIP, std::string("tfg_selftest_powers: ") + hipGetErrorString(e));
  return TFG_OK;
}

#ifdef TFG_WG_TIMING
// diagnostic builds only: the last k_fused<float> launch's per-workgroup
// [start, end, (xcc << 32) | cu] records (tfg_fused.hpp, g_wg_times)
int tfg_debug_wg_times(unsigned long long* out, int n) {
  if (!out || n < 0 || n > TFG_WG_TIMING) return fail(nullptr, TFG_ERR_ARG, "bad arguments");
  HIPCHK(nullptr, hipDeviceSynchronize());
  HIPCHK(nullptr, hipMemcpyFromSymbol(out, HIP_SYMBOL(tfg_kern::g_wg_times), (size_t)n * 24));
  return TFG_OK;
}
#endif

int tfg_nan_safe_launches(tfg_handle* h, int64_t* count) {
  if (!h || !count) return fail(h, TFG_ERR_ARG, "null argument");
  *count = h->ns_launches;
  return TFG_OK;
}

int tfg_sync(tfg_handle* h) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}

int tfg_fill_synthetic(tfg_handle* h, uint64_t seed, int64_t row0, int64_t nx_global, const float* diurnal,
                       int n_frames) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h || !diurnal) return fail(h, TFG_ERR_ARG, "null argument");
  if (n_frames != h->n_frames) return fail(h, TFG_ERR_ARG, "n_frames mismatch");
  if (nx_global != h->nx) return fail(h, TFG_ERR_ARG, "row-block shards must span full rows (nx_global == nx)");
  HIPCHK(h, hipSetDevice(h->device));
  if (!h->d_diurnal) HIPCHK(h, hipMalloc((void**)&h->d_diurnal, (size_t)n_frames * 4));
  HIPCHK(h, hipMemcpyAsync(h->d_diurnal, diurnal, (size_t)n_frames * 4, hipMemcpyHostToDevice, h->stream));
  const int gb = grid_for(h->n);
  if (h->engine == TFG_F32)
    hipLaunchKernelGGL((k_fill_synthetic<float>), gb, 256, 0, h->stream, (float*)h->forc, (float*)h->stat, h->st,
                       h->n, h->n_pad, h->nx, row0, nx_global, seed, h->d_diurnal, n_frames);
  else
    hipLaunchKernelGGL((k_fill_synthetic<double>), gb, 256, 0, h->stream, (double*)h->forc, (double*)h->stat, h->st,
                       h->n, h->n_pad, h->nx, row0, nx_global, seed, h->d_diurnal, n_frames);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->slope_invalid = false;
  h->geo_dirty = true;
  // the generator writes finite forcing, statics and depths
  std::fill(h->plane_state.begin(), h->plane_state.end(), kOk);
  h->elev_state = kOk;
  h->state_state = kOk;
  return tfg_init_state(h);
}

namespace {
int launch_scatter(tfg_handle* h, int frame, const void* dsrc, int src_dtype, int64_t n);
int launch_gather(tfg_handle* h, int hist, void* gdst, int dst_dtype, int64_t n);
}  // namespace

int tfg_set_inputs(tfg_handle* h, int frame, const void* src, int src_dtype, int64_t n, int src_on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!src) return fail(h, TFG_ERR_ARG, "null src");
  if (n != h->n) return fail(h, TFG_ERR_ARG, "n != ny*nx");
  if (frame < 0 || frame >= h->n_frames) return fail(h, TFG_ERR_ARG, "frame index out of range");
  if (src_dtype != TFG_F32 && src_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "src dtype must be TFG_F32/TFG_F64");
  HIPCHK(h, hipSetDevice(h->device));
  const size_t bytes = (size_t)5 * n * dtype_size(src_dtype);
  const void* dsrc = src;
  int b = -1;
  if (!src_on_device) {
    // the host buffer is borrowed for this call only: copy it into a pinned
    // slot whose previous transfer has completed, then transfer asynchronously
    b = h->in_next;
    h->in_next ^= 1;
    if (h->in_ev[b]) HIPCHK(h, hipEventSynchronize(h->in_ev[b]));
    else HIPCHK(h, hipEventCreateWithFlags(&h->in_ev[b], hipEventDisableTiming));
    if (h->in_cap[b] < bytes) {
      if (h->in_h[b]) HIPCHK(h, hipHostFree(h->in_h[b]));
      if (h->in_d[b]) HIPCHK(h, hipFree(h->in_d[b]));
      h->in_h[b] = h->in_d[b] = nullptr;
      h->in_cap[b] = 0;
      HIPCHK(h, hipHostMalloc(&h->in_h[b], bytes, hipHostMallocDefault));
      HIPCHK(h, hipMalloc(&h->in_d[b], bytes));
      h->in_cap[b] = bytes;
    }
    std::memcpy(h->in_h[b], src, bytes);
    HIPCHK(h, hipMemcpyAsync(h->in_d[b], h->in_h[b], bytes, hipMemcpyHostToDevice, h->stream));
    dsrc = h->in_d[b];
  }
  if (h->engine == TFG_F32) {  // finite-data tracking: host inputs are checked here, device inputs later
    static const int map[5] = {F_PA, F_Q, F_P, F_T, F_UZ};  // BMI order -> frame planes
    for (int f = 0; f < 5; ++f) {
      uint8_t st = kUnknown;
      if (!src_on_device)
        st = src_dtype == TFG_F64 ? host_finite_as_f32(static_cast<const double*>(src) + (size_t)f * n, n)
                                  : host_finite(static_cast<const float*>(src) + (size_t)f * n, n);
      h->plane_state[(size_t)frame * kNumForc + map[f]] = st;
    }
  }
  if (int rc = launch_scatter(h, frame, dsrc, src_dtype, n)) return rc;
  if (b >= 0) HIPCHK(h, hipEventRecord(h->in_ev[b], h->stream));
  return TFG_OK;
}

namespace {

// frame <- src[5][n] (device-visible pointer)
int launch_scatter(tfg_handle* h, int frame, const void* dsrc, int src_dtype, int64_t n) {
  char* fr = static_cast<char*>(h->forc) + (size_t)frame * kNumForc * h->n_pad * h->rsz;
  const int gb = grid_for(n);
  if (h->engine == TFG_F32 && src_dtype == TFG_F32)
    hipLaunchKernelGGL((k_scatter_inputs<float, float>), gb, 256, 0, h->stream, (float*)fr, (const float*)dsrc, n, h->n_pad);
  else if (h->engine == TFG_F32)
    hipLaunchKernelGGL((k_scatter_inputs<float, double>), gb, 256, 0, h->stream, (float*)fr, (const double*)dsrc, n, h->n_pad);
  else if (src_dtype == TFG_F32)
    hipLaunchKernelGGL((k_scatter_inputs<double, float>), gb, 256, 0, h->stream, (double*)fr, (const float*)dsrc, n, h->n_pad);
  else
    hipLaunchKernelGGL((k_scatter_inputs<double, double>), gb, 256, 0, h->stream, (double*)fr, (const double*)dsrc, n, h->n_pad);
  HIPCHK(h, hipGetLastError());
  return TFG_OK;
}

// dst[8][n] (device-visible pointer) <- outputs of history slot `hist`
int launch_gather(tfg_handle* h, int hist, void* gdst, int dst_dtype, int64_t n) {
  const char* hs = static_cast<const char*>(h->hist) + (size_t)hist * kNumHist * h->n_pad * h->rsz;
  const int from_state = h->depths_derived ? 0 : 1;
  const int gb = grid_for(n);
  if (h->engine == TFG_F32 && dst_dtype == TFG_F32)
    hipLaunchKernelGGL((k_gather_outputs<float, float>), gb, 256, 0, h->stream, (float*)gdst, (const float*)hs, h->st, n, h->n_pad, from_state);
  else if (h->engine == TFG_F32)
    hipLaunchKernelGGL((k_gather_outputs<float, double>), gb, 256, 0, h->stream, (double*)gdst, (const float*)hs, h->st, n, h->n_pad, from_state);
  else if (dst_dtype == TFG_F32)
    hipLaunchKernelGGL((k_gather_outputs<double, float>), gb, 256, 0, h->stream, (float*)gdst, (const double*)hs, h->st, n, h->n_pad, from_state);
  else
    hipLaunchKernelGGL((k_gather_outputs<double, double>), gb, 256, 0, h->stream, (double*)gdst, (const double*)hs, h->st, n, h->n_pad, from_state);
  HIPCHK(h, hipGetLastError());
  return TFG_OK;
}

}  // namespace

int tfg_get_outputs(tfg_handle* h, int hist, void* dst, int dst_dtype, int64_t n, int dst_on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!dst) return fail(h, TFG_ERR_ARG, "null dst");
  if (n != h->n) return fail(h, TFG_ERR_ARG, "n != ny*nx");
  if (hist < 0 || hist >= h->hist_depth) return fail(h, TFG_ERR_ARG, "history slot out of range");
  if (dst_dtype != TFG_F32 && dst_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "dst dtype must be TFG_F32/TFG_F64");
  HIPCHK(h, hipSetDevice(h->device));
  const size_t bytes = (size_t)8 * n * dtype_size(dst_dtype);
  void* gdst = dst;
  if (!dst_on_device) {
    if (h->out_cap < bytes) {
      if (h->out_d) HIPCHK(h, hipFree(h->out_d));
      if (h->out_h) HIPCHK(h, hipHostFree(h->out_h));
      h->out_d = h->out_h = nullptr;
      h->out_cap = 0;
      HIPCHK(h, hipMalloc(&h->out_d, bytes));
      HIPCHK(h, hipHostMalloc(&h->out_h, bytes, hipHostMallocDefault));
      h->out_cap = bytes;
    }
    gdst = h->out_d;
  }
  if (int rc = launch_gather(h, hist, gdst, dst_dtype, n)) return rc;
  if (!dst_on_device) {
    HIPCHK(h, hipMemcpyAsync(h->out_h, h->out_d, bytes, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    std::memcpy(dst, h->out_h, bytes);
  }
  return TFG_OK;
}

#ifdef TFG_UPDATE_TIMING
// Diagnostic build only (tests/diagnostics/bmi_many_instances.py): where the
// time of tfg_update goes, summed over calls [ns]: input packing, the launch
// call, waiting for the release flags, output unpacking; [4] = calls.
static double g_upd_ns[5];
extern "C" void tfg_update_timing(double* out) {
  for (int i = 0; i < 5; ++i) out[i] = g_upd_ns[i];
}
#define TFG_TSTAMP(v) const auto v = std::chrono::steady_clock::now()
#define TFG_TACC(i, a, b) (g_upd_ns[i] += std::chrono::duration<double, std::nano>((b) - (a)).count())
#else
#define TFG_TSTAMP(v)
#define TFG_TACC(i, a, b)
#endif

namespace {
// Wait for the workgroups' release flags of a tfg_update launch (a few
// microseconds sooner than a stream synchronisation); after ~2 ms fall back to
// the stream wait, which also reports a failed launch.
int wait_flags(tfg_handle* h, size_t flag_off, int blocks, uint32_t seq) {
  const volatile uint32_t* fl = reinterpret_cast<const volatile uint32_t*>(h->io_h + flag_off);
  const auto t0 = std::chrono::steady_clock::now();
  bool done = false;
  for (int64_t spins = 0; !done; ++spins) {
    done = true;
    for (int b = 0; b < blocks && done; ++b) done = fl[b] == seq;
    if (!done && (spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
  }
  if (done) std::atomic_thread_fence(std::memory_order_acquire);
  else HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}
}  // namespace

int tfg_update(tfg_handle* h, int frame, const void* src, int src_dtype, const tfg_uniforms* u, void* dst,
               int dst_dtype, int64_t n) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  TFG_TSTAMP(t_in0);
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!src || !dst) return fail(h, TFG_ERR_ARG, "null src/dst");
  if (n != h->n) return fail(h, TFG_ERR_ARG, "n != ny*nx");
  if (frame < 0 || frame >= h->n_frames) return fail(h, TFG_ERR_ARG, "frame index out of range");
  if (src_dtype != TFG_F32 && src_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "src dtype must be TFG_F32/TFG_F64");
  if (dst_dtype != TFG_F32 && dst_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "dst dtype must be TFG_F32/TFG_F64");
  if (int rc = check_step(h, u, 1)) return rc;
  if (u->frame != frame) return fail(h, TFG_ERR_ARG, "uniforms: frame differs from the input frame");
  HIPCHK(h, hipSetDevice(h->device));
  // One pinned block [forcing kNumForc x n_pad (engine type) | uniforms | outputs 8 x n f64];
  // the call is synchronous, so one block suffices.
  const int64_t np = h->n_pad;
  const size_t in_b = (size_t)kNumForc * np * h->rsz;
  const size_t u_off = (in_b + 255) & ~(size_t)255;
  const size_t out_off = u_off + 256;
  const size_t out_b = (size_t)8 * n * 8;
  const int blocks = fused_blocks(h);
  const size_t flag_off = (out_off + out_b + 255) & ~(size_t)255;
  const size_t total = flag_off + (size_t)blocks * 4;
  if (h->io_cap < total) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->io_h) HIPCHK(h, hipHostFree(h->io_h));
    h->io_h = h->io_d = nullptr;
    h->io_cap = 0;
    HIPCHK(h, hipHostMalloc((void**)&h->io_h, total, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h->io_h, 0, total);  // padding cells read zeros; flags start at 0
    HIPCHK(h, hipHostGetDevicePointer((void**)&h->io_d, h->io_h, 0));
    h->io_cap = total;
    h->io_seq = 0;
  }
  // BMI order (P_air, Hum_sp, P, T_air, uz) -> frame fields, converted to the engine type
  static const int map[5] = {F_PA, F_Q, F_P, F_T, F_UZ};
  if (h->engine == TFG_F64 && n == 1) {
    // one catchment (NextGen's per-catchment model): k_cell, inputs and
    // uniforms as kernel arguments, one workgroup of four waves
    CellIo cio;
    cio.u = *u;
    for (int f = 0; f < 5; ++f)
      cio.in[map[f]] = src_dtype == TFG_F64 ? static_cast<const double*>(src)[f] : (double)static_cast<const float*>(src)[f];
    KArgs a;
    a.p = h->dp;
    a.K = 1;
    a.n_catch = h->n_catch;
    a.n = h->n;
    a.n_pad = h->n_pad;
    a.n_step = h->n_pad;
    a.io_in = nullptr;
    a.io_out = reinterpret_cast<double*>(h->io_d + out_off);
    a.io_flag = reinterpret_cast<uint32_t*>(h->io_d + flag_off);
    a.io_seq = ++h->io_seq == 0 ? ++h->io_seq : h->io_seq;  // never 0, the initial flag value
    TFG_TSTAMP(t_c0);
    TFG_TACC(0, t_in0, t_c0);
    if (int rc = prepare_steps(h)) return rc;
    hipLaunchKernelGGL(k_cell, 1, 64 * tfg::kCellWaves, 0, h->stream, a, cio, reinterpret_cast<const double*>(h->geo), h->catch_id,
                       h->st, h->tot, h->ring, static_cast<double*>(h->forc), static_cast<double*>(h->hist), h->slab,
                       h->qc_on ? static_cast<const double*>(h->qc) : nullptr, h->depths_derived ? 0 : 1);
    HIPCHK(h, hipGetLastError());
    h->depths_derived = true;
    h->last_hist = u->hist;
    TFG_TSTAMP(t_c1);
    TFG_TACC(1, t_c0, t_c1);
    if (int rc = wait_flags(h, flag_off, 1, a.io_seq)) return rc;
    TFG_TSTAMP(t_c2);
    TFG_TACC(2, t_c1, t_c2);
    const double* oh = reinterpret_cast<const double*>(h->io_h + out_off);
    if (dst_dtype == TFG_F64) std::memcpy(dst, oh, out_b);
    else for (int64_t i = 0; i < 8; ++i) static_cast<float*>(dst)[i] = (float)oh[i];
    TFG_TSTAMP(t_c3);
    TFG_TACC(3, t_c2, t_c3);
#ifdef TFG_UPDATE_TIMING
    g_upd_ns[4] += 1;
#endif
    return TFG_OK;
  }
  for (int f = 0; f < 5; ++f) {
    char* o = h->io_h + (size_t)map[f] * np * h->rsz;
    if (src_dtype == TFG_F64) {
      const double* sv = static_cast<const double*>(src) + (size_t)f * n;
      if (h->engine == TFG_F32) for (int64_t i = 0; i < n; ++i) reinterpret_cast<float*>(o)[i] = (float)sv[i];
      else std::memcpy(o, sv, (size_t)n * 8);
    } else {
      const float* sv = static_cast<const float*>(src) + (size_t)f * n;
      if (h->engine == TFG_F32) std::memcpy(o, sv, (size_t)n * 4);
      else for (int64_t i = 0; i < n; ++i) reinterpret_cast<double*>(o)[i] = (double)sv[i];
    }
  }
  std::memcpy(h->io_h + u_off, u, sizeof(tfg_uniforms));
  IoArgs io;
  if (h->engine == TFG_F32) {  // finite-data status of the step's inputs, as the kernel reads them
    io.in_state = kOk;
    for (int f = 0; f < 5; ++f)
      if (host_finite(reinterpret_cast<const float*>(h->io_h + (size_t)map[f] * np * h->rsz), n) != kOk) io.in_state = kDirty;
  }
  TFG_TSTAMP(t_in1);
  TFG_TACC(0, t_in0, t_in1);
  io.in = h->io_d;
  io.out = reinterpret_cast<double*>(h->io_d + out_off);
  io.flag = reinterpret_cast<uint32_t*>(h->io_d + flag_off);
  io.seq = ++h->io_seq == 0 ? ++h->io_seq : h->io_seq;  // never 0, the initial flag value
  if (int rc = launch_steps(h, reinterpret_cast<const tfg_uniforms*>(h->io_d + u_off), u, 1, io)) return rc;
  if (h->engine == TFG_F32)  // the kernel stored the inputs into the frame
    std::fill_n(h->plane_state.begin() + (size_t)frame * kNumForc, kNumForc, io.in_state);
  TFG_TSTAMP(t_l1);
  TFG_TACC(1, t_in1, t_l1);
  if (int rc = wait_flags(h, flag_off, blocks, io.seq)) return rc;
  TFG_TSTAMP(t_w1);
  TFG_TACC(2, t_l1, t_w1);
  const double* oh = reinterpret_cast<const double*>(h->io_h + out_off);
  if (dst_dtype == TFG_F64) std::memcpy(dst, oh, out_b);
  else for (int64_t i = 0; i < 8 * n; ++i) static_cast<float*>(dst)[i] = (float)oh[i];
  TFG_TSTAMP(t_o1);
  TFG_TACC(3, t_w1, t_o1);
#ifdef TFG_UPDATE_TIMING
  g_upd_ns[4] += 1;
#endif
  return TFG_OK;
}

namespace {
// tfg_update_many's pinned, device-mapped block of one device:
// [jobs m x CellJob | outputs m x 8 f64 | release flags m x u32].  Calls are
// synchronous, so one block per device serves every call, under its mutex.
struct ManyBlock {
  std::mutex mu;
  char* h = nullptr;
  char* d = nullptr;
  size_t cap = 0;
  uint32_t seq = 0;
};
constexpr int kMaxDevices = 64;
ManyBlock g_many[kMaxDevices];
}  // namespace

int tfg_update_many(tfg_handle* const* hs, int m, const double* const* src, const tfg_uniforms* const* u,
                    double* const* dst) {
  for (int i = 0; hs && i < m; ++i)
    if (int rc_ = api_sync(hs[i])) return rc_;  // after a split launch's second part
  if (m <= 0) return TFG_OK;
  if (!hs || !src || !u || !dst) return fail(nullptr, TFG_ERR_ARG, "tfg_update_many: null argument");
  tfg_handle* h0 = hs[0];
  if (!h0) return fail(nullptr, TFG_ERR_ARG, "tfg_update_many: null handle 0");
  if (h0->device < 0 || h0->device >= kMaxDevices) return fail(nullptr, TFG_ERR_ARG, "tfg_update_many: device id");
  for (int i = 0; i < m; ++i) {
    tfg_handle* h = hs[i];
    const std::string at = "tfg_update_many: handle " + std::to_string(i) + ": ";
    if (!h || !src[i] || !u[i] || !dst[i]) return fail(nullptr, TFG_ERR_ARG, at + "null handle/src/uniforms/dst");
    if (h->engine != TFG_F64 || h->n != 1) return fail(nullptr, TFG_ERR_ARG, at + "not a one-cell TFG_F64 handle");
    if (h->device != h0->device || h->stream != h0->stream)
      return fail(nullptr, TFG_ERR_ARG, at + "every handle must be on one device and share one stream (tfg_shared_stream)");
    if (int rc = check_step(h, u[i], 1)) return fail(nullptr, rc, at + h->err);
  }
  {  // one step per handle per launch: a handle listed twice would race with itself
    std::vector<const tfg_handle*> v(hs, hs + m);
    std::sort(v.begin(), v.end());
    if (std::adjacent_find(v.begin(), v.end()) != v.end())
      return fail(nullptr, TFG_ERR_ARG, "tfg_update_many: a handle is listed twice");
  }
  ManyBlock& B = g_many[h0->device];
  std::lock_guard<std::mutex> lock(B.mu);
  HIPCHK(nullptr, hipSetDevice(h0->device));
  const size_t job_b = (size_t)m * sizeof(CellJob);
  const size_t out_off = (job_b + 255) & ~(size_t)255;
  const size_t flag_off = (out_off + (size_t)m * 64 + 255) & ~(size_t)255;
  const size_t total = flag_off + (size_t)m * 4;
  if (B.cap < total) {
    const size_t want = std::max(total, B.cap * 2);
    if (B.h) HIPCHK(nullptr, hipHostFree(B.h));
    B.h = B.d = nullptr;
    B.cap = 0;
    HIPCHK(nullptr, hipHostMalloc((void**)&B.h, want, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(B.h, 0, want);
    HIPCHK(nullptr, hipHostGetDevicePointer((void**)&B.d, B.h, 0));
    B.cap = want;
    B.seq = 0;
  }
  CellJob* jobs = reinterpret_cast<CellJob*>(B.h);
  static const int map[5] = {F_PA, F_Q, F_P, F_T, F_UZ};  // BMI order -> device frame order
  for (int i = 0; i < m; ++i) {
    tfg_handle* h = hs[i];
    if (int rc = prepare_steps(h)) return fail(nullptr, rc, "tfg_update_many: " + h->err);
    CellJob& j = jobs[i];
    j.p = h->dp;
    j.u = *u[i];
    for (int f = 0; f < 5; ++f) j.in[map[f]] = src[i][f];
    j.geo = reinterpret_cast<const double*>(h->geo);
    j.catch_id = h->catch_id;
    j.st = h->st;
    j.tot = h->tot;
    j.ring = h->ring;
    j.forc = static_cast<double*>(h->forc);
    j.hist = static_cast<double*>(h->hist);
    j.slab = h->slab;
    j.qc = h->qc_on ? static_cast<const double*>(h->qc) : nullptr;
    j.n_pad = h->n_pad;
    j.read_depths = h->depths_derived ? 0 : 1;
    j.pad_ = 0;
  }
  const uint32_t seq = ++B.seq == 0 ? ++B.seq : B.seq;  // never 0, the initial flag value
  hipLaunchKernelGGL(k_cell_many, m, 64 * tfg::kCellWaves, 0, h0->stream, reinterpret_cast<const CellJob*>(B.d),
                     reinterpret_cast<double*>(B.d + out_off), reinterpret_cast<uint32_t*>(B.d + flag_off), seq);
  HIPCHK(nullptr, hipGetLastError());
  for (int i = 0; i < m; ++i) {
    hs[i]->depths_derived = true;
    hs[i]->last_hist = u[i]->hist;
  }
  // wait for every workgroup's release flag (a stream synchronisation after ~2 ms)
  const volatile uint32_t* fl = reinterpret_cast<const volatile uint32_t*>(B.h + flag_off);
  const auto t0 = std::chrono::steady_clock::now();
  int done = 0;
  for (int64_t spins = 0; done < m; ++spins) {
    while (done < m && fl[done] == seq) ++done;
    if (done < m && (spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
  }
  if (done == m) std::atomic_thread_fence(std::memory_order_acquire);
  else HIPCHK(nullptr, hipStreamSynchronize(h0->stream));
  const double* oh = reinterpret_cast<const double*>(B.h + out_off);
  for (int i = 0; i < m; ++i) std::memcpy(dst[i], oh + (size_t)i * 8, 64);
  return TFG_OK;
}

int tfg_terrain_from_dem(tfg_handle* h, double dx, double dy, const void* halo_north, const void* halo_south,
                         int halo_dtype, int halo_on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!(dx > 0) || !(dy > 0)) return fail(h, TFG_ERR_ARG, "dx and dy must be > 0");
  if (halo_dtype != TFG_F32 && halo_dtype != TFG_F64) return fail(h, TFG_ERR_ARG, "halo dtype must be TFG_F32/TFG_F64");
  HIPCHK(h, hipSetDevice(h->device));
  const int64_t nx = h->nx, ny = h->ny;
  if (!h->halo) HIPCHK(h, hipMalloc((void**)&h->halo, (size_t)2 * nx * 8));
  const size_t rs = h->rsz;
  const char* el = static_cast<const char*>(h->stat);  // TFG_ST_ELEV plane
  // a missing halo replicates the shard's own edge row (domain boundary)
  const void* src[2] = {halo_north, halo_south};
  for (int k = 0; k < 2; ++k) {
    if (src[k]) {
      int rc = upload(h, h->halo + k * nx, TFG_F64, src[k], halo_dtype, nx, halo_on_device);
      if (rc) return rc;
    } else {
      const int64_t row = k == 0 ? 0 : ny - 1;
      int rc = upload(h, h->halo + k * nx, TFG_F64, el + row * nx * rs, h->engine, nx, 1);
      if (rc) return rc;
    }
  }
  char* st = static_cast<char*>(h->stat);
  if (h->engine == TFG_F32)
    hipLaunchKernelGGL((k_terrain<float>), grid_for(h->n), 256, 0, h->stream, (const float*)st, h->halo,
                       (float*)(st + h->n_pad * rs), (float*)(st + 2 * h->n_pad * rs), ny, nx, 1.0 / (8.0 * dx), 1.0 / (8.0 * dy));
  else
    hipLaunchKernelGGL((k_terrain<double>), grid_for(h->n), 256, 0, h->stream, (const double*)st, h->halo,
                       (double*)(st + h->n_pad * rs), (double*)(st + 2 * h->n_pad * rs), ny, nx, 1.0 / (8.0 * dx), 1.0 / (8.0 * dy));
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  h->geo_dirty = true;
  h->slope_invalid = false;  // tan(beta) >= 0 always maps into [0, pi/2)
  return TFG_OK;
}


namespace {
// Ice-flow halos into h->flow_halo; FlowGrid over this shard.
int flow_setup(tfg_handle* h, const double* hn, const double* hs, int on_dev, FlowGrid& g) {
  if (!h->initialised) return fail(h, TFG_ERR_STATE, "tfg_init_state() has not been called");
  const int64_t nx = h->nx;
  if (!h->flow_halo) HIPCHK(h, hipMalloc((void**)&h->flow_halo, (size_t)4 * nx * 8));
  if (hn) HIPCHK(h, hipMemcpyAsync(h->flow_halo, hn, (size_t)2 * nx * 8, on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream));
  if (hs) HIPCHK(h, hipMemcpyAsync(h->flow_halo + 2 * nx, hs, (size_t)2 * nx * 8, on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream));
  g.elev = h->stat;
  g.iwe = h->st + S_HIWE * h->n_pad;
  g.hn = hn ? h->flow_halo : nullptr;
  g.hs = hs ? h->flow_halo + 2 * nx : nullptr;
  g.ny = h->ny;
  g.nx = nx;
  g.wi = h->dp.wi;
  return TFG_OK;
}
}  // namespace

int tfg_ice_flow_edges(tfg_handle* h, double* first, double* last, int on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h || !first || !last) return fail(h, TFG_ERR_ARG, "null argument");
  HIPCHK(h, hipSetDevice(h->device));
  FlowGrid g;
  if (int rc = flow_setup(h, nullptr, nullptr, 0, g)) return rc;
  const int64_t nx = h->nx;
  if (!h->flow_edges) HIPCHK(h, hipMalloc((void**)&h->flow_edges, (size_t)4 * nx * 8));
  const int gb = grid_for(nx);
  if (h->engine == TFG_F32)
    hipLaunchKernelGGL((k_ice_flow_edges<float>), gb, 256, 0, h->stream, g, h->flow_edges, h->flow_edges + 2 * nx);
  else
    hipLaunchKernelGGL((k_ice_flow_edges<double>), gb, 256, 0, h->stream, g, h->flow_edges, h->flow_edges + 2 * nx);
  HIPCHK(h, hipGetLastError());
  const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  HIPCHK(h, hipMemcpyAsync(first, h->flow_edges, (size_t)2 * nx * 8, k, h->stream));
  HIPCHK(h, hipMemcpyAsync(last, h->flow_edges + 2 * nx, (size_t)2 * nx * 8, k, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}

int tfg_ice_flow_dmax(tfg_handle* h, double dx, double dy, const double* halo_north, const double* halo_south,
                      int halo_on_device, double* dmax) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h || !dmax) return fail(h, TFG_ERR_ARG, "null argument");
  if (!(dx > 0) || !(dy > 0)) return fail(h, TFG_ERR_ARG, "dx and dy must be > 0");
  HIPCHK(h, hipSetDevice(h->device));
  FlowGrid g;
  if (int rc = flow_setup(h, halo_north, halo_south, halo_on_device, g)) return rc;
  const dim3 fgrid((unsigned)((h->nx + kFlowTX - 1) / kFlowTX), (unsigned)((h->ny + kFlowRows - 1) / kFlowRows));
  if (fgrid.y > 65535u) return fail(h, TFG_ERR_ARG, "ice flow: too many rows for one shard");
  const int64_t gb = (int64_t)fgrid.x * fgrid.y;
  const FlowTiles ft = flow_tiles(h->nx, (int)fgrid.y);
  const FlowK fk = flow_constants(1.0, dx, dy, h->dp.wi, h->flow_gamma);  // dt unused by the bound
  if (!h->flow_red) HIPCHK(h, hipMalloc((void**)&h->flow_red, (size_t)gb * 8));  // the grid never changes
  if (h->engine == TFG_F32)
    hipLaunchKernelGGL((k_ice_flow<float, true>), flow_blocks(ft), kFlowTX, 0, h->stream, g, fk, h->flow_red, 0, 1, nullptr, ft);
  else
    hipLaunchKernelGGL((k_ice_flow<double, true>), flow_blocks(ft), kFlowTX, 0, h->stream, g, fk, h->flow_red, 0, 1, nullptr, ft);
  HIPCHK(h, hipGetLastError());
  std::vector<double> bm(gb);
  HIPCHK(h, hipMemcpyAsync(bm.data(), h->flow_red, (size_t)gb * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  double m = 0.0;
  for (double v : bm) m = std::max(m, v);
  *dmax = m;
  return TFG_OK;
}

int tfg_ice_flow_step(tfg_handle* h, double dt_years, double dx, double dy, const double* halo_north,
                      const double* halo_south, int halo_on_device, int part) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!(dx > 0) || !(dy > 0) || !(dt_years > 0)) return fail(h, TFG_ERR_ARG, "dt, dx and dy must be > 0");
  if (part != TFG_FLOW_ALL && part != TFG_FLOW_INTERIOR && part != TFG_FLOW_EDGES)
    return fail(h, TFG_ERR_ARG, "part must be TFG_FLOW_ALL, TFG_FLOW_INTERIOR or TFG_FLOW_EDGES");
  if (part == TFG_FLOW_INTERIOR && (halo_north || halo_south))
    return fail(h, TFG_ERR_ARG, "the interior part takes no halo rows");
  HIPCHK(h, hipSetDevice(h->device));
  FlowGrid g;
  if (int rc = flow_setup(h, halo_north, halo_south, halo_on_device, g)) return rc;
  if (!h->wtmp) HIPCHK(h, hipMalloc((void**)&h->wtmp, (size_t)h->n_pad * 8));
  const int64_t strips = (h->ny + kFlowRows - 1) / kFlowRows;
  if (strips > 65535) return fail(h, TFG_ERR_ARG, "ice flow: too many rows for one shard");
  const FlowK fk = flow_constants(dt_years, dx, dy, h->dp.wi, h->flow_gamma);
  // strips [first, first + count*step) by `step`: all of them, the interior
  // ones (no halo row read), or the first and last (the halo readers)
  int first = 0, count = (int)strips, step = 1;
  if (part == TFG_FLOW_INTERIOR) { first = 1; count = (int)std::max<int64_t>(strips - 2, 0); }
  if (part == TFG_FLOW_EDGES) { count = strips > 1 ? 2 : 1; step = (int)std::max<int64_t>(strips - 1, 1); }
  // h_ice (not read by the flow kernels) goes straight to the state plane; the
  // new h_iwe goes to scratch, since neighbouring strips still read the old one
  double* ice = h->st + S_HICE * h->n_pad;
  if (count > 0) {
    const FlowTiles ft = flow_tiles(h->nx, count);
    if (h->engine == TFG_F32)
      hipLaunchKernelGGL((k_ice_flow<float, false>), flow_blocks(ft), kFlowTX, 0, h->stream, g, fk, h->wtmp, first, step, ice, ft);
    else
      hipLaunchKernelGGL((k_ice_flow<double, false>), flow_blocks(ft), kFlowTX, 0, h->stream, g, fk, h->wtmp, first, step, ice, ft);
    HIPCHK(h, hipGetLastError());
  }
  if (part == TFG_FLOW_INTERIOR) return TFG_OK;  // queued; the edges part commits
  hipLaunchKernelGGL(k_flow_commit<false>, grid_for(h->n), 256, 0, h->stream, h->st, h->wtmp, h->n, h->n_pad, h->dp.wi);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}

int tfg_ice_flow_run(tfg_handle* h, double dt_years, double dx, double dy, int n_sub) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!(dx > 0) || !(dy > 0) || !(dt_years > 0) || n_sub < 1) return fail(h, TFG_ERR_ARG, "dt, dx, dy and n_sub must be > 0");
  HIPCHK(h, hipSetDevice(h->device));
  FlowGrid g;
  if (int rc = flow_setup(h, nullptr, nullptr, 0, g)) return rc;
  if (!h->wtmp) HIPCHK(h, hipMalloc((void**)&h->wtmp, (size_t)h->n_pad * 8));
  const int64_t strips = (h->ny + kFlowRows - 1) / kFlowRows;
  if (strips > 65535) return fail(h, TFG_ERR_ARG, "ice flow: too many rows for one shard");
  const FlowK fk = flow_constants(dt_years / n_sub, dx, dy, h->dp.wi, h->flow_gamma);
  const FlowTiles ft = flow_tiles(h->nx, (int)strips);
  // ping-pong between the state plane and the scratch plane: a sub-step that
  // lands in the state plane writes h_ice with it, so only an odd count needs
  // the commit pass at the end
  double* plane = h->st + S_HIWE * h->n_pad;
  double* ice = h->st + S_HICE * h->n_pad;
  for (int k = 0; k < n_sub; ++k) {
    const bool to_state = (k & 1) != 0;
    g.iwe = to_state ? h->wtmp : plane;
    double* dst = to_state ? plane : h->wtmp;
    if (h->engine == TFG_F32)
      hipLaunchKernelGGL((k_ice_flow<float, false>), flow_blocks(ft), kFlowTX, 0, h->stream, g, fk, dst, 0, 1,
                         to_state ? ice : nullptr, ft);
    else
      hipLaunchKernelGGL((k_ice_flow<double, false>), flow_blocks(ft), kFlowTX, 0, h->stream, g, fk, dst, 0, 1,
                         to_state ? ice : nullptr, ft);
    HIPCHK(h, hipGetLastError());
  }
  if (n_sub & 1)
    hipLaunchKernelGGL(k_flow_commit<true>, grid_for(h->n), 256, 0, h->stream, h->st, h->wtmp, h->n, h->n_pad, h->dp.wi);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}

namespace {
// Conduction halos into h->cond_halo; the CondGrid of this shard.
int cond_setup(tfg_handle* h, const double* hn, const double* hs, int on_dev, tfg::CondGrid& g) {
  if (!h->initialised) return fail(h, TFG_ERR_STATE, "tfg_init_state() has not been called");
  const int64_t nx = h->nx, np = h->n_pad;
  if (!h->cond_halo) HIPCHK(h, hipMalloc((void**)&h->cond_halo, (size_t)8 * nx * 8));
  const hipMemcpyKind k = on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  if (hn) HIPCHK(h, hipMemcpyAsync(h->cond_halo, hn, (size_t)4 * nx * 8, k, h->stream));
  if (hs) HIPCHK(h, hipMemcpyAsync(h->cond_halo + 4 * nx, hs, (size_t)4 * nx * 8, k, h->stream));
  static_assert(S_HIWE == S_HSWE + 1 && S_ECCS == S_HSWE + 2 && S_ECCI == S_HSWE + 3,
                "k_conduction reads h_swe, h_iwe, Eccs, Ecci as consecutive planes");
  g.st = h->st + S_HSWE * np;
  g.hn = hn ? h->cond_halo : nullptr;
  g.hs = hs ? h->cond_halo + 4 * nx : nullptr;
  g.ny = h->ny;
  g.nx = nx;
  g.n_pad = np;
  g.ws = h->dp.ws;
  g.wi = h->dp.wi;
  g.T0 = h->dp.T0;
  g.inv_cs = h->inv_cs;
  g.inv_ci = h->inv_ci;
  return TFG_OK;
}
}  // namespace

int tfg_conduction_edges(tfg_handle* h, double* first, double* last, int on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h || !first || !last) return fail(h, TFG_ERR_ARG, "null argument");
  HIPCHK(h, hipSetDevice(h->device));
  tfg::CondGrid g;
  if (int rc = cond_setup(h, nullptr, nullptr, 0, g)) return rc;
  const int64_t nx = h->nx;
  if (!h->cond_edges) HIPCHK(h, hipMalloc((void**)&h->cond_edges, (size_t)8 * nx * 8));
  hipLaunchKernelGGL(tfg::k_conduction_edges, grid_for(nx), 256, 0, h->stream, g, h->cond_edges, h->cond_edges + 4 * nx);
  HIPCHK(h, hipGetLastError());
  const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  HIPCHK(h, hipMemcpyAsync(first, h->cond_edges, (size_t)4 * nx * 8, k, h->stream));
  HIPCHK(h, hipMemcpyAsync(last, h->cond_edges + 4 * nx, (size_t)4 * nx * 8, k, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return TFG_OK;
}

int tfg_conduction_update(tfg_handle* h, double k_snow, double k_ice, double dx, double dy, double q_ground,
                          const double* halo_north, const double* halo_south, int halo_on_device) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  if (!(dx > 0) || !(dy > 0)) return fail(h, TFG_ERR_ARG, "dx and dy must be > 0");
  if (!(k_snow >= 0) || !(k_ice >= 0)) return fail(h, TFG_ERR_ARG, "conductivities must be >= 0");
  // every argument check before cond_setup queues copies from the caller's halo rows
  if (!std::isfinite(q_ground)) return fail(h, TFG_ERR_ARG, "ground heat flux must be finite");
  const int64_t gx = (h->nx + tfg::kCondOut - 1) / tfg::kCondOut, strips = (h->ny + tfg::kCondRows - 1) / tfg::kCondRows;
  const int64_t per_xcd = (gx * strips + 7) / 8;
  if (8 * per_xcd > 0x7fffffff) return fail(h, TFG_ERR_ARG, "conduction: grid too large");
  HIPCHK(h, hipSetDevice(h->device));
  if (int rc = ensure_qc(h)) return rc;
  tfg::CondGrid g;
  if (int rc = cond_setup(h, halo_north, halo_south, halo_on_device, g)) return rc;
  const tfg::CondK K = {k_snow / (dx * dx), k_snow / (dy * dy), k_ice * h->h_active / (dx * dx),
                        k_ice * h->h_active / (dy * dy), q_ground};
  if (h->engine == TFG_F32)
    hipLaunchKernelGGL((tfg::k_conduction<float>), (unsigned)(8 * per_xcd), tfg::kCondTX, 0, h->stream, g, K,
                       (float*)h->qc, (int)gx, (int)strips, (int)per_xcd);
  else
    hipLaunchKernelGGL((tfg::k_conduction<double>), (unsigned)(8 * per_xcd), tfg::kCondTX, 0, h->stream, g, K,
                       (double*)h->qc, (int)gx, (int)strips, (int)per_xcd);
  HIPCHK(h, hipGetLastError());
  // the halo rows are the caller's: finish reading them before returning
  if (halo_north || halo_south) HIPCHK(h, hipStreamSynchronize(h->stream));
  h->qc_on = true;
  // Qc of a finite state is finite; a neighbour's halo rows are not checked here
  h->qc_state = (h->state_state == kOk && !halo_north && !halo_south) ? kOk : kUnknown;
  return TFG_OK;
}

int tfg_conduction_off(tfg_handle* h) {
  if (int rc_ = api_sync(h)) return rc_;  // after a split launch's second part
  if (!h) return fail(nullptr, TFG_ERR_ARG, "null handle");
  h->qc_on = false;
  if (h->qc) {
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemsetAsync(h->qc, 0, (size_t)h->n_pad * h->rsz, h->stream));
  }
  return TFG_OK;
}

const char* tfg_last_error(const tfg_handle* h) { return h ? h->err.c_str() : g_err.c_str(); }

}  // extern "C"
