// tfg_fused.hpp -- the fused multi-step kernel k_fused<R, EXACT, READ_DEPTHS,
// CATCH, QC, C, NS> and its helpers, shared by the two translation units of the
// engine library: tfg_engine.hip (the C ABI, every other kernel, and the fp32
// engine's instantiations) and tfg_fused_f64.hip (the fp64 engine's
// instantiations, compiled with different code-motion flags; see there).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdint>

#include "../../include/tfg.h"
#include "tfg_physics.hpp"

namespace tfg_kern {

using tfg::CellDiag;
using tfg::CellOut;
using tfg::CellState;
using tfg::CellStatic;
using tfg::CellStaticF;
using tfg::DevParams;

constexpr int kBlock = 256;          // threads per workgroup
constexpr int kCellsPerThread = 1;   // cells per lane (the streamed step accesses are per cell)
constexpr int kPrefetchFast = 2;     // time steps of forcing the fast engine requests ahead (HISTORY.md section 5)
constexpr int kWaves = kBlock / 64;
constexpr int kNumForc = 5;   // P, T_air, Hum_sp, P_air, uz  (device frame layout)
constexpr int kNumState = 8;  // h_swe, h_iwe, Eccs, Ecci, n, albedo (fp32 in the fp32 engine), h_snow, h_ice
constexpr int kNumHist = 6;   // h_snow, SM, h_ice, IM, M_total, RH
enum { S_HSWE = 0, S_HIWE, S_ECCS, S_ECCI, S_N, S_ALB, S_HSNOW, S_HICE };
enum { F_P = 0, F_T, F_Q, F_PA, F_UZ };
enum { H_HSNOW = 0, H_SM, H_HICE, H_IM, H_MTOT, H_RH };

// Scalars of a launch (kernarg).  The buffers are separate __restrict__
// kernel parameters: that lets the compiler keep the per-step uniforms in
// scalar registers (s_load) and never order a forcing load behind an output
// store.
struct KArgs {
  DevParams p;
  int K;
  int n_catch;
  int64_t n, n_pad;
  // tfg_update (K == 1): the step's forcing [kNumForc][n_pad] (engine type)
  // is read from io_in, a device-mapped pinned host block, and also written to
  // its frame; the eight BMI outputs go to io_out [8][n] fp64 in the same block.
  // Null for every other launch.
  const void* io_in;
  double* io_out;
  uint32_t* io_flag;  // [gridDim] in the same block: io_seq once a workgroup is done
  uint32_t io_seq;
  // The cells a k_fused launch steps: n_pad, or one part of a split launch
  // (tfg_engine.hip launch_steps: a small grid as two parts on two streams,
  // the second part's buffers offset by its first cell, part_c0).  Two planes
  // are read through a pointer of another width than their buffer's (the fp64
  // geometry planes after the fp32 ones, the fp32 albedo in an fp64 state
  // plane): the kernel corrects those by part_c0.
  int64_t n_step = 0;
  int64_t part_c0 = 0;
};

// TFG_STEP_PARAMS(p): inside a step loop, `p` names the launch's model
// constants (KArgs::p, at offset 0 of the kernel-argument segment) through a
// pointer an empty asm re-defines every step.  The compiler then re-issues
// them as scalar loads (scalar cache hits) each step instead of holding them
// for the whole launch, which spills them to VGPR lanes and reads each back
// with a v_readlane (a VALU instruction) at every use.
static_assert(offsetof(KArgs, p) == 0, "KArgs::p is read at the start of the kernel-argument segment");
#define TFG_STEP_PARAMS(p)                                                                                  \
  auto p##_ks = (const __attribute__((address_space(4))) DevParams*)__builtin_amdgcn_kernarg_segment_ptr(); \
  asm volatile("" : "+s"(p##_ks));                                                                          \
  const DevParams& p = *(const DevParams*)p##_ks

// Vector load/store of C adjacent cells (C*sizeof(T) <= 16 B per lane).
template <class T, int C> struct alignas(C * sizeof(T)) Pack { T v[C]; };

// Every access is (wave-uniform 64-bit field base) + (32-bit per-lane byte
// offset): the global_load/store "saddr" form, one offset VGPR per element
// size instead of a 64-bit address per field (tfg_create keeps n_pad*8 < 2^32).
//
// lane_off re-materialises the 32-bit lane offset at each use (empty asm), so
// instruction selection, which works per basic block, sees base + zext(off)
// and picks the saddr form instead of a per-lane 64-bit add.
__device__ __forceinline__ uint32_t lane_off(uint32_t off) {
  asm volatile("" : "+v"(off));
  return off;
}
template <class T, int C>
__device__ __forceinline__ void vload(const T* __restrict__ base, uint32_t i, T (&v)[C]) {
  const uint32_t off = lane_off(i * (uint32_t)sizeof(T));
  const Pack<T, C> x = *reinterpret_cast<const Pack<T, C>*>(reinterpret_cast<const char*>(base) + off);
#pragma unroll
  for (int j = 0; j < C; ++j) v[j] = x.v[j];
}
template <class T, int C>
__device__ __forceinline__ void vstore(T* __restrict__ base, uint32_t i, const T (&v)[C]) {
  const uint32_t off = lane_off(i * (uint32_t)sizeof(T));
  Pack<T, C> x;
#pragma unroll
  for (int j = 0; j < C; ++j) x.v[j] = v[j];
  *reinterpret_cast<Pack<T, C>*>(reinterpret_cast<char*>(base) + off) = x;
}
// Streamed accesses of the step loop: forcing frames and window slots are read
// once per step and history outputs written once, with far more traffic than
// the caches hold before any reuse.  Stores are non-temporal; non-temporal
// loads measured no better (HISTORY.md section 5).  `off` is the lane's byte
// offset, materialised once per basic block by the caller (lane_off), shared
// by every access of that block.
template <class T>
__device__ __forceinline__ T sload(const T* __restrict__ base, uint32_t off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
}
template <class T>
__device__ __forceinline__ void sstore(T* __restrict__ base, uint32_t off, T v) {
  __builtin_nontemporal_store(v, reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off));
}
template <int C> __device__ __forceinline__ void dload(const double* p, uint32_t i, double (&v)[C]) { vload<double, C>(p, i, v); }
template <int C> __device__ __forceinline__ void dstore(double* p, uint32_t i, const double (&v)[C]) { vstore<double, C>(p, i, v); }
template <int C> __device__ __forceinline__ void iload(const int32_t* p, uint32_t i, int32_t (&v)[C]) { vload<int32_t, C>(p, i, v); }
template <int C> __device__ __forceinline__ void istore(int32_t* p, uint32_t i, const int32_t (&v)[C]) { vstore<int32_t, C>(p, i, v); }
template <int C> __device__ __forceinline__ void lload(const int64_t* p, uint32_t i, int64_t (&v)[C]) { vload<int64_t, C>(p, i, v); }
template <int C> __device__ __forceinline__ void lstore(int64_t* p, uint32_t i, const int64_t (&v)[C]) { vstore<int64_t, C>(p, i, v); }

// the fp64 step's unscaled sums (cell_step_exact, melt_and_mass<true>) times the
// constant factors of :567, :585-623 (da dt) and :1486, :1493 (da dt 3600)
__device__ __forceinline__ void diag_scale(CellDiag& d, const DevParams& p) {
  const double f = p.da_m2 * p.dt, f3600 = p.da_m2 * p.dt * 3600.0;
  d.P *= f;
  d.PR *= f;
  d.PS *= f;
  d.SM *= f3600;
  d.IM *= f3600;
}
__device__ __forceinline__ void diag_zero(CellDiag& d) {
  d.P = d.PR = d.PS = d.SM = d.IM = 0.0;
  d.Pmax = -INFINITY;
}

// Fold the lanes' partial sums into this wave's LDS bins, one pass per
// distinct catchment id present in the wave (normally one).  All 64 lanes
// must be active.  Fixed butterfly order -> deterministic.
__device__ __forceinline__ void wave_flush(double* __restrict__ wbins, int cid, const CellDiag& d, bool has) {
  const int lane = threadIdx.x & 63;
  uint64_t pending = __ballot(has);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const int c = __shfl(cid, leader);
    const bool mine = has && (cid == c);
    double v0 = mine ? d.P : 0.0, v1 = mine ? d.PR : 0.0, v2 = mine ? d.PS : 0.0;
    double v3 = mine ? d.SM : 0.0, v4 = mine ? d.IM : 0.0, m = mine ? d.Pmax : -INFINITY;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      v0 += __shfl_xor(v0, off);
      v1 += __shfl_xor(v1, off);
      v2 += __shfl_xor(v2, off);
      v3 += __shfl_xor(v3, off);
      v4 += __shfl_xor(v4, off);
      m = tfg::npmax(m, __shfl_xor(m, off));
    }
    if (lane == leader) {
      double* b = wbins + 6 * c;
      b[0] += v0; b[1] += v1; b[2] += v2; b[3] += v3; b[4] += v4;
      b[5] = tfg::npmax(b[5], m);
    }
    pending &= ~__ballot(mine);
  }
}

#ifdef TFG_WG_TIMING  // diagnostic builds (tests/diagnostics/wg_timeline.py): for the first
                      // TFG_WG_TIMING workgroups of every k_fused launch, the wall clock
                      // (100 MHz) at start and end and the XCC / CU it ran on
static __device__ unsigned long long g_wg_times[TFG_WG_TIMING][3];
#endif
constexpr int kMinWaves = 4;       // __launch_bounds__ minimum waves per SIMD: fp32 engine, <= 128 VGPRs
constexpr int kMinWavesExact = 2;  // fp64 engine: 256 VGPRs, no scratch spills
// the fp64-flux form: 4 waves per SIMD, spilling 12 VGPRs; 3 waves without spills ran 2.5 % slower (round 6)
constexpr int kMinWavesPrec = 4;
// NS (fast engine only): the NaN-safe form of the step (tfg::cell_step_fast),
// for launches the host could not verify to read only finite values.  PREC
// (fast engine only): the fp64 flux form (tfg_set_flux(TFG_FLUX_F64)).
template <class R, bool EXACT, bool READ_DEPTHS, bool CATCH, bool QC, int C, bool NS = false, bool PREC = false>
__global__ __launch_bounds__(kBlock, EXACT ? kMinWavesExact : (PREC ? kMinWavesPrec : kMinWaves)) void k_fused(const KArgs a, const tfg_uniforms* __restrict__ uni,
                                                  const R* __restrict__ forc,      // [n_frames][5][n_pad]
                                                  const R* __restrict__ stat,      // [3][n_pad]
                                                  const float* __restrict__ geo,   // [kGeoF][n_pad] f32 + [2][n_pad] f64
                                                  const int32_t* __restrict__ catch_id,  // [n_pad] | null
                                                  double* __restrict__ st,         // [8][n_pad]
                                                  int64_t* __restrict__ tot,       // [n_pad]
                                                  int32_t* __restrict__ ring,      // [ring_len][n_pad]
                                                  R* __restrict__ hist,            // [hist_depth][6][n_pad]
                                                  double* __restrict__ slab,       // [gridDim][n_catch][6]
                                                  const R* __restrict__ qcf) {     // [n_pad] Qc [W m-2] (QC) | null
  extern __shared__ double lds_bins[];  // [kWaves][n_catch][6]
#ifdef TFG_WG_TIMING
  const unsigned long long t_wg0 = wall_clock64();
#endif
  const DevParams& p = a.p;
  const int nb = a.n_catch * 6;
  for (int i = threadIdx.x; i < kWaves * nb; i += kBlock) lds_bins[i] = ((i % 6) == 5) ? -INFINITY : 0.0;
  __syncthreads();
  double* wbins = lds_bins + (threadIdx.x >> 6) * nb;

  const int64_t n_pad = a.n_pad;
  // the whole plane stride, the skew's padding cells included (stepping only the cells
  // measured neutral: -0.5 % at 8192^2, +0.6 % at 1024^2, profiles/r4d_ab_skew.json),
  // or one part of a split launch
  const int64_t ngroups = a.n_step / C;
  // Workgroups own whole, aligned chunks of kBlock cell groups, for any grid
  // size: every trip is one full, 64-cell-aligned wave per lane group (a
  // partition in single cells leaves misaligned ranges and a ragged last trip).
  const int64_t nchunks = (ngroups + kBlock - 1) / kBlock;
  const int64_t wg = blockIdx.x;
  const int64_t g0 = (wg * nchunks / gridDim.x) * kBlock;
  const int64_t g1 = std::min<int64_t>(((wg + 1) * nchunks / gridDim.x) * kBlock, ngroups);
  const int64_t trips = (g1 - g0 + kBlock - 1) / kBlock;
  // the pointer arithmetic of a part's float geo moved these by part_c0 / 2 doubles, not part_c0
  const double* geo_d = reinterpret_cast<const double*>(geo + tfg::kGeoF * n_pad) + a.part_c0 / 2;
  // and a part's double st moved the fp32 albedo plane by 2 part_c0 floats, not part_c0
  float* const alb_f = reinterpret_cast<float*>(st + S_ALB * n_pad) - a.part_c0;

  CellDiag acc;
  diag_zero(acc);

  for (int64_t it = 0; it < trips; ++it) {
    const int64_t g = g0 + it * kBlock + threadIdx.x;
    const bool in = g < g1;
    int32_t cid[C];
    CellDiag cacc[CATCH ? C : 1];
    if constexpr (CATCH) {
#pragma unroll
      for (int j = 0; j < C; ++j) { diag_zero(cacc[j]); cid[j] = 0; }
    }
    if (in) {
      const int64_t c0 = g * C;
      const uint32_t lc = (uint32_t)c0;  // element index within every field
      if constexpr (CATCH) iload<C>(catch_id, lc, cid);
      // static geometry: the planes k_prepare_static (exact engine, fp64 in
      // reference op order) or k_prepare_geo (fast engine) wrote
      CellStatic SX[EXACT ? C : 1];
      tfg::CellStaticF SF[EXACT ? 1 : C];
      if constexpr (EXACT) {
        const double* gx = reinterpret_cast<const double*>(geo);
        double v[tfg::kStaticPlanes][C];
#pragma unroll
        for (int f = 0; f < tfg::kStaticPlanes; ++f) dload<C>(gx + f * n_pad, lc, v[f]);
#pragma unroll
        for (int j = 0; j < C; ++j) SX[j] = {v[0][j], v[1][j], v[2][j], v[3][j], v[4][j], v[5][j], v[6][j]};
      } else {
        float gv[tfg::kGeoF][C];
#pragma unroll
        for (int f = 0; f < tfg::kGeoF; ++f) vload<float, C>(geo + f * n_pad, lc, gv[f]);
#pragma unroll
        for (int j = 0; j < C; ++j) SF[j] = {gv[0][j], gv[1][j], gv[2][j], gv[3][j], gv[4][j]};
      }
      // state
      CellState cs[C];
      {
        double v[C];
        dload<C>(st + S_HSWE * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) cs[j].h_swe = v[j];
        dload<C>(st + S_HIWE * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) cs[j].h_iwe = v[j];
        dload<C>(st + S_ECCS * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) cs[j].Eccs = v[j];
        dload<C>(st + S_ECCI * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) cs[j].Ecci = v[j];
        dload<C>(st + S_N * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) cs[j].n = v[j];
        if constexpr (EXACT) {
          dload<C>(st + S_ALB * n_pad, lc, v);
#pragma unroll
          for (int j = 0; j < C; ++j) cs[j].albedo = v[j];
        }
        if constexpr (READ_DEPTHS) {
          dload<C>(st + S_HSNOW * n_pad, lc, v);
#pragma unroll
          for (int j = 0; j < C; ++j) cs[j].h_snow = v[j];
          dload<C>(st + S_HICE * n_pad, lc, v);
#pragma unroll
          for (int j = 0; j < C; ++j) cs[j].h_ice = v[j];
        } else {
#pragma unroll
          for (int j = 0; j < C; ++j) {
            cs[j].h_snow = cs[j].h_swe * p.ws;  // :1711, bit-identical to the last step
            cs[j].h_ice = cs[j].h_iwe * p.wi;   // :1726
          }
        }
        int64_t t[C];
        lload<C>(tot, lc, t);
#pragma unroll
        for (int j = 0; j < C; ++j) cs[j].tot_q = t[j];
        if constexpr (!EXACT) {
          // The fp32 engine's albedo plane holds fp32 (round 6).  Albedo is
          // rebuilt every step from n and the previous depths (:1041-1059);
          // the stored value carries over only where those depths leave it
          // (a NaN or negative snow depth, or no snow over a NaN or negative
          // ice depth), so it is read only in a wave with such a lane: with
          // the model's own depths the plane is written, never read.
          bool carried = false;
#pragma unroll
          for (int j = 0; j < C; ++j) {
            cs[j].albedo = 0.0;
            carried |= !(cs[j].h_snow > 0.0 || (cs[j].h_snow == 0.0 && (cs[j].h_ice > 0.0 || cs[j].h_ice == 0.0)));
          }
          if (__any(carried)) {
            float fa[C];
            vload<float, C>(alb_f, lc, fa);
#pragma unroll
            for (int j = 0; j < C; ++j) cs[j].albedo = (double)fa[j];
          }
        }
      }
      // optional lateral conduction flux, held for the launch (tfg_conduction.hpp)
      R qc[C];
      if constexpr (QC) vload<R, C>(qcf, lc, qc);
      else {
#pragma unroll
        for (int j = 0; j < C; ++j) qc[j] = (R)0;
      }
      // fast engine: fp32 partial sums of this cell over the launch's steps
      tfg::DiagF df[EXACT ? 1 : C];
      if constexpr (!EXACT) {
#pragma unroll
        for (int j = 0; j < C; ++j) df[j] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      }

      // Software pipeline over the fused steps: the forcing frame and the
      // expiring window slot of step k+1 are requested before step k is
      // computed, so their HBM latency overlaps this step's arithmetic.  Two
      // register sets alternate (loop unrolled by two) so no copy has to wait
      // for a load in flight, and every request is unconditional (the last
      // step re-requests its own frame) so the compiler can count loads in
      // flight instead of draining them at a join.  A one-slot window
      // (ring_len == 1) runs unfused (tfg_step): its slot read would otherwise
      // precede the write of the step before.
      struct Frame { R P[C], T[C], Q[C], PA[C], UZ[C]; int32_t q[C]; };
      auto fetch = [&](int k, Frame& f) {
        const tfg_uniforms* un = uni + (k < a.K ? k : a.K - 1);
        const R* __restrict__ fr =
            a.io_in ? static_cast<const R*>(a.io_in) : forc + (int64_t)un->frame * kNumForc * n_pad;
        static_assert(C == 1, "streamed step accesses are per cell");
        static_assert(sizeof(R) == 4 || sizeof(R) == 8, "R is float or double");
        const uint32_t oR = lane_off(lc * (uint32_t)sizeof(R));
        f.P[0] = sload(fr + F_P * n_pad, oR);
        f.T[0] = sload(fr + F_T * n_pad, oR);
        f.Q[0] = sload(fr + F_Q * n_pad, oR);
        f.PA[0] = sload(fr + F_PA * n_pad, oR);
        f.UZ[0] = sload(fr + F_UZ * n_pad, oR);
        f.q[0] = sload(ring + (int64_t)un->slot * n_pad, sizeof(R) == 4 ? oR : lane_off(lc * 4u));
      };
      auto advance = [&](int k, const Frame& f) {
        // SGPR spills 62 -> 56 (fp32) and 170 -> 111 (fp64); same-box A/B:
        // fp32 -0.6 % and fp64 -3.4 % time per launch (HISTORY.md section 5).
        TFG_STEP_PARAMS(p);
        const tfg_uniforms* up = uni + k;
        const tfg_uniforms u = *up;
        int32_t qn[C];
        R o_hs[C], o_sm[C], o_hi[C], o_im[C], o_mt[C], o_rh[C];
#pragma unroll
        for (int j = 0; j < C; ++j) {
          if constexpr (EXACT) {
            CellOut o;
            CellDiag& d = CATCH ? cacc[j] : acc;
            const bool valid = (c0 + j) < a.n;
            const tfg::ParamsAsIs params{p};
            tfg::cell_step_exact<QC>(p, SX[j], u, (double)f.P[j], (double)f.T[j], (double)f.Q[j], (double)f.PA[j],
                                     (double)f.UZ[j], f.q[j], qn[j], cs[j], o, d, valid, (double)qc[j], params);
            o_hs[j] = (R)o.h_snow; o_sm[j] = (R)o.SM; o_hi[j] = (R)o.h_ice;
            o_im[j] = (R)o.IM; o_mt[j] = (R)o.M_total; o_rh[j] = (R)o.RH;
          } else {
            tfg::CellOutF o;
            tfg::cell_step_fast<QC, NS, PREC>(p, SF[j], up, u, geo_d, n_pad, c0 + j, (float)f.P[j], (float)f.T[j],
                                        (float)f.Q[j], (float)f.PA[j], (float)f.UZ[j], f.q[j], qn[j], cs[j], o, df[j],
                                        (float)qc[j]);
            o_hs[j] = (R)o.h_snow; o_sm[j] = (R)o.SM; o_hi[j] = (R)o.h_ice;
            o_im[j] = (R)o.IM; o_mt[j] = (R)o.M_total; o_rh[j] = (R)o.RH;
          }
        }
        const uint32_t oR = lane_off(lc * (uint32_t)sizeof(R));
        sstore(ring + (int64_t)u.slot * n_pad, sizeof(R) == 4 ? oR : lane_off(lc * 4u), qn[0]);
        R* __restrict__ h = hist + (int64_t)u.hist * kNumHist * n_pad;
        sstore(h + H_HSNOW * n_pad, oR, o_hs[0]);
        sstore(h + H_SM * n_pad, oR, o_sm[0]);
        sstore(h + H_HICE * n_pad, oR, o_hi[0]);
        sstore(h + H_IM * n_pad, oR, o_im[0]);
        sstore(h + H_MTOT * n_pad, oR, o_mt[0]);
        sstore(h + H_RH * n_pad, oR, o_rh[0]);
      };
      // The fast engine requests two steps ahead (three register sets, loop
      // unrolled by three, 127 VGPRs): +1.2-2.6 % at 1024^2, 2048^2 and 8192^2
      // in same-box A/Bs against one step ahead, and three steps ahead measured
      // no better (HISTORY.md section 5).  Step
      // k + 2's window slot is then read before steps k and k + 1 write theirs,
      // so a fused launch needs ring_len > 2 (launch_steps runs shorter windows
      // one step per launch).  The conduction (QC) and NaN-safe (NS) forms keep
      // one step ahead: with two they spill 2-4 VGPRs.
      constexpr int kAhead = (QC || NS || PREC) ? 1 : kPrefetchFast;
      Frame fa, fb;
      fetch(0, fa);
      if constexpr (EXACT) {
        // the fp64 step is issue-bound and register-heavy: one copy of its
        // body (not two interleaved) keeps it within 256 VGPRs
        for (int k = 0; k < a.K; ++k) {
          fetch(k + 1, fb);
          advance(k, fa);
          fa = fb;
        }
      } else if constexpr (kAhead == 2) {
        Frame fc;
        fetch(1, fb);
        for (int k = 0; k < a.K; k += 3) {
          fetch(k + 2, fc);
          advance(k, fa);
          fetch(k + 3, fa);
          if (k + 1 < a.K) advance(k + 1, fb);
          fetch(k + 4, fb);
          if (k + 2 < a.K) advance(k + 2, fc);
        }
      } else {
        for (int k = 0; k < a.K; k += 2) {
          fetch(k + 1, fb);
          advance(k, fa);
          fetch(k + 2, fa);
          if (k + 1 < a.K) advance(k + 1, fb);
        }
      }
      if (a.io_in) {  // tfg_update: the frame keeps the inputs, outputs go to the host block
        const int fidx = uni[0].frame, hidx = uni[0].hist;
        R* __restrict__ fr = const_cast<R*>(forc) + (int64_t)fidx * kNumForc * n_pad;
        const uint32_t oR = lane_off(lc * (uint32_t)sizeof(R));
        sstore(fr + F_P * n_pad, oR, fa.P[0]);
        sstore(fr + F_T * n_pad, oR, fa.T[0]);
        sstore(fr + F_Q * n_pad, oR, fa.Q[0]);
        sstore(fr + F_PA * n_pad, oR, fa.PA[0]);
        sstore(fr + F_UZ * n_pad, oR, fa.UZ[0]);
        if (c0 < a.n) {
          const R* hs = hist + (int64_t)hidx * kNumHist * n_pad + c0;
          double* o = a.io_out + c0;
          const int64_t n = a.n;
          o[0 * n] = (double)hs[H_HSNOW * n_pad];
          o[1 * n] = cs[0].h_swe;
          o[2 * n] = (double)hs[H_SM * n_pad];
          o[3 * n] = (double)hs[H_HICE * n_pad];
          o[4 * n] = cs[0].h_iwe;
          o[5 * n] = (double)hs[H_IM * n_pad];
          o[6 * n] = (double)hs[H_MTOT * n_pad];
          o[7 * n] = (double)hs[H_RH * n_pad];
        }
      }
      // fast engine: fold the cell's partial sums into the fp64 accumulators
      // with the constant factors of :567, :585-623, :1486, :1493 (padding
      // cells excluded)
      if constexpr (!EXACT) {
        const double fP = p.da_m2 * p.dt, fSM = p.inv_dt_rhoLf * p.da_m2 * p.dt * 3600.0,
                     fIM = p.da_m2 * p.dt * 3600.0;
#pragma unroll
        for (int j = 0; j < C; ++j) {
          if ((c0 + j) < a.n) {
            CellDiag& d = CATCH ? cacc[j] : acc;
            d.P += (double)df[j].P * fP;
            d.PR += (double)df[j].PR * fP;
            d.PS += (double)df[j].PS * fP;
            d.SM += (double)df[j].Erem_s * fSM;
            d.IM += (double)df[j].IM * fIM;
            d.Pmax = tfg::npmax(d.Pmax, (double)df[j].Pmax);
          }
        }
      }
      // write back state
      {
        double v[C];
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] = cs[j].h_swe;
        dstore<C>(st + S_HSWE * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] = cs[j].h_iwe;
        dstore<C>(st + S_HIWE * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] = cs[j].Eccs;
        dstore<C>(st + S_ECCS * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] = cs[j].Ecci;
        dstore<C>(st + S_ECCI * n_pad, lc, v);
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] = cs[j].n;
        dstore<C>(st + S_N * n_pad, lc, v);
        if constexpr (EXACT) {
#pragma unroll
          for (int j = 0; j < C; ++j) v[j] = cs[j].albedo;
          dstore<C>(st + S_ALB * n_pad, lc, v);
        } else {  // fp32 (the step computes it in fp32)
          float fa[C];
#pragma unroll
          for (int j = 0; j < C; ++j) fa[j] = (float)cs[j].albedo;
          vstore<float, C>(alb_f, lc, fa);
        }
        int64_t t[C];
#pragma unroll
        for (int j = 0; j < C; ++j) t[j] = cs[j].tot_q;
        lstore<C>(tot, lc, t);
      }
    }
    if constexpr (CATCH) {
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if constexpr (EXACT) diag_scale(cacc[j], p);
        wave_flush(wbins, cid[j], cacc[j], in);
      }
    }
  }
  if constexpr (EXACT && !CATCH) diag_scale(acc, p);
  if constexpr (!CATCH) wave_flush(wbins, 0, acc, true);
  __syncthreads();
  // each workgroup accumulates into its own slab row across launches (fixed
  // order, deterministic); tfg_get_diag folds the rows when it is called
  double* bslab = slab + (int64_t)blockIdx.x * nb;
  for (int i = threadIdx.x; i < nb; i += kBlock) {
    double v = lds_bins[i];
    if ((i % 6) == 5) {
      for (int w = 1; w < kWaves; ++w) v = tfg::npmax(v, lds_bins[w * nb + i]);
      bslab[i] = tfg::npmax(bslab[i], v);
    } else {
      for (int w = 1; w < kWaves; ++w) v += lds_bins[w * nb + i];
      bslab[i] += v;
    }
  }
#ifdef TFG_WG_TIMING
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < TFG_WG_TIMING) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID[3:0]
    g_wg_times[blockIdx.x][0] = t_wg0;
    g_wg_times[blockIdx.x][1] = wall_clock64();
    g_wg_times[blockIdx.x][2] = ((unsigned long long)xcc << 32) | (unsigned)__smid();
  }
#endif
  if (a.io_flag) {  // tfg_update: tell the waiting host this workgroup is done
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(a.io_flag + blockIdx.x, a.io_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The buffers of one k_fused launch (tfg_handle's planes; R = the engine type).
struct FusedBufs {
  const tfg_uniforms* uni;
  const void* forc;
  const void* stat;
  const float* geo;
  const int32_t* catch_id;
  double* st;
  int64_t* tot;
  int32_t* ring;
  void* hist;
  double* slab;
  const void* qc;
};

// The fp64 engine's k_fused launch (tfg_fused_f64.hip): the instantiation for
// (read_depths, catchments, qc_on) on `stream`.
hipError_t launch_fused_exact(const KArgs& a, const FusedBufs& b, bool read_depths, bool catchments, bool qc_on,
                              int blocks, size_t lds, hipStream_t stream);
// The fp32 engine's fp64-flux form (tfg_fused_prec.hip): the instantiation for
// (read_depths, catchments, qc_on, nan_safe) on `stream`.
hipError_t launch_fused_prec(const KArgs& a, const FusedBufs& b, bool read_depths, bool catchments, bool qc_on,
                             bool nan_safe, int blocks, size_t lds, hipStream_t stream);

}  // namespace tfg_kern
