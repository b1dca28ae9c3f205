// tfg_conduction.hpp -- optional lateral heat conduction (extension; SURVEY.md
// 8(f) row 4), device side (gfx950).
//
// The reference reserves the conduction term of the energy balance and leaves
// it at zero: update_conduction_heat_flux (bmi_topoflow_glacier.py:936-948)
// is a no-op, Qc = 0 from initialize (:312, :326), and update_net_energy_flux
// adds it last, Q_sum = Qn_SW + Qn_LW + Qh + Qe + Qa + Qc (:1314).  This file
// computes a per-cell Qc [W m-2] from Fourier's law between neighbouring
// cells (the docstring's Qc = Ks (Tx - Ts) / x, applied laterally), which
// k_fused<..., QC = true> then adds to Q_sum in the reference's position.
//
// Pack temperatures follow from the cold contents as the reference defines
// them (Eccs = rho_s Cp_s h_snow (T0 - T), :389-395; Ecci over the active
// ice layer h_active_layer):
//   T_snow = T0 - Eccs / (rho_s Cp_s h_snow)         (h_snow > 0)
//   T_ice  = T0 - Ecci / (rho_i Cp_i h_active_layer)  (h_ice  > 0)
// Face fluxes per unit cell area, for a neighbour j of cell i across a face
// of normal spacing d (dx for west/east, dy for north/south):
//   snow: k_snow * min(h_snow_i, h_snow_j) * (T_snow_j - T_snow_i) / d^2
//         when both cells hold snow;
//   ice:  k_ice * h_active_layer * (T_ice_j - T_ice_i) / d^2
//         when both cells hold ice;
// no flux across the domain edge.  Qc_i sums the snow faces (north, south,
// west, east) and the ice faces, in that order, in fp64, then adds the
// optional ground heat flux: the reference's declared but unused geothermal
// flux Qg (config.py:84, :333) in W m-2.  The two cells of a
// face evaluate the same products of the same values, so their fluxes are
// exact negatives of each other and the domain total is zero up to the
// rounding of the per-cell sums.
//
// The term is operator-split like the ice-flow term: Qc is evaluated from the
// state at the start of a conduction interval and held for its steps, so the
// fused launches keep their K-step register-resident state.  The interval is
// stable for dt_interval <= min(dx, dy)^2 / 8 * min(rho_s Cp_s / k_snow,
// rho_i Cp_i / k_ice) (checked by the config; topoflow_glacier/bmi/config.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfg {

// The state planes a conduction pass reads, and the constants of the
// temperature derivation.  h_swe, h_iwe, Eccs, Ecci are consecutive planes of
// the engine state ([8][n_pad] fp64: S_HSWE .. S_ECCI), so one base pointer
// and the plane stride n_pad address all four.
struct CondGrid {
  const double* st;    // h_swe plane; h_iwe, Eccs, Ecci follow at n_pad strides
  const double* hn;    // north halo [4][nx] (T_snow, h_snow, T_ice, h_ice) or null
  const double* hs;    // south halo [4][nx] or null
  int64_t ny, nx, n_pad;
  double ws, wi;       // rho_H2O/rho_snow, rho_H2O/rho_ice (:385-386)
  double T0;           // T0_cc (:389)
  double inv_cs;       // 1 / (rho_snow Cp_snow)
  double inv_ci;       // 1 / ((rho_ice Cp_ice) h_active_layer)
};

// Face conductances per unit cell area [W m-2 K-1] (snow ones per metre of
// the thinner snowpack).
struct CondK {
  double gsx, gsy;  // k_snow / dx^2, k_snow / dy^2
  double gix, giy;  // k_ice h_active_layer / dx^2, k_ice h_active_layer / dy^2
  double qg;        // ground (geothermal) heat flux [W m-2] added to every cell
};

// A cell as its neighbours see it; an absent neighbour has no snow and no ice.
struct CondCell {
  double Ts, hs, Ti, hi;
};

__device__ __forceinline__ CondCell cond_none() { return {0.0, 0.0, 0.0, 0.0}; }

// (T_snow, h_snow, T_ice, h_ice) from the state values h_swe, h_iwe, Eccs, Ecci.
__device__ __forceinline__ CondCell cond_from_state(const CondGrid& g, double swe, double iwe, double eccs,
                                                    double ecci) {
#pragma clang fp contract(off)
  CondCell c;
  c.hs = swe * g.ws;  // :1711
  c.hi = iwe * g.wi;  // :1726
  c.Ts = c.hs > 0.0 ? g.T0 - (eccs * g.inv_cs) / c.hs : g.T0;
  c.Ti = c.hi > 0.0 ? g.T0 - ecci * g.inv_ci : g.T0;
  return c;
}

// One row's four values at one column as loaded: state values of an
// in-domain row (kind 0), a halo row's cell values (kind 1), or nothing
// beyond the domain edge (kind 2).  The loads are straight-line, from a
// wave-uniform (base, stride) choice, so the compiler keeps them in flight
// instead of waiting at a branch; the values are interpreted only when used.
struct CondRaw {
  double v[4];
  int kind;
};

__device__ __forceinline__ CondRaw cond_fetch(const CondGrid& g, int64_t row, int64_t col) {
  const bool in = row >= 0 && row < g.ny;
  const double* halo = row < 0 ? g.hn : g.hs;
  CondRaw r;
  r.kind = in ? 0 : (halo ? 1 : 2);
  const double* base = r.kind == 0 ? g.st + row * g.nx + col : (r.kind == 1 ? halo + col : g.st + col);
  const int64_t stride = r.kind == 1 ? g.nx : g.n_pad;
#pragma unroll
  for (int k = 0; k < 4; ++k) r.v[k] = base[k * stride];
  return r;
}

__device__ __forceinline__ CondCell cond_cell(const CondGrid& g, const CondRaw& r, bool col_in) {
  if (!col_in || r.kind == 2) return cond_none();
  if (r.kind == 1) return {r.v[0], r.v[1], r.v[2], r.v[3]};
  return cond_from_state(g, r.v[0], r.v[1], r.v[2], r.v[3]);
}

// One face's contribution from neighbour n to cell m (snow and ice sums).
__device__ __forceinline__ void cond_face(const CondCell& m, const CondCell& n, double gs, double gi, double& qs,
                                          double& qi) {
#pragma clang fp contract(off)
  if (m.hs > 0.0 && n.hs > 0.0) qs += (fmin(m.hs, n.hs) * (n.Ts - m.Ts)) * gs;
  if (m.hi > 0.0 && n.hi > 0.0) qi += (n.Ti - m.Ti) * gi;
}

__device__ __forceinline__ void cond_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Tiles of kCondTX threads over kCondOut = kCondTX - 2 output columns (one
// overlapping column each side supplies the west/east neighbours) and
// kCondRows rows.
// Two rows are requested beyond the next one while a row is evaluated (one:
// 514-516 against 510 us at 8192^2, HISTORY.md section 6).
constexpr int kCondTX = 256, kCondOut = kCondTX - 2, kCondRows = 64;

// Qc of a row-block shard.  Each thread walks down one column of its tile with
// the rows above and below in registers and the row after next already in
// flight, so every state value crosses HBM once per tile (plus the two
// overlap columns and the rows just above and below the strip: 1.04 x the
// algorithmic reads at 64-row strips).  Each row's cell
// values go through a double-buffered LDS row, one barrier per row, from which
// a thread reads its west and east neighbours.  Tiles are dealt XCD-aware (the
// ice-flow order, tfg_flow.hpp): XCD k takes the k-th eighth of the tiles in
// row-major order, so vertically adjacent strips share an L2.
template <class R>
__global__ __launch_bounds__(kCondTX) void k_conduction(const CondGrid g, const CondK K, R* __restrict__ qc,
                                                         int gx, int strips, int per_xcd) {
#pragma clang fp contract(off)
  __shared__ double sC[2][4][kCondTX];
  const int64_t tile = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  if (tile >= (int64_t)gx * strips) return;  // the padding of the last eighth (whole workgroup)
  const int t = threadIdx.x;
  const int64_t tx = tile % gx, ty = tile / gx;
  const int64_t c = tx * kCondOut - 1 + t;
  const bool col_in = c >= 0 && c < g.nx;
  const int64_t cl = col_in ? c : (c < 0 ? 0 : g.nx - 1);  // a valid address for the overlap columns
  const bool writes = col_in && t >= 1 && t <= kCondTX - 2;
  const int64_t r0 = ty * kCondRows;
  const int64_t r1 = r0 + kCondRows < g.ny ? r0 + kCondRows : g.ny;
  const int tw = t > 0 ? t - 1 : 0, te = t < kCondTX - 1 ? t + 1 : t;
  CondCell up = cond_cell(g, cond_fetch(g, r0 - 1, cl), col_in);
  CondCell cur = cond_cell(g, cond_fetch(g, r0, cl), col_in);
  CondRaw nxt = cond_fetch(g, r0 + 1, cl);
  CondRaw nx2 = cond_fetch(g, r0 + 2 < r1 ? r0 + 2 : r1, cl);
  for (int64_t r = r0; r < r1; ++r) {
    const int b = (int)(r - r0) & 1;
    // rows past the strip re-read row r1 (a cache hit)
    const CondRaw ahead = cond_fetch(g, r + 3 < r1 ? r + 3 : r1, cl);
    const CondCell dn = cond_cell(g, nxt, col_in);
    sC[b][0][t] = cur.Ts;
    sC[b][1][t] = cur.hs;
    sC[b][2][t] = cur.Ti;
    sC[b][3][t] = cur.hi;
    cond_lds_barrier();  // the row is in buffer b; buffer b^1 (row r-1) is no longer read
    const CondCell w = {sC[b][0][tw], sC[b][1][tw], sC[b][2][tw], sC[b][3][tw]};
    const CondCell e = {sC[b][0][te], sC[b][1][te], sC[b][2][te], sC[b][3][te]};
    double qs = 0.0, qi = 0.0;
    cond_face(cur, up, K.gsy, K.giy, qs, qi);
    cond_face(cur, dn, K.gsy, K.giy, qs, qi);
    cond_face(cur, w, K.gsx, K.gix, qs, qi);
    cond_face(cur, e, K.gsx, K.gix, qs, qi);
    if (writes) qc[r * g.nx + c] = (R)((qs + qi) + K.qg);
    up = cur;
    cur = dn;
    nxt = nx2;
    nx2 = ahead;
  }
}

// This shard's first and last rows as its neighbours' halo rows, [4][nx] each.
__global__ void k_conduction_edges(const CondGrid g, double* __restrict__ first, double* __restrict__ last) {
  const int64_t nx = g.nx;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nx; c += (int64_t)gridDim.x * blockDim.x) {
    const CondCell a = cond_cell(g, cond_fetch(g, 0, c), true);
    const CondCell b = cond_cell(g, cond_fetch(g, g.ny - 1, c), true);
    first[c] = a.Ts; first[nx + c] = a.hs; first[2 * nx + c] = a.Ti; first[3 * nx + c] = a.hi;
    last[c] = b.Ts; last[nx + c] = b.hs; last[2 * nx + c] = b.Ti; last[3 * nx + c] = b.hi;
  }
}

}  // namespace tfg
