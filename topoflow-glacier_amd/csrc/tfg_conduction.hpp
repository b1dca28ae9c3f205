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
// west, east) and the ice faces, in that order, in fp64.  The two cells of a
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
// temperature derivation.
struct CondGrid {
  const double* swe;   // h_swe  [n]
  const double* iwe;   // h_iwe  [n]
  const double* eccs;  // Eccs   [n]
  const double* ecci;  // Ecci   [n]
  const double* hn;    // north halo [4][nx] (T_snow, h_snow, T_ice, h_ice) or null
  const double* hs;    // south halo [4][nx] or null
  int64_t ny, nx;
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
};

// A cell as its neighbours see it; an absent neighbour has no snow and no ice.
struct CondCell {
  double Ts, hs, Ti, hi;
};

__device__ __forceinline__ CondCell cond_cell(const CondGrid& g, int64_t i) {
#pragma clang fp contract(off)
  CondCell c;
  c.hs = g.swe[i] * g.ws;  // :1711
  c.hi = g.iwe[i] * g.wi;  // :1726
  c.Ts = c.hs > 0.0 ? g.T0 - (g.eccs[i] * g.inv_cs) / c.hs : g.T0;
  c.Ti = c.hi > 0.0 ? g.T0 - g.ecci[i] * g.inv_ci : g.T0;
  return c;
}

__device__ __forceinline__ CondCell cond_halo(const double* row, int64_t nx, int64_t c) {
  return {row[c], row[nx + c], row[2 * nx + c], row[3 * nx + c]};
}

__device__ __forceinline__ CondCell cond_none() { return {0.0, 0.0, 0.0, 0.0}; }

// One face's contribution from neighbour n to cell m (snow and ice sums).
__device__ __forceinline__ void cond_face(const CondCell& m, const CondCell& n, double gs, double gi, double& qs,
                                          double& qi) {
#pragma clang fp contract(off)
  if (m.hs > 0.0 && n.hs > 0.0) qs += (fmin(m.hs, n.hs) * (n.Ts - m.Ts)) * gs;
  if (m.hi > 0.0 && n.hi > 0.0) qi += (n.Ti - m.Ti) * gi;
}

constexpr int kCondTX = 256, kCondRows = 32;

// Qc of a row-block shard.  Workgroup tiles of kCondTX columns x kCondRows
// rows; each thread walks down its column with the rows above and below in
// registers (one new row of state per row walked) and reads its west/east
// neighbours from the same cache lines its neighbours load.  Tiles are dealt
// XCD-aware (the ice-flow order, tfg_flow.hpp): XCD k takes the k-th eighth
// of the tiles in row-major order, so vertically adjacent strips share an L2.
template <class R>
__global__ __launch_bounds__(kCondTX) void k_conduction(const CondGrid g, const CondK K, R* __restrict__ qc,
                                                         int gx, int strips, int per_xcd) {
#pragma clang fp contract(off)
  const int64_t tile = (int64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  if (tile >= (int64_t)gx * strips) return;
  const int64_t tx = tile % gx, ty = tile / gx;
  const int64_t c = tx * kCondTX + threadIdx.x;
  if (c >= g.nx) return;  // no barriers below
  const int64_t r0 = ty * kCondRows;
  const int64_t r1 = r0 + kCondRows < g.ny ? r0 + kCondRows : g.ny;
  const int64_t nx = g.nx;
  CondCell up = r0 > 0 ? cond_cell(g, (r0 - 1) * nx + c) : (g.hn ? cond_halo(g.hn, nx, c) : cond_none());
  CondCell cur = cond_cell(g, r0 * nx + c);
  for (int64_t r = r0; r < r1; ++r) {
    const CondCell dn = r + 1 < g.ny ? cond_cell(g, (r + 1) * nx + c) : (g.hs ? cond_halo(g.hs, nx, c) : cond_none());
    const CondCell w = c > 0 ? cond_cell(g, r * nx + c - 1) : cond_none();
    const CondCell e = c + 1 < nx ? cond_cell(g, r * nx + c + 1) : cond_none();
    double qs = 0.0, qi = 0.0;
    cond_face(cur, up, K.gsy, K.giy, qs, qi);
    cond_face(cur, dn, K.gsy, K.giy, qs, qi);
    cond_face(cur, w, K.gsx, K.gix, qs, qi);
    cond_face(cur, e, K.gsx, K.gix, qs, qi);
    qc[r * nx + c] = (R)(qs + qi);
    up = cur;
    cur = dn;
  }
}

// This shard's first and last rows as its neighbours' halo rows, [4][nx] each.
__global__ void k_conduction_edges(const CondGrid g, double* __restrict__ first, double* __restrict__ last) {
  const int64_t nx = g.nx;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nx; c += (int64_t)gridDim.x * blockDim.x) {
    const CondCell a = cond_cell(g, c), b = cond_cell(g, (g.ny - 1) * nx + c);
    first[c] = a.Ts; first[nx + c] = a.hs; first[2 * nx + c] = a.Ti; first[3 * nx + c] = a.hi;
    last[c] = b.Ts; last[nx + c] = b.hs; last[2 * nx + c] = b.Ti; last[3 * nx + c] = b.hi;
  }
}

}  // namespace tfg
