// tfg_flow.hpp -- the optional lateral ice-flow term, device side (gfx950).
//
// Included by tfg_engine.hip after the state-plane layout (S_HIWE, S_HICE);
// the C ABI entry points (tfg_ice_flow_edges / _dmax / _step / _run) live there.
#pragma once

// ---------------------------------------------------------------------------
// Optional lateral ice flow (tfg_ice_flow_*): shallow-ice approximation,
// Glen's law n = 3, explicit flux form on cell faces, fp64, contraction off so
// the face flux two neighbours compute is the same number (exact
// conservation, and sharded == unsharded bit for bit).  The reference declares
// the parameters (glens_A, config.py:64-65) but moves no ice (:936-955).
//   H = h_iwe * wi (ice thickness), s = elev + H (elev is the bed)
//   q = -Gamma * Hf^5 * (gn^2 + gt^2) * gn on a face with normal gradient gn,
//   tangential gradient gt (mean of the two cells' centred differences) and
//   face thickness Hf = (Ha + Hb)/2, limited to |q| <= H_donor * dn / (4 dt).
// Rows outside the shard come from the halo [2][nx] (s, H) when present,
// otherwise the edge row is replicated (domain edge: no face, zero flux).
struct FlowGrid {
  const void* elev;            // R[n_pad]
  const double* iwe;           // st + S_HIWE * n_pad
  const double* hn;            // north halo [2][nx] or null
  const double* hs;            // south halo [2][nx] or null
  int64_t ny, nx;
  double wi;
};
template <class R>
__device__ __forceinline__ double flow_H(const FlowGrid& g, int64_t r, int64_t c) {
  if (r < 0) return g.hn[g.nx + c];
  if (r >= g.ny) return g.hs[g.nx + c];
  return g.iwe[r * g.nx + c] * g.wi;
}
template <class R>
__device__ __forceinline__ double flow_S(const FlowGrid& g, int64_t r, int64_t c) {
#pragma clang fp contract(off)
  c = c < 0 ? 0 : (c >= g.nx ? g.nx - 1 : c);
  if (r < 0) { if (g.hn) return g.hn[c]; r = 0; }
  if (r >= g.ny) { if (g.hs) return g.hs[c]; r = g.ny - 1; }
  const int64_t i = r * g.nx + c;
  return (double)static_cast<const R*>(g.elev)[i] + g.iwe[i] * g.wi;
}
__device__ __forceinline__ double flow_face_D(double Ha, double Hb, double gn, double gt, double gamma) {
#pragma clang fp contract(off)
  const double Hf = 0.5 * (Ha + Hb);
  const double h2 = Hf * Hf;
  const double h5 = (h2 * h2) * Hf;
  return (gamma * h5) * (gn * gn + gt * gt);
}
// lim = dn / (4 dt): a face passes at most a quarter of the donor's ice
__device__ __forceinline__ double flow_face_q(double Ha, double Hb, double gn, double gt, double gamma, double lim) {
#pragma clang fp contract(off)
  double q = -(flow_face_D(Ha, Hb, gn, gt, gamma) * gn);
  const double Hd = q > 0.0 ? Ha : Hb;
  const double qlim = Hd * lim;
  return fmin(fmax(q, -qlim), qlim);
}
// Per-launch constants of a sub-step: the kernel multiplies, it never divides
// (fp64 division would make the stencil issue-bound).
struct FlowK {
  double inv_dx, inv_dy, inv_4dx, inv_4dy;  // 1/dx, 1/dy, 1/(4 dx), 1/(4 dy)
  double lim_x, lim_y;                      // dx/(4 dt), dy/(4 dt)
  double dt_wi;                             // dt / wi
  double gamma;
};
inline FlowK flow_constants(double dt, double dx, double dy, double wi, double gamma) {
  return {1.0 / dx, 1.0 / dy, 1.0 / (4.0 * dx), 1.0 / (4.0 * dy), dx / (4.0 * dt), dy / (4.0 * dt), dt / wi, gamma};
}
// One sub-step, LDS-tiled: a workgroup owns kFlowTX columns x kFlowRows rows
// and walks down its strip with a four-row ring of (s, H) in LDS (one halo
// column each side).  Each thread keeps its own column's values in registers
// and reads the two neighbouring columns from LDS once per row; it evaluates
// its west and east faces itself (the face a neighbour also evaluates comes
// from the same values in the same order, so the two agree bit for bit) and
// carries the south face in a register as the next row's north face.  Faces
// shared by two workgroups (or two shards) agree the same way (restatement:
// tests/harness.py:ice_flow_step_restated).  With four ring slots a row
// costs one workgroup barrier: the slot written in row r (row r+2) was last
// read in row r-1.
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// accesses, not for its global loads and stores (a __syncthreads() fence would
// drain them, and with them the rows prefetched into registers).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// DMAX: instead of stepping, the largest face diffusivity of the workgroup's
// faces goes to out[workgroup] (the CFL bound of tfg_ice_flow_dmax).
constexpr int kFlowTX = 256, kFlowRows = 32;  // 16 and 64 rows measured no better / slower
constexpr int kFlowWaves = 1;  // __launch_bounds__ minimum waves per SIMD (a 7-wave cap measured within 1 %)
// XCD-aware tile order.  Workgroup L of a 1-D launch runs on XCD L mod 8 (the
// dispatcher deals workgroups round-robin over the 8 XCDs, each with its own
// L2), so consecutive tiles of the row-major order would sit on different
// XCDs and every halo column would come from another XCD's L2 or from HBM.
// Instead XCD x takes the x-th eighth of the tiles, in row-major order: left
// and right neighbours share an L2 and run at about the same time, and so do
// the strips above and below (gx tiles later in the same XCD's sequence).
struct FlowTiles {
  int gx;       // tiles per strip (columns of kFlowTX)
  int strips;   // strips in this launch
  int per_xcd;  // ceil(gx * strips / 8)
};
inline FlowTiles flow_tiles(int64_t nx, int strips) {
  const int gx = (int)((nx + kFlowTX - 1) / kFlowTX);
  const int64_t tiles = (int64_t)gx * strips;
  return {gx, strips, (int)((tiles + 7) / 8)};
}
inline unsigned flow_blocks(const FlowTiles& ft) { return 8u * (unsigned)ft.per_xcd; }

template <class R, bool DMAX>
__global__ __launch_bounds__(kFlowTX, kFlowWaves) void k_ice_flow(const FlowGrid g, const FlowK K, double* __restrict__ out,
                                                      int strip0, int strip_step, double* __restrict__ out_ice,
                                                      const FlowTiles ft) {
#pragma clang fp contract(off)
  __shared__ double sS[4][kFlowTX + 2], sH[4][kFlowTX + 2];  // index k = column - (c0 - 1)
  __shared__ double red[DMAX ? kFlowTX : 1];
  const int64_t tile = (int64_t)(blockIdx.x % 8) * ft.per_xcd + blockIdx.x / 8;
  if (tile >= (int64_t)ft.gx * ft.strips) return;  // the padding of the last eighth (whole workgroup)
  const int64_t tx = tile % ft.gx, ty = tile / ft.gx;
  double dmax = 0.0;
  const int t = threadIdx.x;
  const int64_t c0 = tx * kFlowTX;
  const int64_t r0 = ((int64_t)strip0 + ty * strip_step) * kFlowRows;  // this workgroup's strip
  const int64_t r1 = r0 + kFlowRows < g.ny ? r0 + kFlowRows : g.ny;
  const int64_t c = c0 + t;
  auto slot = [&](int64_t rr) { return (int)(rr - r0 + 1) & 3; };
  // One row, as raw values: (elev, h_iwe), or (s, H) from a halo row; a
  // missing row outside the domain repeats the edge row.  Lane t holds its
  // own column (j = 0); lane 0 also holds column c0 - 1 and the other lanes
  // column c0 + kFlowTX (j = 1; put() stores those of lanes 0 and 1).
  // (elev stays in its storage type until put(): converting at fetch time
  // would wait for the load there and serialise the prefetch)
  struct Raw { double a[2], b[2]; R e[2]; bool halo; };
  auto fetch = [&](int64_t rr, Raw& v) {
    // straight-line loads (no branch, so no register merge that would wait
    // for them): a halo row reads (s, H) from the halo; an in-domain row reads
    // (elev, h_iwe), with the halo-s load pointed at the h_iwe row (a cache hit)
    v.halo = (rr < 0 && g.hn) || (rr >= g.ny && g.hs);
    const int64_t rc_ = rr < 0 ? 0 : (rr >= g.ny ? g.ny - 1 : rr);
    const double* hb = v.halo ? (rr < 0 ? g.hn : g.hs) + g.nx : g.iwe + rc_ * g.nx;
    const double* ha = v.halo ? hb - g.nx : hb;
    const R* he = static_cast<const R*>(g.elev) + rc_ * g.nx;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t cc = j == 0 ? c : (t == 0 ? c0 - 1 : c0 + kFlowTX);
      const int64_t cl = cc < 0 ? 0 : (cc >= g.nx ? g.nx - 1 : cc);
      v.e[j] = he[cl];
      v.b[j] = hb[cl];
      v.a[j] = ha[cl];
    }
  };
  // own column's (s, H, h_iwe) of the rows r-1 .. r+2, rolled once per row
  double os[4], oh[4], ow[4];
  auto put = [&](int64_t rr, const Raw& v, int q) {
    const int sl = slot(rr);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const double sv = v.halo ? v.a[j] : (double)v.e[j] + v.b[j] * g.wi;
      const double hv = v.halo ? v.b[j] : v.b[j] * g.wi;
      if (j == 0) {
        sS[sl][t + 1] = sv;
        sH[sl][t + 1] = hv;
        os[q] = sv;
        oh[q] = hv;
        ow[q] = v.b[j];  // h_iwe of an in-domain row (the only rows a workgroup updates)
      } else if (t < 2) {
        const int k = t == 0 ? 0 : kFlowTX + 1;
        sS[sl][k] = sv;
        sH[sl][k] = hv;
      }
    }
  };
  // rows r0-1 .. r0+1 into the ring, row r0+2 in flight in registers
  {
    Raw v;
    fetch(r0 - 1, v);
    put(r0 - 1, v, 0);
    fetch(r0, v);
    put(r0, v, 1);
    fetch(r0 + 1, v);  // r1 >= r0 + 1
    put(r0 + 1, v, 2);
  }
  const bool west_ok = c >= 1 && c < g.nx, east_ok = c + 1 < g.nx;
  double qN = 0.0;
  // one row: `buf` holds row r+2 (fetched earlier); it is refilled with row
  // r+ahead, in flight while this row and the next ahead-3 rows compute
  auto row = [&](int64_t r, Raw& buf, int ahead) {
    lds_barrier();  // rows r-1 .. r+1 are in the ring; row r-2's slot is free
    if (r + 2 <= r1) put(r + 2, buf, 3);
    if (r + ahead <= r1) fetch(r + ahead, buf);
    const int rm = slot(r - 1), rc = slot(r), rp = slot(r + 1);
    const double Lm = sS[rm][t], Lc = sS[rc][t], Lp = sS[rp][t], HL = sH[rc][t];
    const double Rm = sS[rm][t + 2], Rc = sS[rc][t + 2], Rp = sS[rp][t + 2], HR = sH[rc][t + 2];
    const double sm = os[0], sc = os[1], sp = os[2], hc = oh[1];
    // x-faces: west (column c-1 | c) and east (c | c+1), as (left, right)
    double qW = 0.0, qE = 0.0;
    {
      const double gnW = (sc - Lc) * K.inv_dx;
      const double gtW = ((Lp - Lm) + (sp - sm)) * K.inv_4dy;
      const double gnE = (Rc - sc) * K.inv_dx;
      const double gtE = ((sp - sm) + (Rp - Rm)) * K.inv_4dy;
      if constexpr (DMAX) {
        if (west_ok) dmax = fmax(dmax, flow_face_D(HL, hc, gnW, gtW, K.gamma));
        if (east_ok) dmax = fmax(dmax, flow_face_D(hc, HR, gnE, gtE, K.gamma));
      } else {
        if (west_ok) qW = flow_face_q(HL, hc, gnW, gtW, K.gamma, K.lim_x);
        if (east_ok) qE = flow_face_q(hc, HR, gnE, gtE, K.gamma, K.lim_x);
      }
    }
    // y-faces at column c: north (rows r-1 | r) on the strip's first row, then
    // south (r | r+1), carried to the next row as its north face
    auto face_y = [&](double sa, double sb, double ha, double hb, double La, double Ra, double Lb, double Rb) {
      const double gn = (sb - sa) * K.inv_dy;
      const double gt = ((Ra - La) + (Rb - Lb)) * K.inv_4dx;
      if constexpr (DMAX) {
        if (c < g.nx) dmax = fmax(dmax, flow_face_D(ha, hb, gn, gt, K.gamma));
        return 0.0;
      }
      return flow_face_q(ha, hb, gn, gt, K.gamma, K.lim_y);
    };
    if (r == r0) qN = (r > 0 || g.hn) ? face_y(sm, sc, oh[0], hc, Lm, Rm, Lc, Rc) : 0.0;
    const double qS = (r + 1 < g.ny || g.hs) ? face_y(sc, sp, hc, oh[2], Lc, Rc, Lp, Rp) : 0.0;
    if (!DMAX && c < g.nx) {
      const int64_t i = r * g.nx + c;
      const double div = (qE - qW) * K.inv_dx + (qS - qN) * K.inv_dy;
      const double v = fmax(ow[1] - K.dt_wi * div, 0.0);
      out[i] = v;
      if (out_ice) out_ice[i] = v * g.wi;  // writing the state plane: h_ice too (:1726)
    }
    qN = qS;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      os[q] = os[q + 1];
      oh[q] = oh[q + 1];
      ow[q] = ow[q + 1];
    }
  };
  Raw buf;  // one row in flight (two, with 5 waves per SIMD, measured 3 % slower: HISTORY.md section 6)
  if (r0 + 2 <= r1) fetch(r0 + 2, buf);
  for (int64_t r = r0; r < r1; ++r) row(r, buf, 3);
  if constexpr (DMAX) {
    red[t] = dmax;
    __syncthreads();
    for (int w = kFlowTX / 2; w > 0; w >>= 1) {
      if (t < w) red[t] = fmax(red[t], red[t + w]);
      __syncthreads();
    }
    if (t == 0) out[tile] = red[0];  // tile = ty * gx + tx
  }
}

// commit a sub-step: the new h_iwe into the state plane, and (ICE) the next
// step's previous-step ice depth h_ice = h_iwe * wi (:1726) for the state-plane
// read; without ICE the flow kernel has already written h_ice
template <bool ICE>
__global__ void k_flow_commit(double* __restrict__ st, const double* __restrict__ iwe_new, int64_t n, int64_t n_pad,
                              double wi) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = iwe_new[i];
    st[S_HIWE * n_pad + i] = v;
    if constexpr (ICE) st[S_HICE * n_pad + i] = v * wi;
  }
}

// this shard's first / last rows as halo rows [2][nx] (s, H) for its neighbours
template <class R>
__global__ void k_ice_flow_edges(const FlowGrid g, double* __restrict__ first, double* __restrict__ last) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < g.nx; c += (int64_t)gridDim.x * blockDim.x) {
    first[c] = flow_S<R>(g, 0, c);
    first[g.nx + c] = flow_H<R>(g, 0, c);
    last[c] = flow_S<R>(g, g.ny - 1, c);
    last[g.nx + c] = flow_H<R>(g, g.ny - 1, c);
  }
}
