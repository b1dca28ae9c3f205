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
// and walks down its strip with a three-row ring of (s, H) in LDS (one halo
// column each side).  Each face flux is evaluated once per workgroup: the
// row's x-faces into LDS, the y-face below each cell in a register that
// becomes the next row's north face.  A face shared by two workgroups (or two
// shards) is computed by both from the same values in the same order, so they
// agree bit for bit (restatement: tests/harness.py:ice_flow_step_restated).
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// accesses, not for its global loads and stores (a __syncthreads() fence would
// drain them, and with them the rows prefetched into registers).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// DMAX: instead of stepping, the largest face diffusivity of the workgroup's
// faces goes to out[workgroup] (the CFL bound of tfg_ice_flow_dmax).
constexpr int kFlowTX = 256, kFlowRows = 32, kFlowPF = 1;  // kFlowPF rows of loads in flight (2 and 4 measured slower)
template <class R, bool DMAX>
__global__ __launch_bounds__(kFlowTX) void k_ice_flow(const FlowGrid g, const FlowK K, double* __restrict__ out,
                                                      int strip0, int strip_step, double* __restrict__ out_ice) {
#pragma clang fp contract(off)
  __shared__ double sS[3][kFlowTX + 2], sH[3][kFlowTX + 2], sW[3][kFlowTX + 2], qx[kFlowTX + 1];  // sW: h_iwe as read
  double dmax = 0.0;
  const int t = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.x * kFlowTX;
  const int64_t r0 = ((int64_t)strip0 + (int64_t)blockIdx.y * strip_step) * kFlowRows;  // this workgroup's strip
  const int64_t r1 = r0 + kFlowRows < g.ny ? r0 + kFlowRows : g.ny;
  const int64_t c = c0 + t;
  auto slot = [&](int64_t rr) { return (int)(rr - r0 + 1) % 3; };  // 32-bit: rr - r0 + 1 <= kFlowRows + 1
  // A row of (s, H) for columns c0-1 .. c0+kFlowTX, fetched into registers
  // one row ahead and written to LDS a row later, so its HBM latency overlaps
  // the current row's face arithmetic.  Raw values: (elev, h_iwe), or (s, H)
  // from a halo row; a missing row outside the domain repeats the edge row.
  struct Raw { double a[2], b[2]; bool halo; };
  auto fetch = [&](int64_t rr, Raw& v) {
    v.halo = (rr < 0 && g.hn) || (rr >= g.ny && g.hs);
    const double* hr = rr < 0 ? g.hn : g.hs;
    const int64_t rc_ = rr < 0 ? 0 : (rr >= g.ny ? g.ny - 1 : rr);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = t + j * kFlowTX;
      if (k < kFlowTX + 2) {
        const int64_t cc = c0 - 1 + k;
        const int64_t cl = cc < 0 ? 0 : (cc >= g.nx ? g.nx - 1 : cc);
        if (v.halo) {
          v.a[j] = hr[cl];
          v.b[j] = hr[g.nx + cl];
        } else {
          v.a[j] = (double)static_cast<const R*>(g.elev)[rc_ * g.nx + cl];
          v.b[j] = g.iwe[rc_ * g.nx + cl];
        }
      }
    }
  };
  auto put = [&](int64_t rr, const Raw& v) {
    const int sl = slot(rr);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = t + j * kFlowTX;
      if (k < kFlowTX + 2) {
        sS[sl][k] = v.halo ? v.a[j] : v.a[j] + v.b[j] * g.wi;
        sH[sl][k] = v.halo ? v.b[j] : v.b[j] * g.wi;
        sW[sl][k] = v.b[j];  // h_iwe of an in-domain row (the only rows a workgroup updates)
      }
    }
  };
  auto face_y = [&](int a, int b) {  // between the rows in slots a (north) and b (south), column c
    const double gn = (sS[b][t + 1] - sS[a][t + 1]) * K.inv_dy;
    const double gt = ((sS[a][t + 2] - sS[a][t]) + (sS[b][t + 2] - sS[b][t])) * K.inv_4dx;
    if constexpr (DMAX) {
      if (c < g.nx) dmax = fmax(dmax, flow_face_D(sH[a][t + 1], sH[b][t + 1], gn, gt, K.gamma));
      return 0.0;
    }
    return flow_face_q(sH[a][t + 1], sH[b][t + 1], gn, gt, K.gamma, K.lim_y);
  };
  // rows r0-1 and r0 first; rows r0+1 .. r0+kFlowPF in flight in registers
  {
    Raw v;
    fetch(r0 - 1, v);
    put(r0 - 1, v);
    fetch(r0, v);
    put(r0, v);
  }
  Raw buf[kFlowPF];
#pragma unroll
  for (int j = 0; j < kFlowPF; ++j)
    if (r0 + 1 + j <= r1) fetch(r0 + 1 + j, buf[j]);
  double qN = 0.0;
  for (int64_t rb = r0; rb < r1; rb += kFlowPF) {
#pragma unroll
    for (int jj = 0; jj < kFlowPF; ++jj) {
      const int64_t r = rb + jj;
      if (r >= r1) break;
      lds_barrier();  // row r-2's slot and qx are free
      put(r + 1, buf[jj]);
      if (r + 1 + kFlowPF <= r1) fetch(r + 1 + kFlowPF, buf[jj]);  // in flight for the next kFlowPF rows
      lds_barrier();
      const int rm = slot(r - 1), rc = slot(r), rp = slot(r + 1);
      for (int k = t; k < kFlowTX + 1; k += kFlowTX) {  // x-faces between columns c0-1+k and c0+k
        const int64_t fc = c0 - 1 + k;
        double q = 0.0;
        if (fc >= 0 && fc + 1 < g.nx) {
          const double gn = (sS[rc][k + 1] - sS[rc][k]) * K.inv_dx;
          const double gt = ((sS[rp][k] - sS[rm][k]) + (sS[rp][k + 1] - sS[rm][k + 1])) * K.inv_4dy;
          if constexpr (DMAX) dmax = fmax(dmax, flow_face_D(sH[rc][k], sH[rc][k + 1], gn, gt, K.gamma));
          else q = flow_face_q(sH[rc][k], sH[rc][k + 1], gn, gt, K.gamma, K.lim_x);
        }
        qx[k] = q;
      }
      if (r == r0) qN = (r > 0 || g.hn) ? face_y(rm, rc) : 0.0;
      const double qS = (r + 1 < g.ny || g.hs) ? face_y(rc, rp) : 0.0;
      lds_barrier();  // qx complete
      if (!DMAX && c < g.nx) {
        const int64_t i = r * g.nx + c;
        const double div = (qx[t + 1] - qx[t]) * K.inv_dx + (qS - qN) * K.inv_dy;
        const double v = fmax(sW[rc][t + 1] - K.dt_wi * div, 0.0);
        out[i] = v;
        if (out_ice) out_ice[i] = v * g.wi;  // writing the state plane: h_ice too (:1726)
      }
      qN = qS;
    }
  }
  if constexpr (DMAX) {
    __syncthreads();
    qx[t] = dmax;  // reuse qx as the reduction buffer
    __syncthreads();
    for (int w = kFlowTX / 2; w > 0; w >>= 1) {
      if (t < w) qx[t] = fmax(qx[t], qx[t + w]);
      __syncthreads();
    }
    if (t == 0) out[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = qx[0];
  }
}

// commit a sub-step: the new h_iwe into the state plane, and the next step's
// previous-step ice depth h_ice = h_iwe * wi (:1726) for the state-plane read
__global__ void k_flow_commit(double* __restrict__ st, const double* __restrict__ iwe_new, int64_t n, int64_t n_pad,
                              double wi) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = iwe_new[i];
    st[S_HIWE * n_pad + i] = v;
    st[S_HICE * n_pad + i] = v * wi;
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
