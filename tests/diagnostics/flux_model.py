"""A numpy model of the fp32 engine's energy flux (csrc/tfg_physics.hpp
cell_step_fast: Q_sum and the snowfall cold content), for CPU studies of its
accuracy.  Diagnostic only: no test relies on it, and it is not the engine.

fp32 operations are numpy float32 (IEEE round to nearest; fmaf as an fp64
product-sum rounded once).  The gfx950 transcendental instructions are modelled
with their measured error sizes (HISTORY.md section 3: v_exp_f32 max 4e-7,
unbiased; v_log_f32 -0.44 ulp of its result; v_rcp_f32 ~1 ulp): the correctly
rounded value perturbed by a deterministic hash of the argument's bits.

flux_error(variant, ...) evaluates one step at a given state (the oracle's, so
that one-step errors are isolated from trajectory divergence) and returns the
per-cell Q_sum error against the fp64 reference form.  year_metrics() injects a
[steps][cells] error into the numpy oracle's year (through its Qc slot) and
returns the year test's metrics (tests/test_gpu_parity.py
test_fp32_free_run_over_a_year).

  python tests/diagnostics/flux_model.py [variant ...]
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle"), str(ROOT)]

f32, f64 = np.float32, np.float64
NF = 24  # forcing frames (the year test: 24, repeated daily; 8760: no repetition)
LOG2E = 1.4426950408889634
LN2 = 0.6931471805599453


def _hash_u(x, salt):
    """Deterministic uniform(-1, 1) from the bits of an fp32 array."""
    b = np.asarray(x, f32).view(np.uint32).astype(np.uint64)
    z = (b * np.uint64(0x9E3779B97F4A7C15) + np.uint64(salt)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    z ^= z >> np.uint64(29)
    z = (z * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    z ^= z >> np.uint64(32)
    return (z & np.uint64(0xFFFFFF)).astype(f64) / f64(2 ** 23) - 1.0


def fma32(a, b, c):
    return (np.asarray(a, f64) * np.asarray(b, f64) + np.asarray(c, f64)).astype(f32)


IDEAL = bool(int(__import__("os").environ.get("TFG_FM_IDEAL", "0")))  # correctly rounded hardware functions


def hw_exp2(x):
    x = np.asarray(x, f32)
    y = np.exp2(x.astype(f64))
    if IDEAL:
        return y.astype(f32)
    return (y * (1.0 + 1.7e-7 * _hash_u(x, 1))).astype(f32)


def hw_log2(x):
    x = np.asarray(x, f32)
    with np.errstate(divide="ignore", invalid="ignore"):
        y = np.log2(x.astype(f64))
        yr = y.astype(f32)
        if IDEAL:
            return yr
        ulp = np.spacing(np.abs(yr)).astype(f64)
        return (y + ulp * (-0.44 + 0.5 * _hash_u(x, 2))).astype(f32)


def hw_rcp(x):
    x = np.asarray(x, f32)
    if IDEAL:
        return (1.0 / x.astype(f64)).astype(f32)
    return ((1.0 / x.astype(f64)) * (1.0 + 1.0e-7 * _hash_u(x, 3))).astype(f32)


def rcp_nr32(x):
    r = hw_rcp(x)
    return fma32(fma32(-np.asarray(x, f32), r, f32(1.0)), r, r)


def log2_nr32(x):
    y = hw_log2(x)
    return fma32(fma32(x, hw_exp2(-y), f32(-1.0)), f32(LOG2E), y)


class Consts:
    def __init__(self, cfg):
        import tfg_oracle as O
        c = dict(O.CFG_DEFAULTS)
        c.update(cfg)
        self.c = c
        self.eps100, self.ome100 = 100 * c["eps"], 100 * (1 - c["eps"])
        self.gz = c["g"] * 10.0
        self.k2 = (c["kappa"] / np.log(2.0)) ** 2
        self.rhoCp = c["rho_air"] * c["Cp_air"]
        self.qe = c["rho_air"] * c["Lv"] * c["latent_heat_constant"] * 100.0 / c["sea_level_p0"]
        self.dust = c["dust_atten"]
        self.ems_sigma = c["em_surf"] * c["sigma"]
        k = int(round(np.log2(0.7 * 10.0 / c["z0_air"])))
        self.k = k
        self.inv_z0s = np.ldexp(1.0 / c["z0_air"], -k)
        self.l2min = np.ldexp(0.01, -k)
        F, C = c["canopy_factor"], c["cloud_factor"]
        self.ccF = (1 - F) * 1.72 * (1.0 + 0.22 * C * C)
        self.ccFs = self.ccF * 2.0 ** (-10.0 / 7.0)
        self.Fm1 = F - 1.0
        self.ekf = -(-c["M_mass_air"] * c["g"]) / c["uni_gas_const"]  # * elev: the p0 exponent's factor


def flux(variant, K, u, elev, geo, T, Q, PA, uz, h_snow, h_ice, albedo, n_days):
    """Q_sum of one step (fp64 array of the variant's result).  `variant` is a set
    of names of parts computed in fp64 ("base": the kernel as it is).
    geo: dict of fp32 planes sl, cc, cs (k_prepare_geo); u: the step's uniforms."""
    v = set(variant)
    T, Q, PA, uz = (np.asarray(a, f32) for a in (T, Q, PA, uz))
    snow_pos, ice_pos = h_snow > 0, h_ice > 0
    T_K = T + f32(273.15)
    rT = hw_rcp(T_K)
    rA = hw_rcp(T + f32(237.3))
    # dew point
    if "dew" in v:
        e64 = f64(Q) * f64(PA) / (K.eps100 + K.ome100 * f64(Q))
        L = np.log(e64 / 6.1121)
        Td64 = 257.14 * L / (18.678 - L)
        Ts64 = np.where(snow_pos | ice_pos, np.minimum(Td64, 0.0), Td64)
        e_air = e64.astype(f32)
        T_dew = Td64.astype(f32)
        T_surf = Ts64.astype(f32)
        dTs64 = f64(T) - Ts64
    else:
        e_air = Q * PA * rcp_nr32(f32(K.eps100) + f32(K.ome100) * Q)
        log_term = log2_nr32(e_air * f32(1 / 6.1121)) * f32(LN2)
        T_dew = f32(257.14) * log_term * rcp_nr32(f32(18.678) - log_term)
        T_surf = np.where(snow_pos | ice_pos, np.minimum(T_dew, f32(0)), T_dew)
        e64 = f64(e_air)
        Ts64 = f64(T_surf)
        dTs64 = f64(T - T_surf)
    dTs = dTs64.astype(f32)
    # turbulent
    if "turb" in v:
        bot = f64(uz) ** 2 * (f64(T) + 273.15)
        bot = np.where(bot == 0, 0.01, bot)
        Ri = K.gz * dTs64 / bot
        ly = f64(hw_log2(np.maximum((f32(10.0) - h_snow.astype(f32)) * f32(K.inv_z0s), f32(K.l2min))))
        if "turblog" in v:
            ly = np.log2(np.maximum((10.0 - h_snow) * K.inv_z0s, K.l2min))
        L2sq = ly * (ly + 2 * K.k) + K.k * K.k
        Dn = f64(uz) * K.k2 / L2sq
        Dh = np.where(Ri > 0, Dn / (1 + 10 * Ri), Dn * (1 - 10 * Ri))
        Qh = K.rhoCp * Dh * dTs64
    else:
        bot = (uz * uz) * T_K
        bot = np.where(bot == 0, f32(0.01), bot)
        rcp = rcp_nr32 if "rcpnr" in v else hw_rcp  # "rcpnr": Newton-refined reciprocals in Ri, Dn, Dh
        Ri = f32(K.gz) * dTs * rcp(bot)
        ly2 = hw_log2(np.maximum((f32(10.0) - h_snow.astype(f32)) * f32(K.inv_z0s), f32(K.l2min)))
        L2sq = fma32(ly2, ly2 + f32(2 * K.k), f32(K.k * K.k))
        Dn = uz * f32(K.k2) * rcp(L2sq)
        Dh32 = np.where(Ri > 0, Dn * rcp(fma32(f32(10), Ri, f32(1))), Dn * fma32(f32(-10), Ri, f32(1)))
        Dh = f64(Dh32)
        Qh = f64(f32(K.rhoCp) * Dh32 * dTs)
    # latent
    if "lat" in v:
        de = e64 * -np.expm1((-17.3 * 237.3) * dTs64 / ((Ts64 + 237.3) * (f64(T) + 237.3)))
        p0f = np.exp(K.ekf * elev / (f64(T) + 273.15))
        Qe = K.qe * Dh * de * p0f
    else:
        rS = hw_rcp(T_surf + f32(237.3))
        xs2 = f32(-5922.6815) * dTs * rS * rA
        de = fma32(-e_air, hw_exp2(xs2), e_air)
        ek = (K.ekf * elev * LOG2E).astype(f32)
        Qe = f64(f32(K.qe) * Dh.astype(f32) * de * hw_exp2(ek * rT))
    # shortwave
    if "sw" in v:
        Wp = 1.12 * np.exp(0.0614 * f64(T_dew) if "dew" not in v else 0.0614 * Td64)
        mo = u["m_opt"]
        tau = np.clip(np.exp((-0.1240 - 0.0207 * Wp) + (-0.0682 - 0.0248 * Wp) * mo) - K.dust, 0, 1)
        gam = 1 + K.dust - np.exp((-0.0363 - 0.0084 * Wp) + (-0.0572 - 0.0173 * Wp) * mo)
        cwl = u["cos_wth"] * f64(geo["cc"]) - u["sin_wth"] * f64(geo["cs"])
        K_ET = np.maximum(u["isc_e0"] * u["cos_d"] * cwl + u["isc_e0"] * u["sin_d"] * f64(geo["sl"]), 0)
        kf = u["k_et_flat"]
        K_dif = 0.5 * gam * kf
        K_cs = tau * K_ET + K_dif + 0.5 * gam * albedo * (tau * kf + K_dif)
        Qsw = K_cs * (1 - albedo)
    else:
        w = hw_exp2(f32(0.0614 * LOG2E) * T_dew)
        tau = np.minimum(np.maximum(hw_exp2(fma32(f32(u["tau_c1"]), w, f32(u["tau_c0"]))) - f32(K.dust), f32(0)), f32(1))
        gam = f32(1 + K.dust) - hw_exp2(fma32(f32(u["gam_c1"]), w, f32(u["gam_c0"])))
        cwl = f32(u["cos_wth"]) * geo["cc"] - f32(u["sin_wth"]) * geo["cs"]
        K_ET = np.maximum(fma32(f32(u["kc_f"]), cwl, f32(u["ks_f"]) * geo["sl"]), f32(0))
        kf = f32(u["k_et_flat_f"])
        K_dif = f32(0.5) * gam * kf
        r = np.where(T > 0, f32(0.12 * LOG2E), f32(0.05 * LOG2E))
        alb = np.where(h_snow > 0, f32(0.4) + f32(0.44) * hw_exp2(-np.asarray(n_days, f32) * r), albedo.astype(f32))
        K_bs = f32(0.5) * gam * alb * fma32(tau, kf, K_dif)
        K_cs = tau * K_ET + K_dif + K_bs
        Qsw = f64(K_cs * (f32(1) - alb))
        if "alb" in v:  # albedo exact, the rest fp32
            alb = albedo.astype(f32)
            Qsw = f64((tau * K_ET + K_dif + f32(0.5) * gam * alb * fma32(tau, kf, K_dif)) * (f32(1) - alb))
    # the reference's dark test (exact, as the kernel's fallback makes it)
    Qsw = np.where(u["dark"], 0.0, Qsw)
    # long wave
    if "lw" in v:
        em = K.ccF * ((e64 / 10.0) / (f64(T) + 273.15)) ** (1 / 7) + (K.Fm1 + 1)
        TaK, TsK = f64(T) + 273.15, Ts64 + 273.15
        Qlw = K.ems_sigma * ((em - 1) * TaK ** 4 + dTs64 * (TaK + TsK) * (TaK ** 2 + TsK ** 2))
    else:
        em_r = hw_exp2(hw_log2(e_air * f32(102.4) * rT) * f32(1 / 7))
        em_m1 = fma32(f32(K.ccFs), em_r, f32(K.Fm1))
        TsK = T_surf + f32(273.15)
        ta2 = T_K * T_K
        d4 = dTs * (T_K + TsK) * fma32(TsK, TsK, ta2)
        Qlw = f64(f32(K.ems_sigma) * fma32(em_m1, ta2 * ta2, d4))
    if "sum" in v or v & {"dew", "turb", "lat", "lw"}:
        Qs = Qsw + Qlw + Qh + Qe
    else:
        Qs = f64(((Qsw.astype(f32) + Qlw.astype(f32)) + Qh.astype(f32)) + Qe.astype(f32))
    return Qs, {"Qn_SW": Qsw, "Qn_LW": Qlw, "Qh": Qh, "Qe": Qe}


def setup(n=2048, seed=20251001, nf=None):
    import tfg_oracle as O
    from tests.harness import BASE_CFG, synthetic_inputs
    from topoflow_glacier.physics.clock import StepClock

    syn, d = synthetic_inputs(seed, 1, n, nf or NF)
    static = {k: np.asarray(syn[s], f64) for k, s in (("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"),
              ("h0_snow", "h_snow"), ("h0_ice", "h_ice"), ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    cfg = dict(BASE_CFG)
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    lat = c["lat"] * np.pi / 180
    sin_lat, cos_lat = np.sin(lat), np.cos(lat)
    ca, sa = np.sin(static["aspect"]), np.cos(static["aspect"])
    r = 1.0 / np.sqrt(1.0 + static["slope"] ** 2)
    sb, cb = static["slope"] * r, r
    sl = sb * ca * cos_lat + cb * sin_lat
    cl = np.sqrt(np.maximum(1.0 - sl * sl, 0.0))
    t = (sb * sa) / (cb * cos_lat - sb * sin_lat * ca)
    rt = 1.0 / np.sqrt(1.0 + t * t)
    geo = {"sl": sl.astype(f32), "cc": (cl * rt).astype(f32), "cs": (cl * t * rt).astype(f32)}
    return syn, static, cfg, geo


def one_step_errors(variants, steps=8760, n=2048):
    """[variant] -> [steps][n] Q_sum errors at the oracle's own states."""
    import tfg_oracle as O
    from topoflow_glacier.physics.clock import StepClock

    syn, static, cfg, geo = setup(n)
    K = Consts(cfg)
    m = O.OracleGrid(cfg, **static)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    clk = StepClock(cfg["start_time"], cfg["dt"], cfg["lat"], cfg["lon"], None, ring_len=int(72 / cfg["dt"]))
    U = clk.uniforms(0, steps)
    F = {v: syn[v].astype(f64) for v in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    err = {v: np.empty((steps, n), f32) for v in variants}
    terms = {v: {t: np.zeros(n) for t in ("Qn_SW", "Qn_LW", "Qh", "Qe")} for v in variants}
    for k in range(steps):
        f = k % NF
        hs, hi = m.h_snow.copy(), m.h_ice.copy()
        r = m.step(*(F[x][f] for x in F), jd[k], tsn[k])
        u = {name: U[name][k] for name in U.dtype.names}
        u["dark"] = r["Qn_SW"] == 0.0
        for var in variants:
            q, parts = flux(var.split("+") if var != "base" else [], K, u, static["elev"], geo, syn["T_air"][f],
                            syn["Hum_sp"][f], syn["P_air"][f], syn["uz"][f], hs, hi, r["albedo"], r["n"])
            err[var][k] = q - r["Q_sum"]
            for t in parts:
                terms[var][t] += (parts[t] - r[t]) ** 2
    rms = {var: {t: float(np.sqrt(terms[var][t].sum() / (steps * n))) for t in terms[var]} for var in variants}
    for var in variants:
        rms[var]["Q_sum"] = float(np.sqrt(np.mean(err[var].astype(f64) ** 2)))
    return err, rms


def year_metrics(dq, n=2048, steps=8760):
    """The year test's metrics for the oracle with dq [steps][n] added to Q_sum,
    against the unperturbed oracle (and the same for dq = None: 0)."""
    import tfg_oracle as O

    syn, static, cfg, geo = setup(n)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    F = {v: syn[v].astype(f64) for v in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")

    def run(d):
        m = O.OracleGrid(cfg, **static)
        daily = {v: [] for v in HIST}
        runoff = np.zeros(n)
        for k in range(steps):
            if d is not None:
                m.Qc = f64(d[k])
            r = m.step(*(F[x][k % NF] for x in F), jd[k], tsn[k])
            runoff += r["M_total"] * 3600.0
            if k % 24 == 23:
                for v in HIST:
                    daily[v].append(np.array(r[v], copy=True))
        out = {v: np.stack(a) for v, a in daily.items()}
        out["runoff"] = runoff
        return out

    R, G = run(None), run(dq)

    def diverged(v):
        g, r = G[v], R[v]
        s_v = np.percentile(np.abs(r[r != 0]), 99)
        err = np.abs(g - r) / np.maximum(np.maximum(np.abs(r), s_v), 1e-300)
        return float(err.max()), (err > 1e-5).any(axis=0)

    gi = diverged("h_ice")[1] | diverged("IM")[1]
    with np.errstate(divide="ignore", invalid="ignore"):
        rr = np.where(R["runoff"] != 0, np.abs(G["runoff"] - R["runoff"]) / np.abs(R["runoff"]),
                      np.abs(G["runoff"] - R["runoff"]))
    return {"SM_div": int(diverged("SM")[1].sum()), "MT_div": int(diverged("M_total")[1].sum()),
            "MT_nonice": int((diverged("M_total")[1] & ~gi).sum()), "ice_div": int(gi.sum()),
            "runoff_nonice_max": float(rr[~gi].max()), "runoff_nonice_p99": float(np.percentile(rr[~gi], 99))}


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--frames=")]
    NF = int(next((a.split("=")[1] for a in sys.argv[1:] if a.startswith("--frames=")), NF))
    variants = args or ["base"]
    steps = 8760
    err, rms = one_step_errors(variants, steps)
    print(json.dumps(rms, indent=1), flush=True)
    for v in variants:
        print(v, json.dumps(year_metrics(err[v], steps=steps)), flush=True)
