"""Which fp32 energy term causes the fp32 engine's pure-relative 1e-5 misses
(VERDICT r3 "What's weak" 1).  Diagnostic only.

  dump <lib> <out.npz> [rows] [steps]   GPU: run the library at <lib> (TFG_LIB)
        on the first `rows` rows of bench.py's 8192-wide workload, a one-step
        launch then one launch of the rest (as bench.py's parity check), and
        save the six output planes of every step.  With a -DTFG_DEBUG_TERMS
        build the planes hold the step's energy terms (Qn_SW, Qn_LW, Qh, Qe,
        the snowfall cold content, Q_sum); with the production build, the
        outputs (h_snow, SM, h_ice, IM, M_total, RH).
  analyse <terms.npz> <outputs.npz> <out.json>   CPU: the numpy oracle on the
        same cells and steps, unperturbed (the reference) and with the GPU's
        own error in one or several terms injected into its energy balance
        (delta_X = gpu_X - oracle_X per cell and step: added to Q_sum through
        the oracle's Qc slot, :1314, or, for the snowfall cold content, to
        Eccs).  For each injection, the fraction of cell-steps whose outputs
        lie beyond pure-relative 1e-5 of the reference (cells with a melt-out
        flip compared up to the flip, as bench.py does), beside the same
        fractions of the GPU's real outputs and of the fp64 baseline (C
        oracle).  "only X": X's error alone; "all but X": every term's error
        except X's, i.e. what promoting X to exact would leave.
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle"), str(ROOT)]

HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
TERMS = ("Qn_SW", "Qn_LW", "Qh", "Qe", "dEccs", "Q_sum")  # the debug build's planes, in HIST order
NX, SEED = 8192, 20251001


def dump(lib, out, rows=4, steps=129):
    os.environ["TFG_LIB"] = str(lib)
    from tests.harness import BASE_CFG, make_engine
    from topoflow_glacier.synthetic import diurnal_table

    e = make_engine(dict(BASE_CFG), rows, NX, "float32", n_frames=24, hist_depth=steps, fuse_steps=steps - 1)
    e.fill_synthetic(SEED, diurnal_table(24), nx_global=NX)
    e.run(1)
    e.run(steps - 1)
    e.sync()
    planes = np.stack([np.stack([e.get_field(v, index=k, dtype=np.float32) for k in range(steps)]) for v in HIST])
    e.close()
    np.savez(out, planes=planes, rows=rows, steps=steps)


def analyse(terms_f, outs_f, out_json):
    import tfg_oracle as O

    from tests.harness import BASE_CFG, c_oracle_hist, melt_out_flips, valid_mask
    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    T = np.load(terms_f)
    G = np.load(outs_f)
    rows, steps = int(T["rows"]), int(T["steps"])
    gterm = {k: T["planes"][i].astype(np.float64) for i, k in enumerate(TERMS)}
    gout = {k: G["planes"][i].astype(np.float64) for i, k in enumerate(HIST)}
    n = rows * NX
    syn = synthetic_cells(SEED, np.arange(n), diurnal_table(24))
    static = {k: np.asarray(syn[s], np.float64) for k, s in (
        ("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"), ("h0_snow", "h_snow"), ("h0_ice", "h_ice"),
        ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    cfg = dict(BASE_CFG)
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    frames = np.arange(steps) % 24
    forc = {v: syn[v].astype(np.float64) for v in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    ws = np.float64(c["rho_H2O"]) / np.float64(c["rho_snow"])
    rcs = np.float64(c["rho_snow"]) * np.float64(c["Cp_snow"])

    def run(inject=None):
        """inject: dict term -> [steps][n] error to add (None: the reference)."""
        m = O.OracleGrid(cfg, **static)
        out = {v: np.empty((steps, n)) for v in HIST}
        terms = {k: np.empty((steps, n)) for k in TERMS}
        for k in range(steps):
            q = np.zeros(n)
            if inject:
                for t, d in inject.items():
                    if t != "dEccs":
                        q = q + d[k]
            m.Qc = q
            f = [forc[v][frames[k]] for v in ("P", "T_air", "Hum_sp", "P_air", "uz")]
            r = m.step(*f, jd[k], tsn[k])
            P_snow = f[0] * (f[1] <= c["T_rain_snow"])
            RH, Ta = r["RH"], f[1]
            T_wb = (Ta * np.arctan(0.151977 * ((RH + 8.313659) ** 0.5)) + np.arctan(Ta + RH)
                    - np.arctan(RH - 1.676331) + ((0.00391838 * (RH ** 1.5)) * np.arctan(0.023101 * RH)) - 4.86035)
            dE = np.where(P_snow > 0, rcs * ((P_snow * c["dt"]) * ws) * (np.float64(c["T0"]) - T_wb), 0.0)
            if inject and "dEccs" in inject:
                d = inject["dEccs"][k]
                m.Eccs = np.where((P_snow > 0) & (m.Eccs > 0), np.maximum(m.Eccs + d, 0.0), m.Eccs)
            for v in HIST:
                out[v][k] = r[v]
            for t in ("Qn_SW", "Qn_LW", "Qh", "Qe"):
                terms[t][k] = r[t]
            terms["Q_sum"][k] = r["Q_sum"] - q
            terms["dEccs"][k] = dE
        return out, terms

    def misses(g, ref):
        flip, genuine = melt_out_flips(g, ref)
        ok = valid_mask(flip, steps)
        res = {"flips": int((flip >= 0).sum()), "genuine": len(genuine)}
        for v in HIST:
            gv, rv = g[v][ok], ref[v][ok]
            with np.errstate(divide="ignore", invalid="ignore"):
                rel = np.where(rv != 0, np.abs(gv - rv) / np.abs(rv), np.where(gv != rv, np.inf, 0.0))
            res[v] = float(np.mean(rel > 1e-5))
        return res

    t0 = time.time()
    ref, rterm = run()
    delta = {t: gterm[t] - rterm[t] for t in TERMS}
    # the fp32 rounding of the sum itself: Q_sum's error beyond its four terms'
    delta["sum"] = delta["Q_sum"] - (delta["Qn_SW"] + delta["Qn_LW"] + delta["Qh"] + delta["Qe"])
    parts = ("Qn_SW", "Qn_LW", "Qh", "Qe", "sum", "dEccs")
    stats = {}
    for t in parts + ("Q_sum",):
        d, r = delta[t], rterm["Q_sum" if t == "sum" else t]
        nz = r != 0
        rel = d[nz] / np.abs(r[nz]) if nz.any() else np.zeros(1)
        stats[t] = {"mean_abs_err_Wm2": float(np.mean(np.abs(d))), "mean_err_Wm2": float(np.mean(d)),
                    "rms_rel": float(np.sqrt(np.mean(rel ** 2))), "mean_rel": float(np.mean(rel)),
                    "p99_abs_rel": float(np.percentile(np.abs(rel), 99)),
                    "mean_abs_value": float(np.mean(np.abs(r)))}
    res = {"cells": n, "steps": steps, "term_error_stats": stats,
           "gpu_actual": misses(gout, ref)}
    c64 = c_oracle_hist(cfg, static, {v: syn[v] for v in forc}, steps, frames=frames, clock=(jd, tsn))
    res["fp64_baseline"] = misses({v: c64[v] for v in HIST}, ref)
    print(json.dumps({"gpu_actual": res["gpu_actual"], "fp64_baseline": res["fp64_baseline"]}), flush=True)
    runs = {"all": {t: delta[t] for t in parts}}
    for t in parts:
        runs[f"only {t}"] = {t: delta[t]}
        runs[f"all but {t}"] = {u: delta[u] for u in parts if u != t}
    res["injected"] = {}
    for name, inj in runs.items():
        g, _ = run(inj)
        res["injected"][name] = misses(g, ref)
        print(name, json.dumps(res["injected"][name]), flush=True)
    res["seconds"] = time.time() - t0
    Path(out_json).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], sys.argv[3], *(int(a) for a in sys.argv[4:6]))
    elif sys.argv[1] == "analyse":
        analyse(*sys.argv[2:5])
    else:
        raise SystemExit(__doc__)
