"""Accumulated error of each fp32 energy term over a deep launch (GPU + CPU on the box).

With a -DTFG_DEBUG_TERMS build at TFG_LIB, the six output planes of every step
hold that step's Qn_SW, Qn_LW, Qh, Qe, snowfall cold content and Q_sum (the
state evolves as in the production kernel).  This runs bench.py's parity
shape (a one-step launch, then one launch of `steps` - 1 steps, on the first
`rows` rows of an 8192-wide grid), the numpy oracle on the same cells, and
reports per term: the mean per-step error (bias), the rms, and percentiles
over cells of the error summed over all steps -- the energy error that ends
up in the cold content and the depths (the depletion and melt-onset entries
of a deep parity check).  Cells whose Q_sum error ever exceeds 1e-3 W m-2
(melt-out flips: a different albedo or surface temperature) are left out.

  python tests/diagnostics/term_bias.py OUT.json [rows] [steps]
Diagnostic only.
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle"), str(ROOT)]

TERMS = ("Qn_SW", "Qn_LW", "Qh", "Qe", "dEccs", "Q_sum")  # the debug build's planes, in output order
HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
NX, SEED = 8192, 20251001


def main():
    out = sys.argv[1]
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 385
    import tfg_oracle as O

    from tests.harness import BASE_CFG, make_engine
    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    t0 = time.time()
    e = make_engine(dict(BASE_CFG), rows, NX, "float32", n_frames=24, hist_depth=steps, fuse_steps=steps - 1)
    e.fill_synthetic(SEED, diurnal_table(24), nx_global=NX)
    e.run(1)
    e.run(steps - 1)
    e.sync()
    g = {t: np.stack([e.get_field(v, index=k, dtype=np.float32) for k in range(steps)]).astype(np.float64)
         for t, v in zip(TERMS, HIST)}
    e.close()
    n = rows * NX
    syn = synthetic_cells(SEED, np.arange(n), diurnal_table(24))
    static = {k: np.asarray(syn[s], np.float64) for k, s in (
        ("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"), ("h0_snow", "h_snow"), ("h0_ice", "h_ice"),
        ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    cfg = dict(BASE_CFG)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    frames = np.arange(steps) % 24
    m = O.OracleGrid(cfg, **static)
    r = {t: np.empty((steps, n)) for t in ("Qn_SW", "Qn_LW", "Qh", "Qe", "Q_sum", "dEccs")}
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    ws = np.float64(c["rho_H2O"]) / np.float64(c["rho_snow"])
    rcs = np.float64(c["rho_snow"]) * np.float64(c["Cp_snow"])
    for k in range(steps):
        f = [syn[v][frames[k]].astype(np.float64) for v in ("P", "T_air", "Hum_sp", "P_air", "uz")]
        x = m.step(*f, jd[k], tsn[k])
        for t in ("Qn_SW", "Qn_LW", "Qh", "Qe", "Q_sum"):
            r[t][k] = x[t]
        P_snow = f[0] * (f[1] <= c["T_rain_snow"])  # the snowfall cold content (:1507-1537)
        RH, Ta = x["RH"], f[1]
        T_wb = (Ta * np.arctan(0.151977 * ((RH + 8.313659) ** 0.5)) + np.arctan(Ta + RH)
                - np.arctan(RH - 1.676331) + ((0.00391838 * (RH ** 1.5)) * np.arctan(0.023101 * RH)) - 4.86035)
        r["dEccs"][k] = np.where(P_snow > 0, rcs * ((P_snow * c["dt"]) * ws) * (np.float64(c["T0"]) - T_wb), 0.0)
    keep = (np.abs(g["Q_sum"] - r["Q_sum"]) <= 1e-3).all(axis=0)
    res = {"cells": n, "steps": steps, "cells_kept": int(keep.sum()), "lib": str(e.lib._name), "terms": {}}
    for t in ("Qn_SW", "Qn_LW", "Qh", "Qe", "Q_sum", "dEccs"):
        d = (g[t] - r[t])[:, keep]
        acc = np.abs(d.sum(axis=0))
        res["terms"][t] = {"mean_err_Wm2": float(d.mean()), "rms_err_Wm2": float(np.sqrt((d * d).mean())),
                           "mean_abs_value_Wm2": float(np.abs(r[t][:, keep]).mean()),
                           "acc_abs_p50": float(np.percentile(acc, 50)), "acc_abs_p99": float(np.percentile(acc, 99)),
                           "acc_abs_max": float(acc.max())}
    res["seconds"] = time.time() - t0
    Path(out).write_text(json.dumps(res, indent=1) + "\n")
    for t, s in res["terms"].items():
        print(f"{t:6s} bias {s['mean_err_Wm2']:+.3e} rms {s['rms_err_Wm2']:.3e}  sum over steps: p50 {s['acc_abs_p50']:.3e}"
              f" p99 {s['acc_abs_p99']:.3e} max {s['acc_abs_max']:.3e}  (|X| {s['mean_abs_value_Wm2']:.1f})", flush=True)


if __name__ == "__main__":
    main()
