"""How much of the fp32 engine's pure-relative 1e-5 misses a more accurate
Q_sum would remove ("Pure-relative misses"): a CPU
experiment on the numpy oracle, like melt_gate_flips.py.

The numpy oracle (bit-exact to the reference fixtures) runs bench.py's sample
workload (the first N synthetic cells, 96 hourly steps) unperturbed (ref) and
with Q_sum perturbed every cell-step by a relative eps * N(0, 1) (through the
oracle's Qc term, :1314), eps from fp32 size (3e-7) down to 1e-12.  For each
run and output it prints the fraction of values further than 1e-5 relative
from ref (pure relative: |g - r| > 1e-5 |r|), over every cell-step and over the
cells without a melt-out flip (tests/harness.py melt_out_flips), beside the
same fractions for the fp64 baseline (the C oracle, glibc libm).

    python tests/diagnostics/pure_relative.py [N] [out.json]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle"), str(ROOT)]
import tfg_oracle as O  # noqa: E402

from tests.harness import BASE_CFG, c_oracle_hist, melt_out_flips  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table, synthetic_cells  # noqa: E402

HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")


def misses(g, ref, flip):
    """Per output: fraction of cell-steps beyond pure-relative 1e-5, over all
    cells and over the cells that do not flip."""
    keep = flip < 0
    out = {}
    for v in HIST:
        bad = np.abs(g[v] - ref[v]) > 1e-5 * np.abs(ref[v])
        out[v] = {"all": float(bad.mean()), "unflipped": float(bad[:, keep].mean()) if keep.any() else None}
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    steps = 96
    syn = synthetic_cells(20251001, np.arange(n), diurnal_table(24))
    static = {k: np.asarray(syn[s], np.float64) for k, s in (
        ("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"), ("h0_snow", "h_snow"), ("h0_ice", "h_ice"),
        ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    cfg = dict(BASE_CFG)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    forc = {v: syn[v] for v in ("P", "T_air", "Hum_sp", "P_air", "uz")}

    def run(eps=0.0, q_ref=None, seed=1):
        rng = np.random.default_rng(seed)
        m = O.OracleGrid(cfg, **static)
        out, qs = {v: [] for v in HIST}, []
        for k in range(steps):
            m.Qc = np.zeros(n) if q_ref is None else q_ref[k] * eps * rng.standard_normal(n)
            r = m.step(*(forc[v][k % 24].astype(np.float64) for v in forc), jd[k], tsn[k])
            for v in HIST:
                out[v].append(np.array(r[v], copy=True))
            qs.append(np.array(r["Q_sum"], copy=True))
        return {v: np.stack(a) for v, a in out.items()}, qs

    t0 = time.time()
    ref, q_ref = run()
    c = c_oracle_hist(cfg, static, forc, steps, frames=np.arange(steps) % 24, clock=(jd, tsn))
    c = {v: c[v] for v in HIST}
    flip, _ = melt_out_flips(c, ref)
    res = {"cells": n, "steps": steps, "fp64_baseline": {"flips": int((flip >= 0).sum()), "misses": misses(c, ref, flip)},
           "runs": []}
    print(json.dumps(res["fp64_baseline"]), flush=True)
    for eps in (3e-7, 1e-8, 1e-9, 1e-10, 1e-12):
        g, _ = run(eps, q_ref)
        flip, _ = melt_out_flips(g, ref)
        row = {"eps": eps, "flips": int((flip >= 0).sum()), "misses": misses(g, ref, flip)}
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    res["seconds"] = time.time() - t0
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
