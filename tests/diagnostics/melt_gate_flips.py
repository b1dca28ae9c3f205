"""Why the fp32 engine's melt-out flips stay at ~2x the fp64 baseline (DESIGN.md
section 3, "Melt-out flips"): a CPU experiment on the numpy oracle.

The numpy oracle (bit-exact to the reference fixtures) runs bench.py's sample
workload (the first N synthetic cells, 96 hourly steps) three ways:
  ref     unperturbed;
  noise   Q_sum perturbed every cell-step by a relative eps * N(0, 1) (through
          the oracle's Qc term, :1314), eps from fp32 size (3e-7) down to the
          last bit of fp64 (1e-15);
  gated   the same perturbation, except in cell-steps near a melt gate (VERDICT
          r2's proposal: |E_in - Eccs| or |E_in - Ecci| within 1e-5 |E_in|, or
          h_swe below 1e-6 m), i.e. an exact fp64 Q_sum wherever a gate is close.
Melt-out flips of each against ref (tests/harness.py melt_out_flips) are
printed beside the fp64 baseline (the C oracle, glibc libm, against ref).

    python tests/diagnostics/melt_gate_flips.py [N] [out.json]
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    steps = 96
    syn = synthetic_cells(20251001, np.arange(n), diurnal_table(24))
    static = {k: np.asarray(syn[s], np.float64) for k, s in (
        ("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"), ("h0_snow", "h_snow"), ("h0_ice", "h_ice"),
        ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    cfg = dict(BASE_CFG)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])

    def run(mode, eps=0.0, q_ref=None, seed=1):
        rng = np.random.default_rng(seed)
        m = O.OracleGrid(cfg, **static)
        out, qs = {v: [] for v in HIST}, []
        for k in range(steps):
            if mode == "ref":
                m.Qc = np.zeros(n)
            else:
                q = q_ref[k] * eps * rng.standard_normal(n)
                if mode == "gated":
                    e = q_ref[k] * cfg["dt"]
                    near = ((np.abs(e - m.Eccs) < 1e-5 * np.abs(e)) | (np.abs(e - m.Ecci) < 1e-5 * np.abs(e))
                            | (m.h_swe < 1e-6))
                    q = np.where(near, 0.0, q)
                m.Qc = q
            r = m.step(*(syn[v][k % 24].astype(np.float64) for v in ("P", "T_air", "Hum_sp", "P_air", "uz")),
                       jd[k], tsn[k])
            for v in HIST:
                out[v].append(np.array(r[v], copy=True))
            qs.append(np.array(r["Q_sum"], copy=True))
        return {v: np.stack(a) for v, a in out.items()}, qs

    t0 = time.time()
    ref, q_ref = run("ref")
    c = c_oracle_hist(cfg, static, {v: syn[v] for v in ("P", "T_air", "Hum_sp", "P_air", "uz")}, steps,
                      frames=np.arange(steps) % 24, clock=(jd, tsn))
    base = int((melt_out_flips({v: c[v] for v in HIST}, ref)[0] >= 0).sum())
    res = {"cells": n, "steps": steps, "fp64_baseline_flips_c_oracle": base, "runs": []}
    for eps in (3e-7, 1e-9, 1e-12, 1e-15):
        row = {"eps": eps}
        for mode in ("noise", "gated"):
            g, _ = run(mode, eps, q_ref)
            flip, genuine = melt_out_flips(g, ref)
            row[mode + "_flips"] = int((flip >= 0).sum())
            row[mode + "_genuine"] = len(genuine)
        row["noise_over_baseline"] = row["noise_flips"] / base if base else None
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    res["seconds"] = time.time() - t0
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
