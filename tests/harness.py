"""Shared test machinery: golden-fixture loading, the oracle runner, and the
GPU-vs-oracle comparison with the parity tolerance of SURVEY.md 8(d).

Test infrastructure only (imports the oracle as the checker).
"""

from __future__ import annotations

import json
import os
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
for p in (str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

import tfg_oracle as O  # noqa: E402

OUT_NAMES = ["h_snow", "h_swe", "SM", "h_ice", "h_iwe", "IM", "M_total", "RH"]
STATIC_KEYS = ["elev", "slope", "aspect", "h0_snow", "h0_ice", "h0_swe", "h0_iwe"]

# cat-3062920 (tests/integration_test.py:20-38 of the reference)
BASE_CFG = {
    "site_prefix": "cat-3062920", "forcing_file": "data/sample-cat-3062920.csv", "dt": 1,
    "start_time": "2013032000", "end_time": "2013033100", "da": 11.418749923500716,
    "slope": 88.582729, "aspect": 242.8644693769529, "lon": -121.81418, "lat": 46.81953220,
    "elev": 2446.3922737596167, "h_active_layer": 0.125, "h0_snow": 5.0, "h0_ice": 2.0,
    "h0_swe": 0.25, "h0_iwe": 1.834, "T_rain_snow": 0.0,
}


def load_golden(name: str) -> dict:
    z = np.load(GOLDEN / f"{name}.npz")
    cells = json.loads(str(z["cell_cfgs"]))
    F = z["forcing"]
    return {
        "cfg": dict(cells[0]),
        "cells": cells,
        "static": {k: np.array([c[k] for c in cells], dtype=np.float64) for k in STATIC_KEYS},
        "forcing": {n: F[i] for i, n in enumerate(z["in_names"])},  # [nsteps][ncell]
        "outputs": {n: z["outputs"][j] for j, n in enumerate(z["out_names"])},
        "internal": {n: z["internal"][j] for j, n in enumerate(z["internal_names"])},
        "nsteps": F.shape[1],
        "ncell": F.shape[2],
        # the zone the reference's timezonefinder stub returned (make_golden.py)
        "tz_name": str(z["tz_name"]) if "tz_name" in z.files else "America/Los_Angeles",
    }


def cfg_object(cfg: dict):
    """A TopoflowGlacierConfig from a plain dict (product loader)."""
    from topoflow_glacier.bmi.config import TopoflowGlacierConfig

    return TopoflowGlacierConfig.model_validate(cfg)


def oracle_run(cfg: dict, static: dict, forcing: dict, nsteps: int | None = None, catch_id=None,
               tz_name: str = "America/Los_Angeles"):
    out, m = O.run_oracle(cfg, {"elev": static["elev"], "slope": static["slope"], "aspect": static["aspect"],
                                "h0_snow": static["h0_snow"], "h0_ice": static["h0_ice"],
                                "h0_swe": static["h0_swe"], "h0_iwe": static["h0_iwe"]}, forcing, nsteps,
                          tz_name=tz_name)
    return out, m


def scale_floor(ref: np.ndarray) -> float:
    """s_v of SURVEY 8(d): the 99th percentile of |ref|, taken over the
    non-zero entries so that sparse variables (ice melt is zero almost
    everywhere) get a meaningful floor."""
    a = np.abs(np.asarray(ref, dtype=np.float64))
    a = a[a > 0]
    return float(np.percentile(a, 99)) if a.size else 0.0


def parity(gpu: np.ndarray, ref: np.ndarray, rtol: float = 1e-5, mask=None):
    """Floored relative error |gpu-ref| / max(|ref|, s_v).

    Returns (max floored error, fraction of elements above pure-relative rtol).
    `mask` (same shape, bool) selects the elements that are compared.
    """
    gpu = np.asarray(gpu, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    s_v = scale_floor(ref)
    if mask is not None:
        gpu, ref = gpu[mask], ref[mask]
    floor = np.maximum(np.abs(ref), s_v)
    err = np.abs(gpu - ref)
    with np.errstate(divide="ignore", invalid="ignore"):
        fl = np.where(floor > 0, err / floor, np.where(err > 0, np.inf, 0.0))
        rel = np.where(np.abs(ref) > 0, err / np.abs(ref), np.where(err > 0, np.inf, 0.0))
    return float(np.max(fl)) if fl.size else 0.0, float(np.mean(rel > rtol)) if rel.size else 0.0


MELT_OUT_EPS = 1e-9  # m of snow depth: "melt-out" vicinity for the residual-flip rule


OUT_EPS_F32 = 2.0 ** -23  # relative spacing of the fp32 engine's output slots
OUT_EPS_F64 = 2.0 ** -52


def depletion_steps(gpu: dict, ref: dict, cfg: dict, rtol: float = 1e-5, out_eps: float = OUT_EPS_F32) -> np.ndarray:
    """[nsteps][ncell] True at the step a reservoir runs dry, where the melt
    rate is the depth that was left, and the run's rates agree with its depths.

    At the step where the snowpack (or the ice) runs dry in both trajectories
    (its depth at or below the melt-out residual scale MELT_OUT_EPS, after a
    depth above it), update_swe / update_iwe (:1594-1617) cap the melt at what
    is left: SM = min(SM*3600, h_swe + P_snow dt)/3600 and IM =
    min(IM*3600, h_iwe)/3600.  So SM*3600*w_s - P_snow dt w_s and IM*3600*w_i
    ARE the previous step's depth (w = rho_H2O / rho_snow or / rho_ice; the
    snowfall is the same in both runs), and the rate's difference between two
    runs is their depth difference at the step before, divided by 3600 w --
    an identity, not a tolerance.  The depth itself is compared at its own
    floor at the step before; against the rate's floor (p99 of SM, ~1e-6
    m/s) the same difference weighs ~1000x more, so the rate entry is checked
    by the identity instead:
        |G_rate - R_rate| * 3600 * w  <=  |G_h[k-1] - R_h[k-1]|  +  slack,
    slack = 4 out_eps (|R_h[k-1]| + |R_rate| 3600 w) for the rounding of the two
    output slots (out_eps: their relative spacing); M_total's difference must
    be SM's plus IM's to the same rounding (:1441-1443).  Every such entry is
    marked -- those within the rate's own tolerance too -- when the identity
    holds for each rate output of the step, the depths at the step are within
    their own tolerance and RH is; an entry that breaks the identity is
    compared as usual (a defect in the capping shows up there).  Later steps
    are compared as usual."""
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    w = {"snow": float(c["rho_H2O"]) / float(c["rho_snow"]), "ice": float(c["rho_H2O"]) / float(c["rho_ice"])}
    names = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
    G = {v: np.asarray(gpu[v], np.float64) for v in names if v in gpu}
    R = {v: np.asarray(ref[v], np.float64) for v in names if v in ref}
    nsteps, ncell = R["SM"].shape
    bad = {}
    for v in G:
        fl = np.abs(G[v] - R[v]) / np.maximum(np.maximum(np.abs(R[v]), scale_floor(R[v])), 1e-300)
        bad[v] = fl > rtol
    dry, ident = {}, {}
    for res, depth, rate in (("snow", "h_snow", "SM"), ("ice", "h_ice", "IM")):
        prev_r = np.vstack([np.zeros((1, ncell)), R[depth][:-1]])  # depth at the step before (k = 0: not known)
        prev_g = np.vstack([np.zeros((1, ncell)), G[depth][:-1]])
        dry[res] = (np.abs(G[depth]) <= MELT_OUT_EPS) & (np.abs(R[depth]) <= MELT_OUT_EPS) & (prev_r > MELT_OUT_EPS)
        amount = np.abs(G[rate] - R[rate]) * 3600.0 * w[res]
        slack = 4.0 * out_eps * (np.abs(prev_r) + np.abs(R[rate]) * 3600.0 * w[res])
        ident[res] = amount <= np.abs(prev_g - prev_r) + slack
    d_mt = np.abs((G["M_total"] - R["M_total"]) - ((G["SM"] - R["SM"]) + (G["IM"] - R["IM"])))
    ok_mt = d_mt <= 4.0 * out_eps * (np.abs(R["M_total"]) + np.abs(R["SM"]) + np.abs(R["IM"]))
    any_dry = dry["snow"] | dry["ice"]
    rate_ok = {"snow": np.where(dry["snow"], ident["snow"], ~bad["SM"]),
               "ice": np.where(dry["ice"], ident["ice"], ~bad["IM"])}
    rh_ok = ~bad["RH"] if "RH" in bad else np.ones((nsteps, ncell), dtype=bool)
    return any_dry & ~bad["h_snow"] & ~bad["h_ice"] & rh_ok & rate_ok["snow"] & rate_ok["ice"] & ok_mt


def melt_out_flips(gpu: dict, ref: dict, rtol: float = 1e-5, excused: np.ndarray | None = None):
    """Cells whose trajectories part at a melt-out residual.

    The reference tests float state for exact zero in three places:
    ``h_swe == 0 & previous_swe == 0`` gates ice melt (bmi_topoflow_glacier.py:1424),
    ``h_snow == 0`` resets the snowpack cold content (:1562), and ``h_ice == 0``
    resets the ice cold content (:1426).  The depths come from
    h = max(h - (h/3600)*dt*3600, 0), whose sub-ulp residual is 0 or ~1e-19
    depending on the last bit of h, so any engine whose state differs from the
    reference in the last bit can land on the other side of a gate.  Through
    IM that switches ice melt on a step earlier or later; through the reset
    cold content it moves the next melt onset of a thin new snowpack by a step.
    A cell is classified as a flip, and compared only before its flip step,
    when either
      (b) at some step j, exactly one trajectory has a snow (or ice) depth of
          exactly zero and the other a residual within MELT_OUT_EPS: the zero
          gates have diverged.  The flip step is j, whether or not an output
          leaves tolerance later: from j on the two runs follow different
          branches of the reference's own code (round 5; before, such a cell
          was compared until its first step out of tolerance, so its in-
          tolerance post-split entries set the sample's maximum error, for
          the fp64 baseline as much as for the GPU), or
      (a) at its first step k outside tolerance, the IM on/off gate differs
          and one trajectory has a snow depth within MELT_OUT_EPS of zero at
          k or k-1; the flip step is k.
    `excused` ([nsteps][ncell], e.g. depletion_steps) marks entries already
    explained, which are not counted as out of tolerance.
    Returns (flip_step per cell or -1, list of genuinely failing (cell, step, var)).
    """
    names = [v for v in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH") if v in gpu]
    nsteps, ncell = np.asarray(ref[names[0]]).shape
    bad = np.zeros((nsteps, ncell), dtype=bool)
    for v in names:
        g, r = np.asarray(gpu[v], np.float64), np.asarray(ref[v], np.float64)
        fl = np.abs(g - r) / np.maximum(np.maximum(np.abs(r), scale_floor(r)), 1e-300)
        bad |= fl > rtol
    if excused is not None:
        bad &= ~excused
    # (b): first step at which the exact-zero status of a depth diverges at residual scale
    split = np.full(ncell, nsteps)
    for v in ("h_snow", "h_ice"):
        if v not in gpu:
            continue
        g, r = np.abs(np.asarray(gpu[v], np.float64)), np.abs(np.asarray(ref[v], np.float64))
        d = ((g == 0) != (r == 0)) & (np.maximum(g, r) <= MELT_OUT_EPS)
        first = np.where(d.any(axis=0), np.argmax(d, axis=0), nsteps)
        split = np.minimum(split, first)
    flip = np.full(ncell, -1)
    genuine = []
    for c in np.nonzero(bad.any(axis=0) | (split < nsteps))[0]:
        k = int(np.argmax(bad[:, c])) if bad[:, c].any() else nsteps
        if split[c] <= k:  # (b): compared up to the step the gates parted, in or out of tolerance after it
            flip[c] = split[c]
            continue
        gate = (np.asarray(gpu["IM"])[k, c] > 0) != (np.asarray(ref["IM"])[k, c] > 0)
        ks = [k] + ([k - 1] if k > 0 else [])
        near = min(min(abs(float(np.asarray(gpu["h_snow"])[j, c])), abs(float(np.asarray(ref["h_snow"])[j, c]))) for j in ks)
        if gate and near <= MELT_OUT_EPS:
            flip[c] = k
        else:
            genuine.append((int(c), k, [v for v in names if np.abs(np.asarray(gpu[v])[k, c] - np.asarray(ref[v])[k, c])
                                        > rtol * max(abs(np.asarray(ref[v])[k, c]), scale_floor(ref[v]))]))
    return flip, genuine


# One flip budget for every parity check (tests, smoke, bench).  The melt-out
# gates test fp64 state for exact zero, so ANY two implementations that differ in
# the last bit flip some cells.  The yardstick is the fp64 baseline of the same
# cells and steps: the C oracle (glibc libm) against the numpy oracle (numpy's
# SIMD libm, bit-exact to the reference fixtures) -- two fp64 restatements of
# the same operation order.  Measured ratio GPU fp32 / fp64 baseline: 1.94 on
# bench.py's sample (4174 / 2149 of 262 144 cells x 96 steps) and 2.0 on the
# year-long run (ice divergence in 74 / 37 of 2048 cells).  That ratio is the
# floor for any engine whose Q_sum differs from numpy's in the last bit: the
# oracle with Q_sum perturbed by a relative 3e-7 ... 1e-15 flips 1.86-1.91 x the
# baseline, and an exact Q_sum near the melt gates changes nothing
# (tests/diagnostics/melt_gate_flips.py, profiles/r3_melt_gate_flips.json;
# DESIGN.md section 3).  The budget is that ratio plus margin.
FLIP_RATIO_MAX = 2.5
FLIP_SLACK = 3  # absolute allowance for samples whose baseline is a handful of cells


def flip_rule(flips: int, fp64_flips: int) -> dict:
    """The one budget: flips <= FLIP_RATIO_MAX x fp64 baseline flips + FLIP_SLACK."""
    budget = int(FLIP_RATIO_MAX * fp64_flips) + FLIP_SLACK
    return {"flips": int(flips), "fp64_flips": int(fp64_flips), "budget": budget,
            "ratio": (flips / fp64_flips) if fp64_flips else None, "ok": bool(flips <= budget),
            "rule": f"flips <= {FLIP_RATIO_MAX:g} x fp64 baseline (C oracle vs numpy oracle, same cells and steps)"
                    f" + {FLIP_SLACK}"}


def c_oracle_hist(cfg: dict, static: dict, forcing: dict, nsteps: int, frames=None, state=None, clock=None,
                  start_step: int = 0, tz_name: str = "America/Los_Angeles", qc=None, qc_every: int = 1):
    """The C oracle (fp64, glibc libm) over the same cells and steps as a numpy
    oracle run: per-step outputs [nsteps][ncell].  `forcing` is [n_frames][ncell]
    per field and step k reads frames[k] (default k); `state` starts it from a
    numpy-oracle snapshot; `clock` = (jd, tsn) arrays of at least start_step+nsteps."""
    import tfg_oracle_c as OC

    if clock is None:
        jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], start_step + nsteps, cfg["lon"], tz_name)
    else:
        jd, tsn = clock
    jd = np.asarray(jd)[start_step:start_step + nsteps]
    tsn = np.asarray(tsn)[start_step:start_step + nsteps]
    st = {k: np.asarray(static[k], np.float64) for k in STATIC_KEYS}
    f = {k: np.ascontiguousarray(np.asarray(v, np.float64)) for k, v in forcing.items()}
    out, _ = OC.run_oracle_c(cfg, st, f, nsteps, clock=(jd, tsn), frames=frames, hist=True, state=state, qc=qc,
                             qc_every=qc_every)
    return out


def fp64_baseline_flips(c_out: dict, ref: dict, rtol: float = 1e-5, cfg: dict | None = None) -> int:
    """Melt-out flips of the C oracle against the numpy oracle (or the reference);
    with `cfg`, depletion steps (depletion_steps) are explained as for the GPU."""
    names = [v for v in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH") if v in ref]
    c_o, r_o = {v: c_out[v] for v in names}, {v: ref[v] for v in names}
    ex = depletion_steps(c_o, r_o, cfg, rtol, OUT_EPS_F64) if cfg is not None and len(names) == 6 else None
    flip, genuine = melt_out_flips(c_o, r_o, rtol, ex)
    assert not genuine, f"C oracle vs numpy oracle: {genuine[:5]}"
    return int((flip >= 0).sum())


# Melt onset in the fp32 engine.  SM = E_rem / (dt rho_H2O Lf) with E_rem =
# max(Q_sum dt - Eccs, 0) (:1364-1368): where the step's energy just exceeds the
# cold content the difference cancels.  Both sides of it carry the error of
# the fp32 flux terms (a few 1e-7 of their magnitude: hardware exp2/log2/rcp,
# polynomial atan; mean bias -4e-8, HISTORY.md section 3): E_in of this step, and
# Eccs, which integrates E_in over the steps before.  Such a mismatch is
# explained when SM and M_total (:1441) differ by no more than 1e-6 of the
# energy moved so far, sum over steps <= k of |Qn_SW| + |Qn_LW| + |Qh| + |Qe|,
# in melt-rate units (E / (dt rho_H2O Lf) per step of E = Q dt); the cell is
# then compared up to that step, like a melt-out flip.  At most ONSET_FRAC_MAX
# of the cells may need it (the year-long test measures 0.2 % for SM).
ONSET_FRAC_MAX = 0.005


def melt_onsets(gpu: dict, ref: dict, genuine: list, cfg: dict) -> tuple[dict, list]:
    """Split genuine failures into explained melt onsets {cell: step} and the rest."""
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    rho_lf = float(c["rho_H2O"]) * float(c["Lf"])
    onset, rest = {}, []
    for cell, k, vars_ in genuine:
        ok = bool(vars_) and set(vars_) <= {"SM", "M_total"} and all(t in ref for t in ("Qn_SW", "Qn_LW", "Qh", "Qe"))
        if ok:
            moved = sum(np.abs(np.asarray(ref[t])[:k + 1, cell]).sum() for t in ("Qn_SW", "Qn_LW", "Qh", "Qe"))
            bound = 1e-6 * float(moved) / rho_lf
            for v in ("SM", "M_total"):
                d = abs(float(np.asarray(gpu[v])[k, cell]) - float(np.asarray(ref[v])[k, cell]))
                ok &= d <= bound + 1e-7 * abs(float(np.asarray(ref[v])[k, cell]))
        if ok:
            onset[cell] = k
        else:
            rest.append((cell, k, vars_))
    return onset, rest


def valid_mask(flip: np.ndarray, nsteps: int) -> np.ndarray:
    """[nsteps][ncell] True where a cell has not yet flipped."""
    k = np.arange(nsteps)[:, None]
    return (flip[None, :] < 0) | (k < flip[None, :])


def classify_sample(gpu: dict, ref: dict, c64: dict, cfg: dict, tol: float, onsets: bool) -> SimpleNamespace:
    """Every rule of a parity check on one sample, as the GPU suite, smoke and
    each bench rank apply them: depletion steps, melt-out flips (held to the
    fp64 baseline c64 of the same cells and steps), and with `onsets` (the
    fp32 engine) melt onsets.  Returns the per-entry compare mask `ok`
    ([nsteps][ncell]: not excused, cell not yet cut) with the classifications."""
    names = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
    c64 = {v: c64[v] for v in names}
    ex64 = depletion_steps(c64, ref, cfg, tol, OUT_EPS_F64)
    flip64, genuine64 = melt_out_flips(c64, ref, tol, ex64)
    excused = depletion_steps(gpu, ref, cfg, tol, OUT_EPS_F32 if tol >= 1e-7 else OUT_EPS_F64)
    flip, genuine = melt_out_flips(gpu, ref, tol, excused)
    onset = {}
    if onsets and genuine:
        onset, genuine = melt_onsets(gpu, ref, genuine, cfg)
    cut = flip.copy()
    for c_, k_ in onset.items():
        cut[c_] = k_
    nsteps, ncell = np.asarray(ref["SM"]).shape
    return SimpleNamespace(excused=excused, flip=flip, genuine=genuine, onset=onset, cut=cut,
                           ok=valid_mask(cut, nsteps) & ~excused, ex64=ex64, flip64=flip64, genuine64=genuine64,
                           onset_ok=len(onset) <= int(np.ceil(ONSET_FRAC_MAX * ncell)))


# "float32-fluxf64": the fp32 engine's fp64-flux form (tfg_set_flux), as a third engine name of the tests
FLUX_F64_ENGINE = "float32-fluxf64"


def split_engine(engine: str) -> tuple[str, str]:
    """(engine, flux) of a test engine name."""
    return ("float32", "fp64") if engine == FLUX_F64_ENGINE else (engine, "fp32")


def make_engine(cfg: dict, ny: int, nx: int, engine: str, n_frames: int, hist_depth: int, n_catch: int = 1,
                fuse_steps: int = 24, row0: int = 0, flux: str = "fp32", split: str | None = None):
    """split: tfg_set_split's mode; by default "auto", or TFG_TEST_SPLIT ("on": every
    fp32 grid of the suite stepped as two parts on two streams, a stress run)."""
    from topoflow_glacier.engine import GlacierEngine

    split = split or os.environ.get("TFG_TEST_SPLIT", "auto")

    engine, f = split_engine(engine)
    return GlacierEngine(cfg_object(cfg), ny, nx, engine=engine, device=0, n_frames=n_frames,
                         hist_depth=hist_depth, n_catch=n_catch, fuse_steps=fuse_steps, row0=row0,
                         flux=f if f == "fp64" else flux, split=split)


def gpu_run_fields(cfg: dict, static: dict, forcing: dict, ny: int, nx: int, engine: str, nsteps: int,
                   fuse_steps: int = 24, catch_id=None, n_catch: int = 1, chunks=None, window: bool = False):
    """Run the GPU engine on explicit per-step forcing (one frame per step).

    Returns (dict name -> [nsteps][ncell] outputs, state dict, diagnostics),
    plus the snowfall-window slots [ring_len][ncell] when `window`."""
    n = ny * nx
    eng = make_engine(cfg, ny, nx, engine, n_frames=nsteps, hist_depth=nsteps, n_catch=n_catch, fuse_steps=fuse_steps)
    try:
        for k in ("elev", "slope", "aspect"):
            eng.set_field(k, static[k])
        for k in ("h_snow", "h_ice", "h_swe", "h_iwe"):
            eng.set_field(k, static["h0_" + k[2:]])
        if catch_id is not None:
            eng.set_field("catch_id", catch_id)
        eng.init_state()
        for k in range(nsteps):
            for name in ("P", "T_air", "Hum_sp", "P_air", "uz"):
                eng.set_field(name, np.asarray(forcing[name][k]).reshape(n), index=k)
        frames = np.arange(nsteps, dtype=np.int32)
        if chunks is None:
            eng.run(nsteps, frames=frames)
        else:
            done = 0
            for c in chunks:
                eng.run(c, frames=frames[done:done + c])
                done += c
        eng.sync()
        outs = {name: np.stack([eng.get_field(name, index=k) for k in range(nsteps)])
                for name in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")}
        state = {name: eng.get_field(name) for name in ("h_swe", "h_iwe", "Eccs", "Ecci", "albedo", "n")}
        diag = eng.diagnostics()
        window = np.stack([eng.get_field("window", index=j) for j in range(eng.ring_len)]) if window else None
        return (outs, state, diag, window) if window is not None else (outs, state, diag)
    finally:
        eng.close()


def synthetic_inputs(seed: int, ny: int, nx: int, n_frames: int, row0: int = 0):
    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    d = diurnal_table(n_frames)
    cells = (np.arange(ny)[:, None] + row0) * nx + np.arange(nx)[None, :]
    return synthetic_cells(seed, cells.reshape(-1), d), d


def oracle_synthetic(seed: int, ny: int, nx: int, nsteps: int, n_frames: int = 24, row0: int = 0,
                     cfg_over: dict | None = None, cold=None, qc=None, conduction=None):
    """The oracle on the synthetic workload (host mirror of the device
    generator) for rows row0..row0+ny-1 of a grid nx wide.

    Optional lateral conduction (tests of tfg_conduction_*): `cold` = initial
    (Eccs, Ecci) [ncell] replacing initialize()'s; `qc` = a fixed Qc [ncell];
    `conduction` = dict(k_snow, k_ice, dx, dy, every): Qc re-evaluated from the
    oracle's own state every `every` steps (conduction_restated).  The Qc rows
    used are returned as m.qc_rows."""
    cfg = dict(BASE_CFG)
    cfg.update(cfg_over or {})
    syn, _ = synthetic_inputs(seed, ny, nx, n_frames, row0=row0)
    frames = np.arange(nsteps) % n_frames
    forcing = {k: syn[k][frames].astype(np.float64) for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    static = {"elev": syn["elev"], "slope": syn["slope"], "aspect": syn["aspect"],
              "h0_snow": syn["h_snow"], "h0_ice": syn["h_ice"], "h0_swe": syn["h_swe"], "h0_iwe": syn["h_iwe"]}
    static = {k: np.asarray(v, dtype=np.float64) for k, v in static.items()}
    if cold is None and qc is None and conduction is None:
        return oracle_run(cfg, static, forcing, nsteps)
    m = O.OracleGrid(cfg, **static)
    if cold is not None:
        m.Eccs, m.Ecci = (np.asarray(a, np.float64).copy() for a in cold)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], nsteps, cfg["lon"])
    m.qc_rows = []
    if qc is not None:
        m.Qc = np.asarray(qc, np.float64)
        m.qc_rows.append(m.Qc)
    out = {}
    for k in range(nsteps):
        if conduction is not None and k % conduction["every"] == 0:
            shape = (ny, nx)
            m.Qc = conduction_restated(m.h_swe.reshape(shape), m.h_iwe.reshape(shape), m.Eccs.reshape(shape),
                                       m.Ecci.reshape(shape), cfg, conduction["k_snow"], conduction["k_ice"],
                                       conduction["dx"], conduction["dy"]).reshape(-1)
            m.qc_rows.append(m.Qc)
        r = m.step(*(forcing[n][k] for n in ("P", "T_air", "Hum_sp", "P_air", "uz")), jd[k], tsn[k])
        for key, v in r.items():
            out.setdefault(key, []).append(np.array(v, copy=True))
    return {key: np.stack(v) for key, v in out.items()}, m


def catchment_diag(syn: dict, m, cid: np.ndarray, nsteps: int, n_frames: int, n_catch: int, cfg: dict) -> np.ndarray:
    """[n_catch][6] per-catchment vol_P, vol_PR, vol_PS, vol_SM, vol_IM, P_max
    of an oracle run over synthetic cells (:558-624, :1482-1494 summed per
    catchment): the precipitation terms binned from the forcing frames the
    steps read, the melt integrals from the oracle's per-cell contributions."""
    c = dict(BASE_CFG)
    c.update(cfg)
    frames = np.arange(nsteps) % n_frames
    P = syn["P"][frames].astype(np.float64)
    rain = syn["T_air"][frames].astype(np.float64) > float(c["T_rain_snow"])
    f = float(c["da"]) * 1e6 * float(c["dt"])
    out = np.zeros((n_catch, 6))
    for col, w in enumerate((P, np.where(rain, P, 0.0), np.where(rain, 0.0, P))):
        out[:, col] = np.bincount(cid, weights=(w * f).sum(axis=0), minlength=n_catch)
    n = cid.size
    out[:, 3] = np.bincount(cid, weights=np.broadcast_to(m.cell_vol_SM, (n,)), minlength=n_catch)
    out[:, 4] = np.bincount(cid, weights=np.broadcast_to(m.cell_vol_IM, (n,)), minlength=n_catch)
    pmax = P.max(axis=0)
    for k in range(n_catch):
        sel = cid == k
        out[k, 5] = pmax[sel].max() if sel.any() else 0.0
    return out


def oracle_diag(m) -> np.ndarray:
    """[1][6] diagnostics row of an oracle model (vol_P, PR, PS, SM, IM, P_max)."""
    return np.array([[m.vol_P, m.vol_PR, m.vol_PS, m.vol_SM, m.vol_IM, m.P_max]], dtype=np.float64)


def run_gpu_vs_oracle(ny: int, nx: int, nsteps: int, engine: str = "float32", seed: int = 7,
                      n_frames: int = 24, fuse_steps: int = 24, cfg_over: dict | None = None,
                      cold=None, qc=None, conduction=None):
    """Device-generated synthetic workload on the GPU vs the oracle on the same
    fp32 inputs (host mirror).  Returns a report dict.  `cold`, `qc` and
    `conduction` switch on the optional lateral conduction term on both sides
    (oracle_synthetic)."""
    cfg = dict(BASE_CFG)
    cfg.update(cfg_over or {})
    syn, diurnal = synthetic_inputs(seed, ny, nx, n_frames)
    eng = make_engine(cfg, ny, nx, engine, n_frames=n_frames, hist_depth=nsteps, fuse_steps=fuse_steps)
    try:
        eng.fill_synthetic(seed, diurnal)
        if cold is not None:
            eng.set_field("Eccs", cold[0])
            eng.set_field("Ecci", cold[1])
        if qc is not None:
            eng.set_field("Qc", qc)
        if conduction is None:
            eng.run(nsteps)
        else:
            for k0 in range(0, nsteps, conduction["every"]):
                eng.conduction_update(conduction["k_snow"], conduction["k_ice"], conduction["dx"], conduction["dy"])
                eng.run(min(conduction["every"], nsteps - k0))
        eng.sync()
        gpu = {name: np.stack([eng.get_field(name, index=k) for k in range(nsteps)])
               for name in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")}
        gpu["h_swe"] = eng.get_field("h_swe")
        gpu["h_iwe"] = eng.get_field("h_iwe")
        diag = eng.diagnostics()
    finally:
        eng.close()
    ref, m = oracle_synthetic(seed, ny, nx, nsteps, n_frames, cfg_over=cfg_over, cold=cold, qc=qc,
                              conduction=conduction)
    static = {"elev": syn["elev"], "slope": syn["slope"], "aspect": syn["aspect"], "h0_snow": syn["h_snow"],
              "h0_ice": syn["h_ice"], "h0_swe": syn["h_swe"], "h0_iwe": syn["h_iwe"]}
    state = None
    if cold is not None:  # the same initial state for the C oracle, with initialize()'s window and albedo
        m0 = O.OracleGrid(cfg, **{k: np.asarray(v, np.float64) for k, v in static.items()})
        state = {"h_snow": m0.h_snow, "h_ice": m0.h_ice, "h_swe": m0.h_swe, "h_iwe": m0.h_iwe, "Eccs": cold[0],
                 "Ecci": cold[1], "albedo": m0.albedo, "n": m0.n, "ring": m0.ring}
    qc_rows = getattr(m, "qc_rows", None) or None
    c64 = c_oracle_hist(cfg, static, {k: syn[k] for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}, nsteps,
                        frames=np.arange(nsteps) % n_frames, state=state,
                        qc=None if qc_rows is None else np.stack(qc_rows),
                        qc_every=conduction["every"] if conduction is not None else max(nsteps, 1))
    report = {}
    worst = 0.0
    worst_rel = 0.0
    fp32 = split_engine(engine)[0] == "float32"
    tol = 1e-5 if fp32 else 1e-10
    excused = depletion_steps(gpu, ref, cfg, tol, OUT_EPS_F32 if fp32 else OUT_EPS_F64)
    flip, genuine = melt_out_flips(gpu, ref, tol, excused)
    onset = {}
    # TFG_STRICT_ONSET=1: no onset allowance (to list the tests that need it); never for the fp64 flux
    if engine == "float32" and genuine and os.environ.get("TFG_STRICT_ONSET") != "1":
        onset, genuine = melt_onsets(gpu, ref, genuine, cfg)
    cut = flip.copy()
    for cell, k in onset.items():
        cut[cell] = k
    mask = valid_mask(cut, nsteps) & ~excused
    for name in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH"):
        e, frac = parity(gpu[name], ref[name], mask=mask)
        report[name] = (e, frac)
        worst = max(worst, e)
    for name in ("h_swe", "h_iwe"):
        e, frac = parity(gpu[name], ref[name][-1], mask=cut < 0)
        report[name] = (e, frac)
        worst = max(worst, e)
    dref = np.array([m.vol_P, m.vol_PR, m.vol_PS, m.vol_SM, m.vol_IM, m.P_max])
    dg = diag.sum(axis=0)
    dg[5] = diag[:, 5].max()
    with np.errstate(divide="ignore", invalid="ignore"):
        drel = np.where(dref != 0, np.abs(dg - dref) / np.abs(dref), np.abs(dg - dref))
    # vol_IM sums IM over all cells including flipped ones: compare P-volumes strictly
    report["diag"] = (float(np.max(drel[[0, 1, 2, 5]])), 0.0)
    worst_rel = max(worst, report["diag"][0])
    n_flip = int((flip >= 0).sum())
    rule = flip_rule(n_flip, fp64_baseline_flips(c64, ref, tol, cfg))
    onset_ok = len(onset) <= int(np.ceil(ONSET_FRAC_MAX * flip.size))
    ok = worst_rel <= tol and not genuine and rule["ok"] and onset_ok
    summary = (", ".join(f"{k}={v[0]:.2e}" for k, v in report.items())
               + f", melt-out flips={n_flip}/{flip.size} (fp64 baseline {rule['fp64_flips']}, budget {rule['budget']})"
               + (f", melt onsets within fp32 flux rounding={len(onset)}" if onset else ""))
    if genuine:
        summary += f", FAILURES={genuine[:5]}"
    return {"ok": ok, "max_rel": worst_rel, "report": report, "summary": summary, "gpu": gpu, "ref": ref,
            "diag": dg, "diag_ref": dref, "flips": n_flip, "genuine": genuine, "flip_rule": rule, "onsets": onset}


def terrain_dem(ny: int, nx: int) -> np.ndarray:
    """A smooth synthetic DEM [m] (hills and a tilted plane) on 30 m cells, fp32-exact."""
    y, x = np.mgrid[0:ny, 0:nx].astype(np.float64)
    z = 2000.0 + 0.3 * x - 0.2 * y + 150.0 * np.sin(x / 17.0) * np.cos(y / 23.0) + 80.0 * np.exp(-((x - nx / 3) ** 2 + (y - ny / 2) ** 2) / 400.0)
    return z.astype(np.float32).astype(np.float64)


def terrain_oracle(dem: np.ndarray, dx: float, dy: float, north=None, south=None):
    """Horn's 3x3 slope (tan beta) and aspect (downslope direction, radians CCW
    from east), fp64 numpy: the restatement tfg_terrain_from_dem is checked
    against.  Rows run north to south; missing halo rows / edge columns
    replicate the edge."""
    z = np.asarray(dem, dtype=np.float64)
    n = z[0] if north is None else np.asarray(north, dtype=np.float64)
    s_ = z[-1] if south is None else np.asarray(south, dtype=np.float64)
    p = np.vstack([n[None, :], z, s_[None, :]])
    p = np.hstack([p[:, :1], p, p[:, -1:]])
    a, b, c = p[:-2, :-2], p[:-2, 1:-1], p[:-2, 2:]
    d, f = p[1:-1, :-2], p[1:-1, 2:]
    g, h, i = p[2:, :-2], p[2:, 1:-1], p[2:, 2:]
    dzdx = ((c + 2.0 * f + i) - (a + 2.0 * d + g)) * (1.0 / (8.0 * dx))
    dzds = ((g + 2.0 * h + i) - (a + 2.0 * b + c)) * (1.0 / (8.0 * dy))
    slope = np.sqrt(dzdx * dzdx + dzds * dzds)
    aspect = np.where((dzdx == 0) & (dzds == 0), 0.0, np.arctan2(dzds, -dzdx))
    return slope, aspect


def ns(**kw):
    return SimpleNamespace(**kw)


# ---------------------------------------------------------------- optional ice flow (tfg_ice_flow_*)
def ice_flow_gamma(cfg: dict) -> float:
    """Gamma = 2A/5 (rho_ice g)^3 for Glen's law n = 3, as tfg_create folds it."""
    c = cfg_object(cfg)
    rg = c.rho_ice * c.g
    return 2.0 * c.glens_A / 5.0 * (rg * rg * rg)


def _flow_faces(elev, iwe, wi, gamma, dx, dy, north, south):
    """Face normal/tangential gradients and thicknesses of one shard (numpy
    restatement of k_ice_flow's flow_grad_x / flow_grad_y, same op order)."""
    iwe = np.asarray(iwe, np.float64)
    H = iwe * wi
    S = np.asarray(elev, np.float64) + iwe * wi
    Sn = S[0] if north is None else np.asarray(north[0], np.float64)
    Ss = S[-1] if south is None else np.asarray(south[0], np.float64)
    Hn = H[0] if north is None else np.asarray(north[1], np.float64)
    Hs = H[-1] if south is None else np.asarray(south[1], np.float64)
    P = np.vstack([Sn[None], S, Ss[None]])
    P = np.hstack([P[:, :1], P, P[:, -1:]])  # rows -1..ny, columns -1..nx (edge replicated)
    Hp = np.vstack([Hn[None], H, Hs[None]])
    gnx = (P[1:-1, 2:-1] - P[1:-1, 1:-2]) * (1.0 / dx)
    gtx = ((P[2:, 1:-2] - P[:-2, 1:-2]) + (P[2:, 2:-1] - P[:-2, 2:-1])) * (1.0 / (4.0 * dy))
    gny = (P[1:, 1:-1] - P[:-1, 1:-1]) * (1.0 / dy)
    gty = ((P[:-1, 2:] - P[:-1, :-2]) + (P[1:, 2:] - P[1:, :-2])) * (1.0 / (4.0 * dx))
    return H, Hp, gnx, gtx, gny, gty


def _face_D(Ha, Hb, gn, gt, gamma):
    Hf = 0.5 * (Ha + Hb)
    h2 = Hf * Hf
    h5 = (h2 * h2) * Hf
    return (gamma * h5) * (gn * gn + gt * gt)


def _face_q(Ha, Hb, gn, gt, gamma, dn, dt):
    q = -(_face_D(Ha, Hb, gn, gt, gamma) * gn)
    Hd = np.where(q > 0.0, Ha, Hb)
    qlim = Hd * (dn / (4.0 * dt))
    return np.minimum(np.maximum(q, -qlim), qlim)


def ice_flow_step_restated(elev, iwe, wi, gamma, dx, dy, dt, north=None, south=None):
    """One explicit shallow-ice sub-step of a [ny][nx] shard: the numpy
    restatement tfg_ice_flow_step is checked against (test infrastructure)."""
    H, Hp, gnx, gtx, gny, gty = _flow_faces(elev, iwe, wi, gamma, dx, dy, north, south)
    ny, nx = H.shape
    qx = _face_q(H[:, :-1], H[:, 1:], gnx, gtx, gamma, dx, dt)  # faces (r, c+1/2)
    qy = _face_q(Hp[:-1], Hp[1:], gny, gty, gamma, dy, dt)     # faces (r+1/2, c), r = -1..ny-1
    if north is None:
        qy[0] = 0.0
    if south is None:
        qy[-1] = 0.0
    z = np.zeros((ny, 1))
    qE = np.hstack([qx, z])
    qW = np.hstack([z, qx])
    div = (qE - qW) * (1.0 / dx) + (qy[1:] - qy[:-1]) * (1.0 / dy)
    return np.maximum(np.asarray(iwe, np.float64) - (dt / wi) * div, 0.0)


def ice_flow_dmax_restated(elev, iwe, wi, gamma, dx, dy, north=None, south=None):
    H, Hp, gnx, gtx, gny, gty = _flow_faces(elev, iwe, wi, gamma, dx, dy, north, south)
    Dx = _face_D(H[:, :-1], H[:, 1:], gnx, gtx, gamma)
    Dy = _face_D(Hp[:-1], Hp[1:], gny, gty, gamma)
    lo, hi = (0 if north is not None else 1), (Dy.shape[0] if south is not None else Dy.shape[0] - 1)
    return float(max(Dx.max(initial=0.0), Dy[lo:hi].max(initial=0.0)))


class RestatedFlowShard:
    """A CPU stand-in with GlacierEngine's ice_flow_* methods, backed by the
    restatement: lets the sharded orchestration (sharding.ice_flow) run under
    gloo on CPU.  Test infrastructure."""

    def __init__(self, elev, iwe, wi, gamma):
        self.elev = np.asarray(elev, np.float64)
        self.iwe = np.asarray(iwe, np.float64).copy()
        self.wi, self.gamma = wi, gamma
        self.ny, self.nx = self.iwe.shape

    def ice_flow_edges(self):
        S = self.elev + self.iwe * self.wi
        H = self.iwe * self.wi
        return np.stack([S[0], H[0]]), np.stack([S[-1], H[-1]])

    def ice_flow_dmax(self, dx, dy, north=None, south=None):
        return ice_flow_dmax_restated(self.elev, self.iwe, self.wi, self.gamma, dx, dy, north, south)

    def ice_flow_step(self, dt, dx, dy, north=None, south=None, part=0):
        if part == 1:  # FLOW_INTERIOR: the restatement steps whole shards (in the FLOW_EDGES call)
            return
        self.iwe = ice_flow_step_restated(self.elev, self.iwe, self.wi, self.gamma, dx, dy, dt, north, south)


def glacier_valley(ny: int, nx: int, dx: float = 100.0):
    """A bed tilted down-valley with a valley glacier on it: (bed [m] fp32-exact,
    ice water equivalent h_iwe [m])."""
    y, x = np.mgrid[0:ny, 0:nx].astype(np.float64)
    bed = 3000.0 - 0.08 * dx * y + 0.002 * (x - nx / 2) ** 2 * dx
    H = np.maximum(0.0, 220.0 * (1.0 - ((x - nx / 2) / (0.35 * nx)) ** 2 - ((y - 0.4 * ny) / (0.45 * ny)) ** 2))
    return bed.astype(np.float32).astype(np.float64), H * (917.0 / 1000.0)


# ----------------------------------------------------------------------------
# Optional lateral heat conduction (tfg_conduction_*; extension with no
# reference counterpart beyond the reserved Qc term, :936-948, :1314).  numpy
# fp64 restatement of tfg_conduction.hpp, same operation order.
# ----------------------------------------------------------------------------
def conduction_cells(swe, iwe, eccs, ecci, cfg: dict):
    """(T_snow, h_snow, T_ice, h_ice) per cell from the state (:389-395, :1711, :1726)."""
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    ws = np.float64(c["rho_H2O"]) / np.float64(c["rho_snow"])
    wi = np.float64(c["rho_H2O"]) / np.float64(c["rho_ice"])
    inv_cs = 1.0 / (np.float64(c["rho_snow"]) * np.float64(c["Cp_snow"]))
    inv_ci = 1.0 / ((np.float64(c["rho_ice"]) * np.float64(c["Cp_ice"])) * np.float64(c["h_active_layer"]))
    T0 = np.float64(c["T0"])
    hs = np.asarray(swe, np.float64) * ws
    hi = np.asarray(iwe, np.float64) * wi
    with np.errstate(divide="ignore", invalid="ignore"):
        Ts = np.where(hs > 0, T0 - (np.asarray(eccs, np.float64) * inv_cs) / hs, T0)
    Ti = np.where(hi > 0, T0 - np.asarray(ecci, np.float64) * inv_ci, T0)
    return Ts, hs, Ti, hi


def conduction_restated(swe, iwe, eccs, ecci, cfg: dict, k_snow: float, k_ice: float, dx: float, dy: float,
                        north=None, south=None, q_ground: float = 0.0):
    """Qc [W m-2] of a [ny][nx] shard; north/south halo rows [4][nx] (T_snow,
    h_snow, T_ice, h_ice) or None at the domain edge (no flux)."""
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    h_al = np.float64(c["h_active_layer"])
    Ts, hs, Ti, hi = conduction_cells(swe, iwe, eccs, ecci, cfg)
    ny, nx = Ts.shape

    def padded(a, k):
        n = np.zeros(nx) if north is None else np.asarray(north, np.float64).reshape(4, nx)[k]
        s = np.zeros(nx) if south is None else np.asarray(south, np.float64).reshape(4, nx)[k]
        p = np.vstack([n[None], a, s[None]])
        return np.hstack([np.zeros((ny + 2, 1)), p, np.zeros((ny + 2, 1))])

    P = [padded(a, k) for k, a in enumerate((Ts, hs, Ti, hi))]
    gsx, gsy = k_snow / (dx * dx), k_snow / (dy * dy)
    gix, giy = k_ice * h_al / (dx * dx), k_ice * h_al / (dy * dy)
    qs = np.zeros((ny, nx))
    qi = np.zeros((ny, nx))
    for (r, cc), gs, gi in (((0, 1), gsy, giy), ((2, 1), gsy, giy), ((1, 0), gsx, gix), ((1, 2), gsx, gix)):
        nTs, nhs, nTi, nhi = (p[r:r + ny, cc:cc + nx] for p in P)
        ms = (hs > 0) & (nhs > 0)
        qs = np.where(ms, qs + (np.minimum(hs, nhs) * (nTs - Ts)) * gs, qs)
        mi = (hi > 0) & (nhi > 0)
        qi = np.where(mi, qi + (nTi - Ti) * gi, qi)
    return (qs + qi) + q_ground


class RestatedCondShard:
    """A row-block shard of the conduction restatement with the engine's
    conduction_* interface (for sharding.lateral_conduction on CPU)."""

    def __init__(self, swe, iwe, eccs, ecci, cfg: dict):
        self.state = [np.asarray(a, np.float64) for a in (swe, iwe, eccs, ecci)]
        self.cfg = cfg
        self.nx = self.state[0].shape[1]
        self.qc = None

    def conduction_edges(self):
        cells = conduction_cells(*self.state, self.cfg)
        return np.stack([a[0] for a in cells]), np.stack([a[-1] for a in cells])

    def conduction_update(self, k_snow, k_ice, dx, dy, north=None, south=None, q_ground=0.0):
        self.qc = conduction_restated(*self.state, self.cfg, k_snow, k_ice, dx, dy, north, south, q_ground)


def conduction_state(ny: int, nx: int, seed: int = 3):
    """A [ny][nx] state with snow-free and ice-free patches and varied cold
    contents: h_swe, h_iwe [m w.e.], Eccs, Ecci [J m-2]."""
    rng = np.random.default_rng(seed)
    swe = rng.uniform(0.0, 0.5, (ny, nx))
    swe[rng.random((ny, nx)) < 0.2] = 0.0
    iwe = rng.uniform(0.0, 2.0, (ny, nx))
    iwe[rng.random((ny, nx)) < 0.2] = 0.0
    eccs = np.where(swe > 0, rng.uniform(0.0, 2.0e6, (ny, nx)), 0.0)
    ecci = np.where(iwe > 0, rng.uniform(0.0, 1.0e6, (ny, nx)), 0.0)
    return swe, iwe, eccs, ecci
