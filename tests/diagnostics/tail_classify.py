"""Classify the largest compared entries of parity_tail.py dumps (CPU).

For every compared entry (cell not cut, step not excused) above `thr` of the
floored error, the kind of step it sits on:
  depletion  a reservoir empties at this step in the reference (its depth was
             > 0 at the step before and is 0 now): the rate carries the depth's
             error (tests/harness.py depletion_steps)
  split      at or after the step where exactly one trajectory holds a depth
             of exactly zero and the other a sub-1e-9 m residual (the melt-out
             gates diverged; harness.melt_out_flips (b))
  onset      SM starts (reference SM 0 at the step before, > 0 now)
  ordinary   anything else
  python tests/diagnostics/tail_classify.py DUMP.npz [DUMP.npz ...] [--thr 7e-6] [--reclassify]
With --reclassify the dump's cells are classified again by the current
tests/harness.py rules (the dump's own `ok` mask is from the rules of the run
that wrote it), with the whole-sample floors the dump kept.
Diagnostic only.
"""
import sys

from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
NAMES = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")


def reclassify(z):
    """The compare mask of the dump's cells under the current harness rules."""
    sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "topoflow-glacier_amd")]
    import bench
    import tests.harness as H

    fl = dict(zip([str(x) for x in z["names"]], z["floors"]))
    G = {v: np.ascontiguousarray(z["gpu_" + v], dtype=np.float64) for v in NAMES}
    R = {v: np.ascontiguousarray(z["ref_" + v], dtype=np.float64) for v in NAMES}
    C = {v: np.ascontiguousarray(z["c64_" + v], dtype=np.float64) for v in NAMES}
    for t in ("Qn_SW", "Qn_LW", "Qh", "Qe"):
        R[t] = z["ref_" + t]
    ids = {id(R[v]): fl[v] for v in NAMES}
    orig = H.scale_floor
    H.scale_floor = lambda a: ids[id(a)] if id(a) in ids else orig(a)  # the whole sample's floors
    try:
        dt = 0.25 if "--dt 0.25" in str(z["args"]) else 1.0
        cls = H.classify_sample(G, R, C, dict(bench.BASE_CFG, dt=dt), 1e-5, True)
    finally:
        H.scale_floor = orig
    return cls.ok, len(cls.genuine)


def classify(z, thr, ok=None):
    fl = dict(zip([str(x) for x in z["names"]], z["floors"]))
    ok = z["ok"] if ok is None else ok
    G = {v: z["gpu_" + v] for v in NAMES}
    R = {v: z["ref_" + v] for v in NAMES}
    nsteps, ncell = R["SM"].shape
    split = np.full(ncell, nsteps)
    for v in ("h_snow", "h_ice"):
        g, r = np.abs(G[v]), np.abs(R[v])
        d = ((g == 0) != (r == 0)) & (np.maximum(g, r) <= 1e-9)
        split = np.minimum(split, np.where(d.any(axis=0), np.argmax(d, axis=0), nsteps))
    rows = []
    for v in NAMES:
        e = np.abs(G[v] - R[v]) / np.maximum(np.maximum(np.abs(R[v]), fl[v]), 1e-300)
        e = np.where(ok, e, 0.0)
        for k, c in zip(*np.nonzero(e > thr)):
            kind = "ordinary"
            prev = lambda a: a[k - 1, c] if k > 0 else np.nan  # noqa: E731
            if split[c] <= k:
                kind = "split"
            elif v in ("SM", "IM", "M_total") and ((R["h_snow"][k, c] == 0 and prev(R["h_snow"]) > 0)
                                                    or (R["h_ice"][k, c] == 0 and prev(R["h_ice"]) > 0)):
                kind = "depletion"
            elif v in ("SM", "M_total") and prev(R["SM"]) == 0 and R["SM"][k, c] > 0:
                kind = "onset"
            rows.append((float(e[k, c]), v, int(c), int(k), kind))
    rows.sort(reverse=True)
    return rows


def main():
    files = [a for a in sys.argv[1:] if a.endswith(".npz")]
    thr = float(sys.argv[sys.argv.index("--thr") + 1]) if "--thr" in sys.argv else 7e-6
    for f in files:
        z = np.load(f)
        ok, ngen = reclassify(z) if "--reclassify" in sys.argv else (None, None)
        rows = classify(z, thr, ok)
        kinds = {}
        for r in rows:
            kinds.setdefault(r[4], []).append(r[0])
        print(f"{f}: {z['args']}  flips {int(z['n_flips'])}/{int(z['n_flips64'])} excused {int(z['n_excused'])} "
              f"onsets {int(z['n_onsets'])}  max {z['worst'][0]:.4e}  fp64 baseline max {float(z['c64_max_floored']):.4e}"
              + (f"  reclassified: max {rows[0][0] if rows else 0.0:.4e} genuine {ngen}" if ok is not None else ""))
        for kind, es in sorted(kinds.items()):
            print(f"   {kind:9s} entries > {thr:.0e}: {len(es):4d}   max {max(es):.4e}")
        for e, v, c, k, kind in rows[:8]:
            print(f"     {e:.4e} {v:8s} cell {z['cells'][c]:7d} step {k:4d} {kind}")


if __name__ == "__main__":
    main()
