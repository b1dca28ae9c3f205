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
  python tests/diagnostics/tail_classify.py DUMP.npz [DUMP.npz ...] [--thr 7e-6]
Diagnostic only.
"""
import sys

import numpy as np

NAMES = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")


def classify(z, thr):
    fl = dict(zip([str(x) for x in z["names"]], z["floors"]))
    ok = z["ok"]
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
        rows = classify(z, thr)
        kinds = {}
        for r in rows:
            kinds.setdefault(r[4], []).append(r[0])
        print(f"{f}: {z['args']}  flips {int(z['n_flips'])}/{int(z['n_flips64'])} excused {int(z['n_excused'])} "
              f"onsets {int(z['n_onsets'])}  max {z['worst'][0]:.4e}  fp64 baseline max {float(z['c64_max_floored']):.4e}")
        for kind, es in sorted(kinds.items()):
            print(f"   {kind:9s} entries > {thr:.0e}: {len(es):4d}   max {max(es):.4e}")
        for e, v, c, k, kind in rows[:8]:
            print(f"     {e:.4e} {v:8s} cell {z['cells'][c]:7d} step {k:4d} {kind}")


if __name__ == "__main__":
    main()
