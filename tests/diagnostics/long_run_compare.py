"""Compare a GPU long run (tests/diagnostics/gpu_long_run.py) with the oracle on CPU.
Prints, per variable, the floored relative error per month of
model time and the fraction of cells above 1e-5.  Test infrastructure."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle")]
from tests.harness import oracle_synthetic, scale_floor  # noqa: E402

z = np.load(sys.argv[1])
n, steps, seed, every = int(z["n"]), int(z["steps"]), int(z["seed"]), int(z["every"])
t0 = time.time()
ref, m = oracle_synthetic(seed, 1, n, steps)
print(f"oracle {n} cells x {steps} steps: {time.time() - t0:.1f} s", flush=True)
idx = np.arange(every - 1, steps, every)
for k in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH"):
    g = z[f"out_{k}"].astype(np.float64)
    r = np.asarray(ref[k])[idx]
    s_v = scale_floor(r)
    e = np.abs(g - r) / np.maximum(np.maximum(np.abs(r), s_v), 1e-300)
    months = [f"{e[i:i + 30].max():.1e}" for i in range(0, len(idx), 30)]
    print(f"{k:8s} max {e.max():.2e}  cells>1e-5 {(e > 1e-5).any(axis=0).mean():.4f}  monthly max: {' '.join(months)}")
print("h_swe final", np.max(np.abs(z["state_h_swe"] - ref["h_swe"][-1]) / np.maximum(np.abs(ref["h_swe"][-1]), scale_floor(ref["h_swe"][-1]))))
dref = np.array([m.vol_P, m.vol_PR, m.vol_PS, m.vol_SM, m.vol_IM, m.P_max])
print("diag rel", np.abs(z["diag"][0] - dref) / np.abs(dref))
