"""Device time of the one-cell fp64 k_fused launch against the number of steps
it fuses (run under rocprofv3 --kernel-trace): separates the per-step
arithmetic from the per-launch fixed cost (state load/store, the diagnostic
slab, launch).  Diagnostic only.
  rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python tests/diagnostics/one_cell_step_cost.py
then  python tests/diagnostics/one_cell_step_cost.py --summary OUT"""
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle")]
KS = (1, 2, 4, 8)
REPS = 40

if len(sys.argv) > 2 and sys.argv[1] == "--summary":
    rows = []
    for f in glob.glob(f"{sys.argv[2]}/**/*kernel_trace.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "k_fused<double, true" in r["Kernel_Name"] or "k_cell_run" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    d = d[len(d) - len(KS) * REPS:]  # the timed launches (the warm-up ones come first)
    res = {}
    for i, k in enumerate(KS):
        v = sorted(d[i * REPS:(i + 1) * REPS])
        res[k] = {"median_us": v[len(v) // 2], "min_us": v[0]}
    ks = list(res)
    slope = (res[ks[-1]]["median_us"] - res[ks[0]]["median_us"]) / (ks[-1] - ks[0])
    out = {"launch_us_by_steps": res, "per_step_us": slope, "fixed_us": res[1]["median_us"] - slope}
    print(json.dumps(out, indent=1))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from tests.harness import BASE_CFG, make_engine  # noqa: E402

e = make_engine(dict(BASE_CFG), 1, 1, "float64", n_frames=1, hist_depth=8, fuse_steps=8)
for name, v in (("P", 1e-4), ("T_air", -3.0), ("Hum_sp", 0.003), ("P_air", 88000.0), ("uz", 3.0)):
    e.set_field(name, np.float64(v))
for name in ("elev", "slope", "aspect"):
    e.set_field(name, np.float64(BASE_CFG[name]))
for name, key in (("h_snow", "h0_snow"), ("h_ice", "h0_ice"), ("h_swe", "h0_swe"), ("h_iwe", "h0_iwe")):
    e.set_field(name, np.float64(BASE_CFG[key]))
e.init_state()
for _ in range(5):
    e.run(8)
e.sync()
for k in KS:
    for _ in range(REPS):
        e.run(k, frames=np.zeros(k, dtype=np.int32))
        e.sync()
e.close()
print("done")
