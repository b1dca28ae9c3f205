"""Time the optional lateral conduction term on an ny x nx synthetic grid:
one Qc evaluation (tfg_conduction_update: k_conduction) and a K-step fused
launch with the term on against the same launch with it off.  Diagnostic only.
  python tests/diagnostics/conduction_timing.py [ny] [nx] [reps] [fuse]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle")]
import torch  # noqa: E402,F401  (one HIP runtime: torch's)

from tests.harness import BASE_CFG, make_engine  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table  # noqa: E402

ny = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
nx = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
fuse = int(sys.argv[4]) if len(sys.argv) > 4 else 96
e = make_engine(dict(BASE_CFG), ny, nx, "float32", n_frames=24, hist_depth=fuse, fuse_steps=fuse)
e.fill_synthetic(20251001, diurnal_table(24))
e.run(fuse)  # past the first launch (it reads the initial depths)
e.conduction_update(0.1, 2.1, 30.0, 30.0)  # warm-up
e.sync()
t0 = time.perf_counter()
for _ in range(reps):
    e.conduction_update(0.1, 2.1, 30.0, 30.0)
e.sync()
t_cond = (time.perf_counter() - t0) / reps
launch = {}
for on in (True, False, True, False):
    if on:
        e.conduction_update(0.1, 2.1, 30.0, 30.0)
    else:
        e.conduction_off()
    e.sync()
    t0 = time.perf_counter()
    e.run(fuse)
    e.sync()
    launch.setdefault("on" if on else "off", []).append((time.perf_counter() - t0) * 1e3)
n = ny * nx
# algorithmic bytes per cell of k_conduction: h_swe, h_iwe, Eccs, Ecci read (32), Qc written (4)
bpc = 32 + 4
print(json.dumps({"grid": [ny, nx], "conduction_ms": t_cond * 1e3, "bytes_per_cell": bpc,
                  "GBps": n * bpc / t_cond / 1e9, "fused_launch_ms": launch, "fuse": fuse}))
e.close()
