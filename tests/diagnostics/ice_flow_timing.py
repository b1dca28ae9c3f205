"""Time one ice-flow sub-step (tfg_ice_flow_step: k_ice_flow + k_flow_commit)
and the CFL reduction on an ny x nx grid.  Diagnostic only.
  python tests/diagnostics/ice_flow_timing.py [ny] [nx] [reps]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle")]
import torch  # noqa: E402,F401  (one HIP runtime: torch's)

from tests.harness import BASE_CFG, glacier_valley, make_engine  # noqa: E402

ny = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
nx = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
bed, iwe = glacier_valley(ny, nx)
e = make_engine(dict(BASE_CFG), ny, nx, "float32", n_frames=1, hist_depth=1)
e.set_field("elev", bed.reshape(-1).astype(np.float32))
e.set_field("h_iwe", iwe.reshape(-1))
e.init_state()
del bed, iwe
e.ice_flow_step(1e-4, 100.0, 100.0)  # warm-up
t0 = time.perf_counter()
for _ in range(reps):
    e.ice_flow_step(1e-4, 100.0, 100.0)
t_step = (time.perf_counter() - t0) / reps
t0 = time.perf_counter()
for _ in range(reps):
    e.ice_flow_dmax(100.0, 100.0)
t_dmax = (time.perf_counter() - t0) / reps
t0 = time.perf_counter()
e.ice_flow_run(1e-4 * reps, 100.0, 100.0, reps)  # ping-pong sub-steps, one call
t_run = (time.perf_counter() - t0) / reps
n = ny * nx
# algorithmic bytes per cell and sub-step: k_ice_flow reads elev (4) + h_iwe (8),
# writes the new h_iwe (8) to scratch and h_ice (8) to the state plane;
# k_flow_commit reads the new h_iwe (8) and writes it to the state plane (8)
bpc = 4 + 8 + 8 + 8 + 16
print(json.dumps({"grid": [ny, nx], "step_ms": t_step * 1e3, "run_ms_per_sub_step": t_run * 1e3, "dmax_ms": t_dmax * 1e3,
                  "cells_per_s": n / t_step, "bytes_per_cell": bpc, "GBps": n * bpc / t_step / 1e9}))
e.close()
