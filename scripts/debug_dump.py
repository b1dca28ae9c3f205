"""Dump GPU results for offline comparison (debug helper)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle"), str(ROOT)]
from tests.harness import gpu_run_fields, load_golden, run_gpu_vs_oracle  # noqa: E402

out = {}
g = load_golden("grid64")
o, st, dg = gpu_run_fields(g["cfg"], g["static"], g["forcing"], 1, g["ncell"], "float64", g["nsteps"])
for k, v in o.items():
    out["g64_" + k] = v
for k, v in st.items():
    out["g64st_" + k] = v
rep = run_gpu_vs_oracle(32, 64, 48, "float32", seed=11)
for k, v in rep["gpu"].items():
    out["syn_" + k] = v
np.savez_compressed(ROOT / "gpurun_out" / "debug_dump.npz", **out)
print("dumped", len(out))
