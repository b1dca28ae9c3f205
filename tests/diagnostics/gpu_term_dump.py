"""Dump the RH output plane of a TFG_DEBUG_TERM build (a flux term in place
of RH) for `steps` steps of the synthetic workload.  Diagnostic only."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]
from tests.harness import BASE_CFG, make_engine  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table  # noqa: E402

tag, n, steps, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), 20251001
eng = make_engine(dict(BASE_CFG), 1, n, "float32", n_frames=24, hist_depth=steps, fuse_steps=24)
eng.fill_synthetic(seed, diurnal_table(24))
eng.run(steps)
eng.sync()
v = np.stack([eng.get_field("RH", index=k, dtype=np.float32) for k in range(steps)])
np.savez_compressed(ROOT / "gpurun_out" / f"term_{tag}.npz", v=v)
print(tag, "ok", flush=True)
