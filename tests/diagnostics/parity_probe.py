"""Where does the fp32 engine's parity error come from?  Runs the bench's
CPU-baseline sample on the GPU and the oracle, prints the floored error per
variable and the inputs of the worst cells.  Diagnostic only (test infra)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle")]
from tests.harness import run_gpu_vs_oracle, scale_floor, synthetic_inputs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 393216
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 24
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 20251001
rep = run_gpu_vs_oracle(1, n, steps, seed=seed, fuse_steps=24)
print(rep["summary"])
gpu, ref = rep["gpu"], rep["ref"]
syn, _ = synthetic_inputs(seed, 1, n, 24)
for name in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH"):
    g, r = gpu[name], ref[name]
    s_v = scale_floor(r)
    e = np.abs(g - r) / np.maximum(np.abs(r), s_v)
    k, c = np.unravel_index(np.argmax(e), e.shape)
    print(f"{name:8s} max {e.max():.2e} at step {k} cell {c}: gpu {g[k, c]:.9e} ref {r[k, c]:.9e} s_v {s_v:.3e} "
          f"p99.9 {np.percentile(e, 99.9):.2e} frac>1e-6 {(e > 1e-6).mean():.2e}")
    f = k % 24
    print(f"          inputs: P {syn['P'][f, c]:.3e} T {syn['T_air'][f, c]:.3f} q {syn['Hum_sp'][f, c]:.4e} "
          f"Pa {syn['P_air'][f, c]:.1f} uz {syn['uz'][f, c]:.3f} elev {syn['elev'][c]:.1f} slope {syn['slope'][c]:.2f} "
          f"aspect {syn['aspect'][c]:.1f} h_swe0 {syn['h_swe'][c]:.4f} h_iwe0 {syn['h_iwe'][c]:.4f}")
