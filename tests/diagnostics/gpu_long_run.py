"""Free-running long-horizon GPU run for the parity check of SURVEY 8(d):
the fp32 engine on the synthetic workload for `steps` hourly steps; the
outputs of every 24th step and the final state are saved to
gpurun_out/long_run_<cells>x<steps>.npz for a CPU comparison with the oracle
(tests/diagnostics/long_run_compare.py).  Prints progress (flushed) as it goes."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]
from tests.harness import BASE_CFG, make_engine  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8760
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 20251001
every = 24
names = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
eng = make_engine(dict(BASE_CFG), 1, n, "float32", n_frames=24, hist_depth=every, fuse_steps=every)
eng.fill_synthetic(seed, diurnal_table(24))
out = {k: np.empty((steps // every, n), dtype=np.float32) for k in names}
t0 = time.time()
for i in range(steps // every):
    eng.run(every)
    for k in names:
        out[k][i] = eng.get_field(k, index=every - 1, dtype=np.float32)
    if i % 30 == 0:
        print(f"block {i}/{steps // every} ({time.time() - t0:.1f} s)", flush=True)
state = {k: eng.get_field(k) for k in ("h_swe", "h_iwe", "Eccs", "Ecci", "albedo", "n")}
diag = eng.diagnostics()
eng.close()
dst = ROOT / "gpurun_out" / f"long_run_{n}x{steps}.npz"
dst.parent.mkdir(exist_ok=True)
np.savez_compressed(dst, n=n, steps=steps, seed=seed, every=every, diag=diag,
                    **{f"out_{k}": v for k, v in out.items()}, **{f"state_{k}": v for k, v in state.items()})
print("saved", dst, f"{time.time() - t0:.1f} s", flush=True)
