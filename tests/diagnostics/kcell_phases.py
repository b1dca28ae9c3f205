"""Phase times inside k_cell (build with -DTFG_CELL_TIMING, load through
TFG_LIB): state loads, the step's arithmetic, the stores; microseconds at the
100 MHz wall clock, medians over the CSV steps.  Diagnostic only."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd"), str(ROOT / "oracle")]
import torch  # noqa: E402,F401

from tests.harness import BASE_CFG, cfg_object  # noqa: E402
from topoflow_glacier.bmi.bmi_topoflow_glacier import configure_engine, make_engine  # noqa: E402
from topoflow_glacier.forcing import read_forcing_csv  # noqa: E402

cfg = cfg_object(dict(BASE_CFG))
t = read_forcing_csv(ROOT / "tests" / "golden" / "sample-cat-3062920.csv", BASE_CFG["start_time"], BASE_CFG["end_time"])
a = make_engine(cfg)
configure_engine(a, cfg)
out = np.empty((8, 1))
ph = []
for k in range(len(t.times)):
    blk = np.array([[t.inputs[n][k]] for n in ("P_air", "Hum_sp", "P", "T_air", "uz")], dtype=np.float64)
    a.update_io(blk, out)
    ph.append(out[:3, 0].copy())
ph = np.array(ph[5:]) / 100.0  # ticks of 10 ns -> us
print({"loads_us": float(np.median(ph[:, 0])), "step_us": float(np.median(ph[:, 1])), "stores_us": float(np.median(ph[:, 2]))})
