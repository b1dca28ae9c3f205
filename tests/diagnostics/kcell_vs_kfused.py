"""One-cell fp64 step through tfg_update (k_cell) against tfg_step (k_fused,
K = 1) from the same state and inputs, step by step over the reference CSV
forcing: reports the steps whose outputs differ.  Diagnostic only."""
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
a, b = make_engine(cfg), make_engine(cfg)
configure_engine(a, cfg)
configure_engine(b, cfg)
names = ["h_snow", "h_swe", "SM", "h_ice", "h_iwe", "IM", "M_total", "RH"]
out = np.empty((8, 1))
nd = 0
for k in range(len(t.times)):
    blk = np.array([[t.inputs[n][k]] for n in ("P_air", "Hum_sp", "P", "T_air", "uz")], dtype=np.float64)
    a.update_io(blk, out)
    b.set_inputs(blk, 0)
    b.run(1)
    ob = b.get_outputs()
    if not np.array_equal(out, ob):
        nd += 1
        if nd <= 8:
            d = {names[i]: (float(out[i, 0]), float(ob[i, 0])) for i in range(8) if out[i, 0] != ob[i, 0]}
            print(k, {n: f"{x:.17g} / {y:.17g} ({(x - y) / y if y else 0:.2e})" for n, (x, y) in d.items()},
                  "T_air", t.inputs["T_air"][k], "P", t.inputs["P"][k])
        # re-sync b's state to a's so later steps test one step each
        for n in ("h_swe", "h_iwe", "Eccs", "Ecci", "albedo", "n"):
            b.set_field(n, a.get_field(n))
        b.set_field("h_snow", a.get_field("h_snow", index=-1), index=-1)
        b.set_field("h_ice", a.get_field("h_ice", index=-1), index=-1)
print("steps", len(t.times), "differing", nd)
