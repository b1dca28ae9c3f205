"""NextGen's calling pattern at scale: many single-catchment BMI instances in
one process, stepped in turn (7 set_value, update, 8 get_value each).  Reports
creation time and the per-instance step cost.  Diagnostic only.
  python tests/diagnostics/bmi_many_instances.py [instances] [steps] [shared]"""
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import yaml

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]
from tests.harness import BASE_CFG  # noqa: E402
from topoflow_glacier import BmiTopoflowGlacier  # noqa: E402

n_inst = int(sys.argv[1]) if len(sys.argv) > 1 else 500
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 24
tmp = Path(tempfile.mkdtemp())
cfg = tmp / "cfg.yaml"
cfg.write_text(yaml.dump(BASE_CFG))
t0 = time.perf_counter()
models = []
for _ in range(n_inst):
    m = BmiTopoflowGlacier()
    m.initialize(str(cfg))
    models.append(m)
t_create = time.perf_counter() - t0
if len(sys.argv) > 3 and sys.argv[3] == "shared":  # one HIP stream for every instance
    import torch

    shared = torch.cuda.Stream()
    for m in models:
        m._engine.set_stream(shared.cuda_stream)
ins = {"atmosphere_water__liquid_equivalent_precipitation_rate": 1e-7, "land_surface_air__temperature": -2.0,
       "land_surface_radiation~incoming~longwave__energy_flux": 250.0,
       "land_surface_radiation~incoming~shortwave__energy_flux": 100.0, "land_surface_air__pressure": 88000.0,
       "atmosphere_air_water~vapor__relative_saturation": 0.003, "wind_speed_UV": 3.0}
outs = models[0].get_output_var_names()
buf = np.zeros(1)
t_set = t_upd = t_get = 0.0
t0 = time.perf_counter()
for _ in range(steps):
    for m in models:
        a = time.perf_counter()
        for k, v in ins.items():
            m.set_value(k, np.array([v]))
        b = time.perf_counter()
        m.update()
        c = time.perf_counter()
        for k in outs:
            m.get_value(k, buf)
        d = time.perf_counter()
        t_set += b - a
        t_upd += c - b
        t_get += d - c
t_run = time.perf_counter() - t0
ref = models[0].get_value("land_surface_water__runoff_volume_flux", np.zeros(1))[0]
same = all(m.get_value("land_surface_water__runoff_volume_flux", np.zeros(1))[0] == ref for m in models)
for m in models:
    m.finalize()
print(json.dumps({"instances": n_inst, "steps": steps, "extra_shared_stream": len(sys.argv) > 3, "create_s": t_create,
                  "us_per_instance_step": t_run / (n_inst * steps) * 1e6,
                  "us_set_update_get": [round(t / (n_inst * steps) * 1e6, 2) for t in (t_set, t_upd, t_get)],
                  "all_instances_equal": same}))
