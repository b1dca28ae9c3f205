"""NextGen's calling pattern at scale: many single-catchment BMI instances in
one process, stepped in turn (7 set_value, update, 8 get_value each).  Reports
creation time and the steady-state per-instance step cost (after one untimed
round).  Diagnostic only.
  python tests/diagnostics/bmi_many_instances.py [instances] [steps] [shared] [distinct] [defer] [ensemble]
  defer     config defer_update: update() queues, the queued models step in one launch
  ensemble  every model's set_value + update(), then every model's get_value
            (NextGen's order is per model: set, update, get)"""
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
distinct = "distinct" in sys.argv[3:]  # every model its own centroid: no two clocks alike (real catchments)
defer = "defer" in sys.argv[3:]
ensemble = "ensemble" in sys.argv[3:]
base = dict(BASE_CFG, defer_update=defer)
cfg.write_text(yaml.dump(base))
t0 = time.perf_counter()
models = []
for i in range(n_inst):
    m = BmiTopoflowGlacier()
    if distinct:
        c = tmp / f"cfg{i}.yaml"
        c.write_text(yaml.dump(dict(base, lat=BASE_CFG["lat"] + 1e-4 * i, lon=BASE_CFG["lon"] - 1e-4 * i)))
        m.initialize(str(c))
    else:
        m.initialize(str(cfg))
    models.append(m)
t_create = time.perf_counter() - t0
if "shared" in sys.argv[3:]:  # an extra torch stream for every instance
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
# one untimed round: each model's first update() computes (or finds in the
# process-wide cache) its clock's first block of 512 steps of uniforms, a cost
# paid once per 512 steps, not per step
for m in models:
    for k, v in ins.items():
        m.set_value(k, np.array([v]))
    m.update()
for m in models:
    m.get_value(outs[0], buf)
t_set = t_upd = t_get = 0.0
t0 = time.perf_counter()
for _ in range(steps if ensemble else 0):
    a = time.perf_counter()
    for m in models:
        for k, v in ins.items():
            m.set_value(k, np.array([v]))
        m.update()
    b = time.perf_counter()
    for m in models:
        for k in outs:
            m.get_value(k, buf)
    c = time.perf_counter()
    t_upd += b - a  # set_value + update() (queues when deferred)
    t_get += c - b  # get_value (the first one runs the queued launch when deferred)
for _ in range(0 if ensemble else steps):
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
timing = None
try:  # the diagnostic build (-DTFG_UPDATE_TIMING, TFG_LIB=...) splits tfg_update's time
    import ctypes

    from topoflow_glacier import _native

    f = _native.lib().tfg_update_timing
    buf5 = (ctypes.c_double * 5)()
    f.argtypes = [ctypes.c_void_p]
    f(ctypes.cast(buf5, ctypes.c_void_p))
    calls = max(buf5[4], 1)
    timing = {k: round(buf5[i] / calls / 1e3, 2) for i, k in enumerate(("pack_us", "launch_us", "wait_us", "unpack_us"))}
except AttributeError:
    pass
ref = models[0].get_value("land_surface_water__runoff_volume_flux", np.zeros(1))[0]
same = all(m.get_value("land_surface_water__runoff_volume_flux", np.zeros(1))[0] == ref for m in models)
for m in models:
    m.finalize()
print(json.dumps({"instances": n_inst, "steps": steps, "distinct_clocks": distinct, "defer_update": defer,
                  "pattern": "ensemble" if ensemble else "interleaved",
                  "extra_shared_stream": "shared" in sys.argv[3:], "create_s": t_create,
                  "us_per_instance_step": t_run / (n_inst * steps) * 1e6,
                  "us_set_update_get": [round(t / (n_inst * steps) * 1e6, 2) for t in (t_set, t_upd, t_get)],
                  "all_instances_equal": same, "tfg_update_split": timing}))
