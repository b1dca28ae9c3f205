"""Per-step latency of the single-catchment BMI path (set_value x7, update,
get_value x8), as NextGen drives it.  Diagnostic."""
import sys
import time
from pathlib import Path

import numpy as np
import yaml

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]
from tests.harness import BASE_CFG, GOLDEN  # noqa: E402
from topoflow_glacier import BmiTopoflowGlacier  # noqa: E402
from topoflow_glacier.forcing import read_forcing_csv  # noqa: E402
from topoflow_glacier.run import OUT_BMI  # noqa: E402

cfg = Path("/tmp/bmi_lat.yaml")
cfg.write_text(yaml.dump(BASE_CFG))
t = read_forcing_csv(GOLDEN / "sample-cat-3062920.csv", BASE_CFG["start_time"], BASE_CFG["end_time"])
for rep in range(3):
    m = BmiTopoflowGlacier()
    t0 = time.perf_counter()
    m.initialize(cfg)
    t1 = time.perf_counter()
    d = np.zeros(1)
    ts, tu, tg = 0.0, 0.0, 0.0
    for i in range(len(t)):
        a = time.perf_counter()
        t.apply(m, i)
        b = time.perf_counter()
        m.update()
        c = time.perf_counter()
        for name in OUT_BMI.values():
            m.get_value(name, d)
        e = time.perf_counter()
        ts, tu, tg = ts + b - a, tu + c - b, tg + e - c
    m.finalize()
    n = len(t)
    print(f"rep {rep}: initialize {1e3 * (t1 - t0):.1f} ms; per step: set_value x7 {1e6 * ts / n:.1f} us, "
          f"update {1e6 * tu / n:.1f} us, get_value x8 {1e6 * tg / n:.1f} us, total {1e6 * (ts + tu + tg) / n:.1f} us", flush=True)

# breakdown of update(): Python side vs the three native calls
from topoflow_glacier import engine as E  # noqa: E402

acc = {}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
        return r
    return w


E.GlacierEngine.set_inputs = timed("set_inputs", E.GlacierEngine.set_inputs)
E.GlacierEngine.run = timed("run (uniforms + tfg_step)", E.GlacierEngine.run)
E.GlacierEngine.uniforms = timed("  uniforms (Python)", E.GlacierEngine.uniforms)
E.GlacierEngine.get_outputs = timed("get_outputs", E.GlacierEngine.get_outputs)
E.GlacierEngine.update_io = timed("update_io (tfg_update)", E.GlacierEngine.update_io)
m = BmiTopoflowGlacier()
m.initialize(cfg)
t0 = time.perf_counter()
for i in range(len(t)):
    t.apply(m, i)
    m.update()
tot = time.perf_counter() - t0
m.finalize()
n = len(t)
print(f"breakdown per step (us): total incl. set_value {1e6 * tot / n:.1f}; " +
      "; ".join(f"{k} {1e6 * v / n:.1f}" for k, v in acc.items()), flush=True)
