"""Diagnostic (GPU): host time of each tfg_step call and the GPU span of a
split engine's timed launches, after a parity-like prelude of host reads or
without one (bench.py config 2 lost the split's gain after its parity leg)."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT)]


def main():
    import numpy as np
    import torch

    from tests.harness import BASE_CFG, make_engine
    from topoflow_glacier.synthetic import diurnal_table

    for prelude in (sys.argv[1:] or ["reads", "none"]):
        e = make_engine(BASE_CFG, 1024, 1024, "float32", n_frames=24, hist_depth=120, fuse_steps=120)
        e.fill_synthetic(7, diurnal_table(24))
        stream = torch.cuda.Stream(0)
        torch.cuda.set_stream(stream)
        e.set_stream(stream.cuda_stream)
        if prelude.startswith("reads"):
            e.run(1)
            e.sync()
            e.run(120)
            e.sync()
            for v in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH"):
                for j in range(121):
                    e.get_field(v, index=j % 120, dtype=np.float32, cells=262144)
            e.diagnostics()
        e.run(120)
        torch.cuda.synchronize()
        if prelude.endswith("gc"):
            import gc

            gc.collect()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        host = []
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(73):
            t = time.perf_counter()
            e.run(120)
            host.append((time.perf_counter() - t) * 1e3)
        e.join()
        ev1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"prelude": prelude, "split": e.is_split(), "gpu_span_ms": ev0.elapsed_time(ev1), "wall_ms": wall,
                          "host_ms_first5": [round(x, 3) for x in host[:5]], "host_ms_max": round(max(host), 3),
                          "host_ms_mean": round(float(np.mean(host)), 4)}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
