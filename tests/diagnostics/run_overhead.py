"""Host overhead of one engine.run(K) call (uniforms + tfg_step: staging, form
choice, launch) against the launch's GPU time, for small and large grids, with
the GPU idle before each call (the update_until pattern) and back to back.
Diagnostic; prints one JSON line per case."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]
import torch  # noqa: E402

from tests.harness import BASE_CFG, make_engine  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table  # noqa: E402

for engine, ny, nx, K in (("float32", 64, 64, 24), ("float32", 1024, 1024, 24), ("float32", 1024, 1024, 120),
                          ("float32", 8192, 8192, 24), ("float64", 1, 1, 24), ("float64", 512, 512, 24)):
    e = make_engine(BASE_CFG, ny, nx, engine, n_frames=24, hist_depth=max(K, 1), fuse_steps=K)
    try:
        e.fill_synthetic(7, diurnal_table(24))
        stream = torch.cuda.Stream(0)
        e.set_stream(stream.cuda_stream)
        e.run(K)
        e.sync()
        idle_host, idle_wall, idle_gpu = [], [], []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            time.sleep(0.002)  # the GPU idles between calls
            t0 = time.perf_counter()
            a.record(stream)
            e.run(K)
            t1 = time.perf_counter()
            b.record(stream)
            b.synchronize()
            t2 = time.perf_counter()
            idle_host.append((t1 - t0) * 1e6)
            idle_wall.append((t2 - t0) * 1e6)
            idle_gpu.append(a.elapsed_time(b) * 1e3)
        t0 = time.perf_counter()
        n = 20
        for _ in range(n):
            e.run(K)
        t1 = time.perf_counter()
        e.sync()
        t2 = time.perf_counter()
        print(json.dumps({"engine": engine, "grid": f"{ny}x{nx}", "K": K,
                          "idle_call_host_us": float(np.median(idle_host)),
                          "idle_call_wall_us": float(np.median(idle_wall)),
                          "idle_call_event_us": float(np.median(idle_gpu)),
                          "back_to_back_host_us_per_call": (t1 - t0) * 1e6 / n,
                          "back_to_back_wall_us_per_call": (t2 - t0) * 1e6 / n}), flush=True)
    finally:
        e.close()
