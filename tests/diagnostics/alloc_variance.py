"""Does a shard's streaming rate depend on where its buffers landed?  Creates
the engine several times in one process (free, allocate again), times a few
whole launches each time, and prints the rate per allocation.  Diagnostic.
  python tests/diagnostics/alloc_variance.py [ny nx fuse reps]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]
import torch  # noqa: E402

from tests.harness import BASE_CFG, make_engine  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table  # noqa: E402

ny, nx, K, reps = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (4096, 4096, 192, 6)
for rep in range(reps):
    e = make_engine(BASE_CFG, ny, nx, "float32", n_frames=24, hist_depth=K, fuse_steps=K)
    try:
        e.fill_synthetic(7, diurnal_table(24))
        stream = torch.cuda.Stream(0)
        e.set_stream(stream.cuda_stream)
        e.run(K)
        e.sync()
        ms = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            e.run(K)
            b.record(stream)
            ms.append((a, b))
        e.sync()
        t = np.array([a.elapsed_time(b) for a, b in ms])
        print(json.dumps({"alloc": rep, "grid": f"{ny}x{nx}", "K": K, "ms_each": [round(float(x), 3) for x in t],
                          "G_cell_updates_s_steady": ny * nx * K / float(np.median(t[1:])) / 1e6}), flush=True)
    finally:
        e.close()
