"""Per-workgroup timeline of k_fused launches (why config
2's 1024^2 grid streams at 69 % of the HBM spec against 80 % at 8192^2).
Diagnostic only; needs a -DTFG_WG_TIMING=131072 build (diag_libs/_tfg_wgt.so,
TFG_LIB points at it).

For each shape, after warm-up launches, three launches are recorded: every
workgroup's start and end on the 100 MHz wall clock and the XCC it ran on.
Reported per launch: makespan; workgroup duration percentiles; how many
workgroups were resident at once (the "rounds" of waves); the occupancy loss,
1 - sum(durations) / (makespan x peak concurrency), split into the ramp at
the start, the tail at the end and the middle; per-XCC mean durations.

  TFG_LIB=diag_libs/_tfg_wgt.so python tests/diagnostics/wg_timeline.py out.json [ny,nx,K ...]
"""
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]

from tests.harness import BASE_CFG, make_engine  # noqa: E402
from topoflow_glacier import _native as nat  # noqa: E402
from topoflow_glacier.synthetic import diurnal_table  # noqa: E402

TICK_NS = 10.0  # s_memrealtime: 100 MHz


def timeline(rec):
    start, end = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    t0 = start.min()
    s, e = (start - t0) * TICK_NS / 1e3, (end - t0) * TICK_NS / 1e3  # us
    dur = e - s
    span = e.max()
    # concurrency over time
    ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    peak = int(conc.max())
    busy = float(dur.sum())
    # occupancy deficit in the first and last 10 % of the makespan and in between
    grid = np.linspace(0, span, 2001)
    occ = np.interp(grid, ev[:, 0], conc, left=0, right=0)
    mid = (grid > 0.1 * span) & (grid < 0.9 * span)
    loss = lambda m: float(np.trapz(peak - occ[m], grid[m]) / (peak * span)) if m.any() else 0.0  # noqa: E731
    xcc = (rec[:, 2] >> 32).astype(np.int64)
    return {"workgroups": int(len(rec)), "makespan_us": float(span), "peak_concurrent_wg": peak,
            "rounds": float(len(rec) / peak), "dur_us_p5_p50_p95": [float(np.percentile(dur, q)) for q in (5, 50, 95)],
            "occupancy_loss": 1.0 - busy / (span * peak), "loss_first10pct": loss(grid <= 0.1 * span),
            "loss_middle": loss(mid), "loss_last10pct": loss(grid >= 0.9 * span),
            "last_start_us": float(s.max()), "first_end_us": float(e.min()),
            "end_p90_to_max_us": float(span - np.percentile(e, 90)),
            "xcc_mean_dur_us": {int(x): float(dur[xcc == x].mean()) for x in np.unique(xcc)}}


def main():
    out = sys.argv[1]
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or [(1024, 1024, 120), (8192, 8192, 128),
                                                                             (2048, 2048, 384)]
    L = nat.load()
    L.tfg_debug_wg_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    res = {}
    for ny, nx, k in shapes:
        e = make_engine(dict(BASE_CFG), ny, nx, "float32", n_frames=24, hist_depth=k, fuse_steps=k)
        try:
            e.fill_synthetic(20251001, diurnal_table(24), nx_global=nx)
            e.run(k * max(2, 3840 // k))  # warm-up
            e.sync()
            n_work = -(-e.n // 64) * 64  # k_fused steps the plane stride, skew included
            n_work += 512 if n_work >= 1 << 20 else 0
            nwg = min(131072, -(-n_work // 256))  # fused_blocks: one workgroup per 256-cell chunk, capped
            runs = []
            for _ in range(3):
                e.run(k)
                e.sync()
                rec = np.zeros((131072, 3), np.uint64)
                nat.check(L.tfg_debug_wg_times(rec.ctypes.data, 131072))
                runs.append(timeline(rec[:nwg]))
                if nwg <= 20000 and os.environ.get("TFG_WG_RAW"):  # per-workgroup records: start, end (us), XCC, CU
                    r = rec[:nwg]
                    t0 = int(r[:, 0].min())
                    runs[-1]["raw_start_end_xcc_cu"] = [
                        [round((int(a) - t0) * TICK_NS / 1e3, 2), round((int(b) - t0) * TICK_NS / 1e3, 2), int(c >> 32),
                         int(c & 0xFFFFFFFF)] for a, b, c in r]
                print(f"{ny}x{nx} K={k}", json.dumps({kk: v for kk, v in runs[-1].items() if kk != "xcc_mean_dur_us"}),
                      flush=True)
            res[f"{ny}x{nx}_K{k}"] = runs
        finally:
            e.close()
    Path(out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
