"""The tail of a bench parity sample, kept for offline classification.

Runs what one bench rank runs for its parity check (bench.capture_parity on a
fresh handle: a one-step lead-in then one launch of the timed depth; the numpy
and C oracles on the same cells, bench.oracle_sample), then keeps, for the
`top` cells with the largest floored error of any output at any compared step
(tests/harness.py classify_sample: not excused, cell not cut), the GPU,
numpy-oracle and C-oracle outputs at every step, plus every output's whole-
sample floor s_v, so the entries that set max_floored_rel can be classified
on the CPU (depletion steps, melt-out splits, ordinary steps).  Diagnostic
only.

  python tests/diagnostics/parity_tail.py OUT.npz [top] [--rank R --world N] -- <bench.py arguments>

With --rank / --world the sample is rank R's of an N-rank bench line (its own
shard, bench.shard_plan; its parity_plan rows), run here as one process.
"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "topoflow-glacier_amd")]


def main():
    out = sys.argv[1]
    head = sys.argv[:sys.argv.index("--")] if "--" in sys.argv else sys.argv
    top = int(head[2]) if len(head) > 2 and not head[2].startswith("--") else 256
    rank = int(head[head.index("--rank") + 1]) if "--rank" in head else 0
    world = int(head[head.index("--world") + 1]) if "--world" in head else 1
    bargs = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
    import bench

    sys.argv = ["bench.py", *bargs]
    args = bench.parse()
    import torch

    from tests.harness import classify_sample, scale_floor
    from topoflow_glacier.bmi.config import TopoflowGlacierConfig
    from topoflow_glacier.engine import GlacierEngine
    from topoflow_glacier.synthetic import diurnal_table

    plan = bench.shard_plan(args, world, rank)
    if not args.fuse:
        args.fuse = bench.auto_fuse(plan["rows"] * args.nx, 8 if args.engine == "float64" else 4)
    cfg = TopoflowGlacierConfig.model_validate(dict(bench.BASE_CFG, ny=plan["rows"], nx=args.nx, dt=args.dt))
    eng = GlacierEngine(cfg, plan["rows"], args.nx, row0=plan["row0"], engine=args.engine, device=0,
                        n_frames=args.frames, hist_depth=args.fuse, fuse_steps=args.fuse)
    eng.fill_synthetic(args.seed, diurnal_table(args.frames), nx_global=args.nx)
    t0 = time.perf_counter()
    cap = bench.capture_parity(eng, args, plan, world, torch, 0)
    eng.close()
    print(f"captured {cap['plan']} in {time.perf_counter() - t0:.1f} s", flush=True)
    ref, c64, _, pcfg = bench.oracle_sample(args, cap["plan"], bench._cpu_threads())
    gpu = cap["gpu"]
    tol = 1e-5 if args.engine == "float32" else 1e-10
    cls = classify_sample(gpu, ref, c64, pcfg, tol, onsets=args.engine == "float32")
    floors = {v: scale_floor(ref[v]) for v in bench.HIST}
    worst = np.zeros(ref["SM"].shape[1])
    for v in bench.HIST:
        e = np.abs(gpu[v] - ref[v]) / np.maximum(np.maximum(np.abs(ref[v]), floors[v]), 1e-300)
        worst = np.maximum(worst, np.where(cls.ok, e, 0.0).max(axis=0))
    cells = np.argsort(worst)[::-1][:top]
    # the same statistic for the fp64 baseline (C oracle vs numpy oracle, same rules, no onset allowance)
    cls64 = classify_sample(c64, ref, c64, pcfg, tol, onsets=False)
    w64 = max(float(np.where(cls64.ok, np.abs(c64[v] - ref[v]) / np.maximum(np.maximum(np.abs(ref[v]), floors[v]),
                                                                           1e-300), 0.0).max()) for v in bench.HIST)
    keep = {"cells": cells, "worst": worst[cells], "floors": np.array([floors[v] for v in bench.HIST]),
            "names": np.array(bench.HIST), "args": np.array(" ".join(bargs)), "rank": rank, "world": world,
            "global_rows": np.array([cap["plan"]["row0"], cap["plan"]["row0"] + cap["plan"]["rows"] - 1]), "ok": cls.ok[:, cells],
            "excused": cls.excused[:, cells], "flip": cls.flip[cells], "cut": cls.cut[cells],
            "flip64": cls.flip64[cells], "n_flips": (cls.flip >= 0).sum(), "n_flips64": (cls.flip64 >= 0).sum(),
            "n_excused": cls.excused.sum(), "n_genuine": len(cls.genuine), "n_onsets": len(cls.onset),
            "c64_max_floored": w64, "c64_n_genuine": len(cls64.genuine)}
    for v in bench.HIST:
        keep["gpu_" + v] = gpu[v][:, cells]
        keep["ref_" + v] = ref[v][:, cells]
        keep["c64_" + v] = c64[v][:, cells]
    for t in ("Qn_SW", "Qn_LW", "Qh", "Qe"):
        keep["ref_" + t] = ref[t][:, cells]
    np.savez_compressed(out, **keep)
    print(f"kept {len(cells)} cells, worst {worst[cells[0]]:.4e} (fp64 baseline {w64:.4e}), 100th {worst[cells[min(99, len(cells) - 1)]]:.4e}",
          flush=True)


if __name__ == "__main__":
    main()
