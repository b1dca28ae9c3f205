"""Diagnostic (GPU): does splitting a small grid into row blocks stepped on their
own streams fill the end-of-launch drain of k_fused?

DESIGN.md section 5 measures config 2 (1024^2): 1 M cells fill the 1024
resident workgroup slots four times per launch, and ~10 % of the slot-time is
idle, mostly in the drain at the end of each launch.  Row blocks are
independent (the update is pointwise), so S handles of ny/S rows each, every
one on its own stream, let one block's next launch take the slots another
block's launch leaves idle while it drains; only the last launch drains.

Prints one JSON line per (S, repeat): cell-updates/s over L launches of K steps
of every block, wall clock between two device synchronisations.

    python tests/diagnostics/multistream_drain.py --ny 1024 --nx 1024 --fuse 120 --launches 24
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ny", type=int, default=1024)
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--fuse", type=int, default=120)
    ap.add_argument("--launches", type=int, default=24)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--frames", type=int, default=24)
    args = ap.parse_args()

    import torch

    from bench import BASE_CFG
    from topoflow_glacier.bmi.config import TopoflowGlacierConfig
    from topoflow_glacier.engine import GlacierEngine
    from topoflow_glacier.synthetic import diurnal_table

    splits = [int(s) for s in args.splits.split(",")]
    for rep in range(args.repeats):
        for S in splits:
            if args.ny % S:
                raise SystemExit(f"ny={args.ny} does not split into {S} row blocks")
            rows = args.ny // S
            cfg = TopoflowGlacierConfig.model_validate(dict(BASE_CFG, ny=rows, nx=args.nx))
            engs, streams = [], []
            for s in range(S):
                e = GlacierEngine(cfg, rows, args.nx, engine="float32", device=0, n_frames=args.frames,
                                  hist_depth=args.fuse, fuse_steps=args.fuse, row0=s * rows)
                e.fill_synthetic(1234, diurnal_table(args.frames), nx_global=args.nx)
                st = torch.cuda.Stream(0)
                e.set_stream(st.cuda_stream)
                engs.append(e)
                streams.append(st)
            for e in engs:  # warm-up: one lead-in step and two whole launches
                e.run(1)
                e.run(args.fuse)
                e.run(args.fuse)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.launches):
                for e in engs:
                    e.run(args.fuse)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ns = sum(e.nan_safe_launches() for e in engs)
            cells = args.ny * args.nx
            rate = cells * args.fuse * args.launches / dt
            print(json.dumps({"splits": S, "repeat": rep, "grid": [args.ny, args.nx], "fuse": args.fuse,
                              "launches": args.launches, "seconds": round(dt, 5), "G_cell_updates_s": round(rate / 1e9, 3),
                              "frac": round(rate * 52.0 / 8e12 + rate * 132.0 / args.fuse / 8e12, 4),
                              "nan_safe_launches": ns}), flush=True)
            for e in engs:
                e.close()
            del engs, streams
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
