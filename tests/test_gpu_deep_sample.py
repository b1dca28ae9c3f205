"""The deepest launch the bench times, checked exactly as the bench checks it.

At N = 4 the driver's strong-scaling line gives each rank a 2048 x 8192 shard
of the 8192^2 grid (BASELINE config 4) and bench.auto_fuse a 384-step launch:
the longest fp32 launch of any bench line, so the one where the flux error
accumulates furthest.  This runs rank 0's parity check of that line on one GPU
(bench.capture_parity: a one-step lead-in, then ONE 384-step launch over the
whole shard; bench.sample_parity: the numpy oracle on the same cells, the
classification of tests/harness.py) on global rows 0-9 -- a superset of the
rows 0-7 the N = 4 line samples itself -- and holds its max_floored_rel to
8e-6, the 1e-5 tolerance with a 20 % margin.

Every other BASELINE GPU configuration is checked at ITS timed launch depth
the same way: config 3 (4096^2, one 384-step launch) and
config 5's per-GPU slab (rank 3 of 8: rows 6144-8191 of the 16384^2 grid,
dt = 0.25 h, 43 catchments, one 256-step launch), and rank 2 of the N = 4
line, whose own sample had the largest error of any rank in round 5.
"""
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MARGIN_TOL = 8e-6
_FIELDS = ("global_rows", "max_floored_rel", "max_floored_rel_at", "max_floored_rel_fp64_baseline", "melt_out_flips",
           "flips_fp64_baseline", "depletion_steps", "depletion_steps_fp64_baseline", "melt_onsets_explained")


def _record(name, par):
    """Print the sample's parity record and, when $TFG_REPORT_DIR is set, write
    it there as deep_<name>.json (profiles/r6d_deep_samples.json collects them)."""
    import json
    import os

    rec = {k: par.get(k) for k in _FIELDS}
    print(rec)
    d = os.environ.get("TFG_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"deep_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1, default=str)


def test_n4_rank0_deep_launch_sample(monkeypatch):
    import torch

    import bench
    from topoflow_glacier.bmi.config import TopoflowGlacierConfig
    from topoflow_glacier.engine import GlacierEngine
    from topoflow_glacier.synthetic import diurnal_table

    monkeypatch.setattr(sys, "argv", ["bench.py", "--ny", "8192", "--nx", "8192", "--parity-cells", str(10 * 8192)])
    args = bench.parse()
    world, rank = 4, 0
    plan = bench.shard_plan(args, world, rank)
    assert (plan["row0"], plan["rows"]) == (0, 2048)
    args.fuse = bench.auto_fuse(plan["rows"] * args.nx)
    assert args.fuse == 384
    cfg = TopoflowGlacierConfig.model_validate(dict(bench.BASE_CFG, ny=plan["rows"], nx=args.nx, dt=args.dt))
    eng = GlacierEngine(cfg, plan["rows"], args.nx, engine="float32", device=0, n_frames=args.frames,
                        hist_depth=args.fuse, fuse_steps=args.fuse)
    try:
        eng.fill_synthetic(args.seed, diurnal_table(args.frames), nx_global=args.nx)
        cap = bench.capture_parity(eng, args, plan, world, torch, 0)
    finally:
        eng.close()
    assert cap["plan"]["launch_steps"] == [1, 384] and cap["plan"]["rows"] == 10
    par, _ = bench.sample_parity(args, plan, world, rank, bench._cpu_threads(), cap)
    _record("n4_rank0_fp32", par)
    assert par["global_rows"] == [0, 9]
    assert par["ok"], {k: par[k] for k in ("max_floored_rel", "genuine_mismatches", "flip_rule", "mass_balance")}
    assert par["max_floored_rel"] <= MARGIN_TOL, par["max_floored_rel_at"]
    assert par["max_floored_rel_fp64_baseline"] < 1e-12
    assert np.isfinite(par["max_floored_rel_incl_depletion_rates"])
    _exclusions_do_not_grow(par, "fp32")


def _exclusions_do_not_grow(par, flux):
    """The three rules that excuse entries (tests/harness.py classify_sample)
    held to what the round-6 code measures, so that a change of the fp32 step
    cannot widen them unnoticed (VERDICT r5 "What's weak" 2): melt-out flips
    at most 1.75x the fp64 baseline's (measured 1.50-1.58x; the rule's budget
    is 2.5x), depletion steps within 2 % of the fp64 baseline's count (the
    same reservoirs run dry), melt onsets at most 2 cells of the sample for
    the fp32 flux and none for the fp64 flux."""
    if par["flips_fp64_baseline"]:
        assert par["melt_out_flips"] <= 1.75 * par["flips_fp64_baseline"], (par["melt_out_flips"], par["flips_fp64_baseline"])
    base = par["depletion_steps_fp64_baseline"]
    assert abs(par["depletion_steps"] - base) <= 0.02 * base + 10, (par["depletion_steps"], base)
    assert par["melt_onsets_explained"] <= (2 if flux == "fp32" else 0), par["melt_onsets_explained"]


def _timed_depth_sample(monkeypatch, argv, world, rank, want_fuse, want_rows, flux="fp32"):
    """bench.capture_parity + sample_parity of one rank of a bench line, on one
    GPU, at the line's own timed launch depth; returns the parity record."""
    import torch

    import bench
    from topoflow_glacier.bmi.config import TopoflowGlacierConfig
    from topoflow_glacier.engine import GlacierEngine
    from topoflow_glacier.synthetic import diurnal_table

    monkeypatch.setattr(sys, "argv", ["bench.py", *argv, "--flux", flux])
    args = bench.parse()
    plan = bench.shard_plan(args, world, rank)
    assert (plan["row0"], plan["rows"]) == want_rows
    args.fuse = bench.auto_fuse(plan["rows_max"] * args.nx)
    assert args.fuse == want_fuse
    cfg = TopoflowGlacierConfig.model_validate(dict(bench.BASE_CFG, ny=plan["rows"], nx=args.nx, dt=args.dt))
    n_catch = args.catchments + 1 if args.catchments > 0 else 1
    eng = GlacierEngine(cfg, plan["rows"], args.nx, engine="float32", device=0, n_frames=args.frames,
                        hist_depth=args.fuse, fuse_steps=args.fuse, row0=plan["row0"], n_catch=n_catch, flux=flux)
    try:
        eng.fill_synthetic(args.seed, diurnal_table(args.frames), nx_global=args.nx)
        if args.catchments > 0:
            eng.set_field("catch_id", bench.catchment_blocks(plan["row0"], plan["rows"], plan["ny_global"], args.nx,
                                                             args.catchments))
        cap = bench.capture_parity(eng, args, plan, world, torch, 0)
    finally:
        eng.close()
    assert cap["plan"]["launch_steps"] == [1, want_fuse]
    par, _ = bench.sample_parity(args, plan, world, rank, bench._cpu_threads(), cap)
    _record(f"{args.ny}x{args.nx}_n{world}_rank{rank}_{flux}", par)
    assert par["ok"], {k: par[k] for k in ("max_floored_rel", "genuine_mismatches", "flip_rule", "mass_balance")}
    assert par["max_floored_rel"] <= MARGIN_TOL, par["max_floored_rel_at"]
    _exclusions_do_not_grow(par, flux)
    assert par["max_floored_rel_fp64_baseline"] < 1e-12
    if flux == "fp64":  # held without the melt-onset allowance (bench.sample_parity)
        assert par["melt_onsets_explained"] == 0
    return par


def test_config3_at_its_timed_depth(monkeypatch):
    """BASELINE config 3 (4096 x 4096, the bench line's 384-step launches)."""
    par = _timed_depth_sample(monkeypatch, ["--ny", "4096", "--nx", "4096"], 1, 0, 384, (0, 4096))
    assert par["global_rows"][0] == 0


def test_config5_slab_at_its_timed_depth(monkeypatch):
    """BASELINE config 5's per-GPU slab: rank 3 of the 8-GPU 16384 x 16384 line
    (rows 6144-8191), 15-minute steps (a 288-slot window), 43 catchments, the
    line's 256-step launches; the per-catchment mass balance of the launch is
    part of the check (bench.sample_parity)."""
    argv = ["--ny", "16384", "--nx", "16384", "--dt", "0.25", "--catchments", "43"]
    par = _timed_depth_sample(monkeypatch, argv, 8, 3, 256, (6144, 2048))
    assert par["global_rows"][0] == 6144


@pytest.mark.parametrize("rank,rows", [(0, (0, 2048)), (2, (4096, 2048))])
def test_n4_deep_launch_with_the_fp64_flux(monkeypatch, rank, rows):
    """The N = 4 line's rank 0 and rank 2 samples with the fp64-flux form
    (--flux fp64): 8e-6 and no melt onset explained by the fp32-flux allowance."""
    _timed_depth_sample(monkeypatch, ["--ny", "8192", "--nx", "8192"], 4, rank, 384, rows, flux="fp64")


def test_n4_rank2_deep_launch_sample(monkeypatch):
    """Rank 2 of the same N = 4 line, the rank whose own sample (global rows
    4096-4103, the bench's default 65 536 cells) has the largest error of any
    rank of the 2-, 4- and 8-GPU lines (profiles/r5_deep_samples.json,
    other_ranks: 9.56e-6, at a melt onset): the check the driver's line makes
    on that rank, held to the 1e-5 tolerance itself."""
    import torch

    import bench
    from topoflow_glacier.bmi.config import TopoflowGlacierConfig
    from topoflow_glacier.engine import GlacierEngine
    from topoflow_glacier.synthetic import diurnal_table

    monkeypatch.setattr(sys, "argv", ["bench.py", "--ny", "8192", "--nx", "8192"])
    args = bench.parse()
    world, rank = 4, 2
    plan = bench.shard_plan(args, world, rank)
    assert (plan["row0"], plan["rows"]) == (4096, 2048)
    args.fuse = bench.auto_fuse(plan["rows"] * args.nx)
    assert args.fuse == 384
    cfg = TopoflowGlacierConfig.model_validate(dict(bench.BASE_CFG, ny=plan["rows"], nx=args.nx, dt=args.dt))
    eng = GlacierEngine(cfg, plan["rows"], args.nx, engine="float32", device=0, n_frames=args.frames,
                        hist_depth=args.fuse, fuse_steps=args.fuse, row0=plan["row0"])
    try:
        eng.fill_synthetic(args.seed, diurnal_table(args.frames), nx_global=args.nx)
        cap = bench.capture_parity(eng, args, plan, world, torch, 0)
    finally:
        eng.close()
    assert cap["plan"]["launch_steps"] == [1, 384]
    par, _ = bench.sample_parity(args, plan, world, rank, bench._cpu_threads(), cap)
    _record("n4_rank2_fp32", par)
    assert par["global_rows"] == [4096, 4103]
    assert par["ok"], {k: par[k] for k in ("max_floored_rel", "genuine_mismatches", "flip_rule", "mass_balance")}
    assert par["max_floored_rel"] <= 1e-5, par["max_floored_rel_at"]
    assert par["max_floored_rel_fp64_baseline"] < 1e-12
    _exclusions_do_not_grow(par, "fp32")
