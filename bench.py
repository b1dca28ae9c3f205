#!/usr/bin/env python3
"""Benchmark: glacier energy-balance cell-updates/s on MI355X (BASELINE.json).

One "step" = one model time step (BmiTopoflowGlacier.update(),
bmi_topoflow_glacier.py:413-465) applied to every cell of the grid: read that
hour's forcing frame from HBM, run the fused energy/mass balance, write the six
BMI outputs of the step to HBM.  Steps are fused `--fuse` per kernel launch
(state stays in registers between fused steps; every step still streams its
forcing in and its outputs out, to its own history slot: hist_depth = fuse, so
no output write can be absorbed by a cache rewrite).

Workload (N=1): 8192 x 8192 synthetic grid, hourly forcing cycling through 24
HBM-resident frames, fp32 engine (fp64 state), 128 steps per launch (HBM
footprint ~266 GB of the 288 GB: 24 forcing frames 32 GB, 128 output slots
206 GB, 72-slot snowfall window 19 GB, state and geometry 9 GB).  Shards of
2^25 cells or fewer fuse 256 steps per launch (N = 2), 2^24 or fewer 384
(N >= 4; auto_fuse).

--gpus N: one process per GPU (torchrun).  By default the ONE 8192 x 8192 grid
is row-partitioned over the N ranks (strong scaling, BASELINE config 4: 1024 x
8192 per GPU at N = 8); --scaling weak gives every rank its own --ny rows.
There is no data-path collective; value = all cells x steps / max-over-ranks
time between barriers.

The timed region is a whole number of fused launches, at least MIN_LAUNCHES,
covering --steps, and (with the automatic depth) a multiple of 384 steps, so
every N times the same steps of the same grid; the JSON carries
`steps_requested` beside the timed `steps`.

Prints ONE JSON line on rank 0.  Roofline: achieved = algorithmic bytes per
fused launch / mean launch time (HIP events on the engine's stream); traffic
= PMC bytes from the committed profile, only when it was measured on the same
device code (roofline.traffic_source).  Parity spot check: GPU vs the numpy
oracle on a sample, melt-out flips held to the fp64 baseline of the same
sample (tests/harness.py flip_rule).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "topoflow-glacier_amd"), str(ROOT)]

METRIC = "cell-updates/sec (nx·ny·steps) on 8192² fp32 grid; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# algorithmic bytes per cell (DESIGN.md "Bytes per cell-update")
BYTES_PER_STEP = 20 + 4 + 4 + 24  # forcing 5xf32, window slot in+out, 6 outputs f32
BYTES_PER_LAUNCH = 20 + (6 * 8 + 8) * 2  # solar geometry 5xf32; state 6xf64 + window total i64, in and out


def launch_bytes_per_cell(fuse: int) -> int:
    """Algorithmic HBM bytes per cell of one fused launch:
    52 per step + 132 per launch.  (Keeping the window slots that a launch
    reads back itself in LDS would save 8 B per such step, but reserving the
    LDS cost 8 % of throughput on its own: DESIGN.md section 5.)"""
    return BYTES_PER_STEP * fuse + BYTES_PER_LAUNCH

MIN_LAUNCHES = 6
# Why 6: the first launch after the barrier that opens the timed region runs
# 0.5-3.6 ms long at every shape and warm-up length (profiles/r3c_slab_skew_study.jsonl,
# profiles/r3f_slab_depth_study.jsonl); over 6 launches it weighs ~1 % on the
# 1024 x 8192 slab instead of ~2 % over 3.
# auto launch depth by shard size, as deep as ~210 GB of output slots allow
# (hist_depth = launch depth): 128 steps above 2^25 cells (the 8192^2 grid: the
# 128 slots take 206 GB, the whole footprint 266 GB; 96-step launches ran 1.0 %
# slower on the same box, profiles/r3q_fuse128.log), 256 above 2^24 (4096 x 8192,
# N = 2: 206 GB; 121.0-121.4 -> 121.6-121.9 G cell-updates/s from 192 to 256,
# profiles/r3bn_depth_n2_shard.jsonl), 384 at 2^24 and below (N >= 4: a deeper
# launch amortises the per-launch cost; 1024 x 8192 with the plane skew
# 112.6-113.6 -> 115.2-115.7 G cell-updates/s from 192 to 384, profiles/r3ab_slab_k.log)
FUSE_BIG, FUSE_MID, FUSE_SMALL = 128, 256, 384
FUSE_SPLIT_CELLS, FUSE_SMALL_CELLS = 1 << 25, 1 << 24
FUSE_FALLBACK = 96  # if a device cannot hold FUSE_BIG output slots (main())
STEP_QUANTUM = 768  # timed steps are a multiple of every depth: the same total work at every N


def auto_fuse(cells: int, elem: int = 4) -> int:
    """Launch depth by shard size for an engine whose outputs are `elem` bytes
    (the fp64 engine's history slots are twice the fp32 ones, so half as many
    fit the same ~210 GB: 192 steps at 4096^2, 128 at 4096 x 8192)."""
    if cells > FUSE_SPLIT_CELLS:
        k = FUSE_BIG
    else:
        k = FUSE_MID if cells > FUSE_SMALL_CELLS else FUSE_SMALL
    return k * 4 // elem


def warmup_steps(requested: int, fuse: int) -> int:
    """Untimed steps before the timed region: the requested count, and at
    least one whole launch of the timed depth (main() says why)."""
    return max(requested, fuse)


def timed_steps(requested: int, fuse: int, explicit: bool) -> int:
    """Whole launches covering `requested`, at least MIN_LAUNCHES of them.  With
    the automatic depth the count is a multiple of STEP_QUANTUM covering at
    least MIN_LAUNCHES launches of the deepest automatic depth, so N = 1
    (128-step launches), N = 2 (256) and N >= 4 (384) time the same number of
    steps of the same grid."""
    if explicit:
        return max(MIN_LAUNCHES, -(-requested // fuse)) * fuse
    need = max(requested, MIN_LAUNCHES * max(FUSE_BIG, FUSE_MID, FUSE_SMALL))
    return -(-need // STEP_QUANTUM) * STEP_QUANTUM

BASE_CFG = {
    "site_prefix": "synthetic", "forcing_file": "synthetic", "dt": 1, "start_time": "2013032000",
    "end_time": "2014032000", "da": 0.0001, "slope": 50.0, "aspect": 180.0, "lon": -121.81418,
    "lat": 46.81953220, "elev": 2400.0, "h_active_layer": 0.125, "h0_snow": 5.0, "h0_ice": 2.0,
    "h0_swe": 0.25, "h0_iwe": 1.834, "T_rain_snow": 0.0,
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=480)
    ap.add_argument("--warmup", type=int, default=96)
    ap.add_argument("--ny", type=int, default=8192, help="global rows (strong) or rows per GPU (weak)")
    ap.add_argument("--nx", type=int, default=8192)
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--fuse", type=int, default=0,
                    help="steps per launch (= output history slots); 0 = by shard size (auto_fuse)")
    ap.add_argument("--engine", default="float32", choices=["float32", "float64"])
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="strong (default: one --ny x --nx grid row-partitioned over the ranks, BASELINE "
                         "config 4) or weak (--ny rows per rank)")
    ap.add_argument("--seed", type=int, default=20251001)
    ap.add_argument("--cpu-cells", type=int, default=1048576, help="cells in the C CPU-baseline sample")
    ap.add_argument("--cpu-steps", type=int, default=960, help="steps of the C CPU-baseline sample (~10 s on 16 threads)")
    ap.add_argument("--parity-steps", type=int, default=96, help="steps of the GPU-vs-oracle spot check")
    ap.add_argument("--parity-cells", type=int, default=262144,
                    help="cells of the GPU-vs-oracle spot check (also the numpy one-core sample)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pcie", action="store_true",
                    help="add the PCIe-inclusive (host-fed forcing) leg; off by default so that every k_fused "
                         "launch of the 8192^2 shape in a default run is a timed one (rocprof averages = bench's)")
    ap.add_argument("--no-pcie", action="store_true", help=argparse.SUPPRESS)  # the default; kept for old scripts
    ap.add_argument("--dt", type=float, default=1.0, help="time step [h] (BASELINE config 5: 0.25)")
    ap.add_argument("--catchments", type=int, default=0,
                    help="K > 0: per-catchment mass balance over a K-catchment block raster (BASELINE config 5)")
    ap.add_argument("--conduction", action="store_true",
                    help="the optional lateral heat-conduction term: Qc re-evaluated (with the one-row halo swap "
                         "between ranks) before every fused launch, inside the timed region")
    return ap.parse_args()


def _cpu_threads() -> int:
    """Host threads for the C baseline: the process's CPU share (16 on a one-GPU
    box, where OMP_NUM_THREADS is set to it), never the whole machine."""
    env = os.environ.get("OMP_NUM_THREADS")
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    n = int(env) if env and env.isdigit() else avail
    return max(1, min(n, avail, 16))


def _floored_rel(g, r):
    """|gpu - ref| / max(|ref|, s_v), s_v = p99 of the non-zero |ref|."""
    nz = np.abs(r[r != 0])
    s_v = np.percentile(nz, 99) if nz.size else 0.0
    fl = np.maximum(np.maximum(np.abs(r), s_v), 1e-300)
    e = np.abs(g - r) / fl
    return float(np.max(e)), float(np.mean(e > 1e-5))


def cpu_baseline(args, run_gpu_sample):
    """CPU legs on rank 0 at N=1, on the first cells of the shard, same fp32 inputs:
    (1) the C oracle (oracle/tfg_oracle_c.c, fp64, OpenMP over the process's CPU
        share) on --cpu-cells x --cpu-steps: the reported cpu_baseline;
    (2) the numpy oracle (oracle/tfg_oracle.py, fp64, one core) on the first
        --parity-cells x --parity-steps, reported beside it and used as the
        reference of a parity spot check of the GPU on those cells and steps."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import tfg_oracle as O
    import tfg_oracle_c as OC

    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    n = min(args.cpu_cells, args.nx * args.ny)
    steps = max(args.cpu_steps, args.parity_steps)
    syn = synthetic_cells(args.seed, np.arange(n), diurnal_table(args.frames))
    frames = np.arange(steps) % args.frames
    static = dict(elev=syn["elev"], slope=syn["slope"], aspect=syn["aspect"], h0_snow=syn["h_snow"],
                  h0_ice=syn["h_ice"], h0_swe=syn["h_swe"], h0_iwe=syn["h_iwe"])
    static = {k: np.asarray(v, dtype=np.float64) for k, v in static.items()}
    cfg = dict(BASE_CFG, dt=args.dt)
    clock = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    # (1) C oracle, all threads of this process's share
    threads = _cpu_threads()
    forcing = {k: np.ascontiguousarray(syn[k], dtype=np.float64) for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    t0 = time.perf_counter()
    out, _ = OC.run_oracle_c(cfg, static, forcing, args.cpu_steps, clock=(clock[0][:args.cpu_steps], clock[3][:args.cpu_steps]),
                             frames=frames[:args.cpu_steps], hist=False, nthreads=threads)
    t_c = time.perf_counter() - t0
    cpu = {"value": n * args.cpu_steps / t_c, "unit": "cell-updates/s", "cores": threads, "kind": "port",
           "sample": f"oracle/tfg_oracle_c.c (C fp64 restatement of update(), OpenMP, {threads} threads) on the "
                     f"first {n} cells x {args.cpu_steps} hourly steps of the same synthetic workload ({t_c:.1f} s)"}
    # (2) the parity spot check and the one-core numpy leg share one numpy run:
    # the numpy oracle (bit-identical to the reference on every golden fixture)
    # over the first pn cells x ps steps is both the reference the GPU is checked
    # against and the single-core CPU sample.
    from tests.harness import flip_rule, melt_out_flips, valid_mask

    pn = min(args.parity_cells, n)
    ps = args.parity_steps
    fnp = {k: v[frames[:ps], :pn] for k, v in forcing.items()}
    snp = {k: v[:pn] for k, v in static.items()}
    t0 = time.perf_counter()
    ref, _ = O.run_oracle(cfg, snp, fnp, ps, clock=(clock[0], clock[3]))
    t_np = time.perf_counter() - t0
    numpy_leg = {"value": pn * ps / t_np, "unit": "cell-updates/s", "cores": 1, "kind": "port",
                 "sample": f"oracle/tfg_oracle.py (numpy fp64, single thread) on the first {pn} cells x "
                           f"{ps} steps ({t_np:.1f} s)"}
    parity = None
    gpu = run_gpu_sample(pn, ps)
    if gpu is not None:
        # Every step of the first pn cells.  Cells whose trajectories part at a
        # melt-out residual (DESIGN.md "Melt-out flips") are compared up to the
        # flip and counted; the count is held to the fp64 baseline of the same
        # cells and steps: the C oracle against the numpy oracle, two fp64
        # restatements that differ only in their libm (tests/harness.py flip_rule).
        names = sorted(gpu)
        ref = {k: ref[k] for k in names}
        c64, _ = OC.run_oracle_c(cfg, snp, {k: np.ascontiguousarray(v[:, :pn]) for k, v in forcing.items()}, ps,
                                 clock=(clock[0][:ps], clock[3][:ps]), frames=frames[:ps], hist=True, nthreads=threads)
        flip64, genuine64 = melt_out_flips({k: c64[k] for k in names}, ref)
        flip, genuine = melt_out_flips(gpu, ref)
        ok = valid_mask(flip, ps)
        err = max(_floored_rel(g[ok], ref[k][ok])[0] for k, g in gpu.items())
        pure = {}  # the fraction of compared values above pure-relative 1e-5
        for k, g in gpu.items():
            gv, rv = g[ok].astype(np.float64), ref[k][ok]
            with np.errstate(divide="ignore", invalid="ignore"):
                rel = np.where(rv != 0, np.abs(gv - rv) / np.abs(rv), np.where(gv != rv, np.inf, 0.0))
            pure[k] = float(np.mean(rel > 1e-5))
        rule = flip_rule(int((flip >= 0).sum()), int((flip64 >= 0).sum()))
        parity = {"vs": "numpy oracle (fp64; pinned bit-exact to the reference fixtures)", "cells": pn, "steps": ps,
                  "outputs": names, "max_floored_rel": err, "tolerance": 1e-5, "frac_above_pure_rel_1e-5": pure,
                  "melt_out_flips": rule["flips"], "flips_fp64_baseline": rule["fp64_flips"],
                  "flip_ratio": rule["ratio"], "flip_budget": rule["budget"], "flip_rule": rule["rule"],
                  "genuine_mismatches": len(genuine), "fp64_baseline_genuine_mismatches": len(genuine64),
                  "ok": bool(err <= 1e-5 and not genuine and rule["ok"])}
    return cpu, numpy_leg, parity


def shard_plan(args, world: int, rank: int) -> dict:
    """This rank's rows.  The default is strong scaling: the ONE --ny x --nx
    grid of BASELINE config 4 row-partitioned over the ranks (the whole grid at
    N = 1, 1024 x 8192 per GPU at N = 8); --scaling weak gives each rank --ny
    rows of a taller grid."""
    from topoflow_glacier.sharding import row_block

    scaling = args.scaling or "strong"  # the same label at every N of the driver's SCALE series
    if scaling == "weak":
        ny_global, row0, rows = args.ny * world, rank * args.ny, args.ny
    else:
        ny_global = args.ny
        row0, rows = row_block(args.ny, rank, world)
    rows_max = max(row_block(ny_global, r, world)[1] for r in range(world)) if scaling == "strong" else rows
    return {"scaling": scaling, "ny_global": ny_global, "row0": row0, "rows": rows, "rows_max": rows_max,
            "workload": f"{ny_global}x{args.nx} grid ({rows_max}x{args.nx} per GPU)"}


def pmc_traffic(rows, args):
    """HBM bytes per launch from the committed PMC profile of this shard shape
    (scripts/gpu_pmc.sh -> profiles/pmc_<nx>x<rows>_fuse<K>.json), quoted only
    when the profile was measured on the same machine code of the timed kernel
    as the running library's (_native.kernel_code_sha256: the kernel's
    instructions, descriptor and callees, not the other kernels of the
    library); otherwise null, with the reason."""
    from topoflow_glacier import _native as nat

    pmc = ROOT / "profiles" / f"pmc_{args.nx}x{rows}_fuse{args.fuse}.json"
    running = nat.kernel_code_sha256()
    if args.engine != "float32" or args.catchments or args.dt != 1.0 or args.conduction:
        return None, {"profile": None, "reason": "no PMC profile for this variant of the kernel"}
    if not pmc.exists():
        return None, {"profile": None, "reason": f"{pmc.relative_to(ROOT)} not measured"}
    prof = json.loads(pmc.read_text())
    measured = prof.get("kernel_code_sha256")
    src = {"profile": str(pmc.relative_to(ROOT)), "kernel": nat.BENCH_KERNEL, "kernel_code_sha256": measured,
           "running_kernel_code_sha256": running, "match": measured is not None and measured == running,
           "read_scale": corr.get("read_scale") if isinstance(corr := prof.get("correction"), dict) else None}
    return (prof.get("hbm_bytes_per_launch") if src["match"] else None), src


def device_record(torch, local: int) -> dict:
    """The GPU this rank drives: its PCI address (hipDeviceProp_t
    pciDomainID:pciBusID:pciDeviceID, through torch.cuda.get_device_properties)
    and UUID, so a multi-GPU line shows which physical devices ran."""
    p = torch.cuda.get_device_properties(local)
    return {"device": local, "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "uuid": str(p.uuid), "name": p.name}


def rank_report(records: list[dict], backend: str | None) -> dict:
    """What every rank saw, gathered on rank 0: one record per rank (rank,
    local_rank, device, PCI bus id, its launch times and its own timed span),
    the slowest and fastest rank, and whether the ranks drove distinct GPUs.
    Over RCCL two ranks on one GPU are an error (RCCL itself refuses them);
    the gloo rehearsal on one device (TFG_BENCH_ONE_DEVICE) shares one."""
    recs = sorted(records, key=lambda r: r["rank"])
    span = [r["elapsed_s"] for r in recs]
    buses = [r["pci_bus_id"] for r in recs]
    distinct = len(set(buses)) == len(buses)
    if backend == "nccl" and not distinct:
        raise RuntimeError(f"RCCL ranks share a GPU: {buses}")
    slow = max(range(len(recs)), key=lambda i: span[i])
    return {"ranks": recs, "distinct_gpus": distinct, "n_distinct_gpus": len(set(buses)),
            "slowest_rank": recs[slow]["rank"], "rank_time_max_over_min": max(span) / min(span)}


def catchment_blocks(row0, rows, ny_global, nx, k):
    """Global block raster of k catchments (8 x 8 blocks, ids mod k), this
    shard's rows; the per-catchment reduction path of the kernel."""
    r = (np.arange(row0, row0 + rows) * 8 // max(ny_global, 1))[:, None]
    c = (np.arange(nx) * 8 // nx)[None, :]
    return ((r * 8 + c) % k).astype(np.int32).reshape(-1)


def pcie_inclusive(eng, args, torch):
    """Host-fed variant of one fused launch: the fuse frames of forcing are
    first copied from pinned host memory (20 B per cell-update over PCIe,
    synchronous, no overlap), then the launch runs.  Reported beside `value`,
    never as it."""
    from topoflow_glacier import _native as nat

    n = eng.n
    names = ("P", "T_air", "Hum_sp", "P_air", "uz")
    host = torch.empty((len(names), n), dtype=torch.float32, pin_memory=True)
    for i, name in enumerate(names):  # frame 0's values, so the physics stays in range
        host[i].copy_(torch.from_numpy(eng.get_field(name, index=0, dtype=np.float32)))
    eng.sync()
    t0 = time.perf_counter()
    for f in range(args.fuse):
        for i, name in enumerate(names):
            eng._chk(eng.lib.tfg_set_field(eng.h, nat.FIELD[name], f % args.frames, host[i].data_ptr(), nat.F32, n, 0))
    t1 = time.perf_counter()
    eng.run(args.fuse)
    eng.sync()
    t2 = time.perf_counter()
    h2d = len(names) * 4 * n * args.fuse
    return {"value": n * args.fuse / (t2 - t0), "unit": "cell-updates/s", "h2d_GBps": h2d / (t1 - t0) / 1e9,
            "upload_ms": (t1 - t0) * 1e3, "launch_ms": (t2 - t1) * 1e3,
            "sample": f"{args.fuse} steps: {args.fuse} forcing frames (5 x f32 per cell) copied from pinned host "
                      f"memory, synchronously, then one fused launch"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from topoflow_glacier.bmi.config import TopoflowGlacierConfig
    from topoflow_glacier._native import NativeError
    from topoflow_glacier.engine import GlacierEngine
    from topoflow_glacier.sharding import allreduce_diagnostics
    from topoflow_glacier.synthetic import diurnal_table

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal switches for a one-GPU box (not used by the driver): every rank on
    # cuda:0 and gloo for the barrier / max-over-ranks / diagnostics reductions.
    backend = os.environ.get("TFG_BENCH_BACKEND", "nccl")
    if os.environ.get("TFG_BENCH_ONE_DEVICE") == "1":
        local = 0
    # TFG_BENCH_PG=1: a process group at world size 1 too, so the N > 1 barrier,
    # max-over-ranks and diagnostics all-reduce run over RCCL on a one-GPU box
    pg = world > 1 or os.environ.get("TFG_BENCH_PG") == "1"
    if pg:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    plan = shard_plan(args, world, rank)
    args.scaling = plan["scaling"]
    ny_global, row0, rows = plan["ny_global"], plan["row0"], plan["rows"]
    fuse_explicit = args.fuse > 0
    if not fuse_explicit:  # by the largest shard, so every rank fuses alike
        args.fuse = auto_fuse(plan["rows_max"] * args.nx, 8 if args.engine == "float64" else 4)
    cfg = TopoflowGlacierConfig.model_validate(dict(BASE_CFG, ny=rows, nx=args.nx, dt=args.dt))
    n_catch = args.catchments + 1 if args.catchments > 0 else 1
    depth_note = None
    try:
        eng = GlacierEngine(cfg, rows, args.nx, engine=args.engine, device=local, n_frames=args.frames,
                            hist_depth=args.fuse, fuse_steps=args.fuse, row0=row0, n_catch=n_catch)
    except NativeError as e:
        # the 128-step history takes 206 GB of the 266 GB footprint at 8192^2: where a
        # device cannot hold it, the round-2 depth (96 steps, 212 GB) times the same steps
        if fuse_explicit or args.fuse != FUSE_BIG or "memory" not in str(e).lower():
            raise
        depth_note = f"{FUSE_BIG}-step history did not fit ({e}); fused {FUSE_FALLBACK} steps"
        args.fuse = FUSE_FALLBACK
        eng = GlacierEngine(cfg, rows, args.nx, engine=args.engine, device=local, n_frames=args.frames,
                            hist_depth=args.fuse, fuse_steps=args.fuse, row0=row0, n_catch=n_catch)
    eng.fill_synthetic(args.seed, diurnal_table(args.frames), nx_global=args.nx)
    if args.catchments > 0:
        eng.set_field("catch_id", catchment_blocks(row0, rows, ny_global, args.nx, args.catchments))
    stream = torch.cuda.Stream(local)  # a real (non-null) stream shared by the engine and the events
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)

    def barrier():
        torch.cuda.synchronize(local)
        if pg:
            dist.barrier()

    cond_ms = []

    def conduct():
        """The optional conduction term before a launch: edge rows swapped between
        ranks (RCCL over xGMI), Qc evaluated (k_conduction), 30 m cells."""
        from topoflow_glacier.sharding import lateral_conduction

        t = time.perf_counter()
        lateral_conduction(eng, cfg.k_snow, cfg.k_ice, 30.0, 30.0, distributed=world > 1)
        cond_ms.append((time.perf_counter() - t) * 1e3)

    # warmup (untimed): the requested steps, and at least one whole launch of
    # the timed depth.  The first full-depth launch after a short warm-up runs
    # 10-29 ms long on 8192/N-row slabs (scripts/gpu_slab_warmup.sh,
    # profiles/r2p_slab_warmup.json: 1024 x 8192 after --warmup 5: 43.3 ms, then
    # 14.8 and 14.3 ms); after one such launch every later one is steady.
    warm_steps = warmup_steps(args.warmup, args.fuse)
    eng.run(warm_steps)
    barrier()
    ns_before = eng.nan_safe_launches() if args.engine == "float32" else 0
    # Whole fused launches, and at least MIN_LAUNCHES of them, so that a short
    # --steps still gives a multi-launch timed region; the JSON carries the
    # requested count beside the timed one.
    steps = timed_steps(args.steps, args.fuse, fuse_explicit)
    n_launch = steps // args.fuse
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_launch)]
    barrier()
    t0 = time.perf_counter()
    for i in range(n_launch):
        if args.conduction:
            conduct()
        ev[i][0].record(stream)
        eng.run(args.fuse)
        ev[i][1].record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    launch_ms = np.array([a.elapsed_time(b) for a, b in ev])
    own = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), **device_record(torch, local),
           "row0": row0, "rows": rows, "elapsed_s": elapsed, "launch_ms_mean": float(launch_ms.mean()),
           "launch_ms_min": float(launch_ms.min()), "launch_ms_max": float(launch_ms.max())}
    records = [own]
    if pg:
        records = [None] * dist.get_world_size()
        dist.all_gather_object(records, own)
    ranks = rank_report(records, dist.get_backend() if pg else None)
    t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}" if backend == "nccl" else "cpu")
    if pg:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    cells = rows * args.nx
    total_cells = ny_global * args.nx if args.scaling == "strong" else cells * world
    value = total_cells * steps / elapsed
    diag = allreduce_diagnostics(eng.diagnostics()) if pg else eng.diagnostics()

    mean_launch_s = float(launch_ms.mean()) / 1e3
    bytes_launch = cells * launch_bytes_per_cell(args.fuse)
    achieved = bytes_launch / mean_launch_s / 1e9
    # launches of the timed region that ran the fp32 step's NaN-safe form (0: the clean form was timed)
    ns_timed = (eng.nan_safe_launches() - ns_before) if args.engine == "float32" else None
    # the host-fed leg and the CPU baseline run on rank 0 at N=1 only (BASELINE contract)
    pcie = pcie_inclusive(eng, args, torch) if world == 1 and args.pcie else None
    eng.close()

    result = None
    if rank == 0:
        cpu = numpy_leg = parity = None
        if world == 1 and not args.no_cpu_baseline:
            def run_gpu_sample(n, steps):
                # the GPU engine on the CPU sample's cells and steps (a parity spot check)
                scfg = TopoflowGlacierConfig.model_validate(dict(BASE_CFG, ny=1, nx=n, dt=args.dt))
                se = GlacierEngine(scfg, 1, n, engine=args.engine, device=local, n_frames=args.frames,
                                   hist_depth=steps, fuse_steps=args.fuse)
                try:
                    se.fill_synthetic(args.seed, diurnal_table(args.frames), nx_global=n)
                    se.run(steps)
                    se.sync()
                    return {k: np.stack([se.get_field(k, index=j) for j in range(steps)])
                            for k in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")}
                finally:
                    se.close()

            cpu, numpy_leg, parity = cpu_baseline(args, run_gpu_sample)
        traffic, traffic_source = pmc_traffic(rows, args)
        result = {
            "metric": METRIC,
            "value": value,
            "unit": "cell-updates/s",
            "n_gpus": world,
            # what the process group saw (the driver's N > 1 lines): backend and
            # size from torch.distributed itself, not the launcher's environment
            "process_group": ({"backend": dist.get_backend(), "world_size": dist.get_world_size()} if pg else None),
            "ranks": ranks,
            "steps": steps,
            "steps_requested": args.steps,
            "depth_note": depth_note,
            # launches of the timed region that ran the fp32 step's NaN-safe form (0: the clean form was timed)
            "nan_safe_timed_launches": ns_timed,
            "steps_note": None if steps == args.steps else (
                f"timed {n_launch} whole {args.fuse}-step fused launches ({steps} steps) to cover the "
                f"{args.steps} requested: a launch keeps each cell's state in registers across its steps, so the "
                f"timed region is a whole number of launches, at least {MIN_LAUNCHES} (so that the slow first launch after "
                f"the opening barrier weighs ~1 %)"
                + ("" if fuse_explicit else f", and a multiple of {STEP_QUANTUM} steps so that every GPU count "
                                            f"times the same work")),
            "launches": {"count": n_launch, "steps_each": args.fuse, "ms_min": float(launch_ms.min()),
                         "ms_mean": float(launch_ms.mean()), "ms_max": float(launch_ms.max()),
                         "ms_each": [round(float(x), 3) for x in launch_ms]},
            "warmup": args.warmup,
            "warmup_steps_run": warm_steps,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32" if args.engine == "float32" else "f64",
            "data": "synthetic (counter-hash DEM/forcing with CSV statistics, 24 HBM-resident hourly frames)",
            "config": {
                "workload": f"{plan['workload']}, {args.dt:g} h steps, "
                            f"{args.engine} engine (fp64 state), {args.fuse} steps fused per launch"
                            + (f", {args.catchments} catchments" if args.catchments else "")
                            + (", lateral conduction re-evaluated before every launch" if args.conduction else ""),
                "grid_per_gpu": [rows, args.nx],
                "frames": args.frames,
                "fuse_steps": args.fuse,
                "parallelism": f"row-block x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_source,
                "bytes_per_cell_update": bytes_launch / (cells * args.fuse),
                "kernel_ms_per_launch": float(launch_ms.mean()),
                "note": None if args.engine == "float32" else (
                    "the fp64 engine is compute-bound, not HBM-bound: its step issues 1088 VALU instructions per "
                    "wave and cell-step, 81 % of the vector pipe at 4 waves per SIMD (profiles/r3z_issue_counters.json); "
                    "frac is its HBM share only"),
            },
            "cpu_baseline": cpu,
            "cpu_baseline_numpy_1core": numpy_leg,
            "pcie_inclusive": pcie,
            "conduction_host_ms_per_update": (float(np.mean(cond_ms)) if cond_ms else None),
            "sample_parity": parity,
            "mass_balance": {k: float(v) for k, v in zip(["vol_P", "vol_PR", "vol_PS", "vol_SM", "vol_IM", "P_max"], diag[0])},
        }
        print(json.dumps(result), flush=True)
    if pg:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
