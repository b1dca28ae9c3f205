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

--gpus N: one process per GPU.  Under torch.distributed.run (the driver) the
process group must have N ranks; started bare, the bench starts the N ranks
itself as a child torch.distributed.run and relays its line (launch_ranks).
By default the ONE 8192 x 8192 grid
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
import gc
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
HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
FORCING = ("P", "T_air", "Hum_sp", "P_air", "uz")


def bytes_model(elem: int = 4, catchments: bool = False, qc: bool = False) -> tuple[int, int]:
    """Algorithmic HBM bytes per cell of k_fused, as
    (per step, per launch), for an engine whose forcing frames, output slots
    and geometry are `elem`-byte values (4: the fp32 engine, 8: the fp64 one):
      per step:   forcing 5 x elem read, window slot 4 read + 4 written, six
                  outputs 6 x elem written  (fp32 52 B, fp64 96 B);
      per launch: geometry (fp32 engine five f32 planes, fp64 engine seven f64
                  planes), state five f64 + window total i64 read and written,
                  albedo (fp64 engine: f64 read and written; fp32 engine: f32
                  written only -- the step rebuilds it from n and the depths,
                  round 6), the catchment id (i32) and Qc (elem) when the
                  variant reads them  (fp32 120 B, fp64 168 B)."""
    step = 5 * elem + 4 + 4 + 6 * elem
    geo = 5 * 4 if elem == 4 else 7 * 8
    albedo = 4 if elem == 4 else 2 * 8
    launch = geo + 2 * (5 * 8 + 8) + albedo + (4 if catchments else 0) + (elem if qc else 0)
    return step, launch


def launch_bytes_per_cell(fuse: int, elem: int = 4, catchments: bool = False, qc: bool = False) -> int:
    """Algorithmic HBM bytes per cell of one fused launch of `fuse` steps:
    fp32 engine 52 per step + 120 per launch, fp64 engine 96 + 168.  (Keeping
    the window slots that a launch reads back itself in LDS would save 8 B per
    such step, but reserving the LDS cost 8 % of throughput on its own: HISTORY.md.)"""
    step, launch = bytes_model(elem, catchments, qc)
    return step * fuse + launch

PARITY_CELL_STEPS = 262144 * 129
MIN_LAUNCHES = 6
# Why 6: the first launch after the barrier that opens the timed region runs
# 0.5-3.6 ms long at every shape and warm-up length (profiles/r3c_slab_skew_study.jsonl,
# profiles/r3f_slab_depth_study.jsonl); over 6 launches it weighs ~1 % on the
# 1024 x 8192 slab instead of ~2 % over 3 (HISTORY.md section 6).
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


DEVICE_BYTES_BUDGET = 280e9  # of an MI355X's 288 GB HBM: the rest for the runtime and torch
DEPTH_LADDER = (384, 256, 192, 128, 96)  # automatic depths and fallbacks: each divides STEP_QUANTUM


def device_footprint(cells: int, frames: int, hist_depth: int, ring_len: int, n_catch: int = 1, elem: int = 4,
                     catchments: bool = False, cus: int = 256) -> int:
    """Device bytes of one shard's handle, as tfg_create allocates them
    (csrc/tfg_engine.hip, tfg_create) plus the catchment raster: per padded
    cell forcing frames 5 x elem each, static rasters 3 x elem, LW/SW 2 x elem,
    geometry (fp32 engine 5 x f32 + 2 x f64, fp64 engine 7 x f64), state
    8 x f64, window total i64, window slots i32 each, output slots 6 x elem
    each, catchment id i32; plus the per-workgroup diagnostic slab."""
    n_pad = -(-cells // 64) * 64
    if n_pad >= 1 << 20:
        n_pad += 512  # kPlaneSkew
    geo = 5 * 4 + 2 * 8 if elem == 4 else 7 * 8
    per = frames * 5 * elem + 3 * elem + 2 * elem + geo + 8 * 8 + 8 + ring_len * 4 + hist_depth * 6 * elem
    per += 4 if catchments else 0
    blocks = max(256, min(cus * 512, (256 << 20) // (n_catch * 48)))
    blocks = 1 << (blocks.bit_length() - 1)
    blocks = min(blocks, -(-n_pad // 256))
    return n_pad * per + blocks * n_catch * 48 + n_catch * 48


def fit_depth(fuse: int, cells: int, frames: int, ring_len: int, n_catch: int, elem: int, catchments: bool,
              budget: float = DEVICE_BYTES_BUDGET) -> int:
    """The automatic depth, or the next shallower one of DEPTH_LADDER while the
    shard's footprint (history slots = depth) exceeds the device budget."""
    k = fuse
    while device_footprint(cells, frames, k, ring_len, n_catch, elem, catchments) > budget:
        smaller = [d for d in DEPTH_LADDER if d < k]
        if not smaller:
            break
        k = smaller[0]
    return k


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
    ap.add_argument("--flux", default="fp32", choices=["fp32", "fp64"],
                    help="the float32 engine's flux arithmetic (tfg_set_flux): fp64 = the dew point, turbulent "
                         "fluxes and long-wave balance in fp64")
    ap.add_argument("--split", default="auto", choices=["auto", "off", "on"],
                    help="two-part launches of a small fp32 grid on two streams (tfg_set_split; auto: 2^18 .. 2^24 "
                         "cells per GPU)")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="strong (default: one --ny x --nx grid row-partitioned over the ranks, BASELINE "
                         "config 4) or weak (--ny rows per rank)")
    ap.add_argument("--seed", type=int, default=20251001)
    ap.add_argument("--cpu-cells", type=int, default=1048576, help="cells in the C CPU-baseline sample")
    ap.add_argument("--cpu-steps", type=int, default=960, help="steps of the C CPU-baseline sample (~10 s on 16 threads)")
    ap.add_argument("--parity-steps", type=int, default=0,
                    help="steps of the GPU-vs-oracle check after its one-step lead-in launch; 0 = one whole "
                         "launch of the timed depth (--fuse)")
    ap.add_argument("--parity-cells", type=int, default=0,
                    help="cells of each rank's GPU-vs-oracle check (whole rows of its own shard; also the numpy "
                         "one-core sample at N = 1); 0 = 262144 at N = 1, 65536 per rank at N > 1")
    ap.add_argument("--no-parity", action="store_true", help="skip the per-rank GPU-vs-oracle check")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in path legs (per-step update() from device inputs, defer_update instances)")
    ap.add_argument("--dropin-queued", action="store_true",
                    help="add the queued variant of the per-step grid leg (the same steps set into frames, then one "
                         "fused launch); off by default: its short launches of the timed kernel would enter the "
                         "kernel's rocprof average")
    ap.add_argument("--dropin-clean", action="store_true",
                    help="add the clean-form K = 1 launches beside the per-step grid leg (a same-run A/B of the two "
                         "step forms); off by default: they are launches of the timed kernel instance at K = 1, "
                         "which would enter its rocprof average")
    ap.add_argument("--dropin-instances", type=int, default=4096,
                    help="single-catchment BMI models of the defer_update leg")
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


_T0 = time.perf_counter()


def note(msg: str) -> None:
    """A progress line on stderr (stdout carries only the JSON line): a long
    phase (the oracle of a deep parity launch, the CPU baseline) stays visible."""
    print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def _cpu_threads() -> int:
    """Host threads for the C baseline: the process's CPU share (16 on a one-GPU
    box, where OMP_NUM_THREADS is set to it), never the whole machine."""
    env = os.environ.get("OMP_NUM_THREADS")
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    n = int(env) if env and env.isdigit() else avail
    return max(1, min(n, avail, 16))


def _floored_rel(g, r, s_v=None):
    """|gpu - ref| / max(|ref|, s_v), s_v = p99 of the non-zero |ref|
    (pass s_v to take it from the whole sample when g, r are a masked part)."""
    if s_v is None:
        nz = np.abs(r[r != 0])
        s_v = np.percentile(nz, 99) if nz.size else 0.0
    fl = np.maximum(np.maximum(np.abs(r), s_v), 1e-300)
    e = np.abs(g - r) / fl
    return float(np.max(e)), float(np.mean(e > 1e-5))


def cpu_baseline(args):
    """The reported CPU baseline, on rank 0 at N=1: the C oracle
    (oracle/tfg_oracle_c.c, the fp64 restatement of update(), OpenMP over the
    process's CPU share) on the first --cpu-cells cells x --cpu-steps steps of
    the same synthetic workload (the same fp32 inputs as the GPU)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import tfg_oracle as O
    import tfg_oracle_c as OC

    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    n = min(args.cpu_cells, args.nx * args.ny)
    steps = args.cpu_steps
    syn = synthetic_cells(args.seed, np.arange(n), diurnal_table(args.frames))
    static = _static_of(syn)
    cfg = dict(BASE_CFG, dt=args.dt)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    threads = _cpu_threads()
    forcing = {k: np.ascontiguousarray(syn[k], dtype=np.float64) for k in FORCING}
    t0 = time.perf_counter()
    OC.run_oracle_c(cfg, static, forcing, steps, clock=(jd, tsn), frames=np.arange(steps) % args.frames, hist=False,
                    nthreads=threads)
    t_c = time.perf_counter() - t0
    return {"value": n * steps / t_c, "unit": "cell-updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle/tfg_oracle_c.c (C fp64 restatement of update(), OpenMP, {threads} threads) on the "
                      f"first {n} cells x {steps} {args.dt:g} h steps of the same synthetic workload ({t_c:.1f} s)"}


def _static_of(syn: dict) -> dict:
    return {k: np.asarray(syn[s], dtype=np.float64) for k, s in (
        ("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"), ("h0_snow", "h_snow"), ("h0_ice", "h_ice"),
        ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}


def parity_plan(args, plan: dict, world: int) -> dict:
    """The cells and launches of a rank's parity check: whole rows at the top of
    its OWN shard (global rows row0 .. row0 + rows - 1), read from the bench's
    own handle, whose first launches are a one-step lead-in (the k_fused
    instance that reads the initial depths) and then one whole launch of the
    timed depth over the whole shard (capture_parity): the timed kernel
    instance at the timed launch length and shape (at K = 128 the
    three-register-set step loop ends in its two-step tail)."""
    k = args.parity_steps or args.fuse
    # the oracle's work bounded to that of 262144 cells x 129 steps (the N = 1
    # headline check, ~60 s of host time): deeper launches check fewer rows
    want = args.parity_cells or min(262144 if world == 1 else 65536, PARITY_CELL_STEPS // (1 + k))
    rows = max(1, min(plan["rows"], want // args.nx))
    return {"row0": plan["row0"], "rows": rows, "cells": rows * args.nx, "launch_steps": [1, k], "steps": 1 + k}


def capture_parity(eng, args, plan: dict, world: int, torch, local: int) -> dict:
    """The GPU side of this rank's parity check, on the bench's own handle
    before its warm-up: a one-step lead-in launch, then ONE whole launch of
    the timed depth over the whole shard, the same kernel instance and launch
    shape as every timed launch.  Keeps the outputs of the first parity_plan
    cells (a leading block of rows; tfg_get_field reads that prefix) at all
    1 + K steps, and the shard's mass-balance integrals after these steps
    beside fp64 sums of the forcing frames they read (torch on the device,
    per catchment: vol_P, vol_PR, vol_PS, P_max; :558-624)."""
    pp = parity_plan(args, plan, world)
    n, k = pp["cells"], pp["launch_steps"][1]
    if eng.step_index != 0 or k > eng.hist_depth:
        raise RuntimeError("capture_parity runs first on the handle, and keeps at most hist_depth steps")
    ns0 = eng.nan_safe_launches() if args.engine == "float32" else 0
    eng.run(1)  # lead-in: hist slot 0
    eng.sync()
    gpu = {v: [eng.get_field(v, index=0, dtype=np.float32 if args.engine == "float32" else np.float64, cells=n)]
           for v in HIST}
    eng.run(k)  # step j (1..k) writes slot j % hist_depth
    eng.sync()
    for v in HIST:
        gpu[v] += [eng.get_field(v, index=j % eng.hist_depth, dtype=gpu[v][0].dtype, cells=n) for j in range(1, k + 1)]
    gpu = {v: np.stack(x).astype(np.float64) for v, x in gpu.items()}
    ns = (eng.nan_safe_launches() - ns0) if args.engine == "float32" else 0
    diag = eng.diagnostics()
    # what the shard's integrals must be: per-cell fp64 sums of the frames the 1 + k steps read
    kc = max(args.catchments, 1)
    dev = torch.device("cuda", local)
    cnt = np.bincount(np.arange(1 + k) % args.frames, minlength=args.frames)
    P = torch.empty(eng.n, dtype=torch.float32 if args.engine == "float32" else torch.float64, device=dev)
    T = torch.empty_like(P)
    sums = torch.zeros((3, eng.n), dtype=torch.float64, device=dev)
    pcell = torch.full((eng.n,), -float("inf"), dtype=torch.float64, device=dev)
    t_rs = BASE_CFG["T_rain_snow"]
    for f in np.nonzero(cnt)[0]:  # per cell first: elementwise, no two cells share an address
        eng.get_field_device("P", P, index=int(f))
        eng.get_field_device("T_air", T, index=int(f))
        p64 = P.double()
        rain = T.double() > t_rs
        sums[0] += p64 * float(cnt[f])
        sums[1] += torch.where(rain, p64, 0.0) * float(cnt[f])
        sums[2] += torch.where(rain, 0.0, p64) * float(cnt[f])
        torch.maximum(pcell, p64, out=pcell)
    # then per catchment as reductions, not atomics: an index_add_ / scatter_reduce of
    # every cell into one bin serialised on that address (~68 s of a driver run at 8192^2)
    if args.catchments:
        cid = catchment_blocks(plan["row0"], plan["rows"], plan["ny_global"], args.nx, args.catchments)
        order = torch.argsort(torch.from_numpy(cid).to(dev), stable=True)
        lengths = torch.from_numpy(np.bincount(cid, minlength=kc)).to(dev)

        def seg(x, how):
            return torch.segment_reduce(x[order], how, lengths=lengths)
    else:
        def seg(x, how):
            return (x.sum() if how == "sum" else x.max()).reshape(1)
    da_dt = BASE_CFG["da"] * 1e6 * args.dt
    want = torch.stack([seg(sums[i], "sum") for i in range(3)], 1).cpu().numpy() * da_dt
    # P_max starts at 0 (:314, the reference's initial value): a catchment with no cells in this shard (a
    # rank's slab of the 43-catchment block raster holds only some of them) keeps 0
    return {"plan": pp, "gpu": gpu, "nan_safe_launches": ns, "diag": diag, "want_P_PR_PS": want,
            "want_P_max": np.maximum(seg(pcell, "max").cpu().numpy(), 0.0)}


def oracle_sample(args, pp: dict, threads: int):
    """The reference side of a rank's parity check: the numpy oracle
    (oracle/tfg_oracle.py, fp64, bit-exact to the reference fixtures) on the
    host mirror of the synthetic fp32 inputs of parity_plan's cells (global
    cell indices), every output and the four energy terms at every step, and
    the C oracle (the fp64 baseline of the flip rule) on the same cells.
    Returns (ref, c64, the numpy run as a one-core CPU leg, cfg)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import tfg_oracle as O
    import tfg_oracle_c as OC

    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    rows, nx, row0, steps, n = pp["rows"], args.nx, pp["row0"], pp["steps"], pp["cells"]
    cells = ((row0 + np.arange(rows))[:, None] * nx + np.arange(nx)[None, :]).reshape(-1)
    syn = synthetic_cells(args.seed, cells, diurnal_table(args.frames))
    static = _static_of(syn)
    cfg = dict(BASE_CFG, dt=args.dt)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], steps, cfg["lon"])
    frames = np.arange(steps) % args.frames
    forcing = {k: np.ascontiguousarray(syn[k], dtype=np.float64) for k in FORCING}
    ref = {v: np.empty((steps, n)) for v in HIST}
    terms = ("Qn_SW", "Qn_LW", "Qh", "Qe")  # the energy moved, for the melt-onset rule (harness.melt_onsets)
    for t in terms:
        ref[t] = np.empty((steps, n), np.float32)
    t0 = time.perf_counter()
    m = O.OracleGrid(cfg, **static)
    for k in range(steps):
        r = m.step(*(forcing[v][frames[k]] for v in FORCING), jd[k], tsn[k])
        for v in HIST + terms:
            ref[v][k] = r[v]
        if k % 64 == 63:
            note(f"parity: numpy oracle step {k + 1}/{steps} on {n} cells")
    t_np = time.perf_counter() - t0
    numpy_leg = {"value": n * steps / t_np, "unit": "cell-updates/s", "cores": 1, "kind": "port",
                 "sample": f"oracle/tfg_oracle.py (numpy fp64, single thread) on {n} cells x {steps} steps "
                           f"({t_np:.1f} s), the reference of the parity check"}
    note("parity: C oracle (fp64 baseline of the flip rule)")
    c64, _ = OC.run_oracle_c(cfg, static, forcing, steps, clock=(jd, tsn), frames=frames, hist=True, nthreads=threads)
    return ref, {v: c64[v] for v in HIST}, numpy_leg, cfg


def sample_parity(args, plan: dict, world: int, rank: int, threads: int, cap: dict):
    """This rank's GPU-vs-oracle check, outside the timed region (every rank,
    at every N): the outputs capture_parity kept from the bench handle's own
    lead-in and first whole launch, on the first rows of this rank's shard,
    against the numpy oracle (oracle/tfg_oracle.py, fp64, bit-exact to the
    reference fixtures) on the host mirror of the same synthetic fp32 inputs,
    every output at every step.  Cells whose trajectories part at a melt-out
    residual are compared up to the flip and counted, held to the fp64
    baseline of the same cells and steps (the C oracle against the numpy
    oracle; tests/harness.py flip_rule).  The shard's per-catchment
    precipitation integrals and P_max are checked against the sums of the
    forcing it read.

    Returns (parity dict, the numpy run's single-core rate as a CPU leg)."""
    from tests.harness import ONSET_FRAC_MAX, classify_sample, flip_rule, scale_floor, valid_mask

    pp = cap["plan"]
    rows, nx, row0, steps = pp["rows"], args.nx, pp["row0"], pp["steps"]
    n = pp["cells"]
    gpu, diag, ns = cap["gpu"], cap["diag"], cap["nan_safe_launches"]
    ref, c64, numpy_leg, cfg = oracle_sample(args, pp, threads)
    tol = 1e-5 if args.engine == "float32" else 1e-10
    # depletion steps (the rate carries the remaining depth's error), melt-out flips held to the fp64
    # baseline (C oracle vs numpy oracle) and, for the fp32 engine, melt onsets (E_in - Eccs cancelling),
    # classified as the GPU suite does (tests/harness.py classify_sample)
    note("parity: classifying the sample")
    # the melt-onset allowance is the fp32 flux's only (the fp64-flux form is held without it)
    cls = classify_sample(gpu, ref, c64, cfg, tol, onsets=args.engine == "float32" and args.flux == "fp32")
    excused, flip, genuine, onset, ok = cls.excused, cls.flip, cls.genuine, cls.onset, cls.ok
    flip64, genuine64, ex64, onset_ok = cls.flip64, cls.genuine64, cls.ex64, cls.onset_ok
    # each output's floor s_v from the whole sample (as the classifiers take it), not the compared part
    floors = {v: scale_floor(ref[v]) for v in HIST}
    by_out = {v: _floored_rel(gpu[v][ok], ref[v][ok], floors[v])[0] for v in HIST}
    err = max(by_out.values())
    # the same statistic with the depletion steps' rate entries compared at the rate's floor too, and the
    # fp64 baseline's (C oracle vs numpy oracle) under the same rules
    cut_ok = valid_mask(cls.cut, steps)
    err_incl = max(_floored_rel(gpu[v][cut_ok], ref[v][cut_ok], floors[v])[0] for v in HIST)
    ok64 = valid_mask(flip64, steps) & ~ex64
    err64 = max(_floored_rel(c64[v][ok64], ref[v][ok64], floors[v])[0] for v in HIST)
    del c64
    worst = {}  # where the largest floored error sits (diagnosis of the margin)
    vw = max(by_out, key=by_out.get)
    s_v = float(floors[vw])
    e_w = np.where(ok, np.abs(gpu[vw] - ref[vw]) / np.maximum(np.maximum(np.abs(ref[vw]), s_v), 1e-300), 0.0)
    kw, cw = np.unravel_index(int(np.argmax(e_w)), e_w.shape)
    worst = {"output": vw, "cell": int(cw), "global_row": int(row0 + cw // nx), "step": int(kw), "floor_s_v": s_v,
             **{f"{v}_gpu_ref": [float(gpu[v][kw, cw]), float(ref[v][kw, cw])] for v in HIST},
             "h_snow_gpu_ref_step_before": ([float(gpu["h_snow"][kw - 1, cw]), float(ref["h_snow"][kw - 1, cw])]
                                            if kw > 0 else None)}
    pure = {}  # the fraction of compared values above pure-relative 1e-5
    for v in HIST:
        gv, rv = gpu[v][ok], ref[v][ok]
        with np.errstate(divide="ignore", invalid="ignore"):
            rel = np.where(rv != 0, np.abs(gv - rv) / np.abs(rv), np.where(gv != rv, np.inf, 0.0))
        pure[v] = float(np.mean(rel > 1e-5))
    rule = flip_rule(int((flip >= 0).sum()), int((flip64 >= 0).sum()))
    examples = []  # the first genuine mismatches, with the state around them (diagnosis)
    for c, k, vs in genuine[:6]:
        j = [max(k - 2, 0), max(k - 1, 0), k]
        examples.append({"cell": int(c), "global_row": int(row0 + c // nx), "step": int(k), "outputs": vs,
                         **{f"{v}_gpu_ref_steps_k-2_k-1_k": [[float(gpu[v][i, c]), float(ref[v][i, c])] for i in j]
                            for v in ("h_snow", "SM", "h_ice", "IM")}})
    # the shard's mass-balance integrals after the same steps (:558-624), per catchment
    kc = max(args.catchments, 1)
    want = cap["want_P_PR_PS"]
    with np.errstate(divide="ignore", invalid="ignore"):
        p_err = float(np.max(np.where(want != 0, np.abs(diag[:kc, :3] - want) / np.abs(want), np.abs(diag[:kc, :3]))))
    mass = {"catchments": kc, "cells": plan["rows"] * nx, "vol_P_PR_PS_max_rel": p_err,
            "vol_P_PR_PS_tolerance": 1e-6, "P_max_exact": bool(np.array_equal(diag[:kc, 5], cap["want_P_max"])),
            "vs": "fp64 sums of the forcing frames the shard read (torch on the device), per catchment"}
    engine_desc = ("k_fused<float, READ_DEPTHS=false, CATCH=%s, QC=false, clean form%s>"
                   % ("true" if args.catchments else "false", ", fp64 flux" if args.flux == "fp64" else "")
                   if args.engine == "float32" else "k_fused<double, exact, READ_DEPTHS=false>")
    parity = {"vs": "numpy oracle (fp64; pinned bit-exact to the reference fixtures)", "rank": rank,
              "global_rows": [row0, row0 + rows - 1], "cells": n, "steps": pp["launch_steps"][1],
              "lead_in_steps": pp["launch_steps"][0], "steps_compared": steps, "launch_steps": pp["launch_steps"],
              "timed_kernel_instance": engine_desc + f" in a {pp['launch_steps'][1]}-step launch over the whole "
                                                     f"{plan['rows']}x{nx} shard (the bench handle's first, after a "
                                                     f"one-step lead-in launch that reads the initial depths)",
              "nan_safe_launches": ns, "outputs": list(HIST), "max_floored_rel": err,
              "max_floored_rel_incl_depletion_rates": err_incl, "max_floored_rel_fp64_baseline": err64,
              "max_floored_rel_by_output": by_out, "max_floored_rel_at": worst, "tolerance": tol, "frac_above_pure_rel_1e-5": pure,
              "melt_out_flips": rule["flips"], "flips_fp64_baseline": rule["fp64_flips"], "flip_ratio": rule["ratio"],
              "flip_budget": rule["budget"], "flip_rule": rule["rule"], "genuine_mismatches": len(genuine),
              "fp64_baseline_genuine_mismatches": len(genuine64), "genuine_examples": examples,
              "melt_onsets_explained": len(onset), "melt_onset_budget": int(np.ceil(ONSET_FRAC_MAX * n)),
              "melt_onset_rule": "SM / M_total at melt onset within 1e-6 of the energy moved so far, in at most "
                                 f"{ONSET_FRAC_MAX:.1%} of the cells (tests/harness.py melt_onsets)",
              "depletion_steps": int(excused.sum()), "depletion_steps_fp64_baseline": int(ex64.sum()),
              "depletion_rule": "at the step a reservoir runs dry in both runs the melt rate is the depth left at "
                                "the step before: SM / IM checked by that identity (the rate's difference x 3600 "
                                "w = the previous depth's difference, to the outputs' rounding), M_total = SM + IM, "
                                "the depths and RH at their own tolerance (tests/harness.py depletion_steps)",
              "flip_cut": "a cell is compared up to the step its melt-out zero gates part (exact zero in one run, a "
                          "sub-1e-9 m residual in the other), for the GPU and the fp64 baseline alike "
                          "(tests/harness.py melt_out_flips)",
              "mass_balance": mass,
              "ok": bool(err <= tol and not genuine and rule["ok"] and onset_ok and ns == 0 and p_err <= 1e-6
                         and mass["P_max_exact"])}
    return parity, numpy_leg


def parity_summary(per_rank: list[dict]) -> dict:
    """The N > 1 line's parity: every rank's own check (ranks[].sample_parity) folded."""
    ok = [p for p in per_rank if p is not None]
    if not ok:
        return None
    return {"vs": ok[0]["vs"], "ranks_checked": [p["rank"] for p in ok], "cells": sum(p["cells"] for p in ok),
            "steps": ok[0]["steps"], "steps_compared": ok[0]["steps_compared"],
            "max_floored_rel": max(p["max_floored_rel"] for p in ok), "tolerance": ok[0]["tolerance"],
            "max_floored_rel_incl_depletion_rates": max(p.get("max_floored_rel_incl_depletion_rates", 0.0) for p in ok),
            "max_floored_rel_fp64_baseline": max(p.get("max_floored_rel_fp64_baseline", 0.0) for p in ok),
            "melt_out_flips": sum(p["melt_out_flips"] for p in ok),
            "flips_fp64_baseline": sum(p["flips_fp64_baseline"] for p in ok),
            "genuine_mismatches": sum(p["genuine_mismatches"] for p in ok),
            "melt_onsets_explained": sum(p.get("melt_onsets_explained", 0) for p in ok),
            "depletion_steps": sum(p.get("depletion_steps", 0) for p in ok),
            "per_rank": "ranks.ranks[].sample_parity", "ok": all(p["ok"] for p in ok) and len(ok) == len(per_rank)}


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
    and engine (scripts/gpu_pmc.sh -> profiles/pmc_<nx>x<rows>_fuse<K>.json for
    the fp32 engine, ..._f64.json for the fp64 one), quoted only when the
    profile was measured on the same machine code of the timed kernel as the
    running library's (_native.kernel_code_sha256: the kernel's instructions,
    descriptor and callees, not the other kernels of the library); otherwise
    null, with the reason."""
    from topoflow_glacier import _native as nat

    suffix = ("_fluxf64" if args.flux == "fp64" else "") if args.engine == "float32" else "_f64"
    symbol = ((nat.BENCH_KERNEL_PREC if args.flux == "fp64" else nat.BENCH_KERNEL) if args.engine == "float32"
              else nat.BENCH_KERNEL_F64)
    pmc = ROOT / "profiles" / f"pmc_{args.nx}x{rows}_fuse{args.fuse}{suffix}.json"
    if args.catchments or args.dt != 1.0 or args.conduction:
        return None, {"profile": None, "reason": "no PMC profile for this variant of the kernel"}
    if not pmc.exists():
        return None, {"profile": None, "reason": f"{pmc.relative_to(ROOT)} not measured"}
    running = nat.kernel_code_sha256(symbol)
    prof = json.loads(pmc.read_text())
    measured = prof.get("kernel_code_sha256")
    src = {"profile": str(pmc.relative_to(ROOT)), "kernel": symbol, "kernel_code_sha256": measured,
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


def dropin_grid_leg(eng, args, torch, stream, steps: int = 24) -> dict:
    """The grid path NextGen drives (examples/run_topoflow_glacier.py:64-109,
    tests/integration_test.py:102-147 of the reference: set the inputs, then
    update(), every step), with the inputs already on the device: per step
    one tfg_set_inputs from a device [5][n] f32 block (BMI order P_air, Hum_sp,
    P, T_air, uz: 20 B read + 20 B written per cell) and one tfg_step of one
    step (a K = 1 launch: 52 + 120 = 172 B per cell-update).  Beside it the
    same steps queued: the inputs of `steps` steps set into as many frames,
    then one fused launch (what a deferred grid update() would do).  Never
    `value`."""
    names = ("P_air", "Hum_sp", "P", "T_air", "uz")
    n = eng.n
    steps = min(steps, args.frames, args.fuse)
    blk = torch.empty((5, n), dtype=torch.float32, device=f"cuda:{eng.device}")
    for i, name in enumerate(names):  # frame 0's values: the physics stays in range
        eng.get_field_device(name, blk[i], index=0)
    step_b, launch_b = bytes_model(4)
    out = {"cells": n, "steps": steps,
           "protocol": "per step: tfg_set_inputs (device f32 [5][n]) + tfg_step(1)" + (
               f"; queued: the same inputs into {steps} frames, then one {steps}-step launch" if args.dropin_queued
               else "")}
    # --dropin-clean: first the same K = 1 launches in the clean step form, for a same-run A/B of the two forms
    # at 172 B per cell-update: the frames as fill_synthetic wrote them (known finite), no inputs set, each launch
    # between HIP events (before the per-step protocol, whose device-set inputs leave the frames of unknown
    # status).  Off by default: they are launches of the timed kernel instance at K = 1, which would enter its
    # rocprof average (profiles/r5_dropin_form_ab.json holds the A/B)
    c_ms = None
    if args.dropin_clean:
        ns0 = eng.nan_safe_launches()
        ev_c = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize(eng.device)
        for s in range(steps):
            ev_c[s][0].record(stream)
            eng.run(1)
            eng.join()  # a split engine's second part (no-op otherwise)
            ev_c[s][1].record(stream)
        torch.cuda.synchronize(eng.device)
        c_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_c]))
        out["clean_form_step_launch"] = {
            "step_launch_ms": c_ms, "nan_safe_launches": eng.nan_safe_launches() - ns0,
            "step_launch_GBps": n * (step_b + launch_b) / (c_ms / 1e3) / 1e9,
            "note": "per_step's launches read device-set inputs and run the NaN-safe form (device data is not known "
                    "to be finite without a host wait); these read host-checked frames and run the clean form"}
    for mode in ("per_step", "queued") if args.dropin_queued else ("per_step",):
        ns0 = eng.nan_safe_launches()
        ev_k = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(eng.device)
        t0 = time.perf_counter()
        e0.record(stream)
        if mode == "per_step":
            for s in range(steps):
                eng.set_inputs(blk, index=eng.step_index % args.frames)
                ev_k[s][0].record(stream)
                eng.run(1)
                eng.join()  # a split engine's second part (no-op otherwise)
                ev_k[s][1].record(stream)
        else:
            for s in range(steps):
                eng.set_inputs(blk, index=(eng.step_index + s) % args.frames)
            eng.run(steps)
        eng.join()
        e1.record(stream)
        torch.cuda.synchronize(eng.device)
        wall = time.perf_counter() - t0
        dev_ms = e0.elapsed_time(e1)
        rec = {"value": n * steps / wall, "unit": "cell-updates/s", "ms_per_step": wall / steps * 1e3,
               "device_ms_per_step": dev_ms / steps, "nan_safe_launches": eng.nan_safe_launches() - ns0}
        if mode == "per_step":
            k_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_k]))
            rec.update({"step_launch_ms": k_ms, "bytes_per_cell_update": step_b + launch_b,
                        "step_launch_GBps": n * (step_b + launch_b) / (k_ms / 1e3) / 1e9,
                        "bytes_per_cell_update_with_input_copy": step_b + launch_b + 40})
            rec["step_launch_frac"] = rec["step_launch_GBps"] / HBM_PEAK_GBS
        else:
            rec.update({"bytes_per_cell_update": step_b + launch_b / steps + 40})
        rec["device_GBps"] = n * rec["bytes_per_cell_update" if mode == "queued" else
                                     "bytes_per_cell_update_with_input_copy"] / (dev_ms / steps / 1e3) / 1e9
        rec["frac"] = rec["device_GBps"] / HBM_PEAK_GBS
        out[mode] = rec
    if c_ms is not None:
        out["clean_form_step_launch"]["nan_safe_over_clean"] = out["per_step"]["step_launch_ms"] / c_ms
    del blk
    return out


def dropin_instances_leg(args, local: int, steps: int = 8) -> dict:
    """NextGen's many-catchment pattern: one single-catchment BMI model per
    catchment in one process (examples/run_topoflow_glacier.py:64-109 per
    model), with the additive key defer_update: every model's 7 set_value and
    update() (queued), then every model's 8 get_value (the first one runs all
    queued steps: one tfg_update_many call, one k_cell_many launch).  One
    untimed round first.  Never `value`."""
    import tempfile

    import yaml

    from topoflow_glacier import BmiTopoflowGlacier

    with tempfile.TemporaryDirectory() as td:
        cfgf = Path(td) / "cat.yaml"
        cfgf.write_text(yaml.safe_dump(dict(BASE_CFG, defer_update=True, device=local)))
        t0 = time.perf_counter()
        models = []
        for _ in range(args.dropin_instances):
            m = BmiTopoflowGlacier()
            m.initialize(str(cfgf))
            models.append(m)
        t_create = time.perf_counter() - t0
    ins = {"atmosphere_water__liquid_equivalent_precipitation_rate": 1e-7, "land_surface_air__temperature": -2.0,
           "land_surface_air__pressure": 88000.0, "atmosphere_air_water~vapor__relative_saturation": 0.003,
           "wind_speed_UV": 3.0, "land_surface_radiation~incoming~longwave__energy_flux": 250.0,
           "land_surface_radiation~incoming~shortwave__energy_flux": 100.0}
    # numpy scalars, as the reference's driver passes them (examples/run_topoflow_glacier.py:65-73: values of
    # pandas columns, one per step)
    vals = {k: np.float64(v) for k, v in ins.items()}
    outs = models[0].get_output_var_names()
    buf = np.zeros(1)
    t_set = t_get = 0.0
    for r in range(steps + 1):  # round 0 untimed
        a = time.perf_counter()
        for m in models:
            for k, v in vals.items():
                m.set_value(k, v)
            m.update()
        b = time.perf_counter()
        for m in models:
            for k in outs:
                m.get_value(k, buf)
        c = time.perf_counter()
        if r:
            t_set += b - a
            t_get += c - b
    ref = models[0].get_value("land_surface_water__runoff_volume_flux", np.zeros(1))[0]
    same = all(m.get_value("land_surface_water__runoff_volume_flux", np.zeros(1))[0] == ref for m in models)
    for m in models:
        m.finalize()
    per = (t_set + t_get) / (len(models) * steps) * 1e6
    return {"instances": len(models), "steps": steps, "us_per_instance_step": per,
            "instance_steps_per_s": 1e6 / per, "us_set_and_update": t_set / (len(models) * steps) * 1e6,
            "us_get_incl_launch": t_get / (len(models) * steps) * 1e6, "create_s": t_create,
            "all_instances_equal": bool(same),
            "protocol": "ensemble order: every model's 7 set_value (numpy scalars, as the reference's driver) + "
                        "update() (queued), then every model's 8 get_value (the first runs the queued steps in one "
                        "k_cell_many launch)"}


def rank_launch_command(gpus: int, argv: list[str], port: int) -> list[str]:
    """The child that runs this bench as `gpus` ranks, one process per GPU, as
    the driver itself launches N > 1 (torch.distributed.run, 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), *argv]


def launch_ranks(args, argv: list[str]) -> int | None:
    """`--gpus N` is honoured however the bench is started.  Under a launcher
    (WORLD_SIZE set) the process group must have N ranks: a mismatch exits 2
    rather than print a line for another N.  Started bare with N > 1, the bench
    runs N ranks as a CHILD process (torch.distributed.run; this process never
    touches the GPU, so nothing is exec'd after GPU initialisation), relays
    rank 0's one JSON line on stdout and everything else on stderr, and exits
    with the child's code.  Returns None when this process is itself the rank."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks", file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = rank_launch_command(args.gpus, argv, port)
    note(f"--gpus {args.gpus}: starting {args.gpus} ranks: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, cwd=str(ROOT))
    for line in proc.stdout:
        if line.lstrip().startswith("{"):
            print(line.rstrip("\n"), flush=True)
        else:
            print(line, end="", file=sys.stderr, flush=True)
    return proc.wait()


def agree_on_depth(depth: int, pg: bool, torch, dist, local: int, backend: str) -> int:
    """Every rank fuses the same depth: the smallest any rank could allocate
    (a rank whose tfg_create ran out of memory stepped down DEPTH_LADDER).  A
    rank that could allocate none joins with 0, so the collective completes on
    every rank and all of them stop (the caller exits non-zero on 0) instead of
    the others waiting for it until the process-group timeout."""
    if not pg:
        return depth
    t = torch.tensor([depth], dtype=torch.int64, device=f"cuda:{local}" if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def main(args=None):
    args = args or parse()
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
    cfg = TopoflowGlacierConfig.model_validate(dict(BASE_CFG, ny=rows, nx=args.nx, dt=args.dt))
    n_catch = args.catchments + 1 if args.catchments > 0 else 1
    elem = 8 if args.engine == "float64" else 4
    ring_len = int(3 * 24 / args.dt)
    depth_note = None
    if not fuse_explicit:  # by the largest shard, so every rank fuses alike
        auto = auto_fuse(plan["rows_max"] * args.nx, elem)
        args.fuse = fit_depth(auto, plan["rows_max"] * args.nx, args.frames, ring_len, n_catch, elem,
                              args.catchments > 0)
        if args.fuse != auto:
            depth_note = f"{auto}-step history over the {DEVICE_BYTES_BUDGET / 1e9:.0f} GB budget; fused {args.fuse} steps"
    def create(depth: int):
        return GlacierEngine(cfg, rows, args.nx, engine=args.engine, device=local, n_frames=args.frames, flux=args.flux,
                             hist_depth=depth, fuse_steps=depth, row0=row0, n_catch=n_catch, split=args.split)

    eng, create_error = None, None
    while True:
        try:
            eng = create(args.fuse)
            break
        except NativeError as e:
            # a device that cannot hold the history of the automatic depth fuses the
            # next shallower one (each divides the timed step count)
            smaller = [d for d in DEPTH_LADDER if d < args.fuse]
            if fuse_explicit or not smaller or "memory" not in str(e).lower():
                create_error = e
                break
            depth_note = f"{args.fuse}-step history did not fit ({e}); fused {smaller[0]} steps"
            args.fuse = smaller[0]
            torch.cuda.empty_cache()
    # one collective on every rank, the failed ones included (they join with 0)
    agreed = agree_on_depth(0 if eng is None else args.fuse, pg, torch, dist, local, backend)
    if eng is None:
        raise create_error
    if agreed == 0:
        eng.close()
        raise SystemExit(f"rank {rank}: another rank could not create its engine at any depth; stopping")
    if agreed != args.fuse:  # another rank stepped down: this one follows, so every rank times the same launches
        eng.close()
        torch.cuda.empty_cache()
        depth_note = f"another rank could not hold {args.fuse} history slots; every rank fused {agreed} steps"
        args.fuse = agreed
        eng = create(agreed)
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

    # the parity check's GPU side: the handle's first launches (a one-step
    # lead-in, then one whole launch of the timed depth over the whole shard)
    cap = None
    if not args.no_parity:
        cap = capture_parity(eng, args, plan, world, torch, local)
        note(f"parity launches done ({eng.step_index} steps)")
    # warmup (untimed): the requested steps, and at least one whole launch of
    # the timed depth.  The first full-depth launch after a short warm-up runs
    # 10-29 ms long on 8192/N-row slabs (scripts/gpu_slab_warmup.sh,
    # profiles/r2p_slab_warmup.json: 1024 x 8192 after --warmup 5: 43.3 ms, then
    # 14.8 and 14.3 ms); after one such launch every later one is steady.  The
    # parity launches count, but the host reads that follow them leave the GPU
    # idle (the first timed launch then ran 5-11 ms long at 8192^2,
    # profiles/r4e_bench_driver_traced.json), so one more whole launch runs
    # right before the timed region.
    warm_steps = warmup_steps(args.warmup, args.fuse)
    eng.run(max(warm_steps - (eng.step_index - 1), args.fuse) if cap else warm_steps)
    warm_run = eng.step_index
    barrier()
    ns_before = eng.nan_safe_launches() if args.engine == "float32" else 0
    # Whole fused launches, and at least MIN_LAUNCHES of them, so that a short
    # --steps still gives a multi-launch timed region; the JSON carries the
    # requested count beside the timed one.
    steps = timed_steps(args.steps, args.fuse, fuse_explicit)
    n_launch = steps // args.fuse
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_launch)]
    # A split engine (tfg_set_split: a grid of <= 2^24 cells as two parts on two
    # streams) overlaps one part's launch with the other's: per-launch events on
    # the engine's stream would bracket the first parts only, so its launch time
    # is the span of the timed region (both parts joined) over the launches.
    split = eng.is_split()
    # no collector pass inside the timed region: one took 8-11 ms of host time at a
    # random tfg_step call (tests/diagnostics/split_first_launch.py), while the host
    # runs at most two calls ahead of the device -- a tenth of config 2's 80 ms region
    gc.collect()
    gc.disable()
    barrier()
    t0 = time.perf_counter()
    for i in range(n_launch):
        if args.conduction:
            conduct()
        if not split or i == 0:
            ev[i][0].record(stream)
        eng.run(args.fuse)
        if not split:
            ev[i][1].record(stream)
    if split:
        eng.join()
        ev[-1][1].record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    note(f"timed region: {n_launch} launches of {args.fuse} steps in {elapsed:.3f} s")
    if split:
        launch_ms = np.full(n_launch, ev[0][0].elapsed_time(ev[-1][1]) / n_launch)
    else:
        launch_ms = np.array([a.elapsed_time(b) for a, b in ev])
    cells = rows * args.nx
    diag = allreduce_diagnostics(eng.diagnostics()) if pg else eng.diagnostics()
    bytes_launch = cells * launch_bytes_per_cell(args.fuse, elem, args.catchments > 0, args.conduction)
    achieved = bytes_launch / (float(launch_ms.mean()) / 1e3) / 1e9
    # launches of the timed region that ran the fp32 step's NaN-safe form (0: the clean form was timed)
    ns_timed = (eng.nan_safe_launches() - ns_before) if args.engine == "float32" else None
    # the host-fed leg, the drop-in legs and the CPU baseline run on rank 0 at N=1 only (BASELINE contract)
    pcie = pcie_inclusive(eng, args, torch) if world == 1 and args.pcie else None
    dropin_grid = dropin_grid_leg(eng, args, torch, stream) if world == 1 and not args.no_dropin else None
    eng.close()
    torch.cuda.empty_cache()
    # every rank checks its own shard's first rows against the oracle (outside the timed region)
    parity = numpy_leg = None
    if cap is not None:
        parity, numpy_leg = sample_parity(args, plan, world, rank, _cpu_threads(), cap)
        del cap
    own = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), **device_record(torch, local),
           "row0": row0, "rows": rows, "elapsed_s": elapsed, "launch_ms_mean": float(launch_ms.mean()),
           "launch_ms_min": float(launch_ms.min()), "launch_ms_max": float(launch_ms.max()),
           "sample_parity": parity}
    records = [own]
    if pg:
        records = [None] * dist.get_world_size()
        dist.all_gather_object(records, own)
    ranks = rank_report(records, dist.get_backend() if pg else None)
    t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}" if backend == "nccl" else "cpu")
    if pg:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    total_cells = ny_global * args.nx if args.scaling == "strong" else cells * world
    value = total_cells * steps / elapsed

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            note("CPU baseline (C oracle)")
            cpu = cpu_baseline(args)
        dropin_many = None
        if world == 1 and not args.no_dropin and args.dropin_instances > 0:
            note("drop-in leg: defer_update instances")
            dropin_many = dropin_instances_leg(args, local)
        if world > 1:
            parity = parity_summary([r["sample_parity"] for r in ranks["ranks"]]) if not args.no_parity else None
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
            "warmup_steps_run": warm_run,  # untimed steps before the timed region (incl. the parity launches)
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32" if args.engine == "float32" else "f64",
            "data": "synthetic (counter-hash DEM/forcing with CSV statistics, 24 HBM-resident hourly frames)",
            "config": {
                "workload": f"{plan['workload']}, {args.dt:g} h steps, "
                            f"{args.engine} engine (fp64 state"
                            + (", fp64 flux" if args.engine == "float32" and args.flux == "fp64" else "")
                            + f"), {args.fuse} steps fused per launch"
                            + (f", {args.catchments} catchments" if args.catchments else "")
                            + (", lateral conduction re-evaluated before every launch" if args.conduction else ""),
                "grid_per_gpu": [rows, args.nx],
                "frames": args.frames,
                "fuse_steps": args.fuse,
                "launch_parts": 2 if split else 1,
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
                "launch_time_source": ("HIP events on the engine's stream: the span of the timed region (the second "
                                       "part joined) / launches; split launches, two parts on two streams "
                                       "(tfg_set_split), overlap" if split else
                                       "HIP events on the engine's stream around every launch"),
                "bytes_model": dict(zip(("per_step", "per_launch"), bytes_model(elem, args.catchments > 0, args.conduction))),
                "note": None if args.engine == "float32" else (
                    "the fp64 engine is issue-bound, not HBM-bound: its step issues ~680 VALU instructions per "
                    "wave and cell-step (profiles/r5_issue_counters.json); frac is its HBM share only"),
            },
            "cpu_baseline": cpu,
            "cpu_baseline_numpy_1core": numpy_leg if world == 1 else None,
            "pcie_inclusive": pcie,
            "dropin_per_step_grid": dropin_grid,
            "dropin_defer_update_instances": dropin_many,
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
    _args = parse()
    _rc = launch_ranks(_args, sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)
    main(_args)
