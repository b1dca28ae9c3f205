"""Parity at the BASELINE.json GPU configurations' per-GPU sizes.

  * config 4 (the bench): 8192 x 8192, hourly, two launches of the bench's
    automatic depth (bench.auto_fuse: 128 steps).  The first reads the initial
    depths; the second is the timed kernel instance at the timed launch
    length, whose step loop (three register sets) ends in its two-step tail
    (128 = 3 * 42 + 2).  Both are longer than the 72-slot window, so a launch
    reads back window slots it wrote itself;
  * config 3: 4096 x 4096, hourly, two 24-step launches;
  * config 2: 1024 x 1024, a year of hourly steps (8760) in 120-step launches,
    the oracle's daily outputs on about 2048 sampled cells
    (test_config2_year_at_its_own_shape);
  * config 5's per-GPU slab: rows 6144..8191 of the 16384 x 16384 grid over 8
    GPUs (2048 x 16384 cells), dt = 0.25 h (a 288-slot snowfall window), 43
    catchments (256 x 256-cell blocks, ids mod 43), 384 steps in four 96-step
    launches (longer than the window, so slots expire);
  * the largest shard the library accepts: 16383 x 32769 cells (536.9 M, an odd
    count, so the last wave is ragged), where the fp64 state planes' 32-bit
    lane byte offsets reach 4.29e9, just below 2^32.

The oracle cannot run tens of millions of cells, so each case checks what
holds at any size:
  * sampled parity: about 2048 cells spread over the whole shard (first and
    last cell, both sides of every 2^k cell boundary, random others) against
    the oracle on the host mirror of the same synthetic inputs, step by step
    (catches addressing faults at large plane offsets), with melt-out flips
    held to the fp64 baseline of the same cells (tests/harness.py flip_rule);
  * water balance over the whole shard: runoff = rain + snowfall + storage loss;
  * per-catchment mass balance (config 5): the kernel's segmented reduction
    equals a bincount of its own per-cell outputs, per catchment, for every
    integral (vol_P, PR, PS, SM, IM) and P_max;
  * determinism: a second run gives bit-identical state and diagnostics.
"""

import numpy as np
import pytest

import bench
from tests.harness import (BASE_CFG, c_oracle_hist, flip_rule, fp64_baseline_flips, make_engine, melt_out_flips,
                           oracle_run, valid_mask)

pytestmark = pytest.mark.gpu

SEED = 20251001
HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")
CONFIGS = {
    # name: (ny, nx, row0, ny_global, dt, steps, fuse, catchments)
    # the bench's launch shape: two launches of its automatic depth at 8192^2
    "config4_8192sq": (8192, 8192, 0, 8192, 1.0, 2 * bench.auto_fuse(8192 * 8192), bench.auto_fuse(8192 * 8192), 0),
    "config3_4096sq": (4096, 4096, 0, 4096, 1.0, 48, 24, 0),
    "config5_slab_2048x16384_dt0.25_43catch": (2048, 16384, 6144, 16384, 0.25, 384, 96, 43),
    # the largest shard tfg_create accepts (n_pad * 8 < 2^32: fp64 planes at
    # 32-bit lane byte offsets up to 4.29e9), ragged (ny * nx odd), dt = 2 h (a
    # 36-slot window) and 2 forcing frames so that it fits one GPU (~220 GB)
    "max_shard_16383x32769_dt2": (16383, 32769, 0, 16383, 2.0, 8, 4, 0),
}
FRAMES = {"max_shard_16383x32769_dt2": 2}  # forcing frames cycled (default 24)


def _sample_cells(rng, n, nx):
    edges = []
    for k in range(6, 32):
        for c in (2 ** k - 1, 2 ** k):
            if c < n:
                edges.append(c)
    edges += [0, n - 1, n // 2, nx - 1, nx, n - nx]
    edges = np.unique(np.array(edges))
    rest = rng.choice(n, 2048 - len(edges), replace=False)
    return np.unique(np.concatenate([edges, rest]))


def _catchments(row0, rows, nx, k):
    """256 x 256-cell blocks of the global grid, block ids mod k: every one of
    the k catchments appears in a 2048-row slab, each in many pieces."""
    r = ((np.arange(row0, row0 + rows) // 256) * (nx // 256))[:, None]
    c = (np.arange(nx) // 256)[None, :]
    return ((r + c) % k).astype(np.int32).reshape(-1)


def _run(torch, cfg, shape, cells, cid, nf=24):
    """One run of a shard: sampled outputs [steps][cells], runoff sum, storage
    sums before and after, final h_swe on device, diagnostics, and (with
    catchments) per-catchment bincounts of the engine's own outputs."""
    from topoflow_glacier.synthetic import diurnal_table

    ny, nx, row0, _, dt, steps, fuse, ncatch = shape
    n = ny * nx
    torch.cuda.empty_cache()  # the largest shard needs the memory torch keeps cached
    e = make_engine(cfg, ny, nx, "float32", n_frames=nf, hist_depth=fuse, fuse_steps=fuse, row0=row0,
                    n_catch=max(ncatch, 1))

    def dev(name, index, dtype):
        # get_field_device orders the engine-stream copy before torch's reads
        return e.get_field_device(name, torch.empty(n, dtype=dtype, device="cuda:0"), index=index)

    try:
        e.fill_synthetic(SEED, diurnal_table(nf), nx_global=nx)
        if ncatch:
            e.set_field("catch_id", cid)
            # per-cell sums over the run, binned by catchment once at the end
            per = {v: torch.zeros(n, dtype=torch.float64, device="cuda:0") for v in ("P", "PR", "PS", "SM", "IM")}
            pmax = torch.zeros(n, dtype=torch.float64, device="cuda:0")
            P_frames = [dev("P", f, torch.float64) for f in range(24)]
            rain = [dev("T_air", f, torch.float32) > cfg["T_rain_snow"] for f in range(24)]  # :578-604
        idx = torch.as_tensor(cells, device="cuda:0")
        store0 = (float(dev("h_swe", 0, torch.float64).sum()), float(dev("h_iwe", 0, torch.float64).sum()))
        sampled = {v: [] for v in HIST}
        runoff = 0.0
        for launch in range(steps // fuse):
            e.run(fuse)
            e.sync()
            for k in range(fuse):
                step = launch * fuse + k
                for v in HIST:
                    f = dev(v, k, torch.float32)
                    sampled[v].append(f.index_select(0, idx).cpu().numpy())
                    if v == "M_total":
                        runoff += float(f.sum(dtype=torch.float64))
                    if ncatch and v in ("SM", "IM"):
                        per[v] += f.double()
                if ncatch:
                    p = P_frames[step % 24]
                    per["P"] += p
                    per["PR"] += torch.where(rain[step % 24], p, 0.0)
                    per["PS"] += torch.where(rain[step % 24], 0.0, p)
                    torch.maximum(pmax, p, out=pmax)
        swe1 = dev("h_swe", 0, torch.float64)
        store1 = (float(swe1.sum()), float(dev("h_iwe", 0, torch.float64).sum()))
        bins = None
        if ncatch:
            bins = {v: np.bincount(cid, weights=t.cpu().numpy(), minlength=ncatch) for v, t in per.items()}
            pm = pmax.cpu().numpy()
            bins["P_max"] = np.array([pm[cid == c].max() for c in range(ncatch)])
        return ({v: np.stack(a).astype(np.float64) for v, a in sampled.items()}, runoff, store0, store1, swe1,
                e.diagnostics(), bins)
    finally:
        e.close()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_full_size_sampled_parity_water_balance_and_determinism(name):
    import torch

    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    shape = CONFIGS[name]
    ny, nx, row0, ny_global, dt, steps, fuse, ncatch = shape
    nf = FRAMES.get(name, 24)
    cfg = dict(BASE_CFG, dt=dt)
    n = ny * nx
    cells = _sample_cells(np.random.default_rng(5), n, nx)
    cid = _catchments(row0, ny, nx, ncatch) if ncatch else None
    gpu, runoff, s0, s1, swe1, dg, bins = _run(torch, cfg, shape, cells, cid, nf)

    # sampled parity against the oracle on the host mirror of the same fp32 inputs
    syn = synthetic_cells(SEED, cells + row0 * nx, diurnal_table(nf))
    frames = np.arange(steps) % nf
    forcing = {k: syn[k][frames].astype(np.float64) for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    static = {k: np.asarray(syn[s], np.float64) for k, s in (("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"),
              ("h0_snow", "h_snow"), ("h0_ice", "h_ice"), ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    ref, _ = oracle_run(cfg, static, forcing, steps)
    flip, genuine = melt_out_flips(gpu, ref, 1e-5)
    assert not genuine, genuine[:5]
    c64 = c_oracle_hist(cfg, static, {k: syn[k] for k in forcing}, steps, frames=frames)
    rule = flip_rule(int((flip >= 0).sum()), fp64_baseline_flips(c64, ref))
    assert rule["ok"], rule
    ok = valid_mask(flip, steps)
    for v in HIST:
        r = ref[v][ok]
        nz = np.abs(r[r != 0])
        s_v = np.percentile(nz, 99) if nz.size else 0.0
        err = np.abs(gpu[v][ok] - r) / np.maximum(np.maximum(np.abs(r), s_v), 1e-300)
        assert err.max(initial=0.0) <= 1e-5, (v, float(err.max()))

    # water balance over the whole shard: runoff = rain + snowfall + storage loss
    da_m2 = BASE_CFG["da"] * 1e6
    tot = dg.sum(axis=0)
    lhs = runoff * dt * 3600 * da_m2
    rhs = tot[1] + tot[2] + ((s0[0] - s1[0]) + (s0[1] - s1[1])) * da_m2
    assert abs(lhs - rhs) <= 1e-5 * abs(rhs), (lhs, rhs)
    assert tot[0] == pytest.approx(tot[1] + tot[2], rel=1e-6)  # P = rain + snow (fp32 per-launch partials)

    if ncatch:
        # the kernel's per-catchment reduction (:558-624, :1482-1494 per
        # catchment) against bincounts over the catchment raster: the
        # precipitation integrals and P_max exactly from the forcing frames;
        # vol_SM / vol_IM integrate SM and IM before update_swe / update_iwe
        # clamp them (exact per-catchment values against the oracle are in
        # test_catchment_diagnostics), so here they bound the clamped outputs'
        # volumes from above and sum to the domain totals
        assert dg.shape[0] == ncatch
        for col, v in ((0, "P"), (1, "PR"), (2, "PS")):
            want = bins[v] * (da_m2 * dt)
            assert np.all(np.abs(dg[:, col] - want) <= 1e-6 * np.abs(want)), (v, dg[:, col], want)
        assert np.array_equal(dg[:, 5], bins["P_max"].astype(np.float64))
        for col, v in ((3, "SM"), (4, "IM")):
            out_vol = bins[v] * (da_m2 * dt * 3600)
            assert np.all(dg[:, col] >= out_vol * (1 - 1e-6)), (v, dg[:, col], out_vol)
        assert (dg[:, 3] > 0).all() and (dg[:, 0] > 0).all()

    # determinism: a second run, bit for bit
    gpu2, runoff2, _, _, swe2, dg2, _ = _run(torch, cfg, shape, cells, cid, nf)
    assert torch.equal(swe1, swe2) and np.array_equal(dg, dg2) and runoff == runoff2
    for v in HIST:
        assert np.array_equal(gpu[v], gpu2[v]), v


# ---------------------------------------------------------------- config 2: a year at 1024 x 1024
C2_NY = C2_NX = 1024
C2_STEPS, C2_FUSE = 8760, 120  # 73 launches of 120 hourly steps


def _run_year(torch, cfg, cells):
    """Config 2 on the GPU: the whole 1024 x 1024 grid for a year of hourly
    steps in 120-step launches.  Returns the sampled cells' outputs at the last
    step of every day [365][ncell], the whole grid's runoff sum, storage sums
    before and after, the final h_swe on device and the diagnostics."""
    from topoflow_glacier.synthetic import diurnal_table

    n = C2_NY * C2_NX
    e = make_engine(cfg, C2_NY, C2_NX, "float32", n_frames=24, hist_depth=C2_FUSE, fuse_steps=C2_FUSE)

    def dev(name, index, dtype):
        return e.get_field_device(name, torch.empty(n, dtype=dtype, device="cuda:0"), index=index)

    try:
        e.fill_synthetic(SEED, diurnal_table(24), nx_global=C2_NX)
        idx = torch.as_tensor(cells, device="cuda:0")
        store0 = (float(dev("h_swe", 0, torch.float64).sum()), float(dev("h_iwe", 0, torch.float64).sum()))
        daily = {v: [] for v in HIST}
        runoff = torch.zeros((), dtype=torch.float64, device="cuda:0")
        for launch in range(C2_STEPS // C2_FUSE):
            e.run(C2_FUSE)
            e.sync()
            for k in range(C2_FUSE):
                step = launch * C2_FUSE + k
                runoff += dev("M_total", k, torch.float32).sum(dtype=torch.float64)
                if step % 24 == 23:
                    for v in HIST:
                        daily[v].append(dev(v, k, torch.float32).index_select(0, idx).cpu().numpy())
        swe1 = dev("h_swe", 0, torch.float64)
        store1 = (float(swe1.sum()), float(dev("h_iwe", 0, torch.float64).sum()))
        return ({v: np.stack(a).astype(np.float64) for v, a in daily.items()}, float(runoff), store0, store1, swe1,
                e.diagnostics())
    finally:
        e.close()


def test_config2_year_at_its_own_shape():
    """BASELINE config 2 at its own shape: 1024 x 1024 cells, a year of hourly
    steps (16384 waves, four rounds of the chip's resident waves per step).
    Against the oracle's year on ~2048 sampled cells (the first and last cell,
    both sides of every 2^k boundary, random others), compared once a day as
    in test_fp32_free_run_over_a_year: snow depth within the floored 1e-5 and
    RH within 1e-6 everywhere; SM outside 1e-5 (melt onset) in at most 0.5 %
    of the cells; the cells whose ice melt switches at a different step (the
    exact-zero melt-out gate, :1424) held to the flip rule against the fp64
    baseline (the C oracle's year on the same cells); runoff diverging only
    there or at melt onset.  Whole grid: water balance; determinism."""
    import torch

    import tfg_oracle as O
    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    cfg = dict(BASE_CFG)
    n = C2_NY * C2_NX
    cells = _sample_cells(np.random.default_rng(7), n, C2_NX)
    gpu, runoff, s0, s1, swe1, dg = _run_year(torch, cfg, cells)

    syn = synthetic_cells(SEED, cells, diurnal_table(24))
    static = {k: np.asarray(syn[s], np.float64) for k, s in (("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"),
              ("h0_snow", "h_snow"), ("h0_ice", "h_ice"), ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    m = O.OracleGrid(cfg, **static)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], C2_STEPS, cfg["lon"])
    ref = {v: [] for v in HIST}
    for k in range(C2_STEPS):
        f = k % 24
        r = m.step(*(syn[v][f].astype(np.float64) for v in ("P", "T_air", "Hum_sp", "P_air", "uz")), jd[k], tsn[k])
        if k % 24 == 23:
            for v in HIST:
                ref[v].append(np.array(r[v], copy=True))
    ref = {v: np.stack(a) for v, a in ref.items()}
    c = c_oracle_hist(cfg, static, {v: syn[v] for v in ("P", "T_air", "Hum_sp", "P_air", "uz")}, C2_STEPS,
                      frames=np.arange(C2_STEPS) % 24, clock=(jd, tsn))
    c_daily = {v: c[v][23::24] for v in HIST}

    def diverged(A, v):
        g, r = A[v], ref[v]
        s_v = np.percentile(np.abs(r[r != 0]), 99) if np.any(r != 0) else 0.0
        err = np.abs(g - r) / np.maximum(np.maximum(np.abs(r), s_v), 1e-300)
        return float(err.max()), (err > 1e-5).any(axis=0)

    assert diverged(gpu, "h_snow")[0] <= 1e-5
    assert diverged(gpu, "RH")[0] <= 1e-6
    assert diverged(gpu, "SM")[1].mean() <= 0.005
    gi = diverged(gpu, "h_ice")[1] | diverged(gpu, "IM")[1]
    ci = diverged(c_daily, "h_ice")[1] | diverged(c_daily, "IM")[1]
    rule = flip_rule(int(gi.sum()), int(ci.sum()))
    assert rule["ok"], rule
    assert (diverged(gpu, "M_total")[1] & ~gi).mean() <= 0.005

    # water balance over the whole grid: runoff = rain + snowfall + storage loss
    da_m2 = BASE_CFG["da"] * 1e6
    tot = dg.sum(axis=0)
    lhs = runoff * cfg["dt"] * 3600 * da_m2
    rhs = tot[1] + tot[2] + ((s0[0] - s1[0]) + (s0[1] - s1[1])) * da_m2
    assert abs(lhs - rhs) <= 1e-5 * abs(rhs), (lhs, rhs)

    # determinism: a second year, bit for bit
    gpu2, runoff2, _, _, swe2, dg2 = _run_year(torch, cfg, cells)
    assert torch.equal(swe1, swe2) and np.array_equal(dg, dg2) and runoff == runoff2
    for v in HIST:
        assert np.array_equal(gpu[v], gpu2[v]), v
