"""Parity at BASELINE.json's full size: the 8192 x 8192 fp32 grid of the bench.

The oracle cannot run 67 M cells, so this checks what holds at any size:
  * sampled parity: 2048 cells spread over the whole grid (first and last
    cell, both sides of every 2^k cell boundary up to 2^26, random others) are
    compared with the oracle run on the host mirror of the same synthetic
    inputs, step by step (catches addressing faults at large plane offsets:
    the history slots sit up to 154 GB into their buffer);
  * water balance over the whole grid: runoff = rain + snowfall + storage loss;
  * determinism: a second run gives bit-identical state and diagnostics.
Both runs use two launches of 24 fused steps each (48 steps) so the state also
crosses a launch boundary.
"""

import numpy as np
import pytest

from tests.harness import (BASE_CFG, c_oracle_hist, flip_rule, fp64_baseline_flips, make_engine, melt_out_flips,
                           oracle_run, valid_mask)

pytestmark = pytest.mark.gpu

NY = NX = 8192
N = NY * NX
STEPS, FUSE, SEED = 48, 24, 20251001
HIST = ("h_snow", "SM", "h_ice", "IM", "M_total", "RH")


def _sample_cells(rng):
    edges = []
    for k in range(6, 27):
        for c in (2 ** k - 1, 2 ** k):
            if c < N:
                edges.append(c)
    edges += [0, N - 1, N // 2, NX - 1, NX, (NY - 1) * NX]
    rest = rng.choice(N, 2048 - len(set(edges)), replace=False)
    return np.unique(np.concatenate([np.array(edges), rest]))


def _device_field(torch, e, name, index, dtype):
    # GlacierEngine.get_field_device orders the engine-stream copy before
    # torch's reads (a bare tfg_get_field into a device pointer is asynchronous)
    return e.get_field_device(name, torch.empty(N, dtype=dtype, device="cuda:0"), index=index)


def _run(torch, cells):
    """One full-size run: returns (sampled outputs [STEPS][cells], runoff sum,
    swe/iwe sums before and after, final h_swe on device, diagnostics)."""
    from topoflow_glacier.synthetic import diurnal_table

    e = make_engine(BASE_CFG, NY, NX, "float32", n_frames=24, hist_depth=FUSE, fuse_steps=FUSE)
    try:
        e.fill_synthetic(SEED, diurnal_table(24), nx_global=NX)
        idx = torch.as_tensor(cells, device="cuda:0")
        store0 = (float(_device_field(torch, e, "h_swe", 0, torch.float64).sum()),
                  float(_device_field(torch, e, "h_iwe", 0, torch.float64).sum()))
        sampled = {v: [] for v in HIST}
        runoff = 0.0
        for _ in range(STEPS // FUSE):
            e.run(FUSE)
            e.sync()
            for k in range(FUSE):
                for v in HIST:
                    f = _device_field(torch, e, v, k, torch.float32)
                    sampled[v].append(f.index_select(0, idx).cpu().numpy())
                    if v == "M_total":
                        runoff += float(f.sum(dtype=torch.float64))
        swe1 = _device_field(torch, e, "h_swe", 0, torch.float64)
        store1 = (float(swe1.sum()), float(_device_field(torch, e, "h_iwe", 0, torch.float64).sum()))
        return ({v: np.stack(a).astype(np.float64) for v, a in sampled.items()}, runoff, store0, store1,
                swe1, e.diagnostics())
    finally:
        e.close()


def test_full_size_grid_sampled_parity_water_balance_and_determinism():
    import torch

    from topoflow_glacier.synthetic import diurnal_table, synthetic_cells

    cells = _sample_cells(np.random.default_rng(5))
    gpu, runoff, s0, s1, swe1, dg = _run(torch, cells)

    # sampled parity against the oracle on the host mirror of the same fp32 inputs
    syn = synthetic_cells(SEED, cells, diurnal_table(24))
    frames = np.arange(STEPS) % 24
    forcing = {k: syn[k][frames].astype(np.float64) for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    static = {k: np.asarray(syn[s], np.float64) for k, s in (("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"),
              ("h0_snow", "h_snow"), ("h0_ice", "h_ice"), ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    ref, _ = oracle_run(BASE_CFG, static, forcing, STEPS)
    flip, genuine = melt_out_flips(gpu, ref, 1e-5)
    assert not genuine, genuine[:5]
    c64 = c_oracle_hist(BASE_CFG, static, {k: syn[k] for k in forcing}, STEPS, frames=frames)
    rule = flip_rule(int((flip >= 0).sum()), fp64_baseline_flips(c64, ref))
    assert rule["ok"], rule
    ok = valid_mask(flip, STEPS)
    for v in HIST:
        r = ref[v][ok]
        nz = np.abs(r[r != 0])
        s_v = np.percentile(nz, 99) if nz.size else 0.0
        err = np.abs(gpu[v][ok] - r) / np.maximum(np.maximum(np.abs(r), s_v), 1e-300)
        assert err.max(initial=0.0) <= 1e-5, (v, float(err.max()))

    # water balance over all 67 M cells: runoff = rain + snowfall + storage loss
    da_m2, dt = BASE_CFG["da"] * 1e6, 1
    lhs = runoff * dt * 3600 * da_m2
    rhs = dg[0, 1] + dg[0, 2] + ((s0[0] - s1[0]) + (s0[1] - s1[1])) * da_m2
    assert abs(lhs - rhs) <= 1e-5 * abs(rhs), (lhs, rhs)
    assert dg[0, 0] == pytest.approx(dg[0, 1] + dg[0, 2], rel=1e-6)  # P = rain + snow (fp32 per-launch partials)

    # determinism: a second run, bit for bit
    gpu2, runoff2, _, _, swe2, dg2 = _run(torch, cells)
    assert torch.equal(swe1, swe2) and np.array_equal(dg, dg2) and runoff == runoff2
    for v in HIST:
        assert np.array_equal(gpu[v], gpu2[v]), v
