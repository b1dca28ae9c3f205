"""Slope/aspect from a DEM (extension): Horn's stencil on
the GPU (tfg_terrain_from_dem) against the numpy restatement, and the one-row
halo exchange of the row-block shards (torch.distributed; gloo here, RCCL on
the GPU path)."""

from __future__ import annotations

import numpy as np
import pytest

from tests.harness import BASE_CFG, make_engine, terrain_dem, terrain_oracle
from tests.test_sharding import _torchrun


def test_terrain_oracle_conventions():
    """A tilted plane: slope = |grad z|, aspect = direction of steepest descent
    counter-clockwise from east (reference: alpha = pi/2 - aspect, :1086)."""
    y, x = np.mgrid[0:6, 0:7].astype(np.float64)
    dx = dy = 30.0
    # rising to the east by 3 m per cell -> downslope points west (pi)
    s, a = terrain_oracle(3.0 * x, dx, dy)
    I = (slice(1, -1), slice(1, -1))  # interior: replicated edges halve the one-sided difference
    assert np.allclose(s[I], 0.1) and np.allclose(np.abs(a), np.pi) and np.allclose(s[:, 0], 0.05)
    # rising to the south (row index) -> downslope points north (+pi/2)
    s, a = terrain_oracle(6.0 * y, dx, dy)
    assert np.allclose(s[I], 0.2) and np.allclose(a, np.pi / 2)
    # flat -> slope 0, aspect 0
    s, a = terrain_oracle(np.full((4, 4), 100.0), dx, dy)
    assert np.all(s == 0) and np.all(a == 0)
    # halos: the top row of a block with the true north row equals the full-grid result
    z = terrain_dem(40, 30)
    full = terrain_oracle(z, dx, dy)
    top = terrain_oracle(z[10:25], dx, dy, north=z[9], south=z[25])
    assert np.array_equal(top[0], full[0][10:25]) and np.array_equal(top[1], full[1][10:25])


def test_bmi_y_axis_matches_the_terrain_row_order():
    """The BMI grid coordinates and the engine's stencil agree on north: a DEM
    that rises with the BMI y coordinate (get_grid_y) rises to the north in
    the terrain restatement, whose row 0 is the northern edge (halo_north pairs
    with it), so its downslope aspect points south (-pi/2)."""
    from types import SimpleNamespace

    from topoflow_glacier import BmiTopoflowGlacier

    m = BmiTopoflowGlacier()
    m.ny, m.nx, m.n_cells = 6, 7, 42
    m.cfg = SimpleNamespace(da=0.0009, dx=30.0, dy=30.0)
    y = m.get_grid_y(0, np.zeros(6))
    dem = np.repeat((0.1 * y)[:, None], 7, axis=1)  # 0.1 m per metre northward
    s, a = terrain_oracle(dem, 30.0, 30.0)
    I = (slice(1, -1), slice(1, -1))
    assert np.allclose(s[I], 0.1) and np.allclose(a[I], -np.pi / 2)


def test_halo_exchange_gloo_world2(tmp_path):
    ny, nx = 9, 16
    ranks = _torchrun("halo", tmp_path, ny=ny, nx=nx, steps=1)
    z = terrain_dem(ny, nx)
    r0, r1 = ranks
    assert np.all(np.isnan(r0["north"])) and np.array_equal(r0["south"], z[int(r1["row0"])])
    assert np.array_equal(r1["north"], z[int(r1["row0"]) - 1]) and np.all(np.isnan(r1["south"]))


@pytest.mark.gpu
def test_terrain_kernel_matches_restatement():
    ny, nx = 120, 170
    z = terrain_dem(ny, nx)
    for engine, tol in (("float64", 1e-13), ("float32", 2 ** -23)):
        e = make_engine(BASE_CFG, ny, nx, engine, n_frames=1, hist_depth=1)
        try:
            e.set_field("elev", z.reshape(-1))
            e.terrain_from_dem(30.0, 25.0)
            s, a = e.get_field("slope").reshape(ny, nx), e.get_field("aspect").reshape(ny, nx)
        finally:
            e.close()
        rs, ra = terrain_oracle(z, 30.0, 25.0)
        assert np.max(np.abs(s - rs) / np.maximum(np.abs(rs), 1e-12)) <= 2 * tol, engine
        assert np.max(np.abs(a - ra)) <= 2 * np.pi * 2 * tol, engine


@pytest.mark.gpu
def test_sharded_terrain_equals_whole_grid(tmp_path):
    """Row blocks with their neighbours' rows as halos reproduce the unsharded
    rasters bit for bit: in one process, and over torch.distributed (gloo,
    world size 2, both ranks on cuda:0)."""
    ny, nx = 64, 96
    z = terrain_dem(ny, nx)
    whole = make_engine(BASE_CFG, ny, nx, "float32", n_frames=1, hist_depth=1)
    whole.set_field("elev", z.reshape(-1).astype(np.float32))
    whole.terrain_from_dem(30.0, 30.0)
    ws, wa = whole.get_field("slope"), whole.get_field("aspect")
    whole.close()
    parts = []
    for r0, r1 in ((0, 23), (23, 64)):
        e = make_engine(BASE_CFG, r1 - r0, nx, "float32", n_frames=1, hist_depth=1)
        e.set_field("elev", z[r0:r1].reshape(-1).astype(np.float32))
        e.terrain_from_dem(30.0, 30.0, None if r0 == 0 else z[r0 - 1], None if r1 == ny else z[r1])
        parts.append((e.get_field("slope"), e.get_field("aspect")))
        e.close()
    assert np.array_equal(np.concatenate([p[0] for p in parts]), ws)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), wa)
    ranks = _torchrun("gpu_terrain", tmp_path, ny=ny, nx=nx, steps=1)
    assert np.array_equal(np.concatenate([r["slope"] for r in ranks]), ws)
    assert np.array_equal(np.concatenate([r["aspect"] for r in ranks]), wa)
