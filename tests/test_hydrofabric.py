"""Hydrofabric divides -> catchment-ID raster and the
per-catchment mass balance on it."""

from __future__ import annotations

import sqlite3
import struct

import numpy as np
import pytest

from tests.harness import BASE_CFG, GOLDEN, make_engine, oracle_synthetic, synthetic_inputs

FIX = GOLDEN / "hydrofabric_12082500.npz"


def _gp_blob(rings, srs=5070, big_endian=False):
    """A GeoPackage polygon blob (header with an xy envelope + WKB), written
    independently of the reader under test."""
    bo = ">" if big_endian else "<"
    xs = np.concatenate([r[:, 0] for r in rings])
    ys = np.concatenate([r[:, 1] for r in rings])
    flags = (0 if big_endian else 1) | (1 << 1)
    head = b"GP" + bytes([0, flags]) + struct.pack(bo + "i", srs) + struct.pack(bo + "4d", xs.min(), xs.max(), ys.min(), ys.max())
    wkb = bytes([0 if big_endian else 1]) + struct.pack(bo + "II", 3, len(rings))
    for r in rings:
        wkb += struct.pack(bo + "I", len(r)) + r.astype(">f8" if big_endian else "<f8").tobytes()
    return head + wkb


def _square(x, y, s):
    return np.array([[x, y], [x + s, y], [x + s, y + s], [x, y + s], [x, y]], dtype=np.float64)


def test_geopackage_reader_on_a_written_file(tmp_path):
    from topoflow_glacier.hydrofabric import read_divides, ring_area

    db = tmp_path / "t.gpkg"
    con = sqlite3.connect(db)
    con.execute("create table gpkg_geometry_columns (table_name text, column_name text)")
    con.execute("insert into gpkg_geometry_columns values ('divides', 'geom')")
    con.execute("create table divides (fid integer primary key, geom blob, divide_id text, areasqkm real)")
    shell, hole = _square(0, 0, 1000), _square(250, 250, 500)[::-1]
    con.execute("insert into divides values (1, ?, 'cat-1', 0.75)", (_gp_blob([shell, hole]),))
    con.execute("insert into divides values (2, ?, 'cat-2', 1.0)", (_gp_blob([_square(1000, 0, 1000)], big_endian=True),))
    con.commit()
    con.close()
    srs, dv = read_divides(db)
    assert srs == 5070 and [d.divide_id for d in dv] == ["cat-1", "cat-2"]
    p = dv[0].polygons[0]
    assert len(p) == 2 and np.array_equal(p[0], shell) and np.array_equal(p[1], hole)
    assert ring_area(p[0]) - ring_area(p[1]) == 750000.0
    assert np.array_equal(dv[1].polygons[0][0], _square(1000, 0, 1000))


def test_rasterize_squares_with_a_hole():
    from topoflow_glacier.hydrofabric import Divide, catchment_ids, grid_covering, rasterize_divides

    dv = [Divide("a", 0.75, [[_square(0, 0, 1000), _square(250, 250, 500)]]), Divide("b", 1.0, [[_square(1000, 0, 1000)]])]
    x0, y0, ny, nx = grid_covering(dv, 50.0)
    r = rasterize_divides(dv, x0, y0, 50.0, ny, nx)
    assert (r == 0).sum() * 2500 == 750000 and (r == 1).sum() * 2500 == 1000000
    ids, nc = catchment_ids(r)
    assert nc == 3 and ids.min() == 0 and ids.max() == 2 and (ids == 2).sum() == (r < 0).sum()


def test_reference_hydrofabric_divides():
    """The 43 divides of data/12082500.gpkg (fixture extracted by
    tests/golden/make_hydrofabric.py): polygon areas equal the hydrofabric's
    own areasqkm, and a 30 m raster reproduces each divide's area."""
    from topoflow_glacier.hydrofabric import grid_covering, load_divides_npz, rasterize_divides, ring_area

    srs, dv = load_divides_npz(FIX)
    assert srs == 5070 and len(dv) == 43 and dv[0].divide_id == "cat-3062933"
    for d in dv:
        a = sum(ring_area(p[0]) - sum(ring_area(h) for h in p[1:]) for p in d.polygons) / 1e6
        assert abs(a - d.areasqkm) <= 1e-6 * d.areasqkm, d.divide_id
    x0, y0, ny, nx = grid_covering(dv, 30.0)
    r = rasterize_divides(dv, x0, y0, 30.0, ny, nx)
    cnt = np.bincount(r[r >= 0].ravel(), minlength=len(dv))
    areas = np.array([d.areasqkm for d in dv])
    assert np.all(np.abs(cnt * 900 / 1e6 - areas) <= 0.02 * areas)


@pytest.mark.gpu
def test_per_catchment_mass_balance_on_the_hydrofabric():
    """fp32 engine over the 43 divides rasterised at 120 m (+ an 'outside'
    bin): per-catchment volumes from the segmented wave reduction equal the
    oracle's per-cell volumes summed by catchment."""
    from topoflow_glacier.hydrofabric import catchment_ids, grid_covering, load_divides_npz, rasterize_divides

    _, dv = load_divides_npz(FIX)
    x0, y0, ny, nx = grid_covering(dv, 120.0)
    ids, nc = catchment_ids(rasterize_divides(dv, x0, y0, 120.0, ny, nx))
    ids = ids.reshape(-1)
    nsteps, seed = 24, 5
    cfg = dict(BASE_CFG, da=0.0144)  # 120 m cells
    syn, d = synthetic_inputs(seed, ny, nx, 24)
    e = make_engine(cfg, ny, nx, "float32", n_frames=24, hist_depth=1, n_catch=nc)
    try:
        e.fill_synthetic(seed, d)
        e.set_field("catch_id", ids)
        e.run(nsteps)
        e.sync()
        diag = e.diagnostics()
    finally:
        e.close()
    ref, m = oracle_synthetic(seed, ny, nx, nsteps, cfg_over={"da": 0.0144})
    # per catchment: precipitation volume (:567) and maximum, from the same fp32 inputs
    P = syn["P"][np.arange(nsteps) % 24].astype(np.float64)  # [nsteps][ncell]
    vP = np.bincount(ids, weights=P.sum(0), minlength=nc) * (0.0144 * 1e6) * 1
    Pmax = np.array([P[:, ids == c].max() if np.any(ids == c) else 0.0 for c in range(nc)])
    np.testing.assert_allclose(diag[:, 0], vP, rtol=1e-6, atol=0)
    np.testing.assert_array_equal(diag[:, 5], Pmax)
    # domain totals of every integral against the oracle
    for j, v in enumerate((m.vol_P, m.vol_PR, m.vol_PS, m.vol_SM, m.vol_IM)):
        assert diag[:, j].sum() == pytest.approx(float(v), rel=1e-5), j
