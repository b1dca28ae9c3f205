"""The optional lateral ice-flow term (tfg_ice_flow_*; SURVEY.md 8(e) and
8(f) row 4).  The reference declares Glen's-law parameters (config.py:64-65)
but moves no ice, so this term has no reference counterpart: parity is
against its own numpy restatement (tests/harness.py:ice_flow_step_restated),
and the properties checked are the ones the flux form guarantees: ice volume
conserved to rounding, thickness never negative, no flow without a surface
gradient, and row-block shards with exchanged halo rows equal to the whole
grid bit for bit."""

import numpy as np
import pytest

from tests.harness import (BASE_CFG, RestatedFlowShard, glacier_valley, ice_flow_dmax_restated, ice_flow_gamma,
                           ice_flow_step_restated, make_engine)
from tests.test_sharding import _torchrun
from topoflow_glacier.sharding import ice_flow, row_block

WI = 1000.0 / 917.0
DX = DY = 100.0


def test_restated_flow_conserves_ice_and_keeps_it_nonnegative():
    g = ice_flow_gamma(BASE_CFG)
    bed, iwe = glacier_valley(40, 30)
    sh = RestatedFlowShard(bed, iwe, WI, g)
    n = ice_flow(sh, 1.0, DX, DY, distributed=False)
    assert n > 1
    assert abs(sh.iwe.sum() / iwe.sum() - 1.0) <= 1e-13
    assert sh.iwe.min() >= 0.0 and np.abs(sh.iwe - iwe).max() > 1.0  # it did flow
    # ice spreads down-valley: the centre of mass moves to larger row index
    rows = np.arange(40)[:, None]
    assert (rows * sh.iwe).sum() / sh.iwe.sum() > (rows * iwe).sum() / iwe.sum()


def test_restated_flow_is_still_without_gradient_or_ice():
    g = ice_flow_gamma(BASE_CFG)
    flat = np.full((8, 9), 2500.0)
    slab = np.full((8, 9), 50.0)
    assert ice_flow_dmax_restated(flat, slab, WI, g, DX, DY) == 0.0
    np.testing.assert_array_equal(ice_flow_step_restated(flat, slab, WI, g, DX, DY, 0.01), slab)
    bed, _ = glacier_valley(8, 9)
    assert ice_flow(RestatedFlowShard(bed, np.zeros((8, 9)), WI, g), 1.0, DX, DY, distributed=False) == 0


def test_sharded_restated_flow_gloo_world2(tmp_path):
    ny, nx, tenths = 41, 30, 5
    ranks = _torchrun("flow", tmp_path, ny=ny, nx=nx, steps=tenths)
    bed, iwe = glacier_valley(ny, nx)
    whole = RestatedFlowShard(bed, iwe, WI, ice_flow_gamma(BASE_CFG))
    n = ice_flow(whole, tenths / 10.0, DX, DY, distributed=False)
    assert [int(r["n_sub"]) for r in ranks] == [n, n]
    np.testing.assert_array_equal(np.concatenate([r["iwe"] for r in ranks]), whole.iwe.reshape(-1))


# ------------------------------------------------------------------------- GPU
def _engine(bed, iwe, engine="float32", row0=0):
    ny, nx = iwe.shape
    e = make_engine(dict(BASE_CFG), ny, nx, engine, n_frames=1, hist_depth=1, row0=row0)
    e.set_field("elev", bed.reshape(-1).astype(np.float32 if engine == "float32" else np.float64))
    e.set_field("h_iwe", iwe.reshape(-1))
    e.init_state()
    return e


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["float32", "float64"])
def test_gpu_flow_step_matches_restatement(engine):
    g = ice_flow_gamma(BASE_CFG)
    bed, iwe = glacier_valley(48, 40)
    # an interior block with real halo rows on both sides
    b, w = bed[10:30], iwe[10:30]
    H = iwe * WI
    north = np.stack([bed[9] + iwe[9] * WI, H[9]])
    south = np.stack([bed[30] + iwe[30] * WI, H[30]])
    for halos in ((None, None), (north, south)):
        e = _engine(b, w, engine)
        try:
            dmax = e.ice_flow_dmax(DX, DY, *halos)
            assert dmax == ice_flow_dmax_restated(b, w, WI, g, DX, DY, *halos)
            e.ice_flow_step(0.002, DX, DY, *halos)
            got = e.get_field("h_iwe").reshape(w.shape)
            want = ice_flow_step_restated(b, w, WI, g, DX, DY, 0.002, *halos)
            np.testing.assert_array_equal(got, want)
            np.testing.assert_array_equal(e.get_field("h_ice", dtype=np.float64).reshape(w.shape), want * WI)
        finally:
            e.close()


@pytest.mark.gpu
def test_gpu_flow_year_conserves_and_matches_restatement():
    g = ice_flow_gamma(BASE_CFG)
    bed, iwe = glacier_valley(64, 48)
    e = _engine(bed, iwe)
    try:
        n = e.ice_flow(1.0, DX, DY)
        got = e.get_field("h_iwe").reshape(iwe.shape)
    finally:
        e.close()
    ref = RestatedFlowShard(bed, iwe, WI, g)
    assert ice_flow(ref, 1.0, DX, DY, distributed=False) == n > 1
    np.testing.assert_array_equal(got, ref.iwe)
    assert abs(got.sum() / iwe.sum() - 1.0) <= 1e-13 and got.min() >= 0.0


@pytest.mark.gpu
def test_gpu_sharded_flow_gloo_world2_equals_whole_grid(tmp_path):
    ny, nx, tenths = 41, 30, 5
    ranks = _torchrun("gpu_flow", tmp_path, ny=ny, nx=nx, steps=tenths)
    bed, iwe = glacier_valley(ny, nx)
    e = _engine(bed, iwe)
    try:
        n = e.ice_flow(tenths / 10.0, DX, DY)
        whole = e.get_field("h_iwe")
    finally:
        e.close()
    assert [int(r["n_sub"]) for r in ranks] == [n, n]
    assert [int(r["rows"]) for r in ranks] == [row_block(ny, i, 2)[1] for i in range(2)]
    np.testing.assert_array_equal(np.concatenate([r["iwe"] for r in ranks]), whole)
