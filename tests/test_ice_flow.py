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
@pytest.mark.parametrize("shape", [(1, 1), (1, 300), (33, 257), (65, 513)])
def test_gpu_flow_ragged_tiles_match_restatement(shape):
    """Grids that leave a one-row last strip (33 = 32 + 1, 65 = 2*32 + 1) and
    a one-column last workgroup (257, 513): the tile edges of k_ice_flow,
    with and without halo rows, for the step and the CFL bound."""
    g = ice_flow_gamma(BASE_CFG)
    ny, nx = shape
    bed, iwe = glacier_valley(ny + 2, nx)
    b, w = bed[1:-1], iwe[1:-1]
    north = np.stack([bed[0] + iwe[0] * WI, iwe[0] * WI])
    south = np.stack([bed[-1] + iwe[-1] * WI, iwe[-1] * WI])
    for halos in ((None, None), (north, south)):
        e = _engine(b, w)
        try:
            assert e.ice_flow_dmax(DX, DY, *halos) == ice_flow_dmax_restated(b, w, WI, g, DX, DY, *halos)
            e.ice_flow_step(0.001, DX, DY, *halos)
            want = ice_flow_step_restated(b, w, WI, g, DX, DY, 0.001, *halos)
            np.testing.assert_array_equal(e.get_field("h_iwe").reshape(w.shape), want)
        finally:
            e.close()


@pytest.mark.gpu
def test_gpu_flow_interior_then_edges_equals_whole_step():
    """TFG_FLOW_INTERIOR + TFG_FLOW_EDGES (the overlapped sharded sub-step)
    equals TFG_FLOW_ALL and the restatement bit for bit (7 row strips)."""
    from topoflow_glacier import _native as nat

    g = ice_flow_gamma(BASE_CFG)
    bed, iwe = glacier_valley(230, 300)
    b, w = bed[10:210], iwe[10:210]
    north = np.stack([bed[9] + iwe[9] * WI, iwe[9] * WI])
    south = np.stack([bed[210] + iwe[210] * WI, iwe[210] * WI])
    want = ice_flow_step_restated(b, w, WI, g, DX, DY, 0.001, north, south)
    for parts in ((nat.FLOW_ALL,), (nat.FLOW_INTERIOR, nat.FLOW_EDGES)):
        e = _engine(b, w)
        try:
            for part in parts:
                halos = (None, None) if part == nat.FLOW_INTERIOR else (north, south)
                e.ice_flow_step(0.001, DX, DY, *halos, part=part)
            np.testing.assert_array_equal(e.get_field("h_iwe").reshape(w.shape), want)
        finally:
            e.close()


@pytest.mark.gpu
def test_gpu_flow_device_halos_equal_host_halos():
    """Halo rows handed over as CUDA tensors (the RCCL path: edges written by
    the engine into device tensors, read back by device pointer) give the same
    sub-step as host arrays."""
    import torch

    bed, iwe = glacier_valley(200, 90)
    top = _engine(bed[:100], iwe[:100])
    bot = _engine(bed[100:], iwe[100:], row0=100)
    try:
        _, last_h = top.ice_flow_edges()
        first_d, _ = bot.ice_flow_edges(device="cuda:0")
        _, last_d = top.ice_flow_edges(device="cuda:0")
        np.testing.assert_array_equal(last_d.cpu().numpy(), last_h)
        want = ice_flow_step_restated(bed[100:], iwe[100:], WI, ice_flow_gamma(BASE_CFG), DX, DY, 0.001, last_h, None)
        assert bot.ice_flow_dmax(DX, DY, last_d, None) == bot.ice_flow_dmax(DX, DY, last_h, None)
        bot.ice_flow_step(0.001, DX, DY, last_d * 1.0, None)  # a fresh tensor from a torch kernel
        np.testing.assert_array_equal(bot.get_field("h_iwe").reshape(100, 90), want)
        assert first_d.is_cuda and torch.isfinite(first_d).all()
    finally:
        top.close()
        bot.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_sub", [4, 5])
def test_gpu_flow_run_equals_sub_steps(n_sub):
    """tfg_ice_flow_run (sub-steps ping-pong between state and scratch planes)
    equals n_sub separate tfg_ice_flow_step calls bit for bit, h_ice included."""
    bed, iwe = glacier_valley(100, 70)
    got = []
    for run in (True, False):
        e = _engine(bed, iwe)
        try:
            if run:
                e.ice_flow_run(0.01, DX, DY, n_sub)
            else:
                for _ in range(n_sub):
                    e.ice_flow_step(0.01 / n_sub, DX, DY)
            got.append((e.get_field("h_iwe"), e.get_field("h_ice")))
        finally:
            e.close()
    for a, b in zip(*got):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(got[0][1], got[0][0] * WI)


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
    ny, nx, tenths = 150, 30, 5  # 75 rows per rank: 3 strips, so the interior part overlaps the swap
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


def test_config_ice_flow_keys():
    from pydantic import ValidationError

    from tests.harness import cfg_object

    c = cfg_object(BASE_CFG)
    assert c.ice_flow is False and c.ice_flow_interval == 24 and c.dx is None
    with pytest.raises(ValidationError):
        cfg_object(dict(BASE_CFG, ice_flow=True))
    assert cfg_object(dict(BASE_CFG, ice_flow=True, dx=100, dy=100)).dy == 100.0


@pytest.mark.gpu
def test_bmi_ice_flow_every_interval(tmp_path):
    """BMI with ice_flow on: update() and update_until() apply the flow term
    between step k*interval and the next; both paths give the same state as
    running the engine steps and the flow by hand."""
    import yaml

    from topoflow_glacier import BmiTopoflowGlacier

    ny, nx, iv = 12, 10, 3
    bed, iwe = glacier_valley(ny, nx)
    cfg = dict(BASE_CFG, ny=ny, nx=nx, ice_flow=True, ice_flow_interval=iv, dx=DX, dy=DY)
    path = tmp_path / "cfg.yaml"
    path.write_text(yaml.dump(cfg))
    res = []
    for mode in ("update", "update_until"):
        m = BmiTopoflowGlacier()
        m.initialize(str(path))
        m.set_value("land_surface__elevation", bed.reshape(-1))
        m.set_value("glacier__liquid_equivalent_depth", iwe.reshape(-1))
        for name, v in (("land_surface_air__temperature", -5.0), ("land_surface_air__pressure", 88000.0),
                        ("atmosphere_air_water~vapor__relative_saturation", 0.003), ("wind_speed_UV", 3.0),
                        ("atmosphere_water__liquid_equivalent_precipitation_rate", 0.0)):
            m.set_value(name, np.full(ny * nx, v))
        if mode == "update":
            for _ in range(7):
                m.update()
        else:
            m.update_until(7 * m.get_time_step())
        res.append(m.get_value("glacier__liquid_equivalent_depth", np.zeros(ny * nx)).copy())
        m.finalize()
    np.testing.assert_array_equal(res[0], res[1])
    assert np.abs(res[0] - iwe.reshape(-1)).max() > 0.0  # flow ran (at steps 3 and 6)
