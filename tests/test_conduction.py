"""The optional lateral heat-conduction term (tfg_conduction_*; SURVEY.md
8(f) row 4).  The reference reserves the conduction flux Qc in its energy
balance (update_conduction_heat_flux, bmi_topoflow_glacier.py:936-948; Q_sum
adds Qc last, :1314) and leaves it at zero.  Two things are checked:

* the stencil (Fourier's law between neighbouring cells, tfg_conduction.hpp)
  against its numpy restatement (tests/harness.py:conduction_restated) bit for
  bit, with the properties the face form guarantees: zero net energy over the
  domain, zero flux between cells at one temperature, heat flowing from warm
  to cold, and row-block shards with exchanged halo rows equal to the whole
  grid;
* the energy balance with a nonzero Qc against the oracle (and the C oracle
  for the flip baseline), both adding Qc in the reference's position of
  Q_sum: a fixed Qc field, and Qc re-evaluated every interval from each side's
  own state (the operator-split coupling the BMI runs)."""

import numpy as np
import pytest

from tests.harness import (BASE_CFG, FLUX_F64_ENGINE, RestatedCondShard, conduction_cells, conduction_restated,
                           conduction_state, make_engine, run_gpu_vs_oracle, split_engine)
from tests.test_sharding import _torchrun
from topoflow_glacier.sharding import lateral_conduction, row_block

CFG = dict(BASE_CFG)
KS, KI, DX, DY = 0.3, 2.1, 2.0, 3.0


def test_restated_conduction_conserves_energy():
    st = conduction_state(23, 31)
    qc = conduction_restated(*st, CFG, KS, KI, DX, DY)
    scale = np.abs(qc).sum()
    assert scale > 0 and abs(qc.sum()) <= 1e-12 * scale
    # only cells with snow or ice take part
    Ts, hs, Ti, hi = conduction_cells(*st, CFG)
    assert np.all(qc[(hs == 0) & (hi == 0)] == 0.0)


def test_restated_conduction_vanishes_at_one_temperature_and_runs_warm_to_cold():
    ny, nx = 6, 7
    swe = np.full((ny, nx), 0.3)
    iwe = np.full((ny, nx), 1.0)
    # Eccs proportional to h_snow and Ecci constant: one pack temperature everywhere
    z = np.zeros((ny, nx))
    assert np.all(conduction_restated(swe, iwe, z, z, CFG, KS, KI, DX, DY) == 0.0)
    eccs = np.full((ny, nx), 4.0e5)
    eccs[3, 3] = 0.0  # one warm cell (T = T0) among cold ones
    qc = conduction_restated(swe, iwe, eccs, z, CFG, KS, 0.0, DX, DY)
    assert qc[3, 3] < 0.0  # it loses heat
    assert np.all(qc[[2, 4, 3, 3], [3, 3, 2, 4]] > 0.0)  # its four neighbours gain it
    assert qc[2, 3] * DY * DY == pytest.approx(qc[3, 2] * DX * DX, rel=1e-12)  # 1/d^2 per face direction


def test_sharded_restated_conduction_gloo_world2(tmp_path):
    ny, nx = 29, 17
    ranks = _torchrun("cond", tmp_path, ny=ny, nx=nx, steps=1)
    whole = conduction_restated(*conduction_state(ny, nx), CFG, KS, KI, DX, DY)
    np.testing.assert_array_equal(np.concatenate([r["qc"] for r in ranks]), whole.reshape(-1))
    assert [int(r["rows"]) for r in ranks] == [row_block(ny, i, 2)[1] for i in range(2)]


def test_restated_shard_interface_without_a_process_group():
    st = conduction_state(9, 8)
    sh = RestatedCondShard(*st, CFG)
    lateral_conduction(sh, KS, KI, DX, DY, distributed=False)
    np.testing.assert_array_equal(sh.qc, conduction_restated(*st, CFG, KS, KI, DX, DY))


def test_config_conduction_keys():
    from pydantic import ValidationError

    from tests.harness import cfg_object

    c = cfg_object(CFG)
    assert c.lateral_conduction is False and c.conduction_interval == 24 and c.k_snow == 0.1 and c.k_ice == 2.1
    with pytest.raises(ValidationError):
        cfg_object(dict(CFG, lateral_conduction=True))  # needs dx, dy
    # 1 m cells: the ice layer is stable for 31 h of held flux, not 48 h
    with pytest.raises(ValidationError, match="stable"):
        cfg_object(dict(CFG, lateral_conduction=True, dx=1.0, dy=1.0, conduction_interval=48))
    assert cfg_object(dict(CFG, lateral_conduction=True, dx=1.0, dy=1.0, conduction_interval=24)).dx == 1.0
    assert cfg_object(dict(CFG, lateral_conduction=True, dx=1.0, dy=1.0, conduction_interval=48, k_ice=0.0,
                           k_snow=0.0)).k_ice == 0.0


# ------------------------------------------------------------------------- GPU
def _engine(st, engine="float32", row0=0):
    swe, iwe, eccs, ecci = st
    ny, nx = swe.shape
    e = make_engine(dict(CFG), ny, nx, engine, n_frames=1, hist_depth=1, row0=row0)
    e.init_state()
    for name, v in (("h_swe", swe), ("h_iwe", iwe), ("Eccs", eccs), ("Ecci", ecci)):
        e.set_field(name, v.reshape(-1))
    return e


def _as_engine(qc, engine):
    return qc.astype(np.float32).astype(np.float64) if split_engine(engine)[0] == "float32" else qc


def _halos(full, lo, hi):
    """Halo rows [4][nx] of rows lo-1 and hi of a whole-grid state (None outside)."""
    cells = conduction_cells(*full, CFG)
    ny = full[0].shape[0]
    north = np.stack([a[lo - 1] for a in cells]) if lo > 0 else None
    south = np.stack([a[hi] for a in cells]) if hi < ny else None
    return north, south


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["float32", "float64"])
@pytest.mark.parametrize("shape", [(1, 1), (1, 300), (33, 257), (65, 513), (40, 96)])
def test_gpu_conduction_matches_restatement(engine, shape):
    """Qc of k_conduction equals the restatement bit for bit (fp64; the fp32
    engine stores it rounded to fp32), with and without halo rows, on grids
    that leave a one-row last strip and a one-column last workgroup."""
    ny, nx = shape
    full = conduction_state(ny + 2, nx)
    st = tuple(a[1:-1] for a in full)
    for halos in ((None, None), _halos(full, 1, ny + 1)):
        e = _engine(st, engine)
        try:
            assert np.all(e.get_field("Qc") == 0.0)  # the reference's Qc = 0 until a pass runs
            e.conduction_update(KS, KI, DX, DY, *halos)
            want = conduction_restated(*st, CFG, KS, KI, DX, DY, *halos)
            np.testing.assert_array_equal(e.get_field("Qc").reshape(ny, nx), _as_engine(want, engine))
        finally:
            e.close()


@pytest.mark.gpu
def test_gpu_conduction_edges_and_device_halos():
    """Edge rows written by the engine (host arrays or CUDA tensors, the RCCL
    path) are the restatement's cell values, and two shards with exchanged
    halos give the whole grid's Qc."""
    full = conduction_state(120, 70)
    top = _engine(tuple(a[:50] for a in full), "float64")
    bot = _engine(tuple(a[50:] for a in full), "float64", row0=50)
    try:
        first_h, last_h = top.conduction_edges()
        cells = conduction_cells(*full, CFG)
        np.testing.assert_array_equal(first_h, np.stack([a[0] for a in cells]))
        np.testing.assert_array_equal(last_h, np.stack([a[49] for a in cells]))
        first_d, _ = bot.conduction_edges(device="cuda:0")
        _, last_d = top.conduction_edges(device="cuda:0")
        np.testing.assert_array_equal(last_d.cpu().numpy(), last_h)
        top.conduction_update(KS, KI, DX, DY, None, first_d * 1.0)  # device halos (a fresh torch tensor)
        bot.conduction_update(KS, KI, DX, DY, last_h, None)          # host halos
        whole = conduction_restated(*full, CFG, KS, KI, DX, DY)
        got = np.concatenate([top.get_field("Qc"), bot.get_field("Qc")]).reshape(120, 70)
        np.testing.assert_array_equal(got, whole)
    finally:
        top.close()
        bot.close()


@pytest.mark.gpu
def test_gpu_sharded_conduction_gloo_world2_equals_whole_grid(tmp_path):
    ny, nx = 77, 40
    ranks = _torchrun("gpu_cond", tmp_path, ny=ny, nx=nx, steps=1)
    whole = conduction_restated(*conduction_state(ny, nx), CFG, KS, KI, DX, DY)
    np.testing.assert_array_equal(np.concatenate([r["qc"] for r in ranks]), whole.reshape(-1))


def _cold(ny, nx, seed=5):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 2.0e6, ny * nx), rng.uniform(0.0, 3.0e5, ny * nx)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["float32", "float64", FLUX_F64_ENGINE])
def test_gpu_fixed_qc_enters_q_sum_like_the_reference(engine):
    """A given Qc field (set as TFG_ST_QC) enters Q_sum where the reference
    adds its Qc (:1314): the engine matches the oracle run with the same Qc,
    under the same parity rule as every other GPU test."""
    ny, nx, nsteps = 16, 40, 48
    rng = np.random.default_rng(9)
    qc = _as_engine(rng.uniform(-80.0, 80.0, ny * nx), engine)
    r = run_gpu_vs_oracle(ny, nx, nsteps, engine=engine, seed=13, cold=_cold(ny, nx), qc=qc)
    assert r["ok"], r["summary"]
    # the term matters: without it the outputs differ well beyond tolerance
    base = run_gpu_vs_oracle(ny, nx, nsteps, engine=engine, seed=13, cold=_cold(ny, nx))
    assert np.abs(base["gpu"]["SM"] - r["gpu"]["SM"]).max() > 1e-7


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["float32", "float64"])
def test_gpu_coupled_conduction_matches_oracle(engine):
    """Qc re-evaluated every 16 steps from the state (the BMI's operator
    split) on 1 m cells, where the flux is a few W m-2: the engine's run equals
    the oracle's, each side evaluating Qc from its own state."""
    ny, nx, nsteps = 24, 32, 48
    cond = dict(k_snow=KS, k_ice=KI, dx=1.0, dy=1.0, every=16)
    r = run_gpu_vs_oracle(ny, nx, nsteps, engine=engine, seed=17, cold=_cold(ny, nx, 6), conduction=cond)
    assert r["ok"], r["summary"]


@pytest.mark.gpu
def test_gpu_conduction_off_is_the_reference_again():
    """conduction_off() zeroes Qc: the next steps equal a run that never had
    the term, bit for bit (same state in, same kernel)."""
    from topoflow_glacier.synthetic import diurnal_table

    ny, nx = 20, 30
    outs = []
    for with_term in (True, False):
        e = make_engine(dict(CFG), ny, nx, "float32", n_frames=24, hist_depth=24)
        try:
            e.fill_synthetic(3, diurnal_table(24))
            e.set_field("Eccs", _cold(ny, nx)[0])
            if with_term:
                e.conduction_update(KS, KI, 1.0, 1.0)
                assert np.abs(e.get_field("Qc")).max() > 0
                e.conduction_off()
                assert np.all(e.get_field("Qc") == 0.0)
            e.run(24)
            e.sync()
            outs.append([e.get_field(n, index=23) for n in ("h_snow", "SM", "IM", "RH")] + [e.get_field("Eccs")])
        finally:
            e.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_bmi_conduction_every_interval(tmp_path):
    """BMI with lateral_conduction on: update() and update_until() evaluate Qc
    at steps 0, k, 2k ... and give the same state; the term changes the melt."""
    import yaml

    from topoflow_glacier import BmiTopoflowGlacier

    ny, nx, iv = 8, 10, 3
    rng = np.random.default_rng(4)
    swe = rng.uniform(0.05, 0.3, ny * nx)
    res = []
    for mode, on in (("update", True), ("update_until", True), ("update", False)):
        cfg = dict(CFG, ny=ny, nx=nx, lateral_conduction=on, conduction_interval=iv, dx=1.0, dy=1.0, k_snow=0.3)
        path = tmp_path / f"cfg_{mode}_{on}.yaml"
        path.write_text(yaml.dump(cfg))
        m = BmiTopoflowGlacier()
        m.initialize(str(path))
        m.set_value("snowpack__liquid-equivalent_depth", swe)
        m.set_value("snowpack__depth", swe * 20.0)
        for name, v in (("land_surface_air__temperature", -8.0), ("land_surface_air__pressure", 88000.0),
                        ("atmosphere_air_water~vapor__relative_saturation", 0.002), ("wind_speed_UV", 3.0),
                        ("atmosphere_water__liquid_equivalent_precipitation_rate", 0.0)):
            m.set_value(name, np.full(ny * nx, v))
        # cold content varies with depth at one pack temperature, then one warm patch
        m._engine.set_field("Eccs", np.where(np.arange(ny * nx) % 7 == 0, 0.0, 3.0e4 * swe * 20.0))
        if mode == "update":
            for _ in range(7):
                m.update()
        else:
            m.update_until(7 * m.get_time_step())
        res.append((m._engine.get_field("Eccs"), m._engine.get_field("Qc")))
        m.finalize()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    assert np.abs(res[0][1]).max() > 0.0 and np.all(res[2][1] == 0.0)
    assert np.abs(res[0][0] - res[2][0]).max() > 0.0


# ------------------------------------------------------ ground heat flux (Qg)
QG = 1575000.0 / (3600.0 * 24 * 365)  # config.py:84 default [J yr-1 m-2] -> W m-2 (:283, :333)


def test_restated_ground_flux_adds_to_every_cell():
    st = conduction_state(7, 9)
    base = conduction_restated(*st, CFG, KS, KI, DX, DY)
    np.testing.assert_array_equal(conduction_restated(*st, CFG, KS, KI, DX, DY, q_ground=QG), base + QG)
    from tests.harness import cfg_object

    assert cfg_object(CFG).ground_heat_flux is False and cfg_object(dict(CFG, ground_heat_flux=True)).ground_heat_flux


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["float32", "float64"])
def test_gpu_conduction_with_ground_flux_matches_restatement(engine):
    full = conduction_state(35, 70)
    e = _engine(full, engine)
    try:
        e.conduction_update(KS, KI, DX, DY, q_ground=QG)
        want = conduction_restated(*full, CFG, KS, KI, DX, DY, q_ground=QG)
        np.testing.assert_array_equal(e.get_field("Qc").reshape(35, 70), _as_engine(want, engine))
    finally:
        e.close()


@pytest.mark.gpu
def test_bmi_ground_heat_flux_matches_the_oracle(tmp_path):
    """ground_heat_flux: true on the reference's single-catchment workflow
    (one-cell BMI, k_cell): every step adds Qg (config.py:84, :333) to Q_sum
    (:1314); the outputs equal the oracle run with Qc = Qg / sec_per_year to
    1e-10, and differ from the run without it."""
    import yaml

    from tests.harness import GOLDEN, O, load_golden
    from topoflow_glacier.run import run_catchment

    g = load_golden("cat3062920_265")
    res = {}
    for on in (True, False):
        path = tmp_path / f"cat_{on}.yaml"
        path.write_text(yaml.dump(dict(BASE_CFG, ground_heat_flux=on)))
        res[on] = run_catchment(path, forcing=GOLDEN / "sample-cat-3062920.csv", mode="bmi")
    cfg = dict(g["cfg"])
    m = O.OracleGrid(cfg, **g["static"])
    m.Qc = np.float64(QG)
    jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], g["nsteps"], cfg["lon"], g["tz_name"])
    ref = {k: [] for k in ("h_snow", "SM", "M_total", "RH")}
    for k in range(g["nsteps"]):
        r = m.step(*(g["forcing"][n][k] for n in ("P", "T_air", "Hum_sp", "P_air", "uz")), jd[k], tsn[k])
        for v in ref:
            ref[v].append(float(r[v][0]))
    for v, want in ref.items():
        want = np.array(want)
        got = np.asarray(res[True][v], np.float64)
        err = np.abs(got - want) / np.maximum(np.abs(want), 1e-300)
        assert np.all(np.where(want != 0, err, np.abs(got)) <= 1e-10), v
    assert np.abs(np.asarray(res[True]["SM"]) - np.asarray(res[False]["SM"])).max() > 0.0


@pytest.mark.gpu
def test_gpu_coupled_conduction_over_a_year():
    """A year (8760 hourly steps) of the coupled term on 1 m cells, Qc
    re-evaluated every 24 steps from each side's own state: the fp64 engine
    matches the oracle run the same way at 1e-10 every step, with the flip
    rule (the coupling adds no drift).  The fp32 engine's year-long behaviour
    is characterised by test_gpu_parity.py::test_fp32_free_run_over_a_year
    (compared once a day; melt onsets, where E_in - Eccs cancels, are many in
    a year of melt and are not a per-step 1e-5 quantity)."""
    ny, nx, nsteps = 8, 8, 8760
    cond = dict(k_snow=KS, k_ice=KI, dx=1.0, dy=1.0, every=24)
    r = run_gpu_vs_oracle(ny, nx, nsteps, engine="float64", seed=23, cold=_cold(ny, nx, 8), conduction=cond)
    assert r["ok"], r["summary"]
