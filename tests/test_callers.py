"""The callers on either side of the melt update:
forcing ingestion with the reference driver's unit conversions, the mock
routing, and the single-catchment driver in both of its modes."""

from __future__ import annotations

import numpy as np
import pytest
import yaml

from tests.harness import BASE_CFG, GOLDEN, load_golden

CSV = GOLDEN / "sample-cat-3062920.csv"


def test_forcing_csv_matches_the_reference_driver_inputs():
    """The seven per-step inputs equal, bit for bit, what the reference's
    examples/run_topoflow_glacier.py fed set_value() in the golden run
    (tests/golden/make_golden.py recorded them)."""
    from topoflow_glacier.forcing import read_forcing_csv

    g = load_golden("cat3062920_265")
    t = read_forcing_csv(CSV, BASE_CFG["start_time"], BASE_CFG["end_time"])
    assert len(t) == g["nsteps"] == 265
    for name, ref in g["forcing"].items():
        np.testing.assert_array_equal(t.inputs[name], ref[:, 0], err_msg=name)
    assert str(t.times[0])[:13] == "2013-03-20T00" and str(t.times[-1])[:13] == "2013-03-31T00"


def test_forcing_csv_window_and_errors(tmp_path):
    from topoflow_glacier.forcing import INTERNAL, frames_from_table, read_forcing_csv

    t = read_forcing_csv(CSV)  # no window: every row
    assert len(t) == 288
    s = t.step(5)
    assert set(s) == set(INTERNAL.values()) and s["wind_speed_UV"] == t.inputs["uz"][5]
    fr = frames_from_table(t, ncell=3)
    assert fr["P"].shape == (288, 3) and np.array_equal(fr["P"][:, 2], t.inputs["P"])
    bad = tmp_path / "bad.csv"
    bad.write_text("Time,RAINRATE\n2013-03-20 00:00:00,0.0\n")
    with pytest.raises(KeyError):
        read_forcing_csv(bad)


def test_boxcar_route_is_the_20_step_moving_average():
    from topoflow_glacier.routing import boxcar_route

    rng = np.random.default_rng(3)
    x = rng.random(300)
    y = boxcar_route(x)
    ref = np.array([sum(0.05 * x[i - j] for j in range(min(i, 19) + 1)) for i in range(len(x))])
    np.testing.assert_allclose(y, ref, rtol=1e-14, atol=0)
    assert np.array_equal(boxcar_route(np.stack([x, 2 * x], 1))[:, 0], y)
    # causal: an impulse spreads over the next 20 steps only
    imp = np.zeros(50)
    imp[10] = 1.0
    r = boxcar_route(imp)
    assert np.all(r[:10] == 0) and np.allclose(r[10:30], 0.05) and np.all(r[30:] == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["bmi", "bulk"])
def test_run_catchment_reproduces_the_reference_runoff(tmp_path, mode):
    """examples/run_topoflow_glacier.py end to end: runoff [m3 s-1] against the
    reference's golden tests/data/output_m_total.npy (integration_test.py:151-153)."""
    from topoflow_glacier.run import run_catchment

    cfg = tmp_path / "cat.yaml"
    cfg.write_text(yaml.dump(BASE_CFG))
    r = run_catchment(cfg, forcing=CSV, mode=mode)
    ref = np.load(GOLDEN / "ref_output_m_total.npy")
    assert r["runoff"].shape == ref.shape
    rel = np.abs(r["runoff"] - ref) / np.maximum(np.abs(ref), 1e-300)
    assert np.all(np.where(ref != 0, rel, np.abs(r["runoff"])) <= 1e-10)
    g = load_golden("cat3062920_265")
    assert abs(r["h_swe"][-1] - g["outputs"]["h_swe"][-1, 0]) <= 1e-10 * abs(g["outputs"]["h_swe"][-1, 0])


@pytest.mark.gpu
def test_bulk_mode_equals_per_step_bmi(tmp_path):
    """Uploading the window as frames and fusing the steps changes nothing."""
    from topoflow_glacier.run import run_catchment

    cfg = tmp_path / "cat.yaml"
    cfg.write_text(yaml.dump(BASE_CFG))
    a = run_catchment(cfg, forcing=CSV, mode="bmi")
    b = run_catchment(cfg, forcing=CSV, mode="bulk")
    for k in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH"):
        assert np.array_equal(a[k], b[k]), k
    assert a["h_swe"][-1] == b["h_swe"][-1] and a["h_iwe"][-1] == b["h_iwe"][-1]
    assert np.array_equal(a["routed"], b["routed"])


@pytest.mark.gpu
def test_integration_md_binding_stub_runs(tmp_path):
    """The reference-side ctypes binding shown in INTEGRATION.md section 2,
    executed as written (this package aliased as topoflow_glacier_mi355x, the
    reference's _dynamic_input_vars / _output_vars in scope), drives a model
    through the golden window and matches the drop-in BMI bit for bit."""
    import re
    import sys
    import types

    import topoflow_glacier
    import topoflow_glacier._native
    import topoflow_glacier.engine
    import topoflow_glacier.physics.clock
    from topoflow_glacier import BmiTopoflowGlacier
    from topoflow_glacier.bmi import bmi_topoflow_glacier as btg
    from topoflow_glacier.forcing import read_forcing_csv
    from tests.harness import ROOT

    text = (ROOT / "INTEGRATION.md").read_text()
    code = re.search(r"```python\n(# in the reference's bmi_topoflow_glacier.py\n.*?)```", text, re.S).group(1)
    alias = {"topoflow_glacier_mi355x": topoflow_glacier, "topoflow_glacier_mi355x._native": topoflow_glacier._native,
             "topoflow_glacier_mi355x.engine": topoflow_glacier.engine,
             "topoflow_glacier_mi355x.physics.clock": topoflow_glacier.physics.clock}
    saved = {k: sys.modules.get(k) for k in alias}
    sys.modules.update(alias)
    try:
        ns = {"_dynamic_input_vars": btg._dynamic_input_vars, "_output_vars": btg._output_vars}
        exec(compile(code, "INTEGRATION.md", "exec"), ns)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    cfg = tmp_path / "cat.yaml"
    cfg.write_text(yaml.dump(BASE_CFG))
    t = read_forcing_csv(CSV, BASE_CFG["start_time"], BASE_CFG["end_time"])
    host = BmiTopoflowGlacier()  # supplies cfg + the (1,) arrays, like the reference model object
    host.initialize(cfg)
    stub = ns["_GpuUpdate"](host)
    ref = BmiTopoflowGlacier()
    ref.initialize(cfg)
    for i in range(48):
        t.apply(host, i)
        stub.update()
        t.apply(ref, i)
        ref.update()
        for name in ns["OUT_ID"]:
            assert host.get_value_ptr(name)[0] == ref.get_value(name, np.zeros(1))[0], (i, name)
    stub.close()
    host.finalize()
    ref.finalize()


@pytest.mark.gpu
def test_many_bmi_instances_in_one_process_interleaved(tmp_path):
    """NextGen holds one model instance per catchment in one process and steps
    them in turn.  Twelve instances (the reference's catchment configs, two
    each) stepped round-robin through the golden forcing equal each config's
    solo run bit for bit: handles share nothing."""
    from pathlib import Path

    from topoflow_glacier import BmiTopoflowGlacier
    from topoflow_glacier.forcing import read_forcing_csv
    from tests.harness import ROOT

    cfgs = sorted((ROOT / "tests" / "golden" / "config").glob("cat-*.yaml"))
    assert len(cfgs) == 6
    t = read_forcing_csv(CSV, BASE_CFG["start_time"], BASE_CFG["end_time"])
    nsteps = 36
    names = ["snowpack__depth", "glacier_ice__thickness", "land_surface_water__runoff_volume_flux",
             "snowpack__melt_volume_flux", "glacier_ice__melt_volume_flux"]

    def run(models):
        rec = [[] for _ in models]
        for i in range(nsteps):
            for j, m in enumerate(models):
                t.apply(m, i)
                m.update()
                rec[j].append([m.get_value(v, np.zeros(1))[0] for v in names])
        return [np.array(r) for r in rec]

    def make(p: Path):
        m = BmiTopoflowGlacier()
        m.initialize(p)
        return m

    models = [make(p) for p in cfgs for _ in range(2)]
    inter = run(models)
    for m in models:
        m.finalize()
    for j, p in enumerate(cfgs):
        solo = make(p)
        ref = run([solo])[0]
        solo.finalize()
        np.testing.assert_array_equal(inter[2 * j], ref, err_msg=p.name)
        np.testing.assert_array_equal(inter[2 * j + 1], ref, err_msg=p.name)
    assert not np.array_equal(inter[0], inter[-1])  # the configs differ


@pytest.mark.gpu
def test_deferred_updates_equal_per_model_updates(tmp_path, monkeypatch):
    """``defer_update``: fourteen single-catchment models (the six catchment
    configs and one with SATTERLUND and the ground heat flux, twice each)
    stepped as an ensemble -- every model's inputs and
    update(), then every model's outputs -- advance in ONE tfg_update_many
    launch per step (k_cell_many).  Outputs every step, the cold contents,
    albedo, the mass-balance integrals and the clock equal those of models
    stepped one tfg_update at a time, bit for bit.  So do the interleaved
    pattern (each model read right after its update: batches of one), a
    model on its own stream (its own batch), update_until after a queued
    step, and finalize with a step queued."""
    from pathlib import Path

    from topoflow_glacier import BmiTopoflowGlacier, _native
    from topoflow_glacier.bmi import bmi_topoflow_glacier as B
    from topoflow_glacier.engine import UpdateBatch, update_many
    from topoflow_glacier.forcing import read_forcing_csv
    from tests.harness import ROOT

    cfgs = sorted((ROOT / "tests" / "golden" / "config").glob("cat-*.yaml"))
    extra = tmp_path / "satterlund_qg.yaml"  # the alternative vapour formulas and a nonzero Qc
    extra.write_text(yaml.dump(dict(BASE_CFG, SATTERLUND=True, ground_heat_flux=True)))
    cfgs.append(extra)
    deferred = []
    for p in cfgs:
        c = yaml.safe_load(p.read_text())
        c["defer_update"] = True
        q = tmp_path / ("deferred_" + p.name)
        q.write_text(yaml.dump(c))
        deferred.append(q)
    t = read_forcing_csv(CSV, BASE_CFG["start_time"], BASE_CFG["end_time"])
    nsteps = 30
    names = ["snowpack__depth", "snowpack__liquid-equivalent_depth", "snowpack__melt_volume_flux",
             "glacier_ice__thickness", "glacier__liquid_equivalent_depth", "glacier_ice__melt_volume_flux",
             "land_surface_water__runoff_volume_flux", "atmosphere_bottom_air_water-vapor__relative_saturation"]
    batches: list[int] = []
    run = UpdateBatch.run

    def counting(self):
        batches.append(len(self))
        run(self)

    monkeypatch.setattr(UpdateBatch, "run", counting)

    def make(p: Path):
        m = BmiTopoflowGlacier()
        m.initialize(p)
        return m

    def final(m):
        return [m.get_current_time(), float(m.Eccs[0]), float(m.Ecci[0]), float(m.albedo[0]), float(m.n[0]),
                float(m.vol_SM[0]), float(m.vol_IM[0]), float(m.vol_P[0]), float(m.P_max[0])]

    def interleaved(models):
        rec = [[] for _ in models]
        for i in range(nsteps):
            for j, m in enumerate(models):
                t.apply(m, i)
                m.update()
                rec[j].append([m.get_value(v, np.zeros(1))[0] for v in names])
        return [np.array(r) for r in rec], [final(m) for m in models]

    def ensemble(models):
        rec = [[] for _ in models]
        for i in range(nsteps):
            for m in models:
                t.apply(m, i)
                m.update()
            for j, m in enumerate(models):
                rec[j].append([m.get_value(v, np.zeros(1))[0] for v in names])
        return [np.array(r) for r in rec], [final(m) for m in models]

    ref_models = [make(p) for p in cfgs for _ in range(2)]
    ref, ref_final = interleaved(ref_models)
    assert batches == []  # not deferred: one tfg_update per step
    for m in ref_models:
        m.finalize()

    models = [make(p) for p in deferred for _ in range(2)]
    models[-1]._engine.set_stream(None)  # its own stream: a batch of its own
    got, got_final = ensemble(models)
    assert batches[:2] == [2 * len(cfgs) - 1, 1] and len(batches) == 2 * nsteps
    for j in range(len(models)):
        np.testing.assert_array_equal(got[j], ref[j], err_msg=str(j))
    assert got_final == ref_final
    # interleaved on deferred models: batches of one, the same results
    batches.clear()
    models2 = [make(p) for p in deferred for _ in range(2)]
    got2, got2_final = interleaved(models2)
    assert set(batches) == {1}
    for j in range(len(models2)):
        np.testing.assert_array_equal(got2[j], ref[j], err_msg=str(j))
    assert got2_final == ref_final
    # update_until after a queued step, then finalize with a step queued
    t.apply(models[0], nsteps)
    models[0].update()
    models[0].update_until(models[0].get_current_time() + 2 * models[0].get_time_step())
    assert models[0].get_current_time() == (nsteps + 3) * models[0].get_time_step()
    t.apply(models[1], nsteps)
    models[1].update()
    for m in models + models2:
        m.finalize()
    assert not B._BATCHES
    # a handle may appear once per call
    e = make(deferred[0])
    k = e._engine.step_index
    with pytest.raises(_native.NativeError, match="listed twice"):
        update_many([e._engine, e._engine], [e._in_block] * 2, [e._out_block] * 2)
    assert e._engine.step_index == k  # no step ran
    e.finalize()


@pytest.mark.gpu
def test_deferred_update_uses_the_inputs_update_was_given(tmp_path):
    """``defer_update``: update() copies the step's five inputs when it queues
    the step.  A write through a get_value_ptr view between update() and the
    flush changes the NEXT step, not the queued one, as in the reference, whose
    update() uses its inputs at once."""
    from topoflow_glacier import BmiTopoflowGlacier

    cfg_d, cfg_n = tmp_path / "d.yaml", tmp_path / "n.yaml"
    cfg_d.write_text(yaml.dump(dict(BASE_CFG, defer_update=True)))
    cfg_n.write_text(yaml.dump(BASE_CFG))
    models = []
    for c in (cfg_d, cfg_n):
        m = BmiTopoflowGlacier()
        m.initialize(str(c))
        for name, v in (("atmosphere_water__liquid_equivalent_precipitation_rate", 2e-4),
                        ("land_surface_air__temperature", -1.5), ("land_surface_air__pressure", 88000.0),
                        ("atmosphere_air_water~vapor__relative_saturation", 0.004), ("wind_speed_UV", 3.0)):
            m.set_value(name, np.array([v]))
        models.append(m)
    d, n = models
    d.update()  # queued
    d.get_value_ptr("land_surface_air__temperature")[:] = 25.0  # after update(), before the flush
    n.update()
    outs = ("snowpack__melt_volume_flux", "snowpack__liquid-equivalent_depth", "land_surface_water__runoff_volume_flux")
    for name in outs:  # the first read flushes the queued step
        assert d.get_value(name, np.zeros(1)).item() == n.get_value(name, np.zeros(1)).item(), name
    n.set_value("land_surface_air__temperature", np.array([25.0]))
    d.update()
    n.update()
    for name in outs:
        assert d.get_value(name, np.zeros(1)).item() == n.get_value(name, np.zeros(1)).item(), name
    for m in models:
        m.finalize()
