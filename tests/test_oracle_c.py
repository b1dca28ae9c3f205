"""The C oracle (oracle/tfg_oracle_c.c, the multi-core CPU baseline) against the
fixtures made by running the reference (tests/golden/make_golden.py) and
against the numpy oracle.

The C restatement follows the reference's operation order, but its
transcendentals come from glibc, not numpy's SIMD loops, so it differs from the
reference in the last ulp (observed <= 4e-13 relative) instead of matching bit
for bit as the numpy oracle does.  One place turns an ulp into a visible
difference: the melt-out residual of update_swe (:1599), which decides the ice
melt gate (:1424) on an exact zero ("Melt-out flips").  Cells whose
trajectories part there are classified by tests.harness.melt_out_flips and
compared up to the flip; anything else must hold to 1e-12.
"""

import subprocess

import numpy as np
import pytest

from tests.harness import OUT_NAMES, load_golden, melt_out_flips, oracle_run, valid_mask

import tfg_oracle_c as OC  # noqa: E402  (tests/harness puts oracle/ on sys.path)

FIXTURES = ["cat3062920_265", "grid64", "clock_dst_end", "clock_dst_start", "clock_new_year", "dt2", "dt_quarter",
            "satterlund", "params", "clock_phoenix", "clock_anchorage"]
RTOL = 1e-12


def _floored(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    nz = np.abs(b[b != 0])
    s = float(np.percentile(nz, 99)) if nz.size else 0.0
    fl = np.maximum(np.abs(b), s)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(fl > 0, np.abs(a - b) / fl, np.where(a != b, np.inf, 0.0))


def _check(c_out, ref_out, max_flips):
    flip, genuine = melt_out_flips(c_out, ref_out, rtol=RTOL)
    assert not genuine, genuine[:5]
    assert (flip >= 0).sum() <= max_flips
    nsteps = np.asarray(ref_out["h_snow"]).shape[0]
    ok = valid_mask(flip, nsteps)
    for v in OUT_NAMES:
        assert np.max(_floored(c_out[v], ref_out[v])[ok], initial=0.0) <= RTOL, v
    return flip


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not OC.LIB_PATH.exists():  # test infrastructure: build the checker if this tree has not yet
        subprocess.run(["make", "-s", "-C", str(OC.LIB_PATH.parents[1])], check=True)
    OC.load()


@pytest.mark.parametrize("name", FIXTURES)
def test_c_oracle_matches_reference_outputs(name):
    g = load_golden(name)
    out, diag = OC.run_oracle_c(g["cfg"], g["static"], g["forcing"], nthreads=2, tz_name=g["tz_name"])
    flip = _check(out, g["outputs"], max_flips=max(1, g["ncell"] // 32))
    if (flip < 0).all():  # domain integrals: each fixture cell was its own reference model
        for v in ("vol_P", "vol_PR", "vol_PS", "vol_SM", "vol_IM"):
            ref = g["internal"][v].sum(axis=1)[-1]
            assert abs(diag[v] - ref) <= 1e-12 * max(abs(ref), 1e-300), v
    assert diag["P_max"] == g["internal"]["P_max"].max()


def test_c_oracle_matches_numpy_oracle_on_the_synthetic_workload():
    from tests.harness import synthetic_inputs

    syn, _ = synthetic_inputs(20251001, 16, 256, 24)
    nsteps = 60
    frames = np.arange(nsteps) % 24
    cfg = load_golden("cat3062920_265")["cfg"]
    static = {"elev": syn["elev"], "slope": syn["slope"], "aspect": syn["aspect"], "h0_snow": syn["h_snow"],
              "h0_ice": syn["h_ice"], "h0_swe": syn["h_swe"], "h0_iwe": syn["h_iwe"]}
    static = {k: np.asarray(v, np.float64) for k, v in static.items()}
    f_np = {k: syn[k][frames].astype(np.float64) for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    ref, _ = oracle_run(cfg, static, f_np, nsteps)
    f_c = {k: syn[k].astype(np.float64) for k in ("P", "T_air", "Hum_sp", "P_air", "uz")}
    out, diag = OC.run_oracle_c(cfg, static, f_c, nsteps, frames=frames, nthreads=3)
    _check(out, ref, max_flips=4)
    for v in ("vol_P", "vol_PR", "vol_PS", "P_max"):
        assert abs(diag[v] - ref[v][-1]) <= 1e-12 * abs(ref[v][-1]), v


def test_c_oracle_is_thread_count_independent():
    g = load_golden("grid64")
    a, da = OC.run_oracle_c(g["cfg"], g["static"], g["forcing"], nthreads=1)
    b, db = OC.run_oracle_c(g["cfg"], g["static"], g["forcing"], nthreads=5)
    for v in OUT_NAMES:
        assert np.array_equal(a[v], b[v]), v  # cells are independent
    for v in da:
        assert abs(da[v] - db[v]) <= 1e-14 * max(abs(da[v]), 1e-300), v  # only the summation order differs
    last, _ = OC.run_oracle_c(g["cfg"], g["static"], g["forcing"], hist=False, nthreads=3)
    for v in OUT_NAMES:
        assert np.array_equal(last[v], a[v][-1]), v


def test_c_oracle_rejects_negative_slope_and_no_snow_no_ice():
    cfg = dict(load_golden("cat3062920_265")["cfg"])
    f = {"P": np.array([[0.0]]), "T_air": np.array([[5.0]]), "Hum_sp": np.array([[0.003]]),
         "P_air": np.array([[88000.0]]), "uz": np.array([[2.0]])}
    st = dict(elev=cfg["elev"], slope=-1.0, aspect=cfg["aspect"], h0_snow=1.0, h0_ice=1.0, h0_swe=0.05, h0_iwe=0.9)
    with pytest.raises(ValueError):
        OC.run_oracle_c(cfg, st, f, 1)
    st.update(slope=cfg["slope"], h0_snow=0.0, h0_ice=0.0, h0_swe=0.0, h0_iwe=0.0)
    out, _ = OC.run_oracle_c(cfg, st, f, 1)  # integration_test.py:192-243
    assert out["SM"][0, 0] == 0.0 and out["IM"][0, 0] == 0.0


def test_c_oracle_resumes_from_a_numpy_oracle_state():
    """orc_run_from: one step of the C oracle from the numpy oracle's state at
    step 250 (depths, cold contents, albedo, days since snowfall, the 72-slot
    window) equals the numpy oracle's own step 250 to 1e-12.  This is the fp64
    baseline of the one-step state-reinjection GPU test."""
    import tfg_oracle as O

    from tests.harness import BASE_CFG, c_oracle_hist, synthetic_inputs

    syn, _ = synthetic_inputs(20251001, 1, 256, 24)
    static = {k: np.asarray(syn[s], np.float64) for k, s in (
        ("elev", "elev"), ("slope", "slope"), ("aspect", "aspect"), ("h0_snow", "h_snow"), ("h0_ice", "h_ice"),
        ("h0_swe", "h_swe"), ("h0_iwe", "h_iwe"))}
    m = O.OracleGrid(BASE_CFG, **static)
    jd, _, _, tsn = O.oracle_clock(BASE_CFG["start_time"], 1, 260, BASE_CFG["lon"])
    names = ("P", "T_air", "Hum_sp", "P_air", "uz")
    for k in range(251):
        if k == 250:
            snap = {a: np.array(getattr(m, a), copy=True) for a in
                    ("h_swe", "h_iwe", "Eccs", "Ecci", "n", "albedo", "h_snow", "h_ice", "ring")}
        r = m.step(*(syn[v][k % 24].astype(np.float64) for v in names), jd[k], tsn[k])
    c = c_oracle_hist(BASE_CFG, static, {v: syn[v] for v in names}, 1, frames=np.array([250 % 24]), state=snap,
                      clock=(jd, tsn), start_step=250)
    for v in OUT_NAMES:
        assert np.max(_floored(c[v][0], r[v])) <= RTOL, v


def test_depletion_step_rule_checks_the_last_melt_by_the_depth_identity():
    """tests.harness.depletion_steps: at the step a snowpack runs dry in both
    runs, SM*3600*w_s is the depth left at the step before (update_swe caps the
    melt, :1594-1606), so the rate's difference must equal the previous depth's
    difference (to the rounding of the output slots).  Such an entry is marked
    whether or not it is within the rate's own tolerance; a rate that breaks
    the identity, or snow left in one run, is not (the rule no
    longer excuses anything up to the depth's tolerance).  (The driver's
    384-step launches reach such steps: bench.py sample_parity, DESIGN.md
    section 3.)"""
    from tests.harness import BASE_CFG, depletion_steps

    nsteps, ncell = 4, 4000
    rng = np.random.default_rng(3)
    ws = 1000.0 / 50.0  # rho_H2O / rho_snow (config defaults)
    ref = {v: np.zeros((nsteps, ncell)) for v in OUT_NAMES}
    ref["h_snow"][:] = rng.uniform(1.0, 6.0, (1, ncell))  # p99 floor ~6 m of snow
    ref["SM"][:] = rng.uniform(1e-7, 1e-6, (1, ncell))
    ref["h_ice"][:] = 2.0
    ref["RH"][:] = 0.5
    c, c2 = 7, 8
    for cc in (c, c2):
        ref["h_snow"][1, cc], ref["h_snow"][2:, cc] = 0.0038, 0.0  # runs dry at step 2
        ref["SM"][2, cc] = 0.0038 / (3600.0 * ws)
    ref["M_total"][:] = ref["SM"]
    gpu = {v: a.copy() for v, a in ref.items()}
    d_sm = 3.7e-11  # ~1e-5 of the rate's p99 floor: out of the rate's tolerance
    gpu["h_snow"][1, c] += d_sm * 3600.0 * ws  # the depth left one step before differs by exactly that melt
    gpu["SM"][2, c] += d_sm
    gpu["h_snow"][1, c2] += 1e-12 * 3600.0 * ws  # in the rate's tolerance: marked too, by the same identity
    gpu["SM"][2, c2] += 1e-12
    gpu["M_total"][:] = gpu["SM"]
    ex = depletion_steps(gpu, ref, BASE_CFG, 1e-5)
    assert ex[2, c] and ex[2, c2] and ex.sum() == 2
    flip, genuine = melt_out_flips(gpu, ref, 1e-5, ex)
    assert not genuine and (flip < 0).all()
    assert melt_out_flips(gpu, ref, 1e-5)[1]  # without the rule: genuine
    g2 = {v: a.copy() for v, a in gpu.items()}
    g2["SM"][2, c] += 2 * d_sm  # the rate no longer matches the depth it melted: a defect in the capping
    g2["M_total"][2, c] = g2["SM"][2, c]
    assert not depletion_steps(g2, ref, BASE_CFG, 1e-5)[2, c]
    assert melt_out_flips(g2, ref, 1e-5, depletion_steps(g2, ref, BASE_CFG, 1e-5))[1]
    g4 = {v: a.copy() for v, a in gpu.items()}
    g4["M_total"][2, c] += d_sm  # M_total is not SM + IM
    assert not depletion_steps(g4, ref, BASE_CFG, 1e-5)[2, c]
    g3 = {v: a.copy() for v, a in gpu.items()}
    g3["h_snow"][2, c] = 2e-7  # snow left in one run: not a depletion step
    assert not depletion_steps(g3, ref, BASE_CFG, 1e-5)[2, c]
    g5 = {v: a.copy() for v, a in gpu.items()}
    g5["h_snow"][2:, c] = 1e-19  # a melt-out residual in one run: the zero gates part there (a flip at step 2)
    flip5, _ = melt_out_flips(g5, ref, 1e-5, depletion_steps(g5, ref, BASE_CFG, 1e-5))
    assert flip5[c] == 2