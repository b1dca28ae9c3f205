"""The oracle (CPU restatement, oracle/tfg_oracle.py) against fixtures made by
running the reference itself (tests/golden/make_golden.py) and against the
reference's own golden tests/data/output_m_total.npy."""

import numpy as np
import pytest

from tests.harness import GOLDEN, OUT_NAMES, load_golden, oracle_run

FIXTURES = ["cat3062920_265", "grid64", "clock_dst_end", "clock_dst_start", "clock_new_year", "dt2", "dt_quarter",
            "satterlund", "params", "clock_phoenix", "clock_anchorage", "clock_denver", "clock_boise", "clock_chicago",
            "clock_new_york", "clock_honolulu"]
RTOL = 1e-12  # bit-exact here; margin for numpy SIMD paths of other host CPUs


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(b != 0, np.abs(a - b) / np.abs(b), np.abs(a - b))
    return float(np.max(r)) if r.size else 0.0


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_reference_outputs(name):
    g = load_golden(name)
    out, m = oracle_run(g["cfg"], g["static"], g["forcing"], tz_name=g["tz_name"])
    for v in OUT_NAMES:
        assert _rel(out[v], g["outputs"][v]) <= RTOL, v
    for v in ("Q_sum", "Qn_SW", "Qn_LW", "Qh", "Qe", "Eccs", "Ecci", "albedo", "n", "p0", "T_surf", "W_p"):
        assert _rel(out[v], g["internal"][v]) <= RTOL, v
    # domain integrals: each fixture cell was its own reference model
    for i, v in enumerate(("vol_P", "vol_PR", "vol_PS", "vol_SM", "vol_IM")):
        assert _rel(out[v], g["internal"][v].sum(axis=1)) <= 1e-12, v
    assert _rel(out["P_max"], g["internal"]["P_max"].max(axis=1)) == 0.0
    # per-cell melt integrals (the terms a catchment's vol_SM / vol_IM sum):
    # each fixture cell was its own reference model, so they are its vol_SM / vol_IM
    assert _rel(np.broadcast_to(m.cell_vol_SM, (g["ncell"],)), g["internal"]["vol_SM"][-1]) <= 1e-12
    assert _rel(np.broadcast_to(m.cell_vol_IM, (g["ncell"],)), g["internal"]["vol_IM"][-1]) <= 1e-12


def test_reference_known_answer_runoff():
    """integration_test.py:151-153: M_total * da_m2 against output_m_total.npy."""
    g = load_golden("cat3062920_265")
    out, m = oracle_run(g["cfg"], g["static"], g["forcing"])
    runoff = out["M_total"][:, 0] * m.da_m2
    ref = np.load(GOLDEN / "ref_output_m_total.npy")
    assert runoff.shape == ref.shape == (265,)
    assert _rel(runoff, ref) < 1e-13
    assert np.count_nonzero(ref) == 70


def test_oracle_no_snow_no_ice():
    """integration_test.py:192-243: zero depths -> SM == IM == 0."""
    cfg = dict(load_golden("cat3062920_265")["cfg"])
    st = dict(elev=cfg["elev"], slope=cfg["slope"], aspect=cfg["aspect"], h0_snow=0.0, h0_ice=0.0, h0_swe=0.0, h0_iwe=0.0)
    f = {"P": np.array([[0.0]]), "T_air": np.array([[5.0]]), "Hum_sp": np.array([[0.003]]),
         "P_air": np.array([[88000.0]]), "uz": np.array([[2.0]])}
    out, _ = oracle_run(cfg, st, f, 1)
    assert out["SM"][0, 0] == 0.0 and out["IM"][0, 0] == 0.0


def test_oracle_rejects_negative_slope():
    cfg = dict(load_golden("cat3062920_265")["cfg"])
    import tfg_oracle as O

    with pytest.raises(ValueError):
        O.OracleGrid(cfg, elev=2000.0, slope=-1.0, aspect=0.0, h0_snow=1.0, h0_ice=1.0, h0_swe=0.05, h0_iwe=0.9)
