"""The fp64 engine's rewrites of the reference's constant-exponent powers
(csrc/tfg_physics.hpp: pow4, pow1p5, pow_small_root), checked in numpy fp64
against the reference's own `**` over the ranges the physics feeds them:

- T**4.0 of the long-wave terms (bmi_topoflow_glacier.py:1231-1233), T in K;
- RH**1.5 of the Stull wet bulb (:1520), RH a fraction;
- ((e_air/10)/T_air_K)**(1/7) of em_air (:1167).

The bound written here (ulps of the reference's result) is the one DESIGN.md
section 3 states; the GPU fixture tests (test_gpu_parity.py) check the engine
itself at 1e-10 and report ~1e-14.
"""

import numpy as np


def _ulps(a, b):
    return np.abs(a - b) / np.spacing(np.abs(b))


def test_fourth_power_as_products():
    rng = np.random.default_rng(7)
    T = rng.uniform(200.0, 330.0, 200_000)
    x2 = T * T
    assert _ulps(x2 * x2, T ** 4.0).max() <= 2.0


def test_power_one_and_a_half_as_x_sqrt_x():
    rng = np.random.default_rng(8)
    RH = np.concatenate([rng.uniform(0.0, 1.5, 200_000), [0.0, 1.0]])
    ref = RH ** 1.5
    ok = ref > 0
    assert _ulps((RH * np.sqrt(RH))[ok], ref[ok]).max() <= 2.0
    assert (RH * np.sqrt(RH))[~ok].tolist() == ref[~ok].tolist()


def test_seventh_root_as_exp_log():
    rng = np.random.default_rng(9)
    # (e_air / 10) / T_air_K: vapour pressure 0.1-60 mbar over 200-330 K
    x = (rng.uniform(0.1, 60.0, 200_000) / 10.0) / rng.uniform(200.0, 330.0, 200_000)
    inv7 = 1.0 / 7.0
    assert _ulps(np.exp(np.log(x) * inv7), x ** inv7).max() <= 4.0
    with np.errstate(divide="ignore", invalid="ignore"):
        zero, neg = np.float64(0.0), np.float64(-1.0)
        assert np.exp(np.log(zero) * inv7) == zero ** inv7 == 0.0
        assert np.isnan(np.exp(np.log(neg) * inv7)) and np.isnan(neg ** inv7)
