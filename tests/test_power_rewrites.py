"""The fp64 engine's rewrites of the reference's constant-exponent powers
(csrc/tfg_physics.hpp: pow4, pow1p5, root7), checked in numpy fp64
against the reference's own `**` over the ranges the physics feeds them:

- T**4.0 of the long-wave terms (bmi_topoflow_glacier.py:1231-1233), T in K;
- RH**1.5 of the Stull wet bulb (:1520), RH a fraction;
- ((e_air/10)/T_air_K)**(1/7) of em_air (:1167), by one Halley step from an
  fp32 seed (round 5; before: exp(log(x)/7)).

The bound written here (ulps of the reference's result) is the one DESIGN.md
section 3 states; the GPU fixture tests (test_gpu_parity.py) check the engine
itself at 1e-10 and report ~1e-14.
"""

import numpy as np
import pytest


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


def _root7(x):
    """csrc/tfg_physics.hpp root7 restated in numpy: an fp32 seed y0 (numpy's
    float32 exp2 / log2 standing in for v_exp_f32 / v_log_f32) and one Halley
    step y0 - y0 (y0^7 - x) / (4 y0^7 + 3 x) in fp64."""
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        y0 = np.exp2(np.log2(np.float32(x)) * np.float32(1.0 / 7.0)).astype(np.float64)
        y2 = y0 * y0
        y7 = (y2 * y2) * (y2 * y0)
        y = y0 - y0 * ((y7 - x) / (4.0 * y7 + 3.0 * x))
    return np.where((x > 0) & (x < np.inf), y, y0)


ROOT7_ULPS = 2.0


def test_seventh_root_by_halley():
    rng = np.random.default_rng(9)
    # (e_air / 10) / T_air_K: vapour pressure 0.1-60 mbar over 200-330 K
    x = (rng.uniform(0.1, 60.0, 200_000) / 10.0) / rng.uniform(200.0, 330.0, 200_000)
    assert _ulps(_root7(x), x ** (1.0 / 7.0)).max() <= ROOT7_ULPS
    edge = _root7(np.array([0.0, -1.0, np.inf]))
    assert edge[0] == 0.0 and np.isnan(edge[1]) and edge[2] == np.inf


# The Stull wet bulb's atan(0.151977 sqrt(RH + 8.313659)) on RH in [0, 5] as
# the engines evaluate it (csrc/tfg_physics.hpp stull_atan0_poly, wet_bulb_f):
# Horner in t = 0.4 RH - 1 with the coefficients restated here.
STULL64 = [float.fromhex(h) for h in (
    "0x1.da94c1a0c29f5p-2", "0x1.7aac28df5f664p-5", "-0x1.ea2542f0a20c4p-9", "0x1.bc9c3023533e3p-12",
    "-0x1.f1959460701e0p-15", "0x1.3be2008d543e9p-17", "-0x1.b16bbee999fe5p-20", "0x1.38df9b2403c64p-22",
    "-0x1.d44af1ebe2f10p-25", "0x1.686a49a337c49p-27", "-0x1.17d5b0c2a427ap-29", "0x1.acccbc15e0e7fp-32",
    "-0x1.a2f6161678e01p-34", "0x1.b58d687bb4412p-36")]
STULL32 = [0.4634580910205841, 0.046224694699048996, -0.003739525331184268, 0.0004237863759044558,
           -5.9253852668916807e-05, 9.90594708127901e-06, -1.7216859760083025e-06]


def test_stull_arctangent_fits():
    """The fp64 fit is within 2e-14 and the fp32 one within 1.2e-7 (the fp32
    engine's atan is good to 1.5e-7) of arctan(0.151977 sqrt(RH + 8.313659))
    over [0, 5], the range the engines use them on (other RH take atan)."""
    rh = np.linspace(0.0, 5.0, 200_001)
    ref = np.arctan(0.151977 * np.sqrt(rh + 8.313659))
    t = 0.4 * rh - 1.0
    y = np.full_like(t, STULL64[-1])
    for c in STULL64[-2::-1]:
        y = y * t + c
    assert (np.abs(y - ref) / ref).max() <= 2e-14
    t32 = np.float32(0.4) * rh.astype(np.float32) - np.float32(1.0)
    y32 = np.full_like(t32, np.float32(STULL32[-1]))
    for c in STULL32[-2::-1]:
        y32 = (y32 * t32 + np.float32(c)).astype(np.float32)
    assert (np.abs(y32.astype(np.float64) - ref) / ref).max() <= 1.2e-7


def _device(x, which):
    """The engine's own device functions (tfg_selftest_powers: pow4, pow1p5,
    root7 of csrc/tfg_physics.hpp) on x."""
    import ctypes

    from topoflow_glacier import _native

    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    _native.check(_native.load().tfg_selftest_powers(0, x.ctypes.data_as(ctypes.c_void_p), x.size, which,
                                                     out.ctypes.data_as(ctypes.c_void_p)))
    return out


@pytest.mark.gpu
def test_power_rewrites_on_the_device():
    """The same three rewrites as run by the GPU (pow1p5's sqrt_k from the
    v_rsq_f64 seed; root7's hardware seed), against numpy's `**` over the same
    ranges, with the same bounds, and the same zero, NaN and infinity cases."""
    rng = np.random.default_rng(7)
    T = rng.uniform(200.0, 330.0, 200_000)
    assert _ulps(_device(T, 0), T ** 4.0).max() <= 2.0
    RH = np.concatenate([rng.uniform(0.0, 1.5, 200_000), [0.0, 1.0]])
    ref = RH ** 1.5
    got = _device(RH, 1)
    ok = ref > 0
    assert _ulps(got[ok], ref[ok]).max() <= 2.0 and got[~ok].tolist() == ref[~ok].tolist()
    x = (rng.uniform(0.1, 60.0, 200_000) / 10.0) / rng.uniform(200.0, 330.0, 200_000)
    assert _ulps(_device(x, 2), x ** (1.0 / 7.0)).max() <= ROOT7_ULPS
    edge = _device(np.array([0.0, -1.0, np.nan, np.inf]), 2)
    assert edge[0] == 0.0 and np.isnan(edge[1]) and np.isnan(edge[2]) and edge[3] == np.inf
    m = {"pow4_max_ulps": float(_ulps(_device(T, 0), T ** 4.0).max()),
         "pow1p5_max_ulps": float(_ulps(got[ok], ref[ok]).max()),
         "root7_max_ulps": float(_ulps(_device(x, 2), x ** (1.0 / 7.0)).max())}
    import json
    import os

    d = os.environ.get("TFG_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "power_rewrites_device.json"), "w") as f:
            json.dump(m, f)
