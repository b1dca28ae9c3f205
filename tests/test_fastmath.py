"""The fp64 engine's exp, log and constant-divisor division
(topoflow-glacier_amd/csrc/tfg_fastmath.hpp), which replace the device libm's
exp and log and the IEEE division sequence in every fp64 step:

- div_k(x, c, RN(1/c)) equals numpy's x / c bit for bit (correctly rounded),
  over random magnitudes and random divisors, and keeps -0, +-inf and NaN;
- exp_k is within 3 ulp of numpy's np.exp (the reference's exponential,
  e.g. :551-556, :788-802, :919, SF:610, SF:652, :1041) over the arguments the
  physics feeds it and over the whole finite range, and gives inf, 0 and NaN
  where np.exp does; the device computes the host build's bits;
- log_k is within 4 absolute ulp of np.log (:670, :888) over the physics'
  arguments and the whole positive range, with np.log's special values;
- atan_q(n, d) (the wet bulb's arctangent, :1514-1520, from its two operands)
  is within 2 ulp of the arctangent of the exact quotient n / d.

The CPU tests build the same header for the host (g++, std::fma in place of
the device's scalar-operand FMA); the GPU test checks that the device computes
exactly what the host build does.  The fixture tests (test_gpu_parity.py)
check the engine as a whole against the reference at 1e-10.
"""

import ctypes
import subprocess

import numpy as np
import pytest

from tests.harness import ROOT

SRC = ROOT / "tests" / "native" / "fastmath_host.cpp"
HEADER = ROOT / "topoflow-glacier_amd" / "csrc" / "tfg_fastmath.hpp"
EXP, EXP_LIBM, LOG, LOG_LIBM, DIV_61121, DIV_3600, EXP_VGPR, FDIV_BY_73, FDIV_73_BY = 3, 4, 5, 6, 7, 8, 9, 10, 11
ATAN_BY_73, ATAN_M73_BY = 12, 13
EXP_P, LOG_P, EXP_NEAR = 14, 15, 16  # the fp32 engine's fp64-flux form (round 6)

# the bounds HISTORY.md section 5 states (ulps of numpy's result)
EXP_ULPS = 3.0  # degree-10 polynomial since round 5 (the device libm's degree 12: 1 ulp)
LOG_ULPS = 4.0  # absolute, in ulps of max(|log x|, 1): the fp32 seed refined by one exp step (round 5)


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    so = tmp_path_factory.mktemp("fastmath") / "libfastmath_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", str(SRC), "-o", str(so)],
                   check=True)
    lib = ctypes.CDLL(str(so))
    lib.fm_eval.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int]
    lib.fm_div.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    lib.fm_fdiv.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    lib.fm_atan_q.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    lib.fm_fdiv_z.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]

    def ev(x, which):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty_like(x)
        lib.fm_eval(x.ctypes.data, y.ctypes.data, x.size, which)
        return y

    def div(x, c, fn=lib.fm_div):
        x = np.ascontiguousarray(x, dtype=np.float64)
        c = np.ascontiguousarray(c, dtype=np.float64)
        y = np.empty_like(x)
        fn(x.ctypes.data, c.ctypes.data, y.ctypes.data, x.size)
        return y

    div.fdiv = lambda x, c: div(x, c, lib.fm_fdiv)
    div.atan_q = lambda x, c: div(x, c, lib.fm_atan_q)
    div.fdiv_z = lambda x, c: div(x, c, lib.fm_fdiv_z)
    return ev, div


def _ulps(a, b):
    """|a - b| in ulps of b (both finite)."""
    return np.abs(a - b) / np.spacing(np.abs(b))


def _wide(rng, n, lo_exp, hi_exp):
    """Random doubles, log-uniform magnitudes 2^lo_exp .. 2^hi_exp, both signs."""
    m = rng.uniform(1.0, 2.0, n)
    e = rng.integers(lo_exp, hi_exp, n)
    return np.ldexp(m, e) * rng.choice([-1.0, 1.0], n)


def exp_arguments(rng):
    """What the physics feeds exp: the pressure exponent (elev 0-9000 m, 200-330 K),
    Brutsaert's 17.3 T / (T + 237.3), the albedo decay -n r, 0.0614 T_dew, the
    clear-sky a + b m_opt, em_air's log(x) / 7; then the whole finite range."""
    phys = np.concatenate([rng.uniform(-2.0, 0.2, 200_000), rng.uniform(-6.0, 3.5, 200_000),
                           rng.uniform(-130.0, 0.0, 200_000), rng.uniform(-8.0, 0.5, 200_000)])
    return phys, rng.uniform(-745.0, 709.7, 400_000)


def log_arguments(rng):
    """What the physics feeds log: e_air / 6.1121, max((z - h_snow) / z0, 0.01),
    (e_air / 10) / T_air_K; then every positive normal and subnormal magnitude."""
    phys = np.exp(rng.uniform(np.log(1e-8), np.log(1e6), 600_000))
    near_one = 1.0 + rng.uniform(-0.3, 0.3, 200_000)
    return np.concatenate([phys, near_one]), np.abs(_wide(rng, 400_000, -1074, 1024))


SPECIAL = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-320, -1e-320, 5e-324, 1.0, -1.0, 1e308, -1e308,
                    709.78, 709.79, -745.1, -745.2, 1024.5, -1075.5, 1e18, -1e18])


def _same(a, b):
    """Equal as values, NaN where NaN, and the same sign of zero."""
    a, b = np.asarray(a), np.asarray(b)
    return bool(np.all((a == b) & (np.signbit(a) == np.signbit(b)) | (np.isnan(a) & np.isnan(b))))


def test_division_by_a_constant_is_correctly_rounded(host):
    _, div = host
    rng = np.random.default_rng(11)
    x = _wide(rng, 1_000_000, -60, 60)
    c = np.abs(_wide(rng, 1_000_000, -20, 20))
    assert np.array_equal(div(x, c), x / c)
    for c0 in (6.1121, 3600.0, 1000.0, 10.0, 2016.0, 0.001, 0.2617993877991494):  # the engine's divisors
        cc = np.full_like(x, c0)
        assert np.array_equal(div(x, cc), x / cc), c0
    with np.errstate(invalid="ignore", divide="ignore"):
        cc = np.full_like(SPECIAL, 6.1121)
        assert _same(div(SPECIAL, cc), SPECIAL / cc)


def test_variable_division_within_one_ulp(host):
    """fdiv (the fp64 engine's x / y for a variable y: Newton reciprocal and
    one correction) is within 1 ulp of the IEEE quotient -- nearly always equal
    -- over the magnitudes the physics divides, and propagates NaN."""
    _, div = host
    rng = np.random.default_rng(15)
    x = _wide(rng, 1_000_000, -30, 30)
    y = _wide(rng, 1_000_000, -30, 30)
    got, ref = div.fdiv(x, y), x / y
    u = _ulps(got, ref)
    assert u.max() <= 1.0 and np.mean(got == ref) > 0.999, (u.max(), np.mean(got == ref))
    for a, b in ((np.nan, 1.0), (1.0, np.nan)):
        assert np.isnan(div.fdiv(np.array([a]), np.array([b]))[0])
    assert (div.fdiv(np.array([0.0, -0.0]), np.array([5.0, 5.0])) == 0.0).all()  # (the sign of a zero quotient
    # may differ from IEEE's; no comparison or select of the step reads it)


def test_zero_divisor_gives_the_ieee_quotient(host):
    """fdiv_z (kappa / log((z - h_snow)/z0), :670, whose log is 0 at h_snow = z - z0):
    fdiv's quotient for finite nonzero operands, IEEE's inf / 0 / NaN for a zero or
    infinite operand, as the reference's numpy division gives them."""
    _, div = host
    rng = np.random.default_rng(17)
    x, y = _wide(rng, 100_000, -30, 30), _wide(rng, 100_000, -30, 30)
    assert np.array_equal(div.fdiv_z(x, y), div.fdiv(x, y))
    a = np.array([0.408, -0.408, 0.408, 0.408, np.inf, 0.0, 0.0, np.nan, 1.0])
    b = np.array([0.0, 0.0, -0.0, np.inf, 2.0, 0.0, np.inf, 1.0, np.nan])
    assert np.isnan(div.fdiv(a[:1], b[:1])).all()  # the unguarded form's NaN
    with np.errstate(divide="ignore", invalid="ignore"):
        assert _same(div.fdiv_z(a, b), a / b)


def test_exp_within_three_ulp_of_numpy(host):
    ev, _ = host
    rng = np.random.default_rng(12)
    worst = {}
    for name, x in zip(("physics", "finite range"), exp_arguments(rng)):
        ref = np.exp(x)
        ok = ref > 0
        worst[name] = float(_ulps(ev(x, EXP)[ok], ref[ok]).max())
    assert max(worst.values()) <= EXP_ULPS, worst
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        assert _same(ev(SPECIAL[[2, 3, 4, 0, 1, 11, 10]], EXP), np.exp(SPECIAL[[2, 3, 4, 0, 1, 11, 10]]))


def _log_err(got, ref):
    """|got - ref| in ulps of max(|ref|, 1): log_k's error is absolute (~1e-15), not relative near log x = 0."""
    return np.abs(got - ref) / np.spacing(np.maximum(np.abs(ref), 1.0))


def test_log_within_four_absolute_ulp_of_numpy(host):
    ev, _ = host
    rng = np.random.default_rng(13)
    worst = {}
    for name, x in zip(("physics", "positive range"), log_arguments(rng)):
        worst[name] = float(_log_err(ev(x, LOG), np.log(x)).max())
    assert max(worst.values()) <= LOG_ULPS, worst
    with np.errstate(divide="ignore", invalid="ignore"):
        want = np.log(SPECIAL)
        fin = np.isfinite(want) & (SPECIAL != 1.0)
        assert _same(ev(SPECIAL, LOG)[~fin], want[~fin])  # 0, -0, inf, -inf, NaN, negatives, log(1) = 0
        assert _log_err(ev(SPECIAL, LOG)[fin], want[fin]).max() <= LOG_ULPS


def test_flux_form_exp_and_log_within_their_stated_bounds(host):
    """The fp64-flux form's exp_p (degree 7, 5.2e-11 relative), exp_near
    (exp(c + s) / exp(c) for |s| <= 0.41 without reduction, 5.1e-12) and log_p
    (log_k on exp_p, ~6e-11 absolute): sized for the ~1e-9 the flux form needs
    (DESIGN.md section 3), each held with a factor-2 margin on its fit's bound
    plus the fp64 evaluation's rounding, over the physics' arguments; the special
    values as exp_k / log_k."""
    ev, _ = host
    rng = np.random.default_rng(17)
    for name, x in zip(("physics", "finite range"), exp_arguments(rng)):
        ref = np.exp(x)
        ok = (ref > 1e-300) & (ref < 1e300)
        rel = np.abs(ev(x, EXP_P)[ok] - ref[ok]) / ref[ok]
        assert rel.max() <= 1.1e-10, (name, float(rel.max()))
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        assert _same(ev(SPECIAL[[2, 3, 4, 0, 1, 11, 10]], EXP_P), np.exp(SPECIAL[[2, 3, 4, 0, 1, 11, 10]]))
    s = np.concatenate([rng.uniform(-0.41, 0.41, 200000), [-0.41, 0.0, 0.41]])
    rel = np.abs(ev(s, EXP_NEAR) - np.exp(s)) / np.exp(s)
    assert rel.max() <= 1.2e-11, float(rel.max())
    # the dew point's argument e_air / 6.1121 (e_air ~0.01-80 mbar) and a wide positive range
    for x in (np.exp(rng.uniform(np.log(1e-3), np.log(15.0), 200000)), np.exp(rng.uniform(-80.0, 80.0, 200000))):
        err = np.abs(ev(x, LOG_P) - np.log(x))
        assert (err / np.maximum(np.abs(np.log(x)), 1.0)).max() <= 1.5e-10, float(err.max())
    with np.errstate(divide="ignore", invalid="ignore"):
        want = np.log(SPECIAL)
        fin = np.isfinite(want)
        assert _same(ev(SPECIAL, LOG_P)[~fin], want[~fin])


def _atan_exact(n, d):
    """arctan of the exact quotient n / d, rounded to fp64 (mpmath, 30 digits)."""
    import mpmath as mp

    with mp.workdps(30):
        return np.array([float(mp.atan2(mp.mpf(a), mp.mpf(b))) if b > 0 else
                         float(mp.atan(mp.mpf(a) / mp.mpf(b))) for a, b in zip(n, d)])


def wet_bulb_operands(rng, k):
    """The wet bulb's n = T + 1.676331 and d = 1 + (T + RH)(RH - 1.676331): T in
    [-45, 45] degC, RH a fraction in [0, 1.2]."""
    T, RH = rng.uniform(-45.0, 45.0, k), rng.uniform(0.0, 1.2, k)
    return T + 1.676331, 1.0 + (T + RH) * (RH - 1.676331)


def test_atan_from_two_operands_within_two_ulp(host):
    """atan_q(n, d) against the arctangent of the exact quotient, over the wet
    bulb's operands and random magnitudes of both signs (mpmath on a sample;
    numpy's arctan(n / d), which rounds the quotient first, on all of them);
    d = 0 gives +-pi/2, n = 0 a zero of the quotient's sign, NaN propagates."""
    _, div = host
    rng = np.random.default_rng(16)
    for n, d in (wet_bulb_operands(rng, 400_000), (_wide(rng, 400_000, -30, 30), _wide(rng, 400_000, -30, 30))):
        got = div.atan_q(n, d)
        assert _ulps(got, np.arctan(n / d)).max() <= 3.0
        i = rng.choice(n.size, 2000, replace=False)
        assert _ulps(got[i], _atan_exact(n[i], d[i])).max() <= 2.0
    got = div.atan_q(np.array([1.0, -1.0, 0.0, -0.0, np.nan, 1.0]), np.array([0.0, 0.0, 3.0, 3.0, 1.0, np.nan]))
    assert got[0] == np.pi / 2 and got[1] == -np.pi / 2 and got[2] == 0.0 and np.signbit(got[3])
    assert np.isnan(got[4:]).all()


def _device(x, which):
    from topoflow_glacier import _native

    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    _native.check(_native.load().tfg_selftest_powers(0, x.ctypes.data_as(ctypes.c_void_p), x.size, which,
                                                     out.ctypes.data_as(ctypes.c_void_p)))
    return out


@pytest.mark.gpu
def test_fastmath_on_the_device(host):
    """The device computes what the host build computes (bit for bit but for log_k, whose fp32
    seed differs; atan_q included); its exp_k (constants in scalar registers; exp_kv, in vector registers) is
    within 3 ulp of the device libm's exp; its log_k within 4 absolute ulp of the libm's log."""
    ev, _ = host
    rng = np.random.default_rng(14)
    xe = np.concatenate([*exp_arguments(rng), SPECIAL])
    assert _same(_device(xe, EXP), ev(xe, EXP))
    got, libm = _device(xe, EXP), _device(xe, EXP_LIBM)
    fin = np.isfinite(libm) & (libm > 0)
    assert _ulps(got[fin], libm[fin]).max() <= EXP_ULPS and _same(got[~fin], libm[~fin])
    assert _same(_device(xe, EXP_VGPR), _device(xe, EXP))
    xl = np.concatenate([*log_arguments(rng), SPECIAL])
    got = _device(xl, LOG)  # the device's seed (v_log_f32) differs from the host build's (log2f)
    host_ = ev(xl, LOG)
    fin = np.isfinite(host_)
    assert _log_err(got[fin], host_[fin]).max() <= LOG_ULPS and _same(got[~fin], host_[~fin])
    libm = _device(xl, LOG_LIBM)
    ok = np.isfinite(libm)
    assert _log_err(got[ok], libm[ok]).max() <= LOG_ULPS and _same(got[~ok], libm[~ok])
    xd = np.concatenate([_wide(rng, 400_000, -60, 60), SPECIAL])
    for which, c in ((DIV_61121, 6.1121), (DIV_3600, 3600.0)):
        with np.errstate(invalid="ignore"):
            assert _same(_device(xd, which), xd / c)
    xf = np.concatenate([_wide(rng, 400_000, -30, 30), [np.nan]])  # the physics divides finite normal numbers
    for which in (FDIV_BY_73, FDIV_73_BY):
        got = _device(xf, which)
        assert _same(got, ev(xf, which)), which  # the device computes what the host build does
        want = xf / 7.3 if which == FDIV_BY_73 else 7.3 / xf
        fin = np.isfinite(want)
        assert _ulps(got[fin], want[fin]).max() <= 1.0 and np.isnan(got[~fin]).all(), which
    n, _ = wet_bulb_operands(rng, 400_000)
    xa = np.concatenate([n, _wide(rng, 400_000, -30, 30), [0.0, np.nan]])
    for which in (ATAN_BY_73, ATAN_M73_BY):
        assert _same(_device(xa, which), ev(xa, which)), which  # atan_q: the host build's bits
