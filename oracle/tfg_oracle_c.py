"""ORACLE (C) -- ctypes front of oracle/_build/libtfg_oracle_c.so.  TEST INFRASTRUCTURE ONLY.

The C restatement (oracle/tfg_oracle_c.c) of ``BmiTopoflowGlacier.update()``
(bmi_topoflow_glacier.py:413-465), parallel over cells with OpenMP.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it: as a second, independent checker beside the numpy oracle, and as the
multi-core CPU baseline.  Per-step uniforms come from the numpy oracle's clock
(``tfg_oracle.oracle_clock``), which the reference fixtures pin.

Build: ``make -C oracle`` (``__graft_entry__.build()`` runs it).
"""

from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

import tfg_oracle as O

LIB_PATH = Path(__file__).resolve().parent / "_build" / "libtfg_oracle_c.so"
OUT_NAMES = O.OUT_NAMES
DIAG_NAMES = ["vol_P", "vol_PR", "vol_PS", "vol_SM", "vol_IM", "P_max"]
ORC_ERR_SLOPE = 2

_FIELDS = ["dt", "da", "lat", "T_rain_snow", "dust_atten", "canopy_factor", "cloud_factor",
           "rho_air", "rho_snow", "rho_ice", "rho_H2O", "h_active_layer", "T0", "Cp_air", "Cp_ice", "Cp_snow",
           "g", "Lf", "eps", "kappa", "latent_heat_constant", "Lv", "sigma", "sea_level_p0", "uni_gas_const",
           "M_mass_air", "z0_air", "em_surf"]


class OrcParams(ctypes.Structure):
    _fields_ = [(f, ctypes.c_double) for f in _FIELDS] + [("satterlund", ctypes.c_int32), ("pad_", ctypes.c_int32)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(str(LIB_PATH))
        dp = ctypes.POINTER(ctypes.c_double)
        L.orc_run.restype = ctypes.c_int
        L.orc_run.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int64, ctypes.c_int] + [dp] * 7 + [
            ctypes.POINTER(dp), ctypes.POINTER(ctypes.c_int32), dp, dp, dp, dp, dp, ctypes.c_int]
        L.orc_run_from.restype = ctypes.c_int
        L.orc_run_from.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int64, ctypes.c_int] + [dp] * 9 + [
            ctypes.POINTER(dp), ctypes.POINTER(ctypes.c_int32), dp, dp, dp, dp, dp, ctypes.c_int]
        L.orc_run_from_qc.restype = ctypes.c_int
        L.orc_run_from_qc.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int64, ctypes.c_int] + [dp] * 9 + [
            ctypes.POINTER(dp), ctypes.POINTER(ctypes.c_int32), dp, dp, dp, ctypes.c_int, dp, dp, dp, ctypes.c_int]
        L.orc_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def params(cfg: dict) -> OrcParams:
    c = dict(O.CFG_DEFAULTS)
    c.update(cfg)
    p = OrcParams()
    for f in _FIELDS:
        setattr(p, f, float(c[f]))
    p.satterlund = 1 if c["SATTERLUND"] else 0
    return p


def _ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if a is not None else None


STATE_NAMES = ["h_snow", "h_ice", "h_swe", "h_iwe", "Eccs", "Ecci", "albedo", "n"]


def run_oracle_c(cfg: dict, static: dict, forcing: dict, nsteps: int | None = None, clock=None, frames=None,
                 hist: bool = True, nthreads: int = 0, tz_name: str = "America/Los_Angeles", state=None,
                 qc=None, qc_every: int = 1):
    """Same arguments as ``tfg_oracle.run_oracle``; forcing arrays are
    [n_frames][ncell] and step k reads frame ``frames[k]`` (default k).
    ``state``: optional mid-run state to start from instead of initialize()'s,
    a dict with the numpy oracle's attribute names (STATE_NAMES and ``ring``,
    [ncell][ring_len] oldest slot first), e.g. a snapshot of an OracleGrid.
    ``qc``: optional lateral conduction flux [W m-2], [n_intervals][ncell]
    (or [ncell]); step k adds row k // qc_every to Q_sum.
    Returns (outputs, diag): outputs name -> [nsteps][ncell] when ``hist``,
    else name -> [ncell] of the last step; diag name -> float."""
    L = load()
    f = [np.ascontiguousarray(np.asarray(forcing[n], dtype=np.float64)) for n in ("P", "T_air", "Hum_sp", "P_air", "uz")]
    f = [x.reshape(-1, x.shape[-1]) if x.ndim > 1 else x.reshape(1, -1) for x in f]
    n_frames, ncell = f[0].shape
    nsteps = n_frames if nsteps is None else nsteps
    st = {k: np.ascontiguousarray(np.broadcast_to(np.asarray(static[k], dtype=np.float64), (ncell,)))
          for k in ("elev", "slope", "aspect", "h0_snow", "h0_ice", "h0_swe", "h0_iwe")}
    if clock is None:
        jd, _, _, tsn = O.oracle_clock(cfg["start_time"], cfg["dt"], nsteps, cfg["lon"], tz_name)
    else:
        jd, tsn = clock
    jd = np.ascontiguousarray(jd[:nsteps], dtype=np.float64)
    tsn = np.ascontiguousarray(tsn[:nsteps], dtype=np.float64)
    fr = None
    if frames is not None:
        fr = np.ascontiguousarray(frames[:nsteps], dtype=np.int32)
        if fr.size < nsteps or fr.min() < 0 or fr.max() >= n_frames:
            raise ValueError("frames out of range")
    elif nsteps > n_frames:
        raise ValueError("more steps than forcing frames")
    fp = (ctypes.POINTER(ctypes.c_double) * 5)(*[_ptr(x) for x in f])
    last = np.zeros((8, ncell))
    out = np.zeros((nsteps, 8, ncell)) if hist else None
    diag = np.zeros(6)
    p = params(cfg)
    st0 = ring0 = None
    if state is not None:
        st0 = np.ascontiguousarray(np.stack([np.broadcast_to(np.asarray(state[k], np.float64), (ncell,))
                                             for k in STATE_NAMES]))
        ring0 = np.ascontiguousarray(np.asarray(state["ring"], np.float64).reshape(ncell, -1))
        if ring0.shape[1] != int(3 * 24 / float(cfg["dt"])):
            raise ValueError("state ring length != int(72 / dt)")
    q = None
    if qc is not None:
        q = np.ascontiguousarray(np.asarray(qc, np.float64).reshape(-1, ncell))
        if q.shape[0] < (nsteps + qc_every - 1) // qc_every:
            raise ValueError("qc needs one row per conduction interval")
    rc = L.orc_run_from_qc(ctypes.byref(p), ncell, nsteps, *(_ptr(st[k]) for k in ("elev", "slope", "aspect",
                                                                                  "h0_snow", "h0_ice", "h0_swe",
                                                                                  "h0_iwe")),
                           _ptr(st0), _ptr(ring0),
                           fp, fr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) if fr is not None else None,
                           _ptr(jd), _ptr(tsn), _ptr(q), int(qc_every), _ptr(last), _ptr(out), _ptr(diag),
                           int(nthreads))
    if rc == ORC_ERR_SLOPE:
        raise ValueError("some slope angles are out of range (bmi_topoflow_glacier.py:1106-1111)")
    if rc != 0:
        raise RuntimeError(f"orc_run failed ({rc})")
    res = {n: (out[:, j, :] if hist else last[j]) for j, n in enumerate(OUT_NAMES)}
    return res, dict(zip(DIAG_NAMES, diag.tolist()))


def max_threads() -> int:
    return int(load().orc_max_threads())
