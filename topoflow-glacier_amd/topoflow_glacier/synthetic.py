"""Synthetic glacier workload (BASELINE configs 2-5), host mirror.

The device generator ``tfg_fill_synthetic`` (csrc/tfg_engine.hip) fills the
forcing frames, static rasters and initial depths of a shard from a
counter-based hash of (seed, field, frame, global cell).  This module computes
the *same* fp32 values with numpy, cell by cell, so a CPU run (the oracle, or
the CPU baseline) can consume exactly the inputs the GPU consumed, for any
subset of cells, without copying the GPU arrays back.

Statistics follow tests/data/sample-cat-3062920.csv:
T_air -15..15 degC around a per-cell mean with a 24-frame diurnal cycle;
specific humidity 0.0019-0.0061; surface pressure 87.1-89.7 kPa;
wind 0.28-15.8 m/s; precipitation on 24 % of cell-hours, up to 5.2e-7 m per
step (the reference caller's RAINRATE*1e-3, examples/run_topoflow_glacier.py:66);
elevation 1500-3000 m, slope 0.5-100 (tan beta), aspect 0-360;
SWE 0.25 m and IWE 1.834 m with +-20 % jitter.
"""

from __future__ import annotations

import numpy as np

__all__ = ["diurnal_table", "hash_u01", "synthetic_cells", "DEFAULT_SEED"]

DEFAULT_SEED = 20251001
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def hash_u01(seed: int, field: int, frame: int, cell: np.ndarray) -> np.ndarray:
    """fp32 uniform in [0, 1) with 24 random bits (device: hash_u01)."""
    k = (np.uint64(field) << np.uint64(58)) ^ (np.uint64(frame) << np.uint64(42)) ^ cell.astype(np.uint64)
    h = _splitmix64(np.uint64(seed) ^ _splitmix64(k))
    return (h >> np.uint64(40)).astype(np.float32) * np.float32(2.0**-24)


def diurnal_table(n_frames: int) -> np.ndarray:
    """Hourly diurnal factor in [-1, 1], warmest at 15 h (fp32)."""
    h = np.arange(n_frames, dtype=np.float64)
    return np.sin(2 * np.pi * (h - 9.0) / 24.0).astype(np.float32)


def synthetic_cells(seed: int, cells: np.ndarray, diurnal: np.ndarray) -> dict:
    """Inputs of the given global cell indices.

    Returns fp32 arrays: static elev/slope/aspect [ncell]; initial depths
    h_swe/h_iwe/h_snow/h_ice [ncell]; forcing P/T_air/Hum_sp/P_air/uz
    [n_frames][ncell] -- bit-identical to the device generator.
    """
    f32 = np.float32
    c = np.asarray(cells, dtype=np.uint64)
    u = lambda field, frame=0: hash_u01(seed, field, frame, c)  # noqa: E731
    out = {
        "elev": f32(1500.0) + f32(1500.0) * u(7),
        "slope": f32(0.5) + f32(99.5) * u(8),
        "aspect": f32(360.0) * u(9),
    }
    h_swe = f32(0.25) * (f32(0.8) + f32(0.4) * u(10))
    h_iwe = f32(1.834) * (f32(0.8) + f32(0.4) * u(11))
    out.update(h_swe=h_swe, h_iwe=h_iwe, h_snow=h_swe * f32(20.0), h_ice=h_iwe * f32(1.0905125))
    Tbar = f32(-8.0) + f32(16.0) * u(6)
    nf = len(diurnal)
    T = np.empty((nf, c.size), f32)
    Q = np.empty_like(T)
    PA = np.empty_like(T)
    UZ = np.empty_like(T)
    P = np.empty_like(T)
    for f in range(nf):
        T[f] = (Tbar + f32(5.0) * f32(diurnal[f])) + f32(2.0) * (u(0, f) - f32(0.5))
        Q[f] = f32(0.0019) + f32(0.0042) * u(1, f)
        PA[f] = f32(87100.0) + f32(2600.0) * u(2, f)
        UZ[f] = f32(0.28) + f32(15.5) * u(3, f)
        P[f] = np.where(u(4, f) < f32(0.24), f32(5.2e-7) * u(5, f), f32(0.0))
    out.update(T_air=T, Hum_sp=Q, P_air=PA, uz=UZ, P=P)
    return out
