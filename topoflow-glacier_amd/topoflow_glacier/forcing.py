"""Forcing ingestion for the callers of the melt update.

The reference feeds one catchment per step from a NextGen forcing CSV in its
example driver (examples/run_topoflow_glacier.py:30-73).  This module is that
mapping, column for column and with the same unit conversions in the same
operation order, so the values a caller hands to ``set_value`` are bit-identical
to the reference driver's:

  BMI input (_dynamic_input_vars, bmi_topoflow_glacier.py:18-26)   CSV column(s)
  atmosphere_water__liquid_equivalent_precipitation_rate            RAINRATE * 10**(-3)   (mm/h -> m/h, :64-65)
  land_surface_air__temperature                                     K_to_C + T2D          (K -> degC, :66)
  land_surface_radiation~incoming~longwave__energy_flux              LWDOWN                (:67)
  land_surface_radiation~incoming~shortwave__energy_flux             SWDOWN                (:68)
  land_surface_air__pressure                                        PSFC                  (:69)
  atmosphere_air_water~vapor__relative_saturation                   Q2D (specific humidity, :70)
  wind_speed_UV                                                     ((U2D)**2 + (V2D)**2)**0.5  (:45-47)

Rows are selected by ``start_time <= Time <= end_time`` (:33-40).  For grids,
:func:`frames_from_table` broadcasts or stacks per-cell tables into the
``[nsteps][ncell]`` frame arrays :meth:`GlacierEngine.set_field` uploads.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

__all__ = ["BMI_INPUTS", "INTERNAL", "K_TO_C", "ForcingTable", "read_forcing_csv", "frames_from_table"]

K_TO_C = -273.15  # BmiTopoflowGlacier.K_to_C (bmi_topoflow_glacier.py:290)

# BMI input name -> internal name (the engine's field names, _native.FIELD)
BMI_INPUTS = {
    "land_surface_radiation~incoming~longwave__energy_flux": "LW_in",
    "land_surface_air__pressure": "P_air",
    "atmosphere_air_water~vapor__relative_saturation": "Hum_sp",
    "atmosphere_water__liquid_equivalent_precipitation_rate": "P",
    "land_surface_radiation~incoming~shortwave__energy_flux": "SW_in",
    "land_surface_air__temperature": "T_air",
    "wind_speed_UV": "uz",
}
INTERNAL = {v: k for k, v in BMI_INPUTS.items()}


@dataclass
class ForcingTable:
    """Per-step BMI inputs of one catchment (float64, reference units)."""

    times: np.ndarray                      # datetime64[ns], one per step
    inputs: dict = field(default_factory=dict)  # internal name -> [nsteps] float64

    def __len__(self) -> int:
        return len(self.times)

    def step(self, i: int) -> dict:
        """BMI name -> value of step i (what the reference driver set_value()s)."""
        return {INTERNAL[k]: v[i] for k, v in self.inputs.items()}

    def apply(self, model, i: int) -> None:
        """set_value() every input of step i on a BMI model (:63-71)."""
        for name, value in self.step(i).items():
            model.set_value(name, value)


def read_forcing_csv(path: str | Path, start_time: str | None = None, end_time: str | None = None) -> ForcingTable:
    """Read a NextGen forcing CSV (columns Time, RAINRATE, T2D, LWDOWN, SWDOWN,
    PSFC, Q2D, U2D, V2D) between start_time and end_time (YYYYmmddHH, inclusive)."""
    import pandas as pd

    df = pd.read_csv(path)
    missing = {"Time", "RAINRATE", "T2D", "LWDOWN", "SWDOWN", "PSFC", "Q2D", "U2D", "V2D"} - set(df.columns)
    if missing:
        raise KeyError(f"{path}: forcing columns missing: {sorted(missing)}")
    df["Time"] = pd.to_datetime(df["Time"])
    if start_time is not None:
        df = df[df["Time"] >= pd.to_datetime(str(start_time), format="%Y%m%d%H")]
    if end_time is not None:
        df = df[df["Time"] <= pd.to_datetime(str(end_time), format="%Y%m%d%H")]
    df = df.copy()
    wind = (((df["U2D"]) ** 2 + (df["V2D"]) ** 2) ** 0.5).values
    inputs = {
        "P": df["RAINRATE"].values * 10 ** (-3),
        "T_air": K_TO_C + df["T2D"].values,
        "LW_in": df["LWDOWN"].values.astype(np.float64),
        "SW_in": df["SWDOWN"].values.astype(np.float64),
        "P_air": df["PSFC"].values.astype(np.float64),
        "Hum_sp": df["Q2D"].values.astype(np.float64),
        "uz": wind,
    }
    return ForcingTable(times=df["Time"].values, inputs={k: np.asarray(v, dtype=np.float64) for k, v in inputs.items()})


def frames_from_table(table: ForcingTable, ncell: int = 1) -> dict:
    """internal name -> [nsteps][ncell] frames (the table broadcast to ncell cells)."""
    return {k: np.ascontiguousarray(np.broadcast_to(v[:, None], (len(v), ncell))) for k, v in table.inputs.items()}
