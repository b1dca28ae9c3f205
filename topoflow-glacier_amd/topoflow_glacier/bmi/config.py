"""YAML configuration schema (drop-in for config.py:6-115 of the reference).

Every key the reference accepts is accepted here with the same default and the
same validation, so reference YAML files (config/*.yaml) load unchanged.  Two
deliberate, additive differences:

* ``dt`` also accepts a float (the reference types it ``int`` hours,
  config.py:15, which rules out the 15-minute step of BASELINE config 5);
  integer values keep their int type, so arithmetic is unchanged.
* ``start_time`` / ``end_time`` written as bare YAML integers
  (config/cat-3062784.yaml, cat-3062924.yaml, cat-3062927.yaml) are accepted
  as their digit strings; the reference's loader rejects those files.
* grid / engine keys the reference does not have (all optional):
  ``ny``, ``nx`` (grid shape, default 1 x 1 = the reference's single
  catchment), ``engine`` ("float64" | "float32"; default float64 for one cell,
  float32 for grids), ``device`` (HIP device ordinal, default LOCAL_RANK or 0),
  ``time_zone`` (IANA name; default looked up from lat/lon),
  ``fuse_steps`` (time steps fused per kernel launch, default 24),
  ``flux_precision`` ("fp32" | "fp64": the float32 engine's energy-flux
  arithmetic; "fp64" computes the dew point, turbulent fluxes and long-wave
  balance in fp64 so the cold content carries no fp32 rounding into melt
  onset, at a measured throughput cost; default "fp32"),
  ``ice_flow`` / ``ice_flow_interval`` / ``dx`` / ``dy`` (the optional
  shallow-ice flow term, off by default; it moves ice between cells every
  ``ice_flow_interval`` steps on a grid of dx x dy metre cells) and
  ``lateral_conduction`` / ``conduction_interval`` / ``k_snow`` / ``k_ice``
  (the optional lateral heat-conduction term, re-evaluated every
  ``conduction_interval`` steps) and ``ground_heat_flux`` (adds the declared
  ``geothermal_heat_flux`` to every cell's conduction flux), and
  ``defer_update`` (single catchment: ``update()`` queues the step, and the
  steps of every waiting model of the process run in one launch at the first
  call that reads or writes one of them; off by default).

Unknown keys are ignored, as in the reference (pydantic default).
"""

from __future__ import annotations

from typing import Literal

from pydantic import BaseModel, ConfigDict, Field, field_validator, model_validator

__all__ = ["TopoflowGlacierConfig"]


class TopoflowGlacierConfig(BaseModel):
    """Validated model configuration."""

    model_config = ConfigDict(arbitrary_types_allowed=True)

    # --- required (config.py:13-27) ---------------------------------------
    site_prefix: str
    forcing_file: str
    dt: int | float = Field(ge=0, description="time step [hours]")
    start_time: str
    end_time: str
    da: float = Field(description="area [km2] (per cell for grids)")
    slope: float
    lat: float
    lon: float
    h0_snow: float
    h0_ice: float
    h0_swe: float
    h0_iwe: float
    elev: float
    # --- defaulted parameters (config.py:28-33) ----------------------------
    T_rain_snow: float = 1.0
    aspect: float = 0.0
    dust_atten: float = Field(0.08, ge=0.0, le=0.2)
    canopy_factor: float = Field(0.0, ge=0.0, le=1.0)
    cloud_factor: float = Field(0.0, ge=0.0, le=1.0)
    # --- physical constants (config.py:38-62) ------------------------------
    rho_air: float = 1.2614
    rho_snow: float = 50.0
    rho_ice: float = 917.0
    rho_H2O: float = 1000.0
    h_active_layer: float = 0.125
    T0: float = -0.2
    Cp_air: float = 1005.7
    Cp_ice: float = 2060.0
    Cp_snow: float = 2090.0
    g: float = 9.81
    Lf: float = 334000.0
    eps: float = 0.622
    kappa: float = 0.408
    latent_heat_constant: float = 0.622
    Lv: float = 2500000
    sigma: float = 5.67 * 10 ** (-8)
    sea_level_p0: float = 101325.0
    sea_level_T0: float = 288.15
    T_lapse_rate: float = 0.0065
    uni_gas_const: float = 8.3144598
    M_mass_air: float = 0.0289644
    # --- glacier-dynamics fields (config.py:64-85): accepted, unused --------
    min_glacier_thick: float = 1.0
    glens_A: float = 2.142e-16
    B: float = 0.0012
    char_sliding_vel: float = 10.0
    char_tau_bed: float = 100000.0
    depth_to_water_table: float = 20.0
    max_float_fraction: float = 80.0
    Hp_eff: float = 20.0
    init_ELA: float = 3350.0
    ELA_step_size: float = -10.0
    ELA_step_interval: float = 500.0
    grad_Bz: float = 0.01
    max_Bz: float = 2.0
    spinup_time: float = 200.0
    sea_level: float = -100.0
    z0_air: float = Field(0.01, ge=0.0001, le=0.1)
    em_surf: float = Field(0.985, ge=0.9, le=1)
    geothermal_heat_flux: float = 1575000.0
    geothermal_gradient: float = -0.0255
    # --- legacy toggles (config.py:94-101) ---------------------------------
    PRECIP_ONLY: bool = False
    P_factor: float = 1.0
    SATTERLUND: bool = False

    # --- additive keys of this build ---------------------------------------
    ny: int = Field(1, ge=1)
    nx: int = Field(1, ge=1)
    engine: Literal["float64", "float32"] | None = None
    device: int | None = None
    time_zone: str | None = None
    fuse_steps: int = Field(24, ge=1)
    flux_precision: Literal["fp32", "fp64"] = "fp32"  # the float32 engine's flux arithmetic (tfg_set_flux)
    # optional lateral ice flow (extension; tfg_ice_flow_*): off by default,
    # which keeps results identical to the reference
    ice_flow: bool = False
    ice_flow_interval: int = Field(24, ge=1)  # time steps between flow updates
    dx: float | None = Field(None, gt=0)      # grid spacing [m], west-east
    dy: float | None = Field(None, gt=0)      # grid spacing [m], north-south
    # optional lateral heat conduction (extension; tfg_conduction_*): the
    # reference's Qc (:936-948, :1314) from Fourier's law between neighbouring
    # cells, re-evaluated every conduction_interval steps; off by default
    lateral_conduction: bool = False
    conduction_interval: int = Field(24, ge=1)  # time steps between Qc updates
    k_snow: float = Field(0.1, ge=0)  # snow conductivity [W m-1 K-1] (Sturm et al. 1997 at rho_snow = 50 kg m-3)
    k_ice: float = Field(2.1, ge=0)   # ice conductivity [W m-1 K-1] near 0 degC
    # optional ground heat flux: the declared but unused geothermal flux Qg
    # (geothermal_heat_flux [J yr-1 m-2], reference :333) added to every cell's Qc
    ground_heat_flux: bool = False
    # single-catchment models: update() queues the step; all queued models of
    # the process advance together in one launch (tfg_update_many) when one of
    # them is next read or written.  Off by default: update() then returns with
    # the outputs in place, as the reference's does.
    defer_update: bool = False

    @model_validator(mode="after")
    def _flow_needs_spacing(self):
        if self.ice_flow and (self.dx is None or self.dy is None):
            raise ValueError("ice_flow needs the grid spacing dx and dy [m]")
        return self

    @model_validator(mode="after")
    def _conduction_needs_spacing_and_a_stable_interval(self):
        if not self.lateral_conduction:
            return self
        if self.dx is None or self.dy is None:
            raise ValueError("lateral_conduction needs the grid spacing dx and dy [m]")
        # Qc is held over the interval (explicit, operator-split): a cell's pack
        # must not overshoot its neighbours, dt <= d^2/8 * rho Cp / k per layer
        d2 = min(self.dx, self.dy) ** 2
        limits = [d2 / 8.0 * rc / k for rc, k in ((self.rho_snow * self.Cp_snow, self.k_snow),
                                                   (self.rho_ice * self.Cp_ice, self.k_ice)) if k > 0]
        span = self.conduction_interval * float(self.dt) * 3600.0
        if limits and span > min(limits):
            raise ValueError(f"conduction_interval spans {span:.0f} s, above the stable {min(limits):.0f} s "
                             "for this grid spacing; shorten the interval")
        return self

    @field_validator("start_time", "end_time", mode="before")
    @classmethod
    def _digits_as_text(cls, v):
        return str(v) if isinstance(v, int) and not isinstance(v, bool) else v
