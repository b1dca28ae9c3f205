"""BmiTopoflowGlacier -- the reference's BMI surface on the MI355X engine.

Drop-in for src/topoflow_glacier/bmi/bmi_topoflow_glacier.py: same class name,
variable names, units, order and float64 host arrays; same YAML loader
(config.py); same error types.  What changes is where ``update()`` runs: the
46 NumPy calls of :413-465 become one launch of the fused HIP kernel over all
cells of the grid (C ABI include/tfg.h via ctypes).

Modes
  * single catchment (the reference's case, ny = nx = 1): fp64 engine with the
    reference's operation order; inputs/outputs mirrored eagerly, so
    ``get_value_ptr`` references stay live exactly as in the reference.
    With ``defer_update: true`` update() queues the step instead, and every
    queued model of the process advances in one launch (tfg_update_many) at
    the first BMI call that reads or writes one of them, or at
    :func:`flush_updates`; a held ``get_value_ptr`` array shows the new values
    from then on.
  * grid (``ny``/``nx`` in the YAML): fp32 engine by default; BMI arrays have
    ny*nx float64 entries, refreshed from the device when read.

Additive fixes (the reference versions are broken):
``get_current_time``/``get_time_step``/``get_time_units``/``get_end_time``,
``update_until`` (fused multi-step launch), ``get_var_units``,
``get_value_at_indices``, the grid-description functions.
"""

from __future__ import annotations

from datetime import timedelta
from pathlib import Path

import numpy as np
import yaml

from .. import _native as nat
from ..engine import GlacierEngine, UpdateBatch
from ..physics.clock import parse_time
from ..physics.context import Context, build_context
from .bmi_base import BmiBase
from .config import TopoflowGlacierConfig
from .logger import configure_logging, logger

__all__ = ["BmiTopoflowGlacier", "flush_updates"]

# bmi_topoflow_glacier.py:18-37 (names, units, order)
_dynamic_input_vars = [
    ("land_surface_radiation~incoming~longwave__energy_flux", "W m-2"),
    ("land_surface_air__pressure", "Pa"),
    ("atmosphere_air_water~vapor__relative_saturation", "kg kg-1"),
    ("atmosphere_water__liquid_equivalent_precipitation_rate", "mm h-1"),
    ("land_surface_radiation~incoming~shortwave__energy_flux", "W m-2"),
    ("land_surface_air__temperature", "degC"),
    ("wind_speed_UV", "m sec-1"),
]
# Additive, settable static rasters (not in the reference's var lists, which
# stay unchanged): the YAML scalars elev / slope / aspect (config.py:19-28)
# per cell, for gridded runs.  Units and meaning as the reference uses them:
# slope is the tangent of the slope angle labelled m km-1 (:1095-1113), the
# aspect in "degrees" enters the radians formula (:1082-1093).
_static_vars = [
    ("land_surface__elevation", "m"),
    ("land_surface__slope", "m km-1"),
    ("land_surface__aspect_angle", "deg"),
]
_STATIC_FIELD = {"land_surface__elevation": "elev", "land_surface__slope": "slope",
                 "land_surface__aspect_angle": "aspect"}

_output_vars = [
    ("snowpack__depth", "m"),
    ("snowpack__liquid-equivalent_depth", "m"),
    ("snowpack__melt_volume_flux", "m s-1"),
    ("glacier_ice__thickness", "m"),
    ("glacier__liquid_equivalent_depth", "m"),
    ("glacier_ice__melt_volume_flux", "m s-1"),
    ("land_surface_water__runoff_volume_flux", "m s-1"),
    ("atmosphere_bottom_air_water-vapor__relative_saturation", "-"),
]
INTERNAL_NAME_CROSSWALK = {
    "land_surface_radiation~incoming~longwave__energy_flux": "LW_in",
    "land_surface_air__pressure": "P_air",
    "atmosphere_air_water~vapor__relative_saturation": "Hum_sp",
    "atmosphere_water__liquid_equivalent_precipitation_rate": "P",
    "land_surface_radiation~incoming~shortwave__energy_flux": "SW_in",
    "land_surface_air__temperature": "T_air",
    "wind_speed_UV": "uz",
    "snowpack__depth": "h_snow",
    "snowpack__liquid-equivalent_depth": "h_swe",
    "snowpack__melt_volume_flux": "SM",
    "glacier_ice__thickness": "h_ice",
    "glacier__liquid_equivalent_depth": "h_iwe",
    "glacier_ice__melt_volume_flux": "IM",
    "land_surface_water__runoff_volume_flux": "M_total",
    "atmosphere_bottom_air_water-vapor__relative_saturation": "RH",
}
EXTERNAL_NAME_CROSSWALK = {v: k for k, v in INTERNAL_NAME_CROSSWALK.items()}
_PHYSICS_INPUTS = ("P", "T_air", "Hum_sp", "P_air", "uz")  # LW_in / SW_in are never read (:1122, :1235)
_INPUT_BLOCK = ("P_air", "Hum_sp", "P", "T_air", "uz")  # tfg_set_inputs order
_EAGER_MAX_CELLS = 4096


def crosswalk_to_external(name: str) -> str:
    """Reference helper (:93-95); despite its name it maps BMI -> internal."""
    return INTERNAL_NAME_CROSSWALK[name]


def crosswalk_to_interal(name: str) -> str:
    """Reference helper, reference spelling (:98-100); maps internal -> BMI."""
    return EXTERNAL_NAME_CROSSWALK[name]


def _ext(internal: str) -> str:
    return EXTERNAL_NAME_CROSSWALK[internal]


def _int(external: str) -> str:
    return INTERNAL_NAME_CROSSWALK[external]


def first_containing(name: str, *states: Context) -> Context:
    """First context holding `name`, else KeyError (:1896-1901)."""
    for s in states:
        if name in s:
            return s
    raise KeyError(f"unknown name: {name!s}")


def _accessor(external: str, ctx: str):
    def getter(self):
        return self._mirror(external)

    def setter(self, value):
        self.set_value(external, value)

    return property(getter, setter, doc=f"BMI variable {external}")


_SHARED_STREAMS: dict = {}


def _shared_stream(device: int) -> int:
    """One HIP stream per device for every one-cell model of the process
    (tfg_shared_stream: owned by the engine library, no torch needed).
    NextGen steps thousands of catchment instances in turn; one stream instead
    of one per instance saves ~12 us per instance-step at 500 instances
    (tests/diagnostics/bmi_many_instances.py)."""
    if device not in _SHARED_STREAMS:
        import ctypes

        s = ctypes.c_void_p()
        nat.check(nat.lib().tfg_shared_stream(int(device), ctypes.byref(s)))
        _SHARED_STREAMS[device] = s.value
    return _SHARED_STREAMS[device]


# Queued update() steps of single-catchment models (config ``defer_update``),
# one batch per device and stream.
_BATCHES: dict = {}


def flush_updates() -> None:
    """Run every queued ``update()`` of the process (``defer_update`` models):
    one tfg_update_many launch per device and stream advances them all, with
    the results of as many tfg_update calls bit for bit.  Called by the first
    BMI call that reads or writes a queued model; callers may also call it."""
    if not _BATCHES:
        return
    batches = list(_BATCHES.values())
    _BATCHES.clear()
    err = None
    for b in batches:
        owners = b.owners
        for m in owners:
            m._queued = False
        try:
            b.run()
        except Exception as e:  # no step of this batch ran: its models stay at the previous step
            for m in owners:
                m._timestep -= 1
            err = err or e
    if err is not None:
        raise err


def make_engine(cfg, n_frames: int = 1, hist_depth: int = 1) -> GlacierEngine:
    """The device shard a config describes (fp64 engine for one cell, fp32 for grids)."""
    engine = cfg.engine or ("float64" if cfg.ny * cfg.nx == 1 else "float32")
    eng = GlacierEngine(cfg, cfg.ny, cfg.nx, engine=engine, device=cfg.device, n_frames=n_frames,
                        hist_depth=hist_depth, fuse_steps=cfg.fuse_steps)
    if cfg.ny * cfg.nx == 1:
        eng.set_stream(_shared_stream(eng.device))
    return eng


def configure_engine(eng: GlacierEngine, cfg) -> bool:
    """initialize()'s static and state setup (:274-411) on an engine: terrain
    from the YAML scalars, initial depths, cold contents, albedo, window.
    Returns True when the slope is out of range: the reference then logs,
    leaves beta unset, and its first update() fails (:1106-1111)."""
    eng.set_field("elev", np.float64(cfg.elev))
    beta_invalid = False
    try:
        eng.set_field("slope", np.float64(cfg.slope))
    except nat.NativeError as e:
        if e.code != nat.ERR_DOMAIN:
            raise
        logger.error("ERROR: In met_base.py, some slope angles are out of range.  Returning without setting beta.")
        beta_invalid = True
    eng.set_field("aspect", np.float64(cfg.aspect))
    for name, key in (("h_snow", "h0_snow"), ("h_ice", "h0_ice"), ("h_swe", "h0_swe"), ("h_iwe", "h0_iwe")):
        eng.set_field(name, np.float64(getattr(cfg, key)))
    eng.init_state()
    return beta_invalid


class BmiTopoflowGlacier(BmiBase):
    """BMI composition wrapper for TopoflowGlacier on MI355X."""

    def __init__(self) -> None:
        self._dynamic_inputs = build_context(_dynamic_input_vars)
        self._outputs = build_context(_output_vars)
        self._static = build_context(_static_vars)
        self._timestep: int = 0
        self._engine: GlacierEngine | None = None
        self._stale: set[str] = set()
        self._beta_invalid = False
        self._defer = False
        self._queued = False
        configure_logging()

    # reference properties (:124-272)
    P = _accessor("atmosphere_water__liquid_equivalent_precipitation_rate", "in")
    T_air = _accessor("land_surface_air__temperature", "in")
    LW_in = _accessor("land_surface_radiation~incoming~longwave__energy_flux", "in")
    SW_in = _accessor("land_surface_radiation~incoming~shortwave__energy_flux", "in")
    P_air = _accessor("land_surface_air__pressure", "in")
    Hum_sp = _accessor("atmosphere_air_water~vapor__relative_saturation", "in")
    uz = _accessor("wind_speed_UV", "in")
    SM = _accessor("snowpack__melt_volume_flux", "out")
    IM = _accessor("glacier_ice__melt_volume_flux", "out")
    h_swe = _accessor("snowpack__liquid-equivalent_depth", "out")
    h_iwe = _accessor("glacier__liquid_equivalent_depth", "out")
    h_snow = _accessor("snowpack__depth", "out")
    h_ice = _accessor("glacier_ice__thickness", "out")
    M_total = _accessor("land_surface_water__runoff_volume_flux", "out")
    RH = _accessor("atmosphere_bottom_air_water-vapor__relative_saturation", "out")

    # ------------------------------------------------------------------ setup
    def initialize(self, config_file: str | Path) -> None:
        """Read the YAML config and set up state (reference :274-411)."""
        with open(config_file) as f:
            config = yaml.safe_load(f)
        self.cfg = TopoflowGlacierConfig.model_validate(config)
        cfg = self.cfg
        self.hours_per_day = np.float64(24)
        self.seconds_per_Day = np.float64(24) * 3600
        self.sec_per_year = np.float64(3600) * 24 * 365
        self.mps_to_mmph = np.float64(3600000)
        self.mmph_to_mps = np.float64(1) / np.float64(3600000)
        self.dt = cfg.dt
        self.days_per_dt = self.dt / 86400
        self.C_to_K = 273.15
        self.K_to_C = -273.15
        self.twopi = np.float64(2) * np.pi
        self.one_seventh = np.float64(1) / 7
        self.da_km2 = cfg.da
        self.da_m2 = self.da_km2 * 1e6
        self.slopes = cfg.slope
        self.ws_density_ratio = np.float64(cfg.rho_H2O) / np.float64(cfg.rho_snow)
        self.wi_density_ratio = np.float64(cfg.rho_H2O) / np.float64(cfg.rho_ice)
        self.ny, self.nx = cfg.ny, cfg.nx
        n = self.ny * self.nx
        self.n_cells = n
        self._dynamic_inputs = build_context(_dynamic_input_vars, n)
        self._outputs = build_context(_output_vars, n)
        self._static = build_context(_static_vars, n)
        for name, key in (("land_surface__elevation", "elev"), ("land_surface__slope", "slope"),
                          ("land_surface__aspect_angle", "aspect")):
            self._static.set_value(name, np.float64(getattr(cfg, key)))
        self._eager = n <= _EAGER_MAX_CELLS
        # The five physics inputs and the eight outputs are rows of one block
        # each, in tfg_set_inputs / tfg_get_outputs order: the engine reads the
        # inputs and writes the outputs in one transfer, with no copies between
        # the blocks and the BMI variables (set_value copies into the rows,
        # get_value_ptr hands them out).
        self._in_block = np.zeros((5, n), dtype=np.float64)
        self._out_block = np.zeros((8, n), dtype=np.float64)
        for i, name in enumerate(_INPUT_BLOCK):
            self._dynamic_inputs.bind(_ext(name), self._in_block[i])
        for j, (name, _) in enumerate(_output_vars):
            self._outputs.bind(name, self._out_block[j])
        # name -> (host array, internal output name or None): the per-call lookup
        # of set_value / get_value (NextGen makes 15 of them per catchment-step)
        self._arrays = {v.name: (v.value, None) for c in (self._static, self._dynamic_inputs) for v in c}
        self._arrays.update({v.name: (v.value, _int(v.name)) for v in self._outputs})
        self._engine = make_engine(cfg)
        self._beta_invalid = configure_engine(self._engine, cfg)
        # the optional ground heat flux: Qg (:333) in W m-2, held in Qc
        self._q_ground = float(cfg.geothermal_heat_flux) / float(self.sec_per_year) if cfg.ground_heat_flux else 0.0
        if cfg.ground_heat_flux and not cfg.lateral_conduction:
            self._engine.set_field("Qc", np.float64(self._q_ground))
        for name, key in (("h_snow", "h0_snow"), ("h_ice", "h0_ice"), ("h_swe", "h0_swe"), ("h_iwe", "h0_iwe")):
            self._outputs.set_value(_ext(name), np.float64(getattr(cfg, key)))
        self._stale.clear()
        self._dirty_outputs: set[str] = set()
        self._timestep = 0
        self._flowed_at = 0
        self._conducted_at = -1
        start = parse_time(cfg.start_time)
        self.start_year, self.start_month, self.start_day, self.start_hour = start.year, start.month, start.day, start.hour
        end = parse_time(cfg.end_time)
        self.end_year, self.end_month, self.end_day, self.end_hour = end.year, end.month, end.day, end.hour
        self.start_time = start
        self._cal = (0, start, start.year, None, None, None)
        self._clock = self._engine.clock
        self._defer = bool(cfg.defer_update) and n == 1 and self._engine.engine == "float64"
        self._in_addr, self._out_addr = self._in_block.ctypes.data, self._out_block.ctypes.data
        self._queued = False

    # ----------------------------------------------------------------- update
    def _require(self) -> GlacierEngine:
        if self._engine is None:
            raise RuntimeError("initialize() has not been called")
        if self._beta_invalid:
            raise AttributeError("'BmiTopoflowGlacier' object has no attribute 'beta'")
        return self._engine

    def _push_inputs(self) -> None:
        self._engine.set_inputs(self._in_block, 0)  # one transfer for the five inputs (tfg_set_inputs)
        self._push_dirty_outputs()

    def _push_dirty_outputs(self) -> None:
        for name in sorted(self._dirty_outputs):
            self._engine.set_field(name, self._outputs.value(_ext(name)))
        self._dirty_outputs.clear()

    def _after_steps(self, nsteps: int) -> None:
        self._timestep += nsteps
        self._stale = {_int(n) for n, _ in _output_vars}
        if self._eager:
            self._refresh_all()

    # The reference's per-step clock attributes (update_julian_day :957-1004,
    # get_current_datetime :1866-1893), computed when read rather than every step.
    def _calendar(self) -> tuple:
        if self._cal[0] != self._timestep:
            k = self._timestep - 1
            jd, yr, gmt, tsn = self._clock.calendar(k, 1)
            self._cal = (self._timestep, self.start_time + timedelta(hours=self.dt * (k + 1)), int(yr[0]),
                         float(jd[0]), float(gmt[0]), float(tsn[0]))
        return self._cal

    start_datetime = property(lambda self: self._calendar()[1])
    year = property(lambda self: self._calendar()[2])
    julian_day = property(lambda self: self._calendar()[3])
    GMT_offset = property(lambda self: self._calendar()[4])
    TSN_offset = property(lambda self: self._calendar()[5])

    def _flow_if_due(self) -> None:
        """The optional ice-flow term (config ``ice_flow``): between step
        k*ice_flow_interval and the next one, move ice for that interval
        (dt hours / 8760 per year).  Off by default (the reference moves no ice)."""
        c = self.cfg
        if c.ice_flow and self._timestep > 0 and self._timestep % c.ice_flow_interval == 0 \
                and self._flowed_at != self._timestep:
            self._engine.ice_flow(c.ice_flow_interval * c.dt / 8760.0, c.dx, c.dy)
            self._flowed_at = self._timestep
            self._stale = {_int(n) for n, _ in _output_vars}

    def _conduct_if_due(self) -> None:
        """The optional lateral conduction term (config ``lateral_conduction``):
        at step k*conduction_interval (from step 0), evaluate Qc from the
        current state; the steps of that interval add it to Q_sum (:1314).
        Off by default (the reference's Qc = 0, :936-948)."""
        c = self.cfg
        if c.lateral_conduction and self._timestep % c.conduction_interval == 0 \
                and self._conducted_at != self._timestep:
            self._engine.conduction_update(c.k_snow, c.k_ice, c.dx, c.dy, q_ground=self._q_ground)
            self._conducted_at = self._timestep

    def _steps_to_boundary(self, k: int) -> int:
        """k, cut where the next optional split term (ice flow, conduction) is due."""
        c = self.cfg
        if c.ice_flow:
            k = min(k, c.ice_flow_interval - self._timestep % c.ice_flow_interval)
        if c.lateral_conduction:
            k = min(k, c.conduction_interval - self._timestep % c.conduction_interval)
        return k

    def update(self) -> None:
        """Advance one time step (reference :413-465) on the GPU.  Small
        models (eager mirrors) take one synchronous tfg_update call: inputs in,
        one step, all eight outputs back."""
        eng = self._require()
        if not self._eager:
            self._push_inputs()
            self._flow_if_due()
            self._conduct_if_due()
            eng.run(1)
            self._after_steps(1)
            return
        if self._queued:  # defer_update: this model's previous step first
            flush_updates()
        if self._dirty_outputs:
            self._push_dirty_outputs()
        self._flow_if_due()
        self._conduct_if_due()
        if self._defer:
            # queued: runs with every other queued model of the process in one
            # launch when one of them is next read or written (flush_updates)
            key = eng._stream_key()
            b = _BATCHES.get(key)
            if b is None:
                b = _BATCHES[key] = UpdateBatch()
            b.add_addresses(eng, self._in_addr, self._out_addr, self)
            self._queued = True
        else:
            eng.update_io(self._in_block, self._out_block)  # the outputs land in the BMI variables
        self._timestep += 1
        self._stale.clear()

    def update_until(self, time: float) -> None:
        """Advance to `time` [s] with one fused multi-step run (reference :471-490)."""
        if time <= self.get_current_time():
            logger.warning(f"no update performed: {time=} <= current_time={self.get_current_time()}")
            return None
        n_steps, remainder = divmod(time - self.get_current_time(), self.get_time_step())
        if remainder != 0:
            logger.warning(f"time is not multiple of time step size. updating until: {time - remainder=} ")
        n_steps = int(n_steps)
        if n_steps <= 0:
            return None
        eng = self._require()
        if self._queued:
            flush_updates()
        self._push_inputs()
        done = 0
        while done < n_steps:  # in chunks that end where a split term (ice flow, conduction) is due
            self._flow_if_due()
            self._conduct_if_due()
            k = self._steps_to_boundary(n_steps - done)
            eng.run(k)
            self._after_steps(k)
            done += k

    def finalize(self) -> None:
        """Release the device shard (reference :467-469)."""
        if self._queued:
            flush_updates()
        if self._engine is not None:
            for name in list(self._stale):
                self._refresh(name)
            self._engine.close()
            self._engine = None

    # ------------------------------------------------------------- mirrors
    def _refresh_all(self) -> None:
        """All eight outputs in one gather + copy (tfg_get_outputs)."""
        self._engine.get_outputs(out=self._out_block)  # the block's rows are the BMI variables
        self._stale.clear()

    def _refresh(self, internal: str) -> None:
        ext = _ext(internal)
        self._outputs.value(ext)[:] = self._engine.get_field(internal)
        self._stale.discard(internal)

    def _mirror(self, external: str) -> np.ndarray:
        if self._queued:
            flush_updates()
        hit = getattr(self, "_arrays", {}).get(external)
        if hit is not None:
            internal = hit[1]
            if internal is not None and self._engine is not None and internal in self._stale:
                self._refresh(internal)
            return hit[0]
        ctx = first_containing(external, self._outputs, self._dynamic_inputs, self._static)
        if ctx is self._outputs and self._engine is not None:
            internal = _int(external)
            if internal in self._stale:
                self._refresh(internal)
        return ctx.value(external)

    # ------------------------------------------------------------ BMI vars
    def get_component_name(self) -> str:
        return "Topoflow-Glacier"

    def get_input_item_count(self) -> int:
        return len(self._dynamic_inputs)

    def get_output_item_count(self) -> int:
        return len(self._outputs)

    def get_input_var_names(self) -> tuple[str, ...]:
        return tuple(self._dynamic_inputs.names())

    def get_output_var_names(self) -> tuple[str, ...]:
        return tuple(self._outputs.names())

    def _set_static(self, name: str) -> None:
        """Push a static raster to the engine (additive _static_vars).  A slope
        out of range is logged and makes update() fail, as at initialize()
        (reference :1106-1111)."""
        try:
            self._engine.set_field(_STATIC_FIELD[name], self._static.value(name))
            if name == "land_surface__slope":
                self._beta_invalid = False
        except nat.NativeError as e:
            if e.code != nat.ERR_DOMAIN:
                raise
            logger.error("ERROR: In met_base.py, some slope angles are out of range.  Returning without setting beta.")
            self._beta_invalid = True

    def set_value(self, name: str, src) -> None:
        if self._queued:  # the queued step reads this model's input block
            flush_updates()
        if name in _STATIC_FIELD:
            self._static.set_value(name, src)
            self._set_static(name)
            return
        hit = getattr(self, "_arrays", {}).get(name)
        if hit is None:  # before initialize(), or an unknown name (KeyError)
            ctx = first_containing(name, self._outputs, self._dynamic_inputs, self._static)
            ctx.set_value(name, src)
            hit = (None, _int(name) if ctx is self._outputs else None)
        else:
            arr = hit[0]
            if arr.size == 1 and isinstance(src, (float, np.floating)):
                arr[0] = src  # one catchment, a scalar (NextGen's per-step pattern): 0.1 instead of 0.5 us
            else:
                arr[:] = src
        internal = hit[1]
        if internal is not None:
            self._stale.discard(internal)
            self._dirty_outputs.add(internal)

    def set_value_at_indices(self, name: str, inds, src) -> None:
        if self._queued:
            flush_updates()
        if name in _STATIC_FIELD:
            self._static.set_value_at_indices(name, np.asarray(inds), np.asarray(src))
            self._set_static(name)
            return
        self._mirror(name)  # refresh first so the untouched entries stay current
        ctx = first_containing(name, self._outputs, self._dynamic_inputs, self._static)
        ctx.set_value_at_indices(name, np.asarray(inds), np.asarray(src))
        if ctx is self._outputs:
            self._dirty_outputs.add(_int(name))

    def get_value(self, name: str, dest):
        """Copy of a variable, flattened into `dest` (reference :1810-1824)."""
        value = self.get_value_ptr(name)
        try:
            if value.size == 1 and isinstance(dest, np.ndarray) and dest.size == 1:
                dest[0] = value[0]  # one catchment: no flattened view to build
            else:
                dest[:] = value.reshape(-1)
        except Exception as e:
            raise RuntimeError(f"Could not return value {name} as flattened array") from e
        return dest

    def get_value_ptr(self, name: str):
        return self._mirror(name)

    def get_value_at_indices(self, name: str, dest, inds):
        self._mirror(name)
        return first_containing(name, self._outputs, self._dynamic_inputs, self._static).value_at_indices(name, dest, np.asarray(inds))

    def get_var_itemsize(self, name: str) -> int:
        return self.get_value_ptr(name).itemsize

    def get_var_nbytes(self, name: str) -> int:
        return self.get_value_ptr(name).nbytes

    def get_var_type(self, name: str) -> str:
        return str(self.get_value_ptr(name).dtype)

    def get_var_units(self, name: str) -> str:
        return first_containing(name, self._outputs, self._dynamic_inputs, self._static).unit(name)

    def get_var_grid(self, name: str) -> int:
        first_containing(name, self._outputs, self._dynamic_inputs, self._static)
        return 0

    def get_var_location(self, name: str) -> str:
        first_containing(name, self._outputs, self._dynamic_inputs, self._static)
        return "node"

    # ------------------------------------------------------------------ grid
    def get_grid_rank(self, grid: int) -> int:
        return 2

    def get_grid_size(self, grid: int) -> int:
        return int(getattr(self, "n_cells", 1))

    def get_grid_shape(self, grid: int, shape):
        shape[:] = (self.ny, self.nx)
        return shape

    def get_grid_spacing(self, grid: int, spacing):
        # (dy, dx) [m] in shape order, dy NEGATIVE: row 0 is the northern edge,
        # so y falls by |dy| per row from the origin (get_grid_origin, the
        # north-west node), and origin + index * spacing gives every node's
        # coordinates, as get_grid_x / get_grid_y report them.  |dx|, |dy|: the
        # configured spacing of the lateral terms when given, otherwise square
        # cells of area `da` [km2].  (Additive: the reference leaves the grid
        # functions unimplemented.)
        dx, dy = self._cell_size()
        spacing[:] = (-dy, dx)
        return spacing

    def _cell_size(self) -> tuple[float, float]:
        dx, dy = getattr(self.cfg, "dx", None), getattr(self.cfg, "dy", None)
        if dx is not None and dy is not None:
            return float(dx), float(dy)
        d = float(np.sqrt(self.cfg.da) * 1000.0)
        return d, d

    def get_grid_origin(self, grid: int, origin):
        # (y, x) of node 0 (row 0, column 0): the north-west corner node
        origin[:] = ((self.ny - 1) * self._cell_size()[1], 0.0)
        return origin

    def get_grid_type(self, grid: int) -> str:
        return "uniform_rectilinear"

    # Node coordinates and quad topology of the uniform raster (BMI 2.0), for
    # callers that walk every grid the same way.  The reference leaves these
    # unimplemented (bmi_base.py); they are additive.  Nodes are numbered row
    # by row (index = row * nx + col, the layout of every value array), and
    # row 0 is the NORTHERN edge, as in the engine: tfg_terrain_from_dem and
    # the conduction and ice-flow halos pair halo_north with row 0.  So y
    # decreases with the row index: row k sits at y = (ny - 1 - k) * |dy|
    # above the south-west node, i.e. at origin + k * spacing with the origin
    # the north-west node and a negative dy (get_grid_origin, get_grid_spacing).  Edges
    # are the nx - 1 x-edges of each row, then the nx y-edges of each row
    # pair; faces are the cells between four nodes, counter-clockwise in
    # (x, y) from the lower-left node, with edges in the same order.
    def _axis(self, k: int) -> np.ndarray:
        sp = self.get_grid_spacing(0, np.empty(2))
        o = self.get_grid_origin(0, np.empty(2))
        return o[k] + np.arange((self.ny, self.nx)[k], dtype=np.float64) * sp[k]

    def get_grid_x(self, grid: int, x):
        x[:] = self._axis(1)
        return x

    def get_grid_y(self, grid: int, y):
        y[:] = self._axis(0)
        return y

    def get_grid_z(self, grid: int, z):
        raise NotImplementedError("the grid is two-dimensional")

    def get_grid_node_count(self, grid: int) -> int:
        return self.get_grid_size(grid)

    def get_grid_edge_count(self, grid: int) -> int:
        return self.ny * (self.nx - 1) + (self.ny - 1) * self.nx

    def get_grid_face_count(self, grid: int) -> int:
        return (self.ny - 1) * (self.nx - 1)

    def get_grid_edge_nodes(self, grid: int, edge_nodes):
        ny, nx = self.ny, self.nx
        node = np.arange(ny * nx).reshape(ny, nx)
        ex = np.stack([node[:, :-1], node[:, 1:]], axis=-1).reshape(-1, 2)
        ey = np.stack([node[:-1, :], node[1:, :]], axis=-1).reshape(-1, 2)
        edge_nodes[:] = np.concatenate([ex, ey]).ravel()
        return edge_nodes

    def get_grid_face_nodes(self, grid: int, face_nodes):
        node = np.arange(self.ny * self.nx).reshape(self.ny, self.nx)
        # lower-left (row k + 1), lower-right, upper-right (row k), upper-left
        f = np.stack([node[1:, :-1], node[1:, 1:], node[:-1, 1:], node[:-1, :-1]], axis=-1)
        face_nodes[:] = f.ravel()
        return face_nodes

    def get_grid_face_edges(self, grid: int, face_edges):
        ny, nx = self.ny, self.nx
        n_ex = ny * (nx - 1)
        ex = np.arange(n_ex).reshape(ny, nx - 1)
        ey = n_ex + np.arange((ny - 1) * nx).reshape(ny - 1, nx)
        # bottom (row k + 1), right, top (row k), left: edge j joins face nodes j and j + 1
        f = np.stack([ex[1:, :], ey[:, 1:], ex[:-1, :], ey[:, :-1]], axis=-1)
        face_edges[:] = f.ravel()
        return face_edges

    def get_grid_nodes_per_face(self, grid: int, nodes_per_face):
        nodes_per_face[:] = 4
        return nodes_per_face

    # ------------------------------------------------------------------ time
    def get_start_time(self) -> float:
        return 0.0

    def get_time_step(self) -> float:
        return float(self.dt) * 3600.0

    def get_time_units(self) -> str:
        return "s"

    def get_current_time(self) -> float:
        return self._timestep * self.get_time_step()

    def get_end_time(self) -> float:
        return (parse_time(self.cfg.end_time) - parse_time(self.cfg.start_time)).total_seconds()

    # ------------------------------------------------- diagnostics / state
    def _settled(self) -> GlacierEngine:
        if self._queued:
            flush_updates()
        return self._engine

    def _diag(self, i: int) -> np.ndarray:
        self._settled()
        return np.array([self._engine.diagnostics()[:, i].sum() if i < 5 else self._engine.diagnostics()[:, i].max()])

    vol_P = property(lambda self: self._diag(0), doc="sum(P*da*dt) (:558-568)")
    vol_PR = property(lambda self: self._diag(1), doc="sum(P_rain*da*dt) (:606-614)")
    vol_PS = property(lambda self: self._diag(2), doc="sum(P_snow*da*dt) (:616-624)")
    vol_SM = property(lambda self: self._diag(3), doc="sum(SM*da*dt*3600) (:1482-1487)")
    vol_IM = property(lambda self: self._diag(4), doc="sum(IM*da*dt*3600) (:1489-1494)")
    P_max = property(lambda self: self._diag(5), doc="max P (:570-576)")
    Eccs = property(lambda self: self._settled().get_field("Eccs"), doc="snowpack cold content [J m-2]")
    Ecci = property(lambda self: self._settled().get_field("Ecci"), doc="ice cold content [J m-2]")
    albedo = property(lambda self: self._settled().get_field("albedo"), doc="surface albedo")
    n = property(lambda self: self._settled().get_field("n"), doc="days since last major snowfall")
