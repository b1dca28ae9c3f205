"""GlacierEngine: one grid shard of the HIP energy-balance engine.

Thin Python owner of a ``tfg_handle`` (include/tfg.h).  It converts a
validated configuration into ``tfg_params``, moves rasters in and out, and
advances the model with :meth:`run`, which hands a block of per-step uniforms
(:class:`~topoflow_glacier.physics.clock.StepClock`) to ``tfg_step``; the
library fuses up to ``fuse_steps`` steps per kernel launch.

All arithmetic happens in the HIP kernels; this class never computes physics.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _native as nat
from .physics.clock import StepClock

__all__ = ["GlacierEngine", "UpdateBatch", "params_from_config", "update_many"]

_ENGINES = {"float32": nat.F32, "float64": nat.F64}
_NP = {nat.F32: np.float32, nat.F64: np.float64}
_SPLIT = {"auto": 0, "off": 1, "on": 2}  # include/tfg.h TFG_SPLIT_*


def params_from_config(cfg) -> nat.TfgParams:
    """tfg_params from a TopoflowGlacierConfig (or any object with its fields)."""
    p = nat.TfgParams()
    for name, _ in nat.TfgParams._fields_:
        if name in ("da_m2", "sin_lat", "cos_lat", "satterlund", "ring_len"):
            continue
        setattr(p, name, float(getattr(cfg, name)))
    p.da_m2 = float(cfg.da) * 1e6  # :293-294
    lat_rad = cfg.lat * (np.pi / np.float64(180))  # as Equivalent_Latitude computes it
    p.sin_lat = float(np.sin(lat_rad))
    p.cos_lat = float(np.cos(lat_rad))
    p.satterlund = int(bool(cfg.SATTERLUND))
    p.ring_len = int(3 * np.float64(24) / cfg.dt)  # :296
    return p


class GlacierEngine:
    """A ny x nx shard resident on one GPU."""

    def __init__(self, cfg, ny: int, nx: int, engine: str = "float32", device: int | None = None,
                 n_frames: int = 1, hist_depth: int = 1, n_catch: int = 1, fuse_steps: int | None = None,
                 row0: int = 0, flux: str | None = None, split: str = "auto"):
        self.lib = nat.load()
        self.cfg = cfg
        self.ny, self.nx, self.n = int(ny), int(nx), int(ny) * int(nx)
        self.row0 = int(row0)
        self.engine = engine
        self.dtype_code = _ENGINES[engine]
        self.np_dtype = _NP[self.dtype_code]
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", 0))
        self.device = int(device)
        self.n_frames, self.hist_depth, self.n_catch = int(n_frames), int(hist_depth), int(n_catch)
        self.params = params_from_config(cfg)
        self.ring_len = int(self.params.ring_len)
        h = ctypes.c_void_p()
        nat.check(self.lib.tfg_create(ctypes.byref(self.params), self.ny, self.nx, self.dtype_code, self.device,
                                      self.n_frames, self.hist_depth, self.n_catch, ctypes.byref(h)))
        self.h = h
        self.fuse_steps = int(fuse_steps or getattr(cfg, "fuse_steps", 24) or 24)
        nat.check(self.lib.tfg_set_fuse(self.h, self.fuse_steps), self.h)
        # the float32 engine's flux arithmetic (tfg_set_flux): the argument, else the config's flux_precision
        self.flux = flux or getattr(cfg, "flux_precision", None) or "fp32"
        if self.flux not in ("fp32", "fp64"):
            raise ValueError(f"flux must be 'fp32' or 'fp64', not {self.flux!r}")
        nat.check(self.lib.tfg_set_flux(self.h, 1 if self.flux == "fp64" else 0), self.h)
        # two-part launches of a small fp32 grid on two streams (tfg_set_split): "auto", "off" or "on"
        if split not in _SPLIT:
            raise ValueError(f"split must be one of {sorted(_SPLIT)}, not {split!r}")
        if hasattr(self.lib, "tfg_set_split"):
            nat.check(self.lib.tfg_set_split(self.h, _SPLIT[split]), self.h)
        self.clock = StepClock(cfg.start_time, cfg.dt, cfg.lat, cfg.lon, getattr(cfg, "time_zone", None),
                               ring_len=self.ring_len)
        self.step_index = 0  # model steps completed

    # -- lifetime -------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.tfg_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int) -> None:
        nat.check(rc, self.h)

    # -- fields -----------------------------------------------------------------
    def set_field(self, name: str, values, index: int = 0) -> None:
        """Copy a host array (broadcast to n cells) or a torch CUDA tensor into a field."""
        fid = nat.FIELD[name]
        if hasattr(values, "data_ptr") and getattr(values, "is_cuda", False):
            import torch

            t = values.contiguous()
            code = {4: nat.F32, 8: nat.F64}[t.element_size()] if name != "catch_id" else nat.I32
            if t.numel() != self.n:
                raise ValueError(f"{name}: {t.numel()} values for {self.n} cells")
            # the engine copies on its own stream: wait for torch's producer
            # first, and for the copy before `t` (maybe a temporary) is freed
            torch.cuda.current_stream(t.device).synchronize()
            self._chk(self.lib.tfg_set_field(self.h, fid, index, ctypes.c_void_p(t.data_ptr()), code, self.n, 1))
            self.sync()
            return
        if name == "catch_id":
            a = np.ascontiguousarray(np.broadcast_to(np.asarray(values, dtype=np.int32), (self.n,)))
            code = nat.I32
        else:
            a = np.asarray(values)
            a = np.ascontiguousarray(np.broadcast_to(a.astype(np.float32 if a.dtype == np.float32 else np.float64), (self.n,)))
            code = nat.F32 if a.dtype == np.float32 else nat.F64
        self._chk(self.lib.tfg_set_field(self.h, fid, index, a.ctypes.data_as(ctypes.c_void_p), code, self.n, 0))

    def get_field(self, name: str, index: int | None = None, dtype=np.float64, cells: int | None = None) -> np.ndarray:
        """Host copy of a field (its first `cells` cells: a leading block of
        rows; default all).  Outputs default to the newest history slot."""
        fid = nat.FIELD[name]
        n = self.n if cells is None else int(cells)
        if index is None:
            index = self.last_hist if name in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH") else 0
        if name == "catch_id":
            out = np.empty(n, dtype=np.int32)
            code = nat.I32
        else:
            out = np.empty(n, dtype=dtype)
            code = nat.F32 if out.dtype == np.float32 else nat.F64
        self._chk(self.lib.tfg_get_field(self.h, fid, index, out.ctypes.data_as(ctypes.c_void_p), code, n, 0))
        return out

    def get_field_device(self, name: str, out, index: int | None = None):
        """Copy a field into the torch CUDA tensor `out` (n elements; float32,
        float64, or int32 for catch_id).  tfg_get_field with a device pointer
        is asynchronous on the engine's stream, so this waits for the copy
        before torch's stream may read `out`."""
        import torch

        fid = nat.FIELD[name]
        if index is None:
            index = self.last_hist if name in ("h_snow", "SM", "h_ice", "IM", "M_total", "RH") else 0
        if not (out.is_cuda and out.is_contiguous() and out.numel() == self.n):
            raise ValueError(f"{name}: need a contiguous CUDA tensor of {self.n} elements")
        code = {torch.float32: nat.F32, torch.float64: nat.F64, torch.int32: nat.I32}[out.dtype]
        torch.cuda.current_stream(out.device).synchronize()  # `out` may still be in use on torch's stream
        self._chk(self.lib.tfg_get_field(self.h, fid, index, ctypes.c_void_p(out.data_ptr()), code, self.n, 1))
        self.sync()
        return out

    # -- checkpoint / restart ----------------------------------------------------
    _CKPT_STATE = ("h_swe", "h_iwe", "Eccs", "Ecci", "albedo", "n")

    def checkpoint(self, path) -> None:
        """Save what the next step reads, so a restored engine continues bit for
        bit: the fp64 state, the fp64 previous-step depths (TFG_PREV_DEPTH), the
        snowfall window and the step counter (the model clock).  The
        mass-balance integrals are not saved; they restart from zero."""
        st = {k: self.get_field(k) for k in self._CKPT_STATE}
        for k in ("h_snow", "h_ice"):
            st[k] = self.get_field(k, index=nat.PREV_DEPTH)
        st["window"] = np.stack([self.get_field("window", index=j) for j in range(self.ring_len)])
        np.savez(path, step_index=self.step_index, ny=self.ny, nx=self.nx, **st)

    def restore(self, path) -> None:
        """Continue from a checkpoint() of a shard of the same shape.  The
        static rasters and forcing frames are the caller's, as at the start
        of a run; call init_state() (or fill_synthetic) first."""
        z = np.load(path, allow_pickle=False)
        if (int(z["ny"]), int(z["nx"])) != (self.ny, self.nx) or z["window"].shape[0] != self.ring_len:
            raise ValueError("checkpoint of a different grid shape or snowfall-window length")
        for k in self._CKPT_STATE:
            self.set_field(k, z[k])
        for k in ("h_snow", "h_ice"):
            self.set_field(k, z[k], index=nat.PREV_DEPTH)
        for j in range(self.ring_len):
            self.set_field("window", z["window"][j], index=j)
        self.step_index = int(z["step_index"])

    def set_inputs(self, values, index: int = 0) -> None:
        """The five physics inputs of one frame in one call: values [5][n] in
        BMI order P_air, Hum_sp, P, T_air, uz (tfg_set_inputs): a host array,
        or a contiguous float32 / float64 torch CUDA tensor on the engine's
        device, which the engine reads asynchronously on its own stream
        (ordered after torch's current stream when the two differ).  The read
        is recorded on the engine's stream (Tensor.record_stream), so torch's
        caching allocator does not hand the memory out again before the engine
        has read it, even if the caller drops the tensor at once."""
        if getattr(values, "is_cuda", False):
            import torch

            if values.device.index != self.device:
                raise ValueError(f"inputs on {values.device}, the engine runs on cuda:{self.device}")
            if tuple(values.shape) != (5, self.n) or not values.is_contiguous():
                raise ValueError(f"inputs must be a contiguous [5][{self.n}] tensor")
            code = {torch.float32: nat.F32, torch.float64: nat.F64}[values.dtype]
            own = getattr(self, "_stream_ptr", None)
            cur = torch.cuda.current_stream(values.device)
            if own is None or own != cur.cuda_stream:
                cur.synchronize()
            self._chk(self.lib.tfg_set_inputs(self.h, int(index), ctypes.c_void_p(values.data_ptr()), code, self.n, 1))
            ptr = own or self.stream()
            if getattr(self, "_ext_stream", (None, None))[0] != ptr:
                self._ext_stream = (ptr, torch.cuda.ExternalStream(ptr, device=values.device))
            values.record_stream(self._ext_stream[1])
            return
        a = np.ascontiguousarray(values, dtype=np.float64)
        if a.shape != (5, self.n):
            raise ValueError(f"inputs must be [5][{self.n}]")
        self._chk(self.lib.tfg_set_inputs(self.h, int(index), a.ctypes.data_as(ctypes.c_void_p), nat.F64, self.n, 0))

    def get_outputs(self, index: int | None = None, out: np.ndarray | None = None) -> np.ndarray:
        """The eight BMI outputs [8][n] (h_snow, h_swe, SM, h_ice, h_iwe, IM,
        M_total, RH) of history slot `index` (default: the newest) in one call."""
        if out is None:
            out = np.empty((8, self.n), dtype=np.float64)
        idx = self.last_hist if index is None else int(index)
        self._chk(self.lib.tfg_get_outputs(self.h, idx, out.ctypes.data_as(ctypes.c_void_p), nat.F64, self.n, 0))
        return out

    @property
    def last_hist(self) -> int:
        return (self.step_index - 1) % self.hist_depth if self.step_index > 0 else 0

    def init_state(self) -> None:
        """initialize()-time state from the depth rasters (reference :389-395)."""
        self._chk(self.lib.tfg_init_state(self.h))
        self.step_index = 0

    def fill_synthetic(self, seed: int, diurnal: np.ndarray, nx_global: int | None = None) -> None:
        d = np.ascontiguousarray(diurnal, dtype=np.float32)
        self._chk(self.lib.tfg_fill_synthetic(self.h, int(seed), self.row0, int(nx_global or self.nx),
                                              d.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), self.n_frames))
        self.step_index = 0

    # -- time stepping ------------------------------------------------------------
    _UBLOCK = 512  # steps of uniforms computed at once for short runs

    def uniforms(self, nsteps: int, frames=None) -> np.ndarray:
        k0 = self.step_index
        default_frames = frames is None
        hist = (np.arange(k0, k0 + nsteps) % self.hist_depth).astype(np.int32)
        if frames is None:
            frames = (np.arange(k0, k0 + nsteps) % self.n_frames).astype(np.int32)
        b0 = k0 - k0 % self._UBLOCK
        if nsteps <= self._UBLOCK and k0 + nsteps <= b0 + self._UBLOCK:
            # per-step callers (BMI update()): serve from a block computed once
            cache = getattr(self, "_ucache", None)
            if cache is None or cache[0] != b0:
                cache = (b0, self.clock.uniform_block(b0, self._UBLOCK))
                self._ucache = cache
            u = cache[1][k0 - b0:k0 - b0 + nsteps]
            if default_frames and self.n_frames == 1 and self.hist_depth == 1:
                return u  # frame and slot 0: the cached records as they are (tfg_step copies them)
            u = u.copy()
            u["frame"], u["hist"] = frames, hist
            return u
        return self.clock.uniforms(k0, nsteps, frames=frames, hist=hist)

    def run(self, nsteps: int = 1, uniforms: np.ndarray | None = None, frames=None) -> None:
        """Advance nsteps model steps (update() / update_until(), :413-490).
        Asynchronous: returns once the launches are queued."""
        if nsteps <= 0:
            return
        u = self.uniforms(nsteps, frames) if uniforms is None else uniforms
        u = np.ascontiguousarray(u, dtype=nat.UNIFORM_DTYPE)
        if len(u) != nsteps:
            raise ValueError("one uniform record per step")
        self._chk(self.lib.tfg_step(self.h, u.ctypes.data_as(ctypes.c_void_p), nsteps))
        self.step_index += nsteps

    def update_io(self, values: np.ndarray, out: np.ndarray) -> np.ndarray:
        """One synchronous step fed from the host (tfg_update): inputs
        values[5][n] (P_air, Hum_sp, P, T_air, uz), outputs out[8][n] (h_snow,
        h_swe, SM, h_ice, h_iwe, IM, M_total, RH); both C-contiguous float64.
        This is BMI update()'s per-step path (:413-465)."""
        if values.shape != (5, self.n) or out.shape != (8, self.n) or values.dtype != np.float64 \
                or out.dtype != np.float64 or not (values.flags.c_contiguous and out.flags.c_contiguous):
            raise ValueError(f"update_io needs C-contiguous float64 [5][{self.n}] and [8][{self.n}]")
        frame, uptr, keep = self._next_uniform()
        self._chk(self.lib.tfg_update(self.h, frame, values.ctypes.data, nat.F64, uptr, out.ctypes.data, nat.F64, self.n))
        self.step_index += 1
        return out

    def _next_uniform(self):
        """(frame, address of the next step's uniform record, owner of that record)."""
        k0 = self.step_index
        frame = k0 % self.n_frames
        if self.n_frames == 1 and self.hist_depth == 1:
            # the cached block's records have frame = hist = 0: pass one by address
            b0 = k0 - k0 % self._UBLOCK
            cache = getattr(self, "_ucache", None)
            if cache is None or cache[0] != b0:
                cache = (b0, self.clock.uniform_block(b0, self._UBLOCK))
                self._ucache = cache
            return frame, cache[1].ctypes.data + (k0 - b0) * nat.UNIFORM_DTYPE.itemsize, cache[1]
        keep = np.ascontiguousarray(self.uniforms(1), dtype=nat.UNIFORM_DTYPE)
        return frame, keep.ctypes.data, keep

    def _stream_key(self):
        """Engines with equal keys may step in one tfg_update_many call (one
        device, one stream; a handle's own stream is its alone)."""
        s = getattr(self, "_stream_ptr", None)
        return self.device, s if s else ("own", self.h.value)

    def sync(self) -> None:
        self._chk(self.lib.tfg_sync(self.h))

    def join(self) -> None:
        """Order the engine's stream after the second part of split launches
        (tfg_join; no host wait): before work the caller queues on that stream
        itself, e.g. an event that marks the end of the steps."""
        if hasattr(self.lib, "tfg_join"):
            self._chk(self.lib.tfg_join(self.h))

    def is_split(self) -> bool:
        """Whether the next run() steps the grid as two parts on two streams (tfg_get_split)."""
        if not hasattr(self.lib, "tfg_get_split"):
            return False
        v = ctypes.c_int()
        self._chk(self.lib.tfg_get_split(self.h, ctypes.byref(v)))
        return bool(v.value)

    def nan_safe_launches(self) -> int:
        """Launches that ran the fp32 engine's NaN-safe step form (include/tfg.h,
        tfg_nan_safe_launches): missing data, or data not known to be finite."""
        c = ctypes.c_int64()
        self._chk(self.lib.tfg_nan_safe_launches(self.h, ctypes.byref(c)))
        return int(c.value)

    def set_step_form(self, nan_safe: bool) -> None:
        """Run every launch of the fp32 engine in its NaN-safe step form
        (True), or let each launch choose (False, the default; tfg_set_step_form)."""
        self._chk(self.lib.tfg_set_step_form(self.h, 1 if nan_safe else 0))

    def set_stream(self, stream_ptr: int | None) -> None:
        self._chk(self.lib.tfg_set_stream(self.h, ctypes.c_void_p(stream_ptr or 0)))
        self._stream_ptr = stream_ptr or None

    def stream(self) -> int:
        s = ctypes.c_void_p()
        self._chk(self.lib.tfg_get_stream(self.h, ctypes.byref(s)))
        return s.value or 0

    # -- terrain --------------------------------------------------------------------
    def terrain_from_dem(self, dx: float, dy: float, halo_north=None, halo_south=None) -> None:
        """Slope/aspect rasters from the elevation raster (Horn 3x3, tfg_terrain_from_dem).
        Halo rows: numpy arrays or torch CUDA tensors of nx values, None at the domain edge."""
        ptrs, on_dev, dtype = [], 0, nat.F64
        keep = []
        for halo in (halo_north, halo_south):
            if halo is None:
                ptrs.append(None)
                continue
            if hasattr(halo, "data_ptr") and getattr(halo, "is_cuda", False):
                t = halo.contiguous().double()
                keep.append(t)
                ptrs.append(ctypes.c_void_p(t.data_ptr()))
                on_dev = 1
            else:
                a = np.ascontiguousarray(np.asarray(halo, dtype=np.float64).reshape(-1))
                keep.append(a)
                ptrs.append(a.ctypes.data_as(ctypes.c_void_p))
            if (keep[-1].numel() if hasattr(keep[-1], "numel") else keep[-1].size) != self.nx:
                raise ValueError(f"halo rows need nx = {self.nx} values")
        if on_dev and any(isinstance(k, np.ndarray) for k in keep):
            raise ValueError("halo rows must be both host arrays or both device tensors")
        if on_dev:
            import torch

            # RCCL receives complete on torch's stream; the engine reads on its own
            torch.cuda.current_stream(keep[0].device).synchronize()
        self._chk(self.lib.tfg_terrain_from_dem(self.h, float(dx), float(dy), ptrs[0], ptrs[1], dtype, on_dev))

    # -- optional lateral ice flow (tfg_ice_flow_*, off unless called) -----------------
    @staticmethod
    def _halo_args(north, south, nx, rows=2):
        """Halo rows as (keep-alive, north ptr, south ptr, on_device): numpy
        arrays (host) or torch CUDA tensors (device, e.g. straight from an RCCL
        receive), [rows][nx] fp64 each, or None at the domain edge."""
        keep, ptrs, dev = [], [], set()
        dp = ctypes.POINTER(ctypes.c_double)
        for halo in (north, south):
            if halo is None:
                ptrs.append(None)
            elif getattr(halo, "is_cuda", False):
                import torch

                t = halo.reshape(-1).to(torch.float64).contiguous()
                if t.numel() != rows * nx:
                    raise ValueError(f"halo rows need [{rows}][{nx}] values")
                keep.append(t)
                ptrs.append(ctypes.cast(ctypes.c_void_p(t.data_ptr()), dp))
                dev.add(1)
            else:
                a = np.ascontiguousarray(np.asarray(halo, dtype=np.float64).reshape(rows, nx))
                keep.append(a)
                ptrs.append(a.ctypes.data_as(dp))
                dev.add(0)
        if len(dev) > 1:
            raise ValueError("halo rows must be both host arrays or both device tensors")
        if 1 in dev:
            import torch

            torch.cuda.current_stream().synchronize()  # the tensors' producer (RCCL, a cast) is done
        return keep, ptrs[0], ptrs[1], int(1 in dev)

    def ice_flow_edges(self, device=None):
        """This shard's first and last rows as ice-flow halo rows, [2][nx]
        each (surface elevation, ice thickness): numpy arrays, or torch CUDA
        tensors when `device` is given (ready for an RCCL exchange)."""
        dp = ctypes.POINTER(ctypes.c_double)
        if device is not None:
            import torch

            first = torch.empty((2, self.nx), dtype=torch.float64, device=device)
            last = torch.empty((2, self.nx), dtype=torch.float64, device=device)
            torch.cuda.current_stream(first.device).synchronize()
            self._chk(self.lib.tfg_ice_flow_edges(self.h, ctypes.cast(ctypes.c_void_p(first.data_ptr()), dp),
                                                  ctypes.cast(ctypes.c_void_p(last.data_ptr()), dp), 1))
            return first, last  # tfg_ice_flow_edges synchronises the engine stream before returning
        first, last = np.empty((2, self.nx)), np.empty((2, self.nx))
        self._chk(self.lib.tfg_ice_flow_edges(self.h, first.ctypes.data_as(dp), last.ctypes.data_as(dp), 0))
        return first, last

    def ice_flow_dmax(self, dx: float, dy: float, north=None, south=None) -> float:
        """Largest face diffusivity [m2 yr-1] (sets the stable sub-step)."""
        keep, pn, ps, on_dev = self._halo_args(north, south, self.nx)
        out = ctypes.c_double()
        self._chk(self.lib.tfg_ice_flow_dmax(self.h, float(dx), float(dy), pn, ps, on_dev, ctypes.byref(out)))
        return out.value

    def ice_flow_step(self, dt_years: float, dx: float, dy: float, north=None, south=None,
                      part: int = nat.FLOW_ALL) -> None:
        """One explicit shallow-ice sub-step of dt_years (tfg_ice_flow_step).
        part: FLOW_ALL, or FLOW_INTERIOR (queued, no halos) then FLOW_EDGES."""
        keep, pn, ps, on_dev = self._halo_args(north, south, self.nx)
        self._chk(self.lib.tfg_ice_flow_step(self.h, float(dt_years), float(dx), float(dy), pn, ps, on_dev, int(part)))
        del keep

    def ice_flow_run(self, dt_years: float, dx: float, dy: float, n_sub: int) -> None:
        """n_sub sub-steps of dt_years / n_sub on this shard alone, in one call
        (tfg_ice_flow_run: no per-sub-step commit pass)."""
        self._chk(self.lib.tfg_ice_flow_run(self.h, float(dt_years), float(dx), float(dy), int(n_sub)))

    def ice_flow(self, dt_years: float, dx: float, dy: float, cfl: float = 0.5) -> int:
        """Move ice for dt_years on this shard alone (domain edges all round),
        in as many stable sub-steps as needed; returns the sub-step count."""
        from topoflow_glacier.sharding import ice_flow

        return ice_flow(self, dt_years, dx, dy, cfl=cfl, distributed=False)

    # -- optional lateral heat conduction (tfg_conduction_*, off unless called) ------
    def conduction_edges(self, device=None):
        """This shard's first and last rows as conduction halo rows, [4][nx]
        each (T_snow, h_snow, T_ice, h_ice): numpy arrays, or torch CUDA tensors
        when `device` is given (ready for an RCCL exchange)."""
        dp = ctypes.POINTER(ctypes.c_double)
        if device is not None:
            import torch

            first = torch.empty((4, self.nx), dtype=torch.float64, device=device)
            last = torch.empty((4, self.nx), dtype=torch.float64, device=device)
            torch.cuda.current_stream(first.device).synchronize()
            self._chk(self.lib.tfg_conduction_edges(self.h, ctypes.cast(ctypes.c_void_p(first.data_ptr()), dp),
                                                    ctypes.cast(ctypes.c_void_p(last.data_ptr()), dp), 1))
            return first, last  # tfg_conduction_edges synchronises the engine stream before returning
        first, last = np.empty((4, self.nx)), np.empty((4, self.nx))
        self._chk(self.lib.tfg_conduction_edges(self.h, first.ctypes.data_as(dp), last.ctypes.data_as(dp), 0))
        return first, last

    def conduction_update(self, k_snow: float, k_ice: float, dx: float, dy: float, north=None, south=None,
                          q_ground: float = 0.0) -> None:
        """Evaluate the lateral conduction flux Qc from the current state (plus
        a uniform ground heat flux q_ground [W m-2]) and switch the term on:
        every later step adds Qc to Q_sum (:1314) until the next update or
        conduction_off() (tfg_conduction_update)."""
        keep, pn, ps, on_dev = self._halo_args(north, south, self.nx, rows=4)
        self._chk(self.lib.tfg_conduction_update(self.h, float(k_snow), float(k_ice), float(dx), float(dy),
                                                 float(q_ground), pn, ps, on_dev))
        del keep

    def conduction_off(self) -> None:
        """Qc = 0 again: the reference's energy balance (tfg_conduction_off)."""
        self._chk(self.lib.tfg_conduction_off(self.h))

    # -- mass balance -------------------------------------------------------------
    def diagnostics(self) -> np.ndarray:
        """[n_catch][6] = vol_P, vol_PR, vol_PS, vol_SM, vol_IM, P_max of this shard."""
        out = np.zeros((self.n_catch, 6), dtype=np.float64)
        self._chk(self.lib.tfg_get_diag(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), self.n_catch))
        return out

    def reset_diagnostics(self) -> None:
        self._chk(self.lib.tfg_reset_diag(self.h))



class UpdateBatch:
    """Single steps of one-cell fp64 engines that share a device and a stream,
    queued by :meth:`add` and run together by :meth:`run`: one
    tfg_update_many call, one launch (k_cell_many), the results of as many
    ``update_io`` calls bit for bit.  An engine may be queued once per run,
    and must not be closed while queued (the BMI flushes before finalize)."""

    __slots__ = ("engines", "h", "src", "u", "dst", "keep", "owners", "inputs", "n_in")

    _BLOCK = 256  # input rows per staging block

    def __init__(self):
        self.engines, self.h, self.src, self.u, self.dst, self.keep, self.owners = [], [], [], [], [], [], []
        self.inputs, self.n_in = [], 0  # staging blocks [256][5] float64: the queued steps' inputs

    def __len__(self) -> int:
        return len(self.h)

    def add(self, e: GlacierEngine, values: np.ndarray, out: np.ndarray, owner=None) -> None:
        """Queue the next step of `e`: inputs values [5][1] (P_air, Hum_sp, P,
        T_air, uz), outputs out [8][1] (h_snow, h_swe, SM, h_ice, h_iwe, IM,
        M_total, RH), C-contiguous float64 host arrays that must stay alive and
        unmodified until run() returns (it reads and fills them)."""
        if e.n != 1 or e.dtype_code != nat.F64:
            raise ValueError("UpdateBatch: one-cell float64 engines only")
        if values.dtype != np.float64 or out.dtype != np.float64 or values.size != 5 or out.size != 8 \
                or not (values.flags.c_contiguous and out.flags.c_contiguous):
            raise ValueError("UpdateBatch: C-contiguous float64 [5][1] inputs and [8][1] outputs")
        self.add_addresses(e, values.ctypes.data, out.ctypes.data, owner)
        self.keep.append((values, out))

    def add_addresses(self, e: GlacierEngine, src_addr: int, dst_addr: int, owner=None) -> None:
        """add() for a caller that owns fixed, checked blocks (the BMI's input
        and output blocks) and passes their addresses.  The five inputs are
        copied now, into a block the batch owns: the step runs on the values
        update() was given, whatever the caller writes into its own block (a
        get_value_ptr view, say) before the batch runs."""
        _frame, uptr, rec = e._next_uniform()
        row = self.n_in % self._BLOCK
        if row == 0:
            self.inputs.append(np.empty((self._BLOCK, 5), dtype=np.float64))
        blk = self.inputs[-1]
        ctypes.memmove(blk.ctypes.data + row * 40, src_addr, 40)
        self.n_in += 1
        self.engines.append(e)
        self.h.append(e.h.value)
        self.src.append(blk.ctypes.data + row * 40)
        self.u.append(uptr)
        self.dst.append(dst_addr)
        self.keep.append(rec)
        self.owners.append(owner)
        e.step_index += 1

    def run(self) -> None:
        """The queued steps, in one synchronous call.  On an error no step has
        run and the engines' step counters are rolled back."""
        m = len(self.h)
        if m == 0:
            return
        arr = ctypes.c_void_p * m
        engines = self.engines
        try:
            nat.check(engines[0].lib.tfg_update_many(arr(*self.h), m, arr(*self.src), arr(*self.u), arr(*self.dst)))
        except Exception:
            for e in engines:
                e.step_index -= 1
            raise
        finally:
            self.engines, self.h, self.src, self.u, self.dst, self.keep, self.owners = [], [], [], [], [], [], []
            self.inputs, self.n_in = [], 0


def update_many(engines, values, outs) -> None:
    """One step of each one-cell fp64 engine in ONE launch (tfg_update_many):
    for engine i, the same as ``engines[i].update_io(values[i], outs[i])``
    and bit for bit the same result.  values[i] [5][1] and outs[i] [8][1] are
    C-contiguous float64 host arrays, read and filled by the call.  The engines
    share one device and one stream (the BMI's tfg_shared_stream); each appears
    once."""
    b = UpdateBatch()
    for e, v, o in zip(engines, values, outs):
        b.add(e, v, o)
    b.run()
