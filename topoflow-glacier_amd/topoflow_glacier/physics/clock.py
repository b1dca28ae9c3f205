"""Model clock and the per-step uniform scalars of the hot path.

For a grid with one latitude/longitude (the reference's catchment centroid,
config.py:21-22) everything in ``update_julian_day`` (bmi_topoflow_glacier.py
:957-1004) and the latitude-only part of ``Clear_Sky_Radiation``
(solar_funcs.py:894-953) is the same for every cell.  ``StepClock`` evaluates
it on the host once per step, in float64 numpy with the reference's operation
order (so the fp64 engine sees bit-identical values), vectorised over a block
of steps, and packs it into ``tfg_uniforms`` records for the kernel.

Time convention (reference :1866-1893): the model datetime is advanced by
``dt`` hours *before* it is used, so step k (0-based) uses start + (k+1)*dt.
The UTC offset is DST-aware (zoneinfo, SF:1616-1637); the IANA zone comes from
``cfg.time_zone`` or from :func:`zone_for` (timezonefinder is not available
offline).
"""

from __future__ import annotations

from collections import OrderedDict
from datetime import datetime, timedelta
from functools import lru_cache
from zoneinfo import ZoneInfo

import numpy as np

from .._native import UNIFORM_DTYPE

__all__ = ["StepClock", "zone_for", "parse_time", "PERIHELION"]

_RAD = np.pi / np.float64(180)
_OMEGA = (np.float64(360) / np.float64(24)) * (np.pi / np.float64(180))  # SF:257-258

# Day-of-January and hour of Earth's perihelion, 1981-2060 (SF:1167-1248).
_TP = (
    "2:2 4:11 2:15 3:22 3:20 2:5 4:23 3:0 1:22 4:17 3:3 3:15 4:3 2:6 4:11 4:7 2:0 4:21 3:13 3:5 "
    "4:9 2:14 4:5 4:18 2:1 4:15 3:20 3:0 4:15 3:0 3:19 5:0 2:5 4:12 4:7 2:23 4:14 3:6 3:5 5:8 "
    "2:14 4:7 4:16 3:1 4:13 3:17 3:3 5:12 2:18 3:10 4:21 3:5 4:12 4:5 3:1 5:14 3:4 3:5 5:7 3:12 "
    "3:22 4:9 2:22 5:13 3:15 3:1 5:12 3:18 3:10 4:20 3:6 5:9 3:22 2:18 5:12 4:4 3:3 5:4 3:11 4:23"
)
PERIHELION = {1981 + i: tuple(int(x) for x in v.split(":")) for i, v in enumerate(_TP.split())}

# IANA zones by lat/lon box, for points where a box can be justified: every
# box lies wholly inside territory with ONE set of UTC offsets (borders and the
# water beyond them included), so a point in it gets the offsets the
# reference's timezonefinder + zoneinfo lookup gives.  The zone name is that of
# the US territory; the Eastern box also covers southern Ontario, whose
# America/Toronto has the same offsets and DST dates as America/New_York.  Where zones meet irregularly -- the Idaho and Oregon Pacific /
# Mountain line, the Navajo Nation (DST) inside Arizona (no DST), the Alaska
# panhandle against British Columbia and Yukon, the Central / Eastern line,
# Indiana -- no box reaches, and the caller must set `time_zone`.  The
# reference resolves the zone with timezonefinder polygons (solar_funcs.py
# :1616-1637), which are not available offline.  (lat0, lat1, lon0, lon1).
_ZONES = [
    # Pacific: Washington (and the Idaho panhandle) north of the Columbia, west of 117.1 W
    ((45.6, 49.0, -124.8, -117.1), "America/Los_Angeles"),
    # Pacific: Oregon west of Malheur County
    ((42.0, 46.3, -124.6, -119.0), "America/Los_Angeles"),
    # Pacific: California and western Nevada, clear of Arizona (Colorado River) and Mexico
    ((32.72, 42.0, -124.5, -115.0), "America/Los_Angeles"),
    # Pacific: Nevada north of Lake Mead, west of West Wendover (Mountain) and Utah
    ((36.2, 42.0, -120.0, -114.1), "America/Los_Angeles"),
    # Mountain, DST: Utah, Colorado, Wyoming, New Mexico
    ((37.0, 42.0, -114.05, -109.05), "America/Denver"),
    ((37.0, 41.0, -109.05, -102.05), "America/Denver"),
    ((41.0, 45.0, -111.05, -104.05), "America/Denver"),
    ((32.0, 37.0, -109.05, -103.07), "America/Denver"),  # clear of the Texas line at 103.064 W
    ((31.79, 32.0, -109.05, -106.65), "America/Denver"),  # southern New Mexico, clear of Chihuahua
    # Mountain, DST: Montana east of the Bitterroot divide, and north of 48 N east of the 116.05 W line
    ((45.0, 49.0, -113.0, -104.05), "America/Denver"),
    ((48.0, 49.0, -116.0, -104.05), "America/Denver"),
    # Mountain, DST: southern Idaho and Malheur County, Oregon (the state line at
    # 117.03 W up to the Snake's mouth of the Owyhee, 43.8 N); north of 43.8 N the
    # box stays east of the Snake River, beyond which Baker County, Oregon keeps Pacific time
    ((42.0, 43.8, -117.0, -111.05), "America/Boise"),
    ((43.8, 44.8, -116.8, -111.05), "America/Boise"),
    # Arizona outside the Navajo Nation: Mountain, no DST
    ((31.34, 34.8, -111.0, -109.05), "America/Phoenix"),
    ((32.5, 35.0, -114.0, -111.0), "America/Phoenix"),
    ((35.0, 37.0, -114.0, -112.0), "America/Phoenix"),
    # Alaska west of the Yukon border (141 W) and east of the Aleutian (Adak) zone
    ((51.2, 71.5, -169.0, -141.0), "America/Anchorage"),
    ((18.5, 23.0, -161.0, -154.0), "Pacific/Honolulu"),
    # Central: Texas to Minnesota, clear of the Mountain line, Mexico, Michigan and Indiana
    ((29.0, 45.0, -99.5, -88.5), "America/Chicago"),
    # Eastern: east of Indiana, Kentucky's and Tennessee's Central parts, south of New Brunswick
    ((25.0, 45.0, -84.0, -67.0), "America/New_York"),
]


def zone_for(lat: float, lon: float) -> str:
    """IANA time zone of a point inside one of the boxes above; elsewhere
    ValueError, asking for `time_zone` (the reference raises when it finds
    no zone, SF:1629-1630)."""
    for (la0, la1, lo0, lo1), name in _ZONES:
        if la0 <= lat <= la1 and lo0 <= lon <= lo1:
            return name
    raise ValueError(f"No unambiguous time zone for lat={lat}, lon={lon} in the built-in table; "
                     "set `time_zone` (an IANA name) in the config.")


def parse_time(s) -> datetime:
    """'YYYYMMDDHH' or 'YYYYMMDD-HH' (reference :512-517)."""
    s = str(s).strip()
    return datetime.strptime(s, "%Y%m%d-%H" if "-" in s else "%Y%m%d%H")


def _julian_day_of_january(day: int, hour: int) -> np.float64:
    # Julian_Day(1, day, hour) with year=None (SF:958-1009)
    return np.float64(0) + np.maximum(day - 1, 0) + (hour / np.float64(24))


@lru_cache(maxsize=None)
def _perihelion_jd(year: int) -> np.float64:
    if year not in PERIHELION:
        # the reference silently substitutes the wall-clock year (SF:1158-1162);
        # that makes results depend on when they are run, so refuse instead.
        raise ValueError(f"Earth perihelion table covers 1981-2060, got year {year}")
    d, h = PERIHELION[year]
    return _julian_day_of_january(d, h)


def _equation_of_time_hours(JD: np.ndarray, years: np.ndarray) -> np.ndarray:
    """Equation_Of_Time(JD, year) in hours (SF:1301-1429), vectorised."""
    e = np.float64(0.016713)
    eps = np.float64(23.4397) * (np.pi / np.float64(180))
    dpy = np.float64(365.2425)
    twopi = np.float64(2) * np.pi
    uy, inv = np.unique(years, return_inverse=True)
    Tp = np.array([_perihelion_jd(int(y)) for y in uy])[inv]
    M = (twopi / dpy) * (JD - Tp)
    M = (M + twopi) % twopi
    VE = np.float64(79.3125) + dpy * (years.astype(np.float64) - np.float64(2000))
    PT = (np.float64(365) + Tp) - VE
    L = M + twopi * (PT / dpy)
    TE = (-2.0 * e * np.sin(M)) + (np.sin(2 * L) * (eps / 2) ** 2.0)
    return TE / (np.float64(2) * np.pi / np.float64(24))


_BLOCKS: "OrderedDict[tuple, np.ndarray]" = OrderedDict()  # StepClock.uniform_block, least recently used first
_BLOCKS_MAX = 256  # blocks of 512 records (80 KB each)


class StepClock:
    """Uniform scalars for model steps k = 0, 1, 2, ... of one run."""

    def __init__(self, start_time, dt_hours, lat: float, lon: float, time_zone: str | None = None,
                 ring_len: int = 72):
        self.start = parse_time(start_time)
        self.dt = dt_hours
        self.lat = lat
        self.lon = lon
        self.tz = ZoneInfo(time_zone or zone_for(lat, lon))
        self.ring_len = int(ring_len)

    # -- calendar ----------------------------------------------------------
    def calendar(self, k0: int, n: int):
        """(julian_day, year, GMT_offset, TSN_offset) for steps k0..k0+n-1
        (update_julian_day :957-1004).  Short requests are served from blocks
        of 512 steps computed once."""
        B = 512
        b0 = k0 - k0 % B
        if n <= B and k0 + n <= b0 + B:
            cache = getattr(self, "_cal_cache", None)
            if cache is None or cache[0] != b0:
                cache = (b0, self._calendar(b0, B))
                self._cal_cache = cache
            i = k0 - b0
            return tuple(a[i:i + n] for a in cache[1])
        return self._calendar(k0, n)

    def _calendar(self, k0: int, n: int):
        """Vectorised where the step is a whole number of seconds that the
        float product dt*(k+1) hits exactly (dt a multiple of 1/1024 h, e.g.
        1 h or 0.25 h): the same values as the per-step datetime loop
        (_calendar_loop, the reference's own arithmetic), bit for bit
        (tests/test_host.py::test_vectorised_calendar_equals_the_loop)."""
        step_s = self.dt * 3600.0
        if not (n > 0 and step_s == int(step_s) and self.dt * 1024.0 == int(self.dt * 1024.0)
                and (k0 + n) * self.dt < 2.0 ** 40):
            return self._calendar_loop(k0, n)
        secs = (np.arange(k0 + 1, k0 + n + 1, dtype=np.int64) * int(step_s)).astype("timedelta64[s]")
        t = np.datetime64(self.start, "s") + secs  # naive, read as UTC as the loop does
        day = t.astype("datetime64[D]")
        yr = t.astype("datetime64[Y]").astype(np.int64) + 1970
        yday0 = (day - t.astype("datetime64[Y]").astype("datetime64[D]")).astype(np.int64)  # tm_yday - 1
        sod = (t - day).astype(np.int64)
        hour, minute, second = sod // 3600, (sod % 3600) // 60, sod % 60
        # J = tm_yday - 1 + hour/24 + minute/1440 + second/86400, left to right (:985-990)
        jd = ((yday0.astype(np.float64) + hour / 24) + minute / 1440) + second / 86400
        clock_hour = (jd - np.trunc(jd)) * np.float64(24)
        gmt = self._utc_offsets(t, day)
        LC = ((gmt * np.float64(15)) - self.lon) / np.float64(15)  # SF:1466-1468
        solar_noon = np.float64(12) + LC + _equation_of_time_hours(jd, yr)  # SF:1471
        return jd, yr, gmt, clock_hour - solar_noon

    def _utc_offsets(self, t: np.ndarray, day: np.ndarray) -> np.ndarray:
        """UTC offset [h] of the zone at each UTC instant t (SF:1616-1637's
        zoneinfo lookup): looked up once per UTC day where the offset is the
        same at the day's first and last second, per step on a day with a
        transition."""
        utc = ZoneInfo("UTC")

        def off(dt64) -> float:
            d = dt64.astype("datetime64[s]").astype(datetime).replace(tzinfo=utc)
            return d.astimezone(self.tz).utcoffset().total_seconds() / 3600.0

        gmt = np.empty(len(t))
        days, inv = np.unique(day, return_inverse=True)
        for j, d in enumerate(days):
            a, b = off(d), off(d + np.timedelta64(86399, "s"))
            sel = inv == j
            if a == b:
                gmt[sel] = a
            else:
                gmt[sel] = [off(x) for x in t[sel]]
        return gmt

    def _calendar_loop(self, k0: int, n: int):
        jd = np.empty(n)
        yr = np.empty(n, dtype=np.int64)
        gmt = np.empty(n)
        clock_hour = np.empty(n)
        utc = ZoneInfo("UTC")
        for i in range(n):
            t = self.start + timedelta(hours=self.dt * (k0 + i + 1))
            J = t.timetuple().tm_yday - 1 + t.hour / 24 + t.minute / 1440 + t.second / 86400
            jd[i] = J
            yr[i] = t.year
            clock_hour[i] = (J - int(J)) * np.float64(24)
            gmt[i] = t.replace(tzinfo=utc).astimezone(self.tz).utcoffset().total_seconds() / 3600.0
        LC = ((gmt * np.float64(15)) - self.lon) / np.float64(15)  # SF:1466-1468
        solar_noon = np.float64(12) + LC + _equation_of_time_hours(jd, yr)  # SF:1471
        return jd, yr, gmt, clock_hour - solar_noon

    # -- per-step uniforms --------------------------------------------------
    def key(self) -> tuple:
        """Everything the uniforms depend on: equal keys give equal records."""
        return (self.start, float(self.dt), float(self.lat), float(self.lon), self.tz.key, self.ring_len)

    def uniform_block(self, b0: int, n: int) -> np.ndarray:
        """uniforms(b0, n) with frame = hist = 0, read-only and shared by every
        clock of the process with the same key (NextGen runs one model per
        catchment: an ensemble, or catchments that share a centroid clock,
        then compute each block once, not once per model)."""
        k = (self.key(), int(b0), int(n))
        u = _BLOCKS.get(k)
        if u is None:
            u = self.uniforms(b0, n)
            u.flags.writeable = False
            _BLOCKS[k] = u
            if len(_BLOCKS) > _BLOCKS_MAX:
                _BLOCKS.popitem(last=False)
        else:
            _BLOCKS.move_to_end(k)
        return u

    def uniforms(self, k0: int, n: int, frames=None, hist=None) -> np.ndarray:
        """tfg_uniforms records for steps k0..k0+n-1.

        frames: forcing frame per step (default 0); hist: output-history slot
        per step (default 0).  The snowfall-window slot is (k mod ring_len).
        """
        jd, _, _, th = self.calendar(k0, n)
        u = np.zeros(n, dtype=UNIFORM_DTYPE)
        lat = self.lat
        G = (2 * np.pi) * jd / np.float64(365)  # Day_Angle SF:176
        delta = (np.float64(0.006918) - (np.float64(0.399912) * np.cos(G)) + (np.float64(0.070257) * np.sin(G))
                 - (np.float64(0.006758) * np.cos(np.float64(2) * G)) + (np.float64(0.000907) * np.sin(np.float64(2) * G))
                 - (np.float64(0.002697) * np.cos(np.float64(3) * G)) + (np.float64(0.001480) * np.sin(np.float64(3) * G)))
        E0 = (np.float64(1.000110) + (np.float64(0.034221) * np.cos(G)) + (np.float64(0.001280) * np.sin(G))
              + (np.float64(0.000719) * np.cos(np.float64(2) * G)) + (np.float64(0.000077) * np.sin(np.float64(2) * G)))
        lat_rad = lat * _RAD
        # Optical_Air_Mass (Kasten & Young; SF:540-570), gamma clamped >= 0
        Z = np.arccos(np.sin(lat_rad) * np.sin(delta) + np.cos(lat_rad) * np.cos(delta) * np.cos(_OMEGA * th))
        gamma = np.maximum(90.0 - Z * (180 / np.pi), 0.0)
        m_opt = np.float64(1) / (np.sin(gamma * (np.pi / 180)) + 0.50572 / (gamma + 6.07995) ** 1.6364)
        # ET_Radiation_Flux on the flat (SF:383-413)
        k_flat = np.float64(1361.5) * E0 * (np.cos(delta) * np.cos(lat_rad) * np.cos(_OMEGA * th)
                                            + np.sin(delta) * np.sin(lat_rad))
        k_flat = np.maximum(k_flat, 0.0)
        # Sunrise/Sunset_Offset at the centroid latitude (SF:319-358)
        arg = -np.float64(1) * np.tan(lat_rad) * np.tan(delta)
        arg = np.minimum(np.maximum(-1, arg), 1)
        flat_sr = -np.float64(1) * np.arccos(arg) / _OMEGA
        flat_ss = np.arccos(arg) / _OMEGA
        wth = _OMEGA * th
        u["th"], u["omega_th"], u["cos_wth"], u["sin_wth"] = th, wth, np.cos(wth), np.sin(wth)
        u["sin_d"], u["cos_d"], u["tan_d"] = np.sin(delta), np.cos(delta), np.tan(delta)
        u["isc_e0"] = np.float64(1361.5) * E0
        u["m_opt"], u["k_et_flat"], u["flat_sr"], u["flat_ss"] = m_opt, k_flat, flat_sr, flat_ss
        # fp32-engine coefficients (tfg.h): fp64 here, rounded once
        log2e = np.float64(1.4426950408889634)
        u["cos_wth_f"], u["sin_wth_f"], u["omega_th_f"] = u["cos_wth"], u["sin_wth"], wth
        u["tan_d_f"] = u["tan_d"]
        u["kc_f"] = u["isc_e0"] * u["cos_d"]
        u["ks_f"] = u["isc_e0"] * u["sin_d"]
        u["k_et_flat_f"] = k_flat
        # a + b*m_opt with a, b affine in W_p = 1.12*w (SF:606-613, SF:648-655)
        u["tau_c0"] = log2e * (-0.1240 - 0.0682 * m_opt)
        u["tau_c1"] = log2e * 1.12 * (-0.0207 - 0.0248 * m_opt)
        u["gam_c0"] = log2e * (-0.0363 - 0.0572 * m_opt)
        u["gam_c1"] = log2e * 1.12 * (-0.0084 - 0.0173 * m_opt)
        u["flat_dark"] = ((th <= flat_sr) | (th >= flat_ss)).astype(np.int32)
        u["frame"] = 0 if frames is None else frames
        u["hist"] = 0 if hist is None else hist
        u["slot"] = (np.arange(k0, k0 + n) % self.ring_len).astype(np.int32)
        return u
