"""Catchment divides of a NextGen hydrofabric -> catchment-ID raster
(SURVEY.md 8(f) row 2).

The reference runs one model instance per catchment, with the catchment area
`da` from the hydrofabric's `divides` layer (data/12082500.gpkg, column
`areasqkm`, one row per `cat-*` divide; config.py:11).  On a grid the same
catchments become an int32 raster: the fused kernel's per-catchment reduction
(k_fused<..., CATCH>) then yields every catchment's vol_P / vol_PR / vol_PS /
vol_SM / vol_IM / P_max in one launch.

GeoPackage is SQLite with OGC geometry blobs; no GIS library is available
offline, so the reader is written here against the published formats:
  * GeoPackage binary header (OGC 12-128r18 section 2.1.3): b"GP", version,
    flags (bit 0 byte order, bits 1-3 envelope code, bit 4 empty), int32 srs_id,
    then an envelope of 0/4/6/6/8 doubles;
  * ISO/OGC WKB (OGC 06-103r4): byte order, uint32 type (Polygon 3,
    MultiPolygon 6; +1000/2000/3000 for Z/M/ZM), rings of points.
The database is opened read-only and immutable; nothing in it is executed.
"""

from __future__ import annotations

import sqlite3
import struct
from dataclasses import dataclass
from pathlib import Path

import numpy as np

__all__ = ["Divide", "read_divides", "load_divides_npz", "parse_gpkg_geometry", "ring_area", "grid_covering",
           "rasterize_divides", "catchment_ids"]


@dataclass
class Divide:
    divide_id: str
    areasqkm: float
    polygons: list  # [polygon][ring] -> float64 [k, 2] (x, y); ring 0 is the shell


def _wkb_polygons(b: memoryview, off: int):
    """Parse one WKB geometry at `off`; returns (list of polygons, new offset)."""
    bo = "<" if b[off] == 1 else ">"
    (gtype,) = struct.unpack_from(bo + "I", b, off + 1)
    off += 5
    base = gtype % 1000
    dims = {0: 2, 1: 3, 2: 3, 3: 4}[gtype // 1000]
    if base == 3:
        (nrings,) = struct.unpack_from(bo + "I", b, off)
        off += 4
        rings = []
        for _ in range(nrings):
            (npts,) = struct.unpack_from(bo + "I", b, off)
            off += 4
            pts = np.frombuffer(b, dtype=np.dtype(np.float64).newbyteorder(bo), count=npts * dims, offset=off)
            rings.append(pts.reshape(npts, dims)[:, :2].astype(np.float64))
            off += 8 * npts * dims
        return [rings], off
    if base == 6:
        (npoly,) = struct.unpack_from(bo + "I", b, off)
        off += 4
        polys = []
        for _ in range(npoly):
            p, off = _wkb_polygons(b, off)
            polys.extend(p)
        return polys, off
    raise ValueError(f"unsupported WKB geometry type {gtype} (Polygon/MultiPolygon only)")


def parse_gpkg_geometry(blob: bytes) -> tuple[int, list]:
    """(srs_id, polygons) of a GeoPackage geometry blob."""
    b = memoryview(blob)
    if bytes(b[:2]) != b"GP":
        raise ValueError("not a GeoPackage geometry blob")
    flags = b[3]
    bo = "<" if flags & 1 else ">"
    (srs_id,) = struct.unpack_from(bo + "i", b, 4)
    env = (flags >> 1) & 7
    if env > 4:
        raise ValueError(f"invalid GeoPackage envelope code {env}")
    off = 8 + 8 * (0, 4, 6, 6, 8)[env]
    if flags & 16:  # empty geometry
        return srs_id, []
    polys, _ = _wkb_polygons(b, off)
    return srs_id, polys


def read_divides(path: str | Path, layer: str = "divides") -> tuple[int, list]:
    """(srs_id, [Divide]) of a hydrofabric GeoPackage, ordered by fid."""
    con = sqlite3.connect(f"file:{Path(path)}?mode=ro&immutable=1", uri=True)
    try:
        cur = con.cursor()
        (gcol,) = cur.execute("select column_name from gpkg_geometry_columns where table_name = ?", (layer,)).fetchone()
        rows = cur.execute(f'select divide_id, areasqkm, "{gcol}" from "{layer}" order by fid').fetchall()
    finally:
        con.close()
    out, srs = [], None
    for did, area, blob in rows:
        s, polys = parse_gpkg_geometry(blob)
        srs = s if srs is None else srs
        out.append(Divide(str(did), float(area), polys))
    return srs, out


def ring_area(ring: np.ndarray) -> float:
    """Unsigned shoelace area of a closed or open ring [m2 in a projected CRS]."""
    x, y = ring[:, 0], ring[:, 1]
    return 0.5 * abs(float(np.dot(x, np.roll(y, -1)) - np.dot(y, np.roll(x, -1))))


def grid_covering(divides: list, cell: float, pad: int = 1):
    """(x0, y0, ny, nx): a north-up grid of `cell`-metre cells covering every
    divide; (x0, y0) is the upper-left corner, row 0 at the top."""
    xs = np.concatenate([r[:, 0] for d in divides for p in d.polygons for r in p])
    ys = np.concatenate([r[:, 1] for d in divides for p in d.polygons for r in p])
    x0 = np.floor(xs.min() / cell) * cell - pad * cell
    y0 = np.ceil(ys.max() / cell) * cell + pad * cell
    nx = int(np.ceil((xs.max() - x0) / cell)) + pad
    ny = int(np.ceil((y0 - ys.min()) / cell)) + pad
    return float(x0), float(y0), ny, nx


def _inside(px: np.ndarray, py: np.ndarray, ring: np.ndarray) -> np.ndarray:
    """Even-odd crossing test of points against one ring."""
    x, y = ring[:, 0], ring[:, 1]
    x2, y2 = np.roll(x, -1), np.roll(y, -1)
    inside = np.zeros(px.shape, dtype=bool)
    for a, b, c, d in zip(x, y, x2, y2):
        if b == d:
            continue
        cond = (b > py) != (d > py)
        xc = a + (py - b) * (c - a) / (d - b)
        inside ^= cond & (px < xc)
    return inside


def rasterize_divides(divides: list, x0: float, y0: float, cell: float, ny: int, nx: int) -> np.ndarray:
    """int32 [ny, nx] raster of divide index (position in `divides`) at cell
    centres, -1 outside every divide.  Shells include, holes exclude."""
    ids = np.full((ny, nx), -1, dtype=np.int32)
    for k, d in enumerate(divides):
        for poly in d.polygons:
            sh = poly[0]
            c0 = max(int(np.floor((sh[:, 0].min() - x0) / cell)), 0)
            c1 = min(int(np.ceil((sh[:, 0].max() - x0) / cell)) + 1, nx)
            r0 = max(int(np.floor((y0 - sh[:, 1].max()) / cell)), 0)
            r1 = min(int(np.ceil((y0 - sh[:, 1].min()) / cell)) + 1, ny)
            if c0 >= c1 or r0 >= r1:
                continue
            px = x0 + (np.arange(c0, c1) + 0.5) * cell
            py = y0 - (np.arange(r0, r1) + 0.5) * cell
            PX, PY = np.meshgrid(px, py)
            m = _inside(PX, PY, sh)
            for hole in poly[1:]:
                m &= ~_inside(PX, PY, hole)
            sub = ids[r0:r1, c0:c1]
            sub[m] = k
    return ids


def load_divides_npz(path: str | Path) -> tuple[int, list]:
    """(srs_id, [Divide]) from the vertex-array form tests/golden/make_hydrofabric.py writes."""
    z = np.load(path)
    off, ring_poly, poly_div = z["ring_off"], z["ring_poly"], z["poly_div"]
    polys = [[] for _ in range(len(poly_div))]
    for r in range(len(ring_poly)):
        polys[ring_poly[r]].append(z["xy"][off[r]:off[r + 1]])
    out = [Divide(str(i), float(a), []) for i, a in zip(z["divide_id"], z["areasqkm"])]
    for p, k in zip(polys, poly_div):
        out[k].polygons.append(p)
    return int(z["srs"]), out


def catchment_ids(raster: np.ndarray) -> tuple[np.ndarray, int]:
    """Engine catchment ids from a divide raster: divide k -> k, outside -> the
    last id (a bin for cells that belong to no divide).  Returns (ids, n_catch)."""
    n = int(raster.max()) + 1 if raster.size else 0
    ids = np.where(raster < 0, n, raster).astype(np.int32)
    return ids, n + 1
