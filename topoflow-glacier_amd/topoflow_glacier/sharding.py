"""Row-block decomposition of a raster over the GPUs of one node.

Cells are independent in the reference physics (no lateral term: Qc = Qa = 0,
bmi_topoflow_glacier.py:936-955), so a time step of the energy balance needs
no data exchange between shards.  Its only cross-shard operation is the
mass-balance diagnostics (vol_P/PR/PS/SM/IM sums and the P_max max,
:558-624, :1482-1494), combined on demand with one all-reduce over
``torch.distributed`` (RCCL over xGMI on MI355X; gloo in CPU tests).

Three optional stencils (none in the reference
physics) need the rows on each side of a shard, swapped point-to-point
between neighbouring ranks by :func:`exchange_halo_rows` (RCCL send/recv
over xGMI on the GPU path): slope/aspect from a DEM (once,
:func:`terrain_from_dem_sharded`), lateral heat conduction (once per
conduction interval, :func:`lateral_conduction`) and ice flow (before every
sub-step, overlapped with the interior strips, :func:`ice_flow`).
"""

from __future__ import annotations

import numpy as np

__all__ = ["row_block", "allreduce_diagnostics", "exchange_halo_rows", "terrain_from_dem_sharded", "ice_flow",
           "lateral_conduction"]


def row_block(ny_global: int, rank: int, world: int) -> tuple[int, int]:
    """(row0, rows) of `rank`'s block; rows differ by at most one."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(int(ny_global), int(world))
    rows = base + (1 if rank < extra else 0)
    row0 = rank * base + min(rank, extra)
    return row0, rows


def allreduce_diagnostics(diag: np.ndarray, group=None, device=None) -> np.ndarray:
    """Combine per-shard [n_catch][6] diagnostics: sum of columns 0-4, max of
    column 5.  One all-reduce of the sums plus one of the maxima."""
    import torch
    import torch.distributed as dist

    d = np.asarray(diag, dtype=np.float64)
    if not (dist.is_available() and dist.is_initialized()):
        return d.copy()
    dev = device if device is not None else ("cuda" if dist.get_backend(group) == "nccl" else "cpu")
    sums = torch.from_numpy(np.ascontiguousarray(d[:, :5])).to(dev)
    maxs = torch.from_numpy(np.ascontiguousarray(d[:, 5])).to(dev)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(maxs, op=dist.ReduceOp.MAX, group=group)
    out = np.empty_like(d)
    out[:, :5] = sums.cpu().numpy()
    out[:, 5] = maxs.cpu().numpy()
    return out


def exchange_halo_rows(first_row, last_row, group=None):
    """(north, south) halo rows of this rank's row block: the last row of rank
    r-1 and the first row of rank r+1 (None at the domain edges).  first_row /
    last_row are torch tensors (CUDA for the nccl backend); one batched
    point-to-point exchange, no collective."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return None, None
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    north = torch.empty_like(first_row) if rank > 0 else None
    south = torch.empty_like(last_row) if rank < world - 1 else None
    peer = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    ops = []
    if rank > 0:
        ops += [dist.P2POp(dist.isend, first_row.contiguous(), peer(rank - 1), group),
                dist.P2POp(dist.irecv, north, peer(rank - 1), group)]
    if rank < world - 1:
        ops += [dist.P2POp(dist.isend, last_row.contiguous(), peer(rank + 1), group),
                dist.P2POp(dist.irecv, south, peer(rank + 1), group)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return north, south


def terrain_from_dem_sharded(eng, dx: float, dy: float, group=None) -> None:
    """Slope/aspect of a row-block shard (GlacierEngine) with its neighbours'
    boundary rows as halos: equal to the unsharded result."""
    import torch
    import torch.distributed as dist

    elev = eng.get_field("elev").reshape(eng.ny, eng.nx)
    dev = "cpu"
    if dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "nccl":
        dev = f"cuda:{torch.cuda.current_device()}"
    first = torch.from_numpy(np.ascontiguousarray(elev[0])).to(dev)
    last = torch.from_numpy(np.ascontiguousarray(elev[-1])).to(dev)
    north, south = exchange_halo_rows(first, last, group)
    eng.terrain_from_dem(dx, dy, north, south)


def ice_flow(eng, dt_years: float, dx: float, dy: float, cfl: float = 0.5, group=None, distributed=None,
             max_substeps: int = 100000) -> int:
    """The optional shallow-ice flow term over a row-block sharded grid
    (tfg_ice_flow_*; extension).

    Each sub-step needs the neighbour shards' adjacent rows (surface elevation
    and ice thickness), swapped by one batched point-to-point exchange (RCCL
    over xGMI on the GPU path, gloo on CPU).  The sub-step count comes from the
    largest face diffusivity over all ranks (one MAX all-reduce), so every
    rank takes the same steps and the sharded result equals the unsharded one
    bit for bit.  `eng` is a GlacierEngine (or anything with its ice_flow_*
    methods and `nx`).  Returns the number of sub-steps.
    """
    import math

    import torch
    import torch.distributed as dist

    on = distributed if distributed is not None else (
        dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1)
    dev = "cpu"
    if on and dist.get_backend(group) == "nccl":
        dev = f"cuda:{torch.cuda.current_device()}"

    FLOW_INTERIOR, FLOW_EDGES = 1, 2  # tfg_ice_flow_step parts (include/tfg.h)

    # On the GPU path the halo rows never leave the devices: the engine writes
    # its edge rows into CUDA tensors, RCCL swaps them over xGMI, and the
    # engine reads the received tensors by device pointer.
    def edges():
        return eng.ice_flow_edges(device=dev) if dev != "cpu" else eng.ice_flow_edges()

    def swap(first, last):
        t = (lambda a: a.reshape(-1)) if dev != "cpu" else (lambda a: torch.from_numpy(a.reshape(-1)))
        n, s = exchange_halo_rows(t(first), t(last), group)
        if dev != "cpu":
            return n, s  # device tensors; the engine orders its copy after torch's stream
        return (None if n is None else n.numpy().reshape(2, -1), None if s is None else s.numpy().reshape(2, -1))

    def halos():
        return swap(*edges()) if on else (None, None)

    north, south = halos()
    dmax = float(eng.ice_flow_dmax(dx, dy, north, south))
    if on:
        t = torch.tensor([dmax], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dmax = float(t.item())
    if not dmax > 0.0:
        return 0  # no ice or no slope anywhere: nothing moves
    dt_stable = cfl * min(dx, dy) ** 2 / (4.0 * dmax)
    n_sub = max(1, math.ceil(dt_years / dt_stable))
    if n_sub > max_substeps:
        raise ValueError(f"ice flow needs {n_sub} sub-steps (> {max_substeps}); shorten the interval")
    if not on and hasattr(eng, "ice_flow_run"):
        eng.ice_flow_run(dt_years, dx, dy, n_sub)  # one shard: sub-steps ping-pong on the device
        return n_sub
    dt = dt_years / n_sub
    for k in range(n_sub):
        if k == 0 or not on:
            eng.ice_flow_step(dt, dx, dy, north, south)  # halos of the CFL pass are current
            continue
        # the interior rows run on the GPU while the halo rows cross between ranks
        first, last = edges()
        eng.ice_flow_step(dt, dx, dy, part=FLOW_INTERIOR)
        north, south = swap(first, last)
        eng.ice_flow_step(dt, dx, dy, north, south, part=FLOW_EDGES)
    return n_sub


def lateral_conduction(eng, k_snow: float, k_ice: float, dx: float, dy: float, group=None, distributed=None,
                       q_ground: float = 0.0) -> None:
    """The optional lateral heat-conduction term over a row-block sharded grid
    (tfg_conduction_*; extension): each shard swaps its
    edge rows' pack temperatures and depths with its neighbours (one batched
    point-to-point exchange, RCCL over xGMI on the GPU path, gloo on CPU), then
    evaluates its Qc field, which the following steps add to Q_sum.  The
    sharded Qc equals the unsharded one bit for bit.  `eng` is a GlacierEngine
    (or anything with its conduction_* methods)."""
    import torch
    import torch.distributed as dist

    on = distributed if distributed is not None else (
        dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1)
    if not on:
        eng.conduction_update(k_snow, k_ice, dx, dy, q_ground=q_ground)
        return
    if dist.get_backend(group) == "nccl":  # the rows stay on the devices
        first, last = eng.conduction_edges(device=f"cuda:{torch.cuda.current_device()}")
        north, south = exchange_halo_rows(first.reshape(-1), last.reshape(-1), group)
    else:
        first, last = eng.conduction_edges()
        north, south = exchange_halo_rows(torch.from_numpy(first.reshape(-1)), torch.from_numpy(last.reshape(-1)), group)
        north = None if north is None else north.numpy()
        south = None if south is None else south.numpy()
    eng.conduction_update(k_snow, k_ice, dx, dy, north, south, q_ground=q_ground)
