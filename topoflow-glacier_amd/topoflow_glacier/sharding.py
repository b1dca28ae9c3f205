"""Row-block decomposition of a raster over the GPUs of one node.

Cells are independent in the reference physics (no lateral term: Qc = Qa = 0,
bmi_topoflow_glacier.py:936-955), so a time step needs no data exchange
between shards.  The only cross-shard operation is the mass-balance
diagnostics (vol_P/PR/PS/SM/IM sums and the P_max max, :558-624,
:1482-1494), combined on demand with one all-reduce over
``torch.distributed`` (RCCL over xGMI on MI355X; gloo in CPU tests).
"""

from __future__ import annotations

import numpy as np

__all__ = ["row_block", "allreduce_diagnostics"]


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
