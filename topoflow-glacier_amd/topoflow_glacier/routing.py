"""Mock routing downstream of the melt runoff.

The reference's example driver compares against the original TopoFlow by
routing the catchment runoff [m3 s-1] through a 20-tap boxcar
(examples/run_topoflow_glacier.py:129-131): weights 0.05, full convolution,
truncated to the input length (a causal 20-step moving average).  Host-side
and tiny (one series per catchment), so it stays on the CPU.
"""

from __future__ import annotations

import numpy as np

__all__ = ["boxcar_route"]


def boxcar_route(runoff: np.ndarray, taps: int = 20) -> np.ndarray:
    """Route a runoff series [nsteps] or a stack [nsteps][ncatch] along time."""
    x = np.asarray(runoff, dtype=np.float64)
    weights = np.zeros(taps) + 1.0 / taps  # 0.05 for the reference's 20 taps (:129)
    if x.ndim == 1:
        return np.convolve(x, weights, mode="full")[: len(x)]
    return np.stack([np.convolve(x[:, j], weights, mode="full")[: x.shape[0]] for j in range(x.shape[1])], axis=1)
