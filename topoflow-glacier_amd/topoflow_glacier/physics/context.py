"""Named BMI variable store (counterpart of physics/context.py:9-88).

Each variable is a float64 host array of the grid's cell count (shape (1,) for
the reference's single catchment) with a unit.  ``set_value`` copies into the
existing array so references handed out by ``get_value_ptr`` stay valid.
"""

from __future__ import annotations

from collections.abc import Iterable, Iterator
from dataclasses import dataclass

import numpy as np

__all__ = ["Var", "Context", "build_context"]


@dataclass
class Var:
    name: str
    unit: str
    value: np.ndarray


class Context:
    def __init__(self, vars: Iterable[Var]):
        self._vars: dict[str, Var] = {v.name: v for v in vars}

    def unit(self, name: str) -> str:
        return self._vars[name].unit

    def value(self, name: str) -> np.ndarray:
        return self._vars[name].value

    def value_at_indices(self, name: str, dest: np.ndarray, indices: np.ndarray) -> np.ndarray:
        if dest.shape[0] < indices.shape[0]:
            raise ValueError("dest smaller than indices")
        dest[: indices.shape[0]] = self.value(name)[indices]
        return dest

    def set_value(self, name: str, value) -> None:
        self._vars[name].value[:] = value

    def bind(self, name: str, array: np.ndarray) -> None:
        """Back a variable by `array` (e.g. one row of a block the engine fills
        in one transfer), keeping its current values."""
        array[:] = self._vars[name].value
        self._vars[name].value = array

    def set_value_at_indices(self, name: str, inds: np.ndarray, src: np.ndarray) -> None:
        if src.shape[0] < inds.shape[0]:
            raise ValueError("inds larger than src")
        self.value(name)[inds] = src[: inds.shape[0]]

    def names(self) -> Iterator[str]:
        yield from self._vars

    def vars(self) -> Iterator[Var]:
        yield from self._vars.values()

    def __contains__(self, name: str) -> bool:
        return name in self._vars

    def __iter__(self) -> Iterator[Var]:
        return iter(self.vars())

    def __len__(self) -> int:
        return len(self._vars)


def build_context(vars: Iterable[tuple[str, str]], size: int = 1) -> Context:
    return Context(Var(name=n, unit=u, value=np.zeros(size, dtype=np.float64)) for n, u in vars)
