"""Minimal BMI base (counterpart of bmi/bmi_base.py).

The CSDMS ``bmipy.Bmi`` ABC is used when it is installed; otherwise a plain
object base stands in (bmipy carries no arithmetic).  Methods this model does
not support raise NotImplementedError, as in the reference; the grid
topology the reference leaves unimplemented there is BmiTopoflowGlacier's.
"""

from __future__ import annotations

try:  # pragma: no cover - depends on the environment
    from bmipy import Bmi as _Bmi
except ImportError:  # bmipy 2.0.1 is not installable offline
    class _Bmi:  # type: ignore[no-redef]
        pass

__all__ = ["BmiBase"]


class BmiBase(_Bmi):
    def get_component_name(self) -> str:
        return self.__class__.__name__

    def get_value(self, name, dest):
        dest[:] = self.get_value_ptr(name)
        return dest

    def get_var_nbytes(self, name) -> int:
        return self.get_value_ptr(name).nbytes

    def get_var_type(self, name) -> str:
        return str(self.get_value_ptr(name).dtype)
