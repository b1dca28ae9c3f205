"""Minimal BMI base (counterpart of bmi/bmi_base.py).

The CSDMS ``bmipy.Bmi`` ABC is used when it is installed; otherwise a plain
object base stands in (bmipy carries no arithmetic).  Methods this model does
not support raise NotImplementedError, as in the reference.
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

    # grid topology beyond the uniform raster is not modelled
    def get_grid_edge_count(self, grid):
        raise NotImplementedError()

    def get_grid_edge_nodes(self, grid, edge_nodes):
        raise NotImplementedError()

    def get_grid_face_count(self, grid):
        raise NotImplementedError()

    def get_grid_face_edges(self, grid, face_edges):
        raise NotImplementedError()

    def get_grid_face_nodes(self, grid, face_nodes):
        raise NotImplementedError()

    def get_grid_node_count(self, grid):
        raise NotImplementedError()

    def get_grid_nodes_per_face(self, grid, nodes_per_face):
        raise NotImplementedError()

    def get_grid_x(self, grid, x):
        raise NotImplementedError()

    def get_grid_y(self, grid, y):
        raise NotImplementedError()

    def get_grid_z(self, grid, z):
        raise NotImplementedError()
