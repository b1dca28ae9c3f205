"""MI355X-native engine for the topoflow-glacier energy balance.

Drop-in import path of the reference package (src/topoflow_glacier/__init__.py):
``from topoflow_glacier import BmiTopoflowGlacier``.  The per-cell physics runs
in hand-written HIP kernels for gfx950 (``_tfg.so``, C ABI include/tfg.h).
"""

from .bmi.bmi_topoflow_glacier import BmiTopoflowGlacier
from .bmi.logger import configure_logging, logger

__version__ = "0.1.0+mi355x"

__all__ = ["__version__", "BmiTopoflowGlacier", "configure_logging", "logger"]
