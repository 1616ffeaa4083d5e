"""gpmdm_amd -- MI355X-native GPMDM particle-filter inference.

Drop-in for the reference's import surface (``from gpmdm import GPMDM, GPMDM_PF``,
/root/reference/gpmdm/__init__.py:1-2): the same classes, computed by hand-written fp64
HIP kernels for gfx950 in ``libgpmdm_hip.so``.
"""
from .model import GPMDM
from .pf import GPMDM_PF
from .bank import GPMDM_PF_Bank

__all__ = ["GPMDM", "GPMDM_PF", "GPMDM_PF_Bank"]
__version__ = "0.1.0"
