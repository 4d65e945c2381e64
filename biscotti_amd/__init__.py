"""biscotti_amd -- MI355X-native Multi-Krum engine for Biscotti's verifier path.

The engine is libbk.so (HIP kernels for gfx950 + a C ABI, include/bk.h).  This
package holds its build recipe, the ctypes binding, the host-side mirror of the
reference's verifier interface (krum.py) and the dimension-sharded multi-GPU
driver (dist.py).
"""
from . import _lib  # noqa: F401
from .krum import (Engine, KRUMValidator, Update, default_engine, get_krum_scores,  # noqa: F401
                   krum, krum_mean)

__version__ = "0.1.0"
