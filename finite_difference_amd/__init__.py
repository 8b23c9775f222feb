"""MI355X-native Crank-Nicolson finite-difference engine (fdcn).

Drop-in for the time-stepping hot path of rwx-gigaba-sonwabo/Finite_Difference:
the batched CN / Rannacher / knock-out / Ikonen-Toivanen march runs in HIP
kernels for gfx950 (libfdcn.so, C ABI in include/fdcn.h); the pricer façades
keep the reference's constructor arguments and methods.
"""
__version__ = "0.1.0"

from . import capi  # noqa: F401
from .engine import Engine, Solve, Boundary, default_engine  # noqa: F401
