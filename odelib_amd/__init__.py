"""odelib_amd — MI355X-native batched ODE-in-MCMC engine with ODElib's API.

    from odelib_amd import ModelFramework, parameter      # as `import ODElib`

Compute runs only in libodelib_amd.so (HIP, gfx950); see DESIGN.md.
"""
from . import Statistics  # noqa: F401
from .Framework import ModelFramework, parameter, rawstats  # noqa: F401
from .engine import Engine, FitProblem  # noqa: F401

__version__ = "0.1.0"
