from . import Samplers, stats  # noqa: F401  (ODElib/Statistics/__init__.py:1)
