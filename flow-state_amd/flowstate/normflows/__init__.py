"""Drop-in for the reference's ``normflows`` surface on the hot path
(NF/normflows/core.py, flows/neural_spline/wrapper.py, Energy/Uniform.py)."""
from . import Energy, flows  # noqa: F401
from .core import NormalizingFlow  # noqa: F401
