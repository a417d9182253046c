"""leanfe_amd: MI355X-native (gfx950) backend for leanfe's fixed-effects
demean + solve hot path.  ``leanfe(..., backend="hip")`` mirrors the reference
``leanfe()`` API (jorgenhost/leanfe, python/leanfe/__init__.py)."""
from .api import leanfe
from .formula import FormulaComponents, parse_formula
from .hip_impl import leanfe_hip
from .result import LeanFEResult

__version__ = "0.1.0"
__all__ = ["leanfe", "leanfe_hip", "parse_formula", "FormulaComponents", "LeanFEResult"]
