"""GPU (gfx950) operators: the columnar state-store query accelerator."""
from .columnar import ColumnarIndex, Program, Unsupported

__all__ = ["ColumnarIndex", "Program", "Unsupported"]
