"""w+ prologue modules (reference `modules/__init__.py`)."""
from .leam import LEAM
from .semantic_pe import SemanticPE
from .layer_wise_norm import LayerWiseNorm

__all__ = ["LEAM", "SemanticPE", "LayerWiseNorm"]
