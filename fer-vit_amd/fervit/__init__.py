"""fervit — MI355X-native (gfx950) training path for the FER-ViT models.

Layers: `_lib` (ctypes binding of libfervit.so) -> `ops` (tensor wrappers) ->
`layers` (autograd functions, one per transformer layer) -> `blocks` / `module`
(parameter containers with the reference's names) -> `models_fer_vit`, `modules`
(the reference's public constructors) ; `optim` (fused AdamW), `loss`, `ddp` (RCCL
data parallel).
"""
from .runtime import manual_seed, next_seed

__version__ = "0.1.0"


def library_version() -> str:
    from ._lib import lib

    return lib().fer_version().decode()
