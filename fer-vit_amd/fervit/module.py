"""FerModule: nn.Module base that owns (or shares) a FlatParams store.

The outermost FerModule that runs a forward owns the flat buffers of all its
parameters (nested FerModules share the owner's). The store is (re)built lazily on
the module's device, so `model.cuda()` / `model.to(dev)` keep working: the
Parameter objects stay the same (optimizers hold them), only their `.data` is
re-pointed at the flat views.
"""
from __future__ import annotations

import weakref
from typing import List, Optional

import torch
import torch.nn as nn

from .runtime import FlatParams, default_precision


class FerModule(nn.Module):
    def __init__(self):
        super().__init__()
        object.__setattr__(self, "_fer_flat", None)
        object.__setattr__(self, "_fer_owner", None)
        object.__setattr__(self, "fer_precision", default_precision())

    # ---- ordering hook: modules may reorder their parameters in the flat buffer
    def fer_param_order(self) -> List[nn.Parameter]:
        seen, out = set(), []
        for m in self.modules():
            hook = getattr(m, "_fer_local_order", None)
            if hook is not None:
                for p in hook():
                    if id(p) not in seen:
                        seen.add(id(p))
                        out.append(p)
        for p in self.parameters():
            if id(p) not in seen:
                seen.add(id(p))
                out.append(p)
        return out

    def _apply(self, fn, recurse=True):
        r = super()._apply(fn, recurse)
        for m in self.modules():
            if isinstance(m, FerModule):
                object.__setattr__(m, "_fer_flat", None)
                object.__setattr__(m, "_fer_owner", None)
        return r

    def fer_flat(self) -> FlatParams:
        owner = self._fer_owner() if self._fer_owner is not None else None
        if owner is not None and owner._fer_flat is not None:
            flat = owner._fer_flat
            if not flat.owner_active:
                # a child module run on its own (e.g. `model.backbone(x)`), not inside the owner's
                # forward: start a pass so the bf16 shadow re-checks the parameters' versions
                # (they may have been changed in place since the owner's last pass)
                flat.begin_pass()
            return flat
        if self._fer_flat is not None:
            self._fer_flat.begin_pass()
            return self._fer_flat
        if self._fer_flat is None:
            params = self.fer_param_order()
            if not params:
                raise RuntimeError("fervit: module has no parameters")
            if not params[0].is_cuda:
                raise RuntimeError("fervit: move the model to a ROCm device first (no CPU path)")
            flat = FlatParams(params)
            object.__setattr__(self, "_fer_flat", flat)
            for h in getattr(self, "_fer_hooks", ()):
                h.remove()

            def _enter(_m, _inp, flat=flat):
                flat.owner_active = True

            def _leave(_m, _inp, _out, flat=flat):
                flat.owner_active = False

            object.__setattr__(self, "_fer_hooks", (self.register_forward_pre_hook(_enter),
                                                    self.register_forward_hook(_leave, always_call=True)))
            ref = weakref.ref(self)
            for m in self.modules():
                if m is not self and isinstance(m, FerModule):
                    object.__setattr__(m, "_fer_owner", ref)
                    object.__setattr__(m, "_fer_flat", None)
        return self._fer_flat

    def set_precision(self, precision: str):
        """'bf16' (MFMA fast path, fp32 accumulation) or 'fp32' (exact parity path)."""
        if precision not in ("bf16", "fp32"):
            raise ValueError(precision)
        for m in self.modules():
            if isinstance(m, FerModule):
                object.__setattr__(m, "fer_precision", precision)
        return self

    def compute_dtype(self) -> torch.dtype:
        return torch.bfloat16 if self.fer_precision == "bf16" else torch.float32

    @staticmethod
    def need_grad(x: Optional[torch.Tensor], params) -> bool:
        if not torch.is_grad_enabled():
            return False
        if x is not None and x.requires_grad:
            return True
        return any(p.requires_grad for p in params)
