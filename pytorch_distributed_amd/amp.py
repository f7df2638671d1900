"""Native dynamic loss scaling (replacement for the reference's "Apex" path).

The reference's ``resnet_ddp_apex.py`` uses ``torch.cuda.amp.GradScaler`` with
defaults (``resnet_ddp_apex.py:107``; ``torch/amp/grad_scaler.py:126-129``):
init scale 2**16, x2 after 2000 consecutive finite steps, x0.5 and skip the
step on inf/nan. :class:`LossScaler` reproduces that state machine with the
same public API (``scale``, ``step``, ``update``, ``unscale_``, ``state_dict``,
``load_state_dict``, ``get_scale``) but keeps all state on the device:

* with the native :class:`~pytorch_distributed_amd.models.native.NativeSGD` the
  non-finite check and the scale update run in ONE kernel (``amp_scan``, csrc/misc.hip:
  its last workgroup publishes found_inf / 1/scale and updates scale + growth tracker),
  and the unscale + conditional skip inside the fused SGD -- two launches, **no host sync
  per step** (GradScaler's ``_maybe_opt_step`` does ``found_inf.item()``,
  ``torch/amp/grad_scaler.py:348-358``, and ``update`` is a third kernel);
* with any other optimizer it falls back to torch's ``_amp_*`` ATen kernels and
  a host sync, exactly like GradScaler.
"""
from __future__ import annotations

from typing import Optional

import torch

__all__ = ["LossScaler"]


class LossScaler:
    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000,
                 enabled: bool = True, device=None) -> None:
        self.enabled = enabled
        self.growth_factor = growth_factor
        self.backoff_factor = backoff_factor
        self.growth_interval = growth_interval
        self._init_scale = init_scale
        self._device = device
        self._scale: Optional[torch.Tensor] = None
        self._growth_tracker: Optional[torch.Tensor] = None
        self._found_inf: Optional[torch.Tensor] = None
        self._unscaled = False
        self._stepped = False
        self._updated_in_step = False   # the fused native step already ran the scale update

    # -- state -----------------------------------------------------------------------------
    def _lazy_init(self, device) -> None:
        if self._scale is None:
            self._scale = torch.full((1,), self._init_scale, dtype=torch.float32, device=device)
            self._growth_tracker = torch.full((1,), getattr(self, "_pending_tracker", 0),
                                              dtype=torch.int32, device=device)
            self._found_inf = torch.zeros((1,), dtype=torch.float32, device=device)

    def get_scale(self) -> float:
        if not self.enabled:
            return 1.0
        return self._init_scale if self._scale is None else float(self._scale.item())

    @property
    def scale_tensor(self) -> torch.Tensor:
        return self._scale

    @property
    def found_inf(self) -> torch.Tensor:
        return self._found_inf

    # -- API -------------------------------------------------------------------------------
    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        if not self.enabled:
            return loss
        self._lazy_init(loss.device)
        return loss * self._scale.to(loss.dtype)

    def _grads(self, optimizer):
        for g in optimizer.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    yield p.grad

    def unscale_(self, optimizer) -> None:
        if not self.enabled or self._unscaled:
            return
        if hasattr(optimizer, "amp_unscale_"):
            optimizer.amp_unscale_(self._scale, self._found_inf)
        else:
            inv = self._scale.double().reciprocal().float()
            self._found_inf.zero_()
            grads = list(self._grads(optimizer))
            if grads:
                torch._amp_foreach_non_finite_check_and_unscale_(grads, self._found_inf, inv)
        self._unscaled = True

    def step(self, optimizer, *args, **kwargs):
        if not self.enabled:
            return optimizer.step(*args, **kwargs)
        if self._scale is None:
            return optimizer.step(*args, **kwargs)
        if self._updated_in_step:
            # the fused native step already scanned for infs AND moved the scale/growth tracker
            # this iteration; a second optimizer would unscale by the updated scale (GradScaler
            # updates once per iteration, in update())
            raise RuntimeError("LossScaler.step() called twice before update(): the fused native "
                               "step updates the loss scale in-kernel; use one native optimizer per "
                               "iteration or call update() between steps")
        self._stepped = True
        if hasattr(optimizer, "step_amp") and not self._unscaled:
            # fused: inf check + scale update (one kernel), unscale + conditional step in the SGD
            self._updated_in_step = True
            return optimizer.step_amp(self._scale, self._found_inf, self._growth_tracker,
                                      self.growth_factor, self.backoff_factor,
                                      self.growth_interval)
        self.unscale_(optimizer)
        if hasattr(optimizer, "step_if_finite"):
            return optimizer.step_if_finite(self._found_inf)
        if self._found_inf.item() == 0:                      # GradScaler semantics: host sync
            return optimizer.step(*args, **kwargs)
        return None

    def update(self, new_scale: Optional[float] = None) -> None:
        if not self.enabled or self._scale is None:
            return
        if new_scale is not None:
            self._scale.fill_(float(new_scale))
        elif not self._updated_in_step:
            torch._amp_update_scale_(self._scale, self._growth_tracker, self._found_inf,
                                     self.growth_factor, self.backoff_factor, self.growth_interval)
        if not self._updated_in_step:
            self._found_inf.zero_()     # (the native scan republishes it every step)
        self._unscaled = False
        self._stepped = False
        self._updated_in_step = False

    def state_dict(self) -> dict:
        if not self.enabled:
            return {}
        return {
            "scale": self.get_scale(),
            "growth_factor": self.growth_factor,
            "backoff_factor": self.backoff_factor,
            "growth_interval": self.growth_interval,
            "_growth_tracker": 0 if self._growth_tracker is None else int(self._growth_tracker.item()),
        }

    def load_state_dict(self, sd: dict) -> None:
        if not sd:
            return
        self._init_scale = float(sd["scale"])
        self.growth_factor = float(sd["growth_factor"])
        self.backoff_factor = float(sd["backoff_factor"])
        self.growth_interval = int(sd["growth_interval"])
        if self._scale is not None:
            self._scale.fill_(self._init_scale)
            self._growth_tracker.fill_(int(sd["_growth_tracker"]))
        else:
            self._pending_tracker = int(sd["_growth_tracker"])
