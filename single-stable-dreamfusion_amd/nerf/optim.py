"""GradScaler + Adam step of the train loop as one native call (csrc/optim.hip).

The reference steps `scaler.step(optimizer); scaler.update()` with
torch.optim.Adam (nerf/utils.py:708-713).  With a fused torch Adam that is
~15 launches and ~0.4 ms of host Python per step, which on a graph-replayed
step is the host's largest cost.  `NativeAdamAmp.step()` does the same update
with three launches: the non-finite check, the Adam update of every tensor
(skipped on inf) and the scale / step-count update.  It reads and writes the
torch objects' own state (Adam's `step` / `exp_avg` / `exp_avg_sq` per
parameter, GradScaler's `_scale` / `_growth_tracker`), so state_dict /
load_state_dict and checkpoints are unchanged.

Without a GradScaler (bf16 autocast, the C5 option: torch.amp.GradScaler is
disabled) the same launches run against a private unit scale that never
changes: the update is torch Adam's, except that a step whose gradients are
not finite is skipped instead of writing non-finite parameters.
"""
import ctypes

import torch

import _dfhip

_MAX_TENSORS = 24


def eligible(optimizer, scaler, unit_scale=False):
    """True when NativeAdamAmp reproduces scaler.step(optimizer) +
    scaler.update().  A disabled GradScaler is accepted only with
    unit_scale=True (the bf16 trainer): the unit-scale form skips a step with
    non-finite gradients where torch Adam would write them into the
    parameters, so plain fp32 training keeps torch's optimizer."""
    if not isinstance(optimizer, torch.optim.Adam) or type(optimizer) is not torch.optim.Adam:
        return False
    if scaler is None or (not scaler.is_enabled() and not unit_scale):
        return False
    if scaler.is_enabled() and (scaler._growth_factor, scaler._backoff_factor) != (2.0, 0.5):
        return False
    n = 0
    for g in optimizer.param_groups:
        if g.get("amsgrad") or g.get("maximize") or g.get("differentiable"):
            return False
        if torch.is_tensor(g["lr"]):
            return False
        for p in g["params"]:
            if not (p.is_cuda and p.dtype == torch.float32):
                return False
            n += 1
    return 0 < n <= _MAX_TENSORS


class NativeAdamAmp:
    def __init__(self, optimizer, scaler):
        self.optimizer = optimizer
        self.scaler = scaler
        self.found_inf = None
        self._unit = None  # (scale 1.0, growth tracker) when the scaler is disabled
        self._ptr_key = None
        self._arrays = None

    def _state(self, p):
        st = self.optimizer.state[p]
        if not st:  # torch fused Adam's lazy init (adam.py _init_group)
            st["step"] = torch.tensor(0.0, dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        elif not st["step"].is_cuda:
            st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
        return st

    def step(self):
        """One scaler.step(optimizer) + scaler.update() (parameters without a
        gradient are skipped, as torch does)."""
        sc = self.scaler
        if sc.is_enabled():
            if sc._scale is None:
                return  # scale() never called: nothing was back-propagated
            scale, tracker = sc._scale, sc._growth_tracker
            growth, backoff, interval = sc._growth_factor, sc._backoff_factor, sc._growth_interval
        else:
            if self._unit is None:
                dev = next(p.device for g in self.optimizer.param_groups for p in g["params"])
                self._unit = (torch.ones(1, dtype=torch.float32, device=dev),
                              torch.zeros(1, dtype=torch.int32, device=dev))
            scale, tracker = self._unit
            growth, backoff, interval = 1.0, 1.0, 1 << 30
        if self.found_inf is None:
            self.found_inf = torch.zeros(1, dtype=torch.float32, device=scale.device)
        # fast path: same parameters / gradient buffers as last step (the graph-
        # replayed step keeps its gradients in place) -> only the lrs are new
        # (a reloaded optimizer state is a new dict: its identity is part of the key)
        key = (id(self.optimizer.state), len(self.optimizer.state),
               *(p.grad.data_ptr() if p.grad is not None else 0
                 for g in self.optimizer.param_groups for p in g["params"]))
        if key != self._ptr_key:
            self._rebuild(key)
        if self._arrays is None:
            return
        n, P, G, M, V, S, N, B1, B2, E, WD, groups = self._arrays
        lr = (ctypes.c_float * n)(*[float(self.optimizer.param_groups[i]["lr"]) for i in groups])
        rc = self._fn(n, P, G, M, V, S, N, lr, B1, B2, E, WD, scale.data_ptr(),
                      tracker.data_ptr(), self.found_inf.data_ptr(), float(growth),
                      float(backoff), int(interval), _dfhip.stream())
        if rc != 0:
            raise RuntimeError(f"dfhip_adam_amp_step failed ({rc}): "
                               f"{_dfhip.load().dfhip_last_error().decode()}")
        self.optimizer._opt_called = True  # what LRScheduler checks for "stepped"

    def group_lrs(self):
        """Current learning rate of every param group (host floats)."""
        return [float(g["lr"]) for g in self.optimizer.param_groups]

    def device_lr_launch(self, lr_dev):
        """The step as a closure over device-resident learning rates (tensor k
        reads lr_dev[its group]): captured once in the native train step's
        HIP graph (nerf/graph.py), while the prologue launch writes lr_dev
        every step from group_lrs().  Built against the current gradient
        buffers and optimizer state, like step()'s fast path."""
        sc = self.scaler
        if sc.is_enabled():
            if sc._scale is None:
                raise RuntimeError("device_lr_launch: the GradScaler has no scale yet")
            scale, tracker = sc._scale, sc._growth_tracker
            growth, backoff, interval = sc._growth_factor, sc._backoff_factor, sc._growth_interval
        else:
            if self._unit is None:
                dev = next(p.device for g in self.optimizer.param_groups for p in g["params"])
                self._unit = (torch.ones(1, dtype=torch.float32, device=dev),
                              torch.zeros(1, dtype=torch.int32, device=dev))
            scale, tracker = self._unit
            growth, backoff, interval = 1.0, 1.0, 1 << 30
        if self.found_inf is None:
            self.found_inf = torch.zeros(1, dtype=torch.float32, device=scale.device)
        key = (id(self.optimizer.state), len(self.optimizer.state),
               *(p.grad.data_ptr() if p.grad is not None else 0
                 for g in self.optimizer.param_groups for p in g["params"]))
        self._rebuild(key)
        if self._arrays is None:
            raise RuntimeError("device_lr_launch: no parameter has a gradient")
        if len(self.optimizer.param_groups) > 8:
            raise RuntimeError("device_lr_launch: at most 8 param groups")
        n, P, G, M, V, S, N, B1, B2, E, WD, groups = self._arrays
        slots = (ctypes.c_int32 * n)(*groups)
        fn = _dfhip.load().dfhip_adam_amp_step_lr_dev
        found_inf, opt = self.found_inf, self.optimizer
        keep = (slots, self._arrays, lr_dev, scale, tracker, found_inf)

        def launch():
            rc = fn(n, P, G, M, V, S, N, slots, lr_dev.data_ptr(), B1, B2, E, WD,
                    scale.data_ptr(), tracker.data_ptr(), found_inf.data_ptr(), float(growth),
                    float(backoff), int(interval), _dfhip.stream())
            if rc != 0:
                raise RuntimeError(f"dfhip_adam_amp_step_lr_dev failed ({rc}): "
                                   f"{_dfhip.load().dfhip_last_error().decode()}")
            opt._opt_called = True
        launch.keep = keep  # the host arrays the launch reads stay alive with it
        return launch

    def _rebuild(self, key):
        ts = []
        for gi, g in enumerate(self.optimizer.param_groups):
            b1, b2 = g["betas"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self._state(p)
                ts.append((p, p.grad, st["exp_avg"], st["exp_avg_sq"], st["step"], gi, b1, b2,
                           g["eps"], g["weight_decay"]))
        self._ptr_key = key
        if not ts:
            self._arrays = None
            return
        n = len(ts)
        vp = ctypes.c_void_p * n
        f = ctypes.c_float * n
        ptrs = [vp(*[t[i].data_ptr() for t in ts]) for i in range(5)]
        hyper = [f(*[float(t[i]) for t in ts]) for i in range(6, 10)]
        self._arrays = (n, *ptrs, (ctypes.c_uint64 * n)(*[t[0].numel() for t in ts]), *hyper,
                        [t[5] for t in ts])
        self._fn = _dfhip.load().dfhip_adam_amp_step
