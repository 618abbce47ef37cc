"""Fused gradient-clip + Adam on the MI355X (one norm pass + one update pass over all tensors).

Replaces Lightning's ``gradient_clip_val`` (torch clip_grad_norm_, configs/base_training.yaml:51)
followed by ``torch.optim.Adam(lr, weight_decay)`` (base_training.yaml:56-59, instantiated at
src/training/engine.py:300).  Numerics follow torch's single-tensor Adam: L2 decay added to the
(clipped) gradient, ``exp_avg.lerp_(g, 1-beta1)``, ``exp_avg_sq = beta2*v + (1-beta2) g^2``,
``p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)``.  The clip coefficient is computed on the device,
so the step never synchronises with the host.
"""
from __future__ import annotations

import math
import weakref

import numpy as np
import torch
from torch.optim.optimizer import register_optimizer_step_pre_hook

from ..miaudio import kernels as K
from ..miaudio import lib as L


def _materialise_for_other_optimizers(opt, args, kwargs):
    """Global optimizer step pre-hook: an optimizer other than FusedAdam about to step a parameter whose
    weight gradient was deferred gets the gradient materialised into ``p.grad`` first (the same GEMM), and
    the parameter stops deferring -- so torch.optim.Adam built after a FusedAdam updates FC1 from its
    first step instead of silently skipping it."""
    if isinstance(opt, FusedAdam):
        return
    for grp in opt.param_groups:
        for p in grp["params"]:
            if getattr(p, "_mia_fused_adam", None) is not None:
                p._mia_fused_adam = None
            if getattr(p, "_mia_deferred", None) is not None:
                K.materialise_deferred_grad(p)


register_optimizer_step_pre_hook(_materialise_for_other_optimizers)


class FusedAdam(torch.optim.Optimizer):
    # torch.optim.Adam options the fused kernel implements only at their defaults
    _DEFAULT_ONLY = {"amsgrad": False, "maximize": False, "capturable": False, "differentiable": False,
                     "decoupled_weight_decay": False}
    _IGNORED = ("foreach", "fused")  # implementation selectors of torch's Adam: this is the fused one

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, clip: float = 0.0, **kw):
        for k, v in kw.items():
            if k in self._IGNORED:
                continue
            if k not in self._DEFAULT_ONLY:
                raise TypeError(f"FusedAdam got an unexpected keyword argument {k!r}")
            if bool(v) != self._DEFAULT_ONLY[k]:
                raise ValueError(f"FusedAdam implements torch.optim.Adam with {k}={self._DEFAULT_ONLY[k]} only "
                                 f"(got {k}={v}); use torch.optim.Adam for this option")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.clip = float(clip or 0.0)
        self.last_total_norm = None
        self.last_precomputed = 0  # tensors whose norm came from their GEMM's per-tile sums (last step)
        self._table_key = None     # pointer table of the last step (host pinned + device copy)
        self._table = None
        self.table_builds = 0
        self.last_deferred = 0     # weight gradients applied by their fused Adam GEMM (last step)
        ref = weakref.ref(self)
        for p in self.param_groups[0]["params"]:
            # models may defer a wide Linear's weight gradient to this optimizer (K.defer_weight_grad) while
            # it is alive; another optimizer stepping the parameter first materialises the gradient
            # (_materialise_for_other_optimizers), and takes the parameter over
            p._mia_fused_adam = ref

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if len(self.param_groups) != 1:
            raise RuntimeError("FusedAdam drives one parameter group (the reference configures one)")
        grp = self.param_groups[0]
        ps = [p for p in grp["params"] if p.grad is not None or getattr(p, "_mia_deferred", None) is not None]
        if not ps:
            return loss
        dev = ps[0].device
        L.require_device(ps[0], "FusedAdam")
        deferred = [getattr(p, "_mia_deferred", None) for p in ps]
        for p, d in zip(ps, deferred):
            shard = getattr(p, "_mia_shard", None)
            if shard is not None and (d is None or "row0" not in d):
                # the last steps updated only this rank's row slice (GradAllReducer fc1_exchange="shard"):
                # bring every rank's rows of the parameter and moments back before a whole-tensor update
                shard[0].sync_param(p)
            if d is not None and p.grad is not None:
                raise RuntimeError("a parameter has both a gradient and a deferred weight gradient")
            if p.dtype != torch.float32 or (d is None and p.grad.dtype != torch.float32):
                raise TypeError("FusedAdam keeps f32 master parameters and gradients")
            st = self.state[p]
            if not st:
                st["step"] = torch.zeros((), dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["step"] += 1
        # torch's Adam keeps one step count per parameter; they differ only after a parameter missed
        # gradients, and then the kernel takes the per-tensor counts
        steps = [int(self.state[p]["step"].item()) for p in ps]
        step = steps[0]
        per_tensor_steps = any(v != step for v in steps)
        gs = [None if d is not None else (p.grad if p.grad.is_contiguous() else p.grad.contiguous())
              for p, d in zip(ps, deferred)]
        # parameters with a live bf16 operand copy (K.bf16_shadow) get it rewritten in the update pass
        shadows = [getattr(p, "_mia_bf16", None) if getattr(p, "_mia_bf16_ver", None) == p._version else None
                   for p in ps]
        # gradients whose producing GEMM left per-tile sums of squares (K.sqsum_slots) skip the norm read;
        # a deferred one is in the table with a NULL gradient: norm from its sums, update by its GEMM
        pre = [d["sq"] if d is not None else K.valid_sqsum(p, g) for p, g, d in zip(ps, gs, deferred)]
        self.last_precomputed = sum(q is not None for q in pre)
        self.last_deferred = sum(d is not None for d in deferred)
        have_pre = self.last_precomputed > 0
        rows = [[p.data_ptr() for p in ps], [0 if g is None else g.data_ptr() for g in gs],
                [self.state[p]["exp_avg"].data_ptr() for p in ps],
                [self.state[p]["exp_avg_sq"].data_ptr() for p in ps],
                [0 if sh is None else sh.data_ptr() for sh in shadows],
                [p.numel() for p in ps]]
        if have_pre:
            rows += [[0 if q is None else q.data_ptr() for q in pre], [0 if q is None else q.numel() for q in pre]]
        # the device pointer table is rebuilt only when a pointer changed: in steady state the caching
        # allocator hands every gradient the same storage step after step
        key = tuple(map(tuple, rows))
        if key != self._table_key:
            host = torch.tensor(rows, dtype=torch.int64).pin_memory()
            self._table = (host, host.to(dev, non_blocking=True))
            self._table_key = key
            self.table_builds += 1
        table = self._table[1]
        steps_host = torch.tensor(steps, dtype=torch.int32).pin_memory() if per_tensor_steps else None
        steps_dev = steps_host.to(dev, non_blocking=True) if per_tensor_steps else None
        n = len(ps)
        lib = L.load()
        ws = K.workspace(lib.mia_adam_workspace_bytes(n), dev, "adam")
        tot = torch.empty(1, dtype=torch.float32, device=dev)
        b1, b2 = grp["betas"]
        # algorithmic HBM bytes: grad read by the norm pass (4 B/param) + Adam's p, g, m, v read and
        # p, m, v written (28 B/param) + the bf16 operand copies rewritten (2 B/param where shadowed)
        # (a sharded deferred gradient: only this rank's rows are updated and read)
        upd = [d["M"] * d["N"] if d is not None else p.numel() for p, d in zip(ps, deferred)]
        nbytes = 32 * sum(upd) + 2 * sum(u for u, sh in zip(upd, shadows) if sh is not None)
        nbytes -= 4 * sum(u for u, q in zip(upd, pre) if q is not None)  # no norm read of those
        for u, d in zip(upd, deferred):  # no gradient read either; the GEMM reads its two bf16 operands
            if d is not None:
                nbytes += -4 * u + 2 * d["K"] * (d["M"] + d["N"])
        with K.probe("optim.step", 0.0, nbytes):
            L.check(lib.mia_clip_adam(table[0].data_ptr(), table[1].data_ptr(), table[2].data_ptr(),
                                      table[3].data_ptr(), table[4].data_ptr(), table[5].data_ptr(), n,
                                      max((p.numel() for p, d in zip(ps, deferred) if d is None), default=1),
                                      max((p.numel() for p, q in zip(ps, pre) if q is None), default=1),
                                      float(grp["lr"]), float(b1), float(b2), float(grp["eps"]),
                                      float(grp["weight_decay"]), step, self.clip, tot.data_ptr(), ws.data_ptr(),
                                      table[6].data_ptr() if have_pre else None,
                                      table[7].data_ptr() if have_pre else None,
                                      steps_dev.data_ptr() if per_tensor_steps else None,
                                      L.stream_ptr()), "mia_clip_adam")
            coef = ws.data_ptr() + int(lib.mia_adam_coef_offset(n))
            for p, d, sh, st in zip(ps, deferred, shadows, steps):
                if d is None:
                    continue
                # the bias corrections exactly as mia_clip_adam forms them: f32 lr / betas, double pow
                lr32, b1_32, b2_32 = (float(np.float32(v)) for v in (grp["lr"], b1, b2))
                lr_bc1 = lr32 / (1.0 - math.pow(b1_32, st))
                bc2_sqrt = math.sqrt(1.0 - math.pow(b2_32, st))
                off = d.get("row0", 0) * d["N"]  # a sharded gradient covers rows [row0, row0 + M) only
                L.check(lib.mia_gemm_adam(d["A"], d["B"], d["M"], d["N"], d["K"], p.data_ptr() + 4 * off,
                                          self.state[p]["exp_avg"].data_ptr() + 4 * off,
                                          self.state[p]["exp_avg_sq"].data_ptr() + 4 * off,
                                          0 if sh is None else sh.data_ptr() + 2 * off, d["N"], coef, lr_bc1,
                                          bc2_sqrt, float(b1), float(b2), float(grp["eps"]),
                                          float(grp["weight_decay"]), L.stream_ptr()),
                        "mia_gemm_adam")
                if "row0" in d:
                    d["shard"].after_shard_update(p, sh, d)
        self.last_total_norm = tot
        for p, sh in zip(ps, shadows):
            if sh is not None:
                p._mia_bf16_ver = p._version  # the copy now matches the updated parameter
        for p in ps:
            p._mia_sqsum = None  # consumed (or stale): the next step's gradient brings its own
            p._mia_deferred = None
        self._keep = (gs, pre, steps_host, steps_dev, deferred)  # alive until the next step (async use)
        return loss
