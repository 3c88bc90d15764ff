"""Adam on the device in one launch (ngnn_adam_step): the update over every
parameter tensor; its last workgroup advances the step count.

Same rule and hyper-parameters as ``torch.optim.Adam`` (the reference's
optimiser, model.py:66-69; amsgrad / maximize / foreach variants not
offered); the step count is a device tensor, so the step is capturable in a
HIP graph (``ngnn.graphs.GraphedTrainStep``).  State keys follow torch:
``step``, ``exp_avg``, ``exp_avg_sq``.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


# (gate word, generation word) of the graph slot whose step is being
# captured (ngnn.graphs sets it around a one-rank capture): the captured
# Adam launch skips the update of a block that broke the slot's contract
# (ABI 20; include/ngnn.h ngnn_adam_step)
_slot_gate = None


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      capturable=True))
        self._tickets: dict = {}  # step tensor address -> device ticket
        # per group: (parameter addresses, the launch's pointer arrays) -- the
        # eager step is host-bound, and only the gradient addresses change
        # from step to step
        self._arrays: dict = {}

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            # (address, numel, dtype, contiguity) per parameter: a parameter
            # replaced by one of another size or dtype that the caching
            # allocator placed at the same address re-runs the checks and
            # rebuilds the arrays
            pkey = tuple((p.data_ptr(), p.numel(), p.dtype, p.is_contiguous()) for p in ps)
            cached = self._arrays.get(gi)
            if cached is None or cached[0][0] != pkey:
                cached = None
                for p in ps:  # (the parameters' own checks: once per parameter set)
                    if not p.is_cuda or p.dtype not in (torch.float32, torch.bfloat16) \
                            or not p.is_contiguous():
                        raise RuntimeError("ngnn.optim.Adam: contiguous float32 / bfloat16 GPU "
                                           "parameters only")
            for p in ps:
                g = p.grad
                if g.dtype != p.dtype:
                    raise RuntimeError("ngnn.optim.Adam: gradient dtype differs from the parameter")
                if g.is_sparse:
                    raise RuntimeError("ngnn.optim.Adam: dense gradients only")
            st0 = self.state[ps[0]]
            if "step" not in st0:
                step = torch.zeros((), dtype=torch.float32, device=ps[0].device)
                for p in ps:
                    st = self.state[p]
                    st["step"] = step  # one device counter per group
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
            step = self.state[ps[0]]["step"]
            ticket = self._tickets.get(step.data_ptr())
            if ticket is None:  # zero once; the kernel re-zeroes it after every use
                ticket = torch.zeros(1024, dtype=torch.int32, device=step.device)  # (ABI 21: two levels, a line per group)
                self._tickets[step.data_ptr()] = ticket
            grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in ps]
            n = len(ps)
            G = (ctypes.c_void_p * n)(*[g.data_ptr() for g in grads])
            sts = [self.state[p] for p in ps]
            # (the moments' addresses belong to the key: a state reload --
            # load_state_dict -- makes new tensors)
            key = (pkey, tuple(st["exp_avg"].data_ptr() for st in sts),
                   tuple(st["exp_avg_sq"].data_ptr() for st in sts))
            if cached is None or cached[0] != key:
                cached = (key, (ctypes.c_void_p * n)(*[k[0] for k in pkey]),
                          (ctypes.c_void_p * n)(*key[1]), (ctypes.c_void_p * n)(*key[2]),
                          (ctypes.c_int64 * n)(*[p.numel() for p in ps]),
                          (ctypes.c_int32 * n)(*[_lib.BF16 if p.dtype == torch.bfloat16 else _lib.F32
                                                 for p in ps]))
                self._arrays[gi] = cached
            _, P, M, V, N, D = cached
            b1, b2 = group["betas"]
            _lib.check(lib.ngnn_adam_step(n, P, G, M, V, N, D, step.data_ptr(), ticket.data_ptr(),
                                          float(group["lr"]),
                                          float(b1), float(b2), float(group["eps"]),
                                          float(group["weight_decay"]),
                                          *(_slot_gate if _slot_gate is not None else (None, None)),
                                          _lib.stream_handle(ps[0].device)), "ngnn_adam_step")
        return loss
