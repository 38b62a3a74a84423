"""The reference loop's clip + optimizer step as one HIP launch.

train_flow.py:265-267 runs ``torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)`` and then
``optimizer.step()`` of ``torch.optim.Adam`` (configs/train_SNN.yml:45-47: Adam, lr 2e-4).
``ClipAdam`` is that pair: ``torch.optim.Adam``'s constructor and per-parameter state
(``step``, ``exp_avg``, ``exp_avg_sq``) with an optional ``max_norm``; ``step()`` clips the gradients
in place and applies Adam with the reference's arithmetic (``_single_tensor_adam``: ``lerp_`` for the
first moment, fp64 bias corrections) in ``snnflow_clip_adam``, one block over the engine's flat
gradient buffer (FireNetEngine hands every parameter's gradient out as a view of one buffer).  The
moments live in two persistent flat buffers (parameter order; the gradient buffer may move between
steps, e.g. one per captured HIP graph); ``self.state[p]`` holds views of them, so ``state_dict()``
/ ``load_state_dict()`` round-trip like torch's Adam (loaded states are copied back into the flat
buffers on the next step).  No CPU path: gradients must be the engine's
flat CUDA buffer (``snnflow.dp.flat_grad_buffer``)."""
import ctypes

import torch

from . import _lib
from .dp import flat_grad_buffer


class ClipAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_norm=None,
                 clip_eps=1e-6):
        if lr < 0.0 or eps < 0.0 or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0 or weight_decay < 0.0:
            raise ValueError("ClipAdam: invalid hyper-parameter")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, max_norm=max_norm,
                        clip_eps=clip_eps)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("ClipAdam: one parameter group (the clip norm spans all parameters)")
        self._moments = None     # (parameter ids, exp_avg, exp_avg_sq, step, state offsets)
        self.last_total_norm = None

    def _state(self, params):
        """Persistent flat moment buffers (parameter order) and the device step counter; the
        per-parameter state entries are views of them.  Rebuilt only when the parameter set
        changes or a loaded state dict replaced the views (values copied over)."""
        ids = tuple(id(p) for p in params)
        m = self._moments
        if m is not None and m[0] == ids and all(self.state[p].get("exp_avg") is not None and
                                                 self.state[p]["exp_avg"].data_ptr() == m[1].data_ptr() + 4 * o
                                                 for p, o in zip(params, m[4])):
            return m
        dev = params[0].device
        offs, total = [], 0
        for p in params:
            offs.append(total)
            total += p.numel()
        ea = torch.zeros(total, device=dev)
        es = torch.zeros(total, device=dev)
        step = torch.zeros((), dtype=torch.float32, device=dev)
        for p, o in zip(params, offs):
            st, n = self.state[p], p.numel()
            if "exp_avg" in st:  # carried over (another parameter set, or a loaded state dict)
                ea[o:o + n].copy_(st["exp_avg"].reshape(-1))
                es[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                step.copy_(torch.as_tensor(st["step"], dtype=torch.float32))
            st["exp_avg"] = ea[o:o + n].view_as(p)
            st["exp_avg_sq"] = es[o:o + n].view_as(p)
            st["step"] = step
        self._moments = (ids, ea, es, step, offs)
        return self._moments

    def zero_grad(self, set_to_none=True):
        """torch.optim.Optimizer.zero_grad without its per-call profiler / foreach machinery (the
        eager per-window loop calls it once per step: ~60 us of host time for ~40 parameters)."""
        for p in self.param_groups[0]["params"]:
            if p.grad is None:
                continue
            if set_to_none:
                p.grad = None
            else:
                if p.grad.grad_fn is not None:
                    p.grad.detach_()
                else:
                    p.grad.requires_grad_(False)
                p.grad.zero_()

    def _fast_args(self, params, grads):
        """The launch arguments of the previous step, reused when the parameter set, the hyper-
        parameters, the moments and the gradient layout relative to the buffer start are unchanged
        (the eager loop gets a new gradient buffer every step, at the same relative offsets).  One pass
        over the parameters (the per-window loop calls this once per step)."""
        c = self.__dict__.get("_args_cache")
        if c is None or c[0] != tuple(map(id, params)) or self._moments is None or c[4] is not self._moments:
            return None
        ptrs = tuple(g.data_ptr() for g in grads)
        base = min(ptrs)
        if (c[1] != tuple(x - base for x in ptrs) or c[2] != self._hyper() or c[5] != grads[0].device
                or c[6] != tuple(p.data_ptr() for p in params)):
            return None
        return c[3], base

    def state_dict(self):
        """torch.optim.Adam's state-dict form: every parameter's ``step`` is its own CPU float32
        tensor (a copy of the shared device counter, which stays internal).  A shared tensor would
        be incremented once per parameter by torch's Adam after ``load_state_dict`` (the reference
        saves ``optimizer.state_dict()`` in its checkpoints, train_flow.py:131-150)."""
        sd = super().state_dict()
        state = {}
        for k, st in sd["state"].items():
            st = dict(st)  # super() hands out this optimizer's own per-parameter dicts
            if isinstance(st.get("step"), torch.Tensor):
                st["step"] = st["step"].detach().to("cpu", torch.float32, copy=True)
            state[k] = st
        sd["state"] = state
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._args_cache = None  # the loaded moments replace the flat buffers' views (re-read by _state)

    def _hyper(self):
        g = self.param_groups[0]
        return (g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"], g["max_norm"], g["clip_eps"])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        group = self.param_groups[0]
        allp = group["params"]
        grads = [p.grad for p in allp]
        if any(g is None for g in grads):
            params = [p for p, g in zip(allp, grads) if g is not None]
            grads = [g for g in grads if g is not None]
        else:
            params = allp
        if not params:
            return loss
        fast = self._fast_args(params, grads)
        if fast is not None:
            a, base = fast
            a.grad = base
            _lib.call("clip_adam", _lib.lib.snnflow_clip_adam, ctypes.byref(a), _lib.stream_ptr(params[0].device))
            return loss
        if len(params) > _lib.ADAM_MAX_TENSORS:
            raise _lib.SnnflowError(f"ClipAdam: at most {_lib.ADAM_MAX_TENSORS} parameter tensors")
        grad = flat_grad_buffer(params)
        if grad is None or not grad.is_cuda or grad.dtype != torch.float32:
            raise _lib.SnnflowError("ClipAdam: the gradients must be the engine's flat fp32 CUDA buffer")
        if grad.numel() > _lib.CLIP_ADAM_MAX_N:
            raise _lib.SnnflowError("ClipAdam: more than SNNFLOW_CLIP_ADAM_MAX_N parameters")
        for p in params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device != grad.device:
                raise _lib.SnnflowError("ClipAdam: fp32 contiguous parameters on the gradients' device")
        _, ea, es, step, offs = self._state(params)
        if self.last_total_norm is None or self.last_total_norm.device != grad.device:
            self.last_total_norm = torch.zeros((), device=grad.device)
            self._scratch = torch.empty(513, dtype=torch.float64, device=grad.device)  # SNNFLOW_CLIP_SCRATCH
        a = _lib.ClipAdamArgs()
        a.grad, a.exp_avg, a.exp_avg_sq, a.step = grad.data_ptr(), ea.data_ptr(), es.data_ptr(), step.data_ptr()
        a.total_out, a.n = self.last_total_norm.data_ptr(), grad.numel()
        a.lr = float(group["lr"])
        a.beta1, a.beta2 = float(group["betas"][0]), float(group["betas"][1])
        a.eps, a.weight_decay = float(group["eps"]), float(group["weight_decay"])
        mn = group["max_norm"]
        a.max_norm, a.clip_eps = (float(mn) if mn is not None else 0.0), float(group["clip_eps"])
        a.ntensors = len(params)
        a.scratch = self._scratch.data_ptr()
        base = grad.data_ptr()
        order = sorted(range(len(params)), key=lambda k: params[k].grad.data_ptr())  # gradient order
        for i, k in enumerate(order):
            p, t = params[k], a.t[i]
            t.param, t.offset, t.state_offset, t.numel = p.data_ptr(), (p.grad.data_ptr() - base) // 4, offs[k], p.numel()
        _lib.call("clip_adam", _lib.lib.snnflow_clip_adam, ctypes.byref(a), _lib.stream_ptr(grad.device))
        self._args_cache = (tuple(map(id, params)), tuple(p.grad.data_ptr() - base for p in params), self._hyper(), a,
                            self._moments, grad.device, tuple(p.data_ptr() for p in params))
        return loss
