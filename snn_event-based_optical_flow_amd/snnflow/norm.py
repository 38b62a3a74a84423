"""TEBN / MPBN normalisation (``models/SNNtorch_spiking_submodules.py:18-121``) and the 1x1
``ConvLayer`` as standalone HIP ops (csrc/norm.hip).

* ``TEBN``: ``BatchNorm2d(x) * p[t]`` with ``p`` [T, C, 1, 1] learnable, ``p.mean(0)`` when no
  valid time step is given (the reference's cells are always called without one,
  ``models/model.py:172-180``).  Inside a cell the product folds into the BatchNorm affine
  parameters (``weight * p_t``, ``bias * p_t``), so the fused conv/LIF kernels run unchanged and
  autograd carries the gradient to ``bn.weight``, ``bn.bias`` and ``p``.
* ``MPBN``: ``BatchNorm2d`` of the membrane after the detached LIF update
  (``:313-317`` / ``:558-562``); ``get_effective_threshold`` as in the reference (``:97-121``).
"""
import ctypes

import torch
import torch.nn as nn

from . import _lib
from ._lib import lib, ptr

_SCRATCH = {}


def _scratch(n, dev):
    t = _SCRATCH.get(dev)
    if t is None or t.numel() < n:
        t = torch.empty(n, dtype=torch.float64, device=dev)
        _SCRATCH[dev] = t
    return t


def _bn_train(bn):
    return bn.training or bn.running_mean is None


class BatchNormRowsFn(torch.autograd.Function):
    """``bn`` (an ``nn.BatchNorm2d``) over [P, C] channel-fastest rows; weight/bias are passed as
    inputs so that callers may hand in derived (e.g. TEBN-scaled) affine parameters."""

    @staticmethod
    def forward(ctx, x, weight, bias, bn):
        _lib.require_device(x, "BatchNorm input")
        Pn, C = x.shape
        dev = x.device
        s = _lib.stream_ptr(dev)
        y = torch.empty_like(x)
        mean = torch.empty(C, device=dev)
        invstd = torch.empty(C, device=dev)
        train = _bn_train(bn)
        a = _lib.BnFwdArgs()
        a.P, a.C, a.train = Pn, C, 1 if train else 0
        a.x, a.y, a.weight, a.bias = ptr(x), ptr(y), ptr(weight), ptr(bias)
        if bn.running_mean is not None:
            a.running_mean, a.running_var = ptr(bn.running_mean), ptr(bn.running_var)
            if bn.training:
                a.num_batches_tracked = ptr(bn.num_batches_tracked)
        else:
            a.running_mean = a.running_var = None
        if not bn.training and bn.running_mean is None:
            raise _lib.SnnflowError("BatchNorm in eval mode needs running statistics")
        if bn.training and bn.running_mean is not None and bn.momentum is None:
            raise NotImplementedError("BatchNorm momentum=None (cumulative average) is not implemented")
        a.momentum, a.eps = float(bn.momentum or 0.0), float(bn.eps)
        a.save_mean, a.save_invstd = ptr(mean), ptr(invstd)
        a.scratch = ptr(_scratch(lib.snnflow_bn_scratch_doubles(C), dev))
        _lib.call("bn_fwd", lib.snnflow_bn_fwd, ctypes.byref(a), s)
        ctx.train = train
        ctx.save_for_backward(x, weight, mean, invstd)
        ctx.set_materialize_grads(False)
        return y

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None, None
        x, weight, mean, invstd = ctx.saved_tensors
        Pn, C = x.shape
        dev = x.device
        g = g.contiguous().float()
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gw = torch.empty(C, device=dev) if (weight is not None and ctx.needs_input_grad[1]) else None
        gb = torch.empty(C, device=dev) if ctx.needs_input_grad[2] else None
        a = _lib.BnBwdArgs()
        a.P, a.C, a.train = Pn, C, 1 if ctx.train else 0
        a.x, a.g, a.weight, a.save_mean, a.save_invstd = ptr(x), ptr(g), ptr(weight), ptr(mean), ptr(invstd)
        a.g_x, a.g_weight, a.g_bias = ptr(gx), ptr(gw), ptr(gb)
        a.scratch = ptr(_scratch(lib.snnflow_bn_scratch_doubles(C), dev))
        _lib.call("bn_bwd", lib.snnflow_bn_bwd, ctypes.byref(a), _lib.stream_ptr(dev))
        return gx, gw, gb, None


def batch_norm_nchw(x, bn, weight=None, bias=None):
    """``bn(x)`` for x [B, C, H, W] through the rows kernel; the result is a channels_last tensor."""
    B, C, H, W = x.shape
    rows = x.permute(0, 2, 3, 1).contiguous().float().view(B * H * W, C)
    w = bn.weight if weight is None else weight
    b = bn.bias if bias is None else bias
    y = BatchNormRowsFn.apply(rows, w, b, bn)
    return y.view(B, H, W, C).permute(0, 3, 1, 2)


class TEBN(nn.Module):
    """``models/SNNtorch_spiking_submodules.py:18-63``: same submodule/parameter names
    (``bn``, ``p`` [T, C, 1, 1]) and ``forward(x, timestep=None)``."""

    def __init__(self, num_features, num_timesteps=4, momentum=0.1, eps=1e-5):
        super().__init__()
        self.bn = nn.BatchNorm2d(num_features, momentum=momentum, eps=eps)
        self.register_parameter("p", nn.Parameter(torch.ones(num_timesteps, num_features, 1, 1)))
        self.num_timesteps = num_timesteps

    def p_t(self, timestep=None):
        """[C] temporal weight: p[timestep] for a valid step, else the mean over steps (:56-60)."""
        if timestep is not None and 0 <= timestep < self.num_timesteps:
            return self.p[timestep].reshape(-1)
        return self.p.mean(dim=0).reshape(-1)

    def affine(self, timestep=None):
        """The BatchNorm affine parameters with the temporal weight folded in."""
        pt = self.p_t(timestep)
        return self.bn.weight * pt, self.bn.bias * pt

    def forward(self, x, timestep=None):
        w, b = self.affine(timestep)
        return batch_norm_nchw(x, self.bn, w, b)


class MPBN(nn.Module):
    """``models/SNNtorch_spiking_submodules.py:66-121``."""

    def __init__(self, num_features, momentum=0.1, eps=1e-5):
        super().__init__()
        self.bn = nn.BatchNorm2d(num_features, momentum=momentum, eps=eps)

    def forward(self, mem):
        return batch_norm_nchw(mem, self.bn)

    def get_effective_threshold(self, threshold):
        if self.bn.training:
            return threshold
        mean = self.bn.running_mean.view(1, -1, 1, 1)
        std = torch.sqrt(self.bn.running_var.view(1, -1, 1, 1) + self.bn.eps)
        return (threshold * std) + mean


def _flat(st):
    """1-D view of an NHWC-storage state [2, B, C, H, W] in storage order (no copy)."""
    return st.permute(0, 1, 3, 4, 2).view(-1)


class MPBNStateFn(torch.autograd.Function):
    """stack([MPBN(mem), spk]) of a cell state [2, B, C, H, W] held in NHWC storage (the cells'
    layout): the membrane half through the BatchNorm rows kernel, the spike half passed on."""

    @staticmethod
    def forward(ctx, state, weight, bias, bn):
        from .engine import as_nhwc_state, empty_state
        two, B, C, H, W = state.shape
        st = as_nhwc_state(state)
        Pn = B * H * W
        rows = _flat(st)[:Pn * C].view(Pn, C)  # mem half of the NHWC storage
        y = BatchNormRowsFn.forward(ctx, rows, weight, bias, bn)
        out = empty_state(B, C, H, W, state.device)
        _flat(out)[:Pn * C].copy_(y.view(-1))
        _flat(out)[Pn * C:].copy_(_flat(st)[Pn * C:])
        ctx.dims = (B, C, H, W)
        return out

    @staticmethod
    def backward(ctx, g):
        from .engine import as_nhwc_state, empty_state
        if g is None:
            return None, None, None, None
        B, C, H, W = ctx.dims
        Pn = B * H * W
        gn = as_nhwc_state(g)
        g_mem = _flat(gn)[:Pn * C].view(Pn, C)
        gx, gw, gb, _ = BatchNormRowsFn.backward(ctx, g_mem)
        g_in = None
        if ctx.needs_input_grad[0]:
            g_in = empty_state(B, C, H, W, g.device)
            if gx is not None:
                _flat(g_in)[:Pn * C].copy_(gx.view(-1))
            else:
                _flat(g_in)[:Pn * C].zero_()
            _flat(g_in)[Pn * C:].copy_(_flat(gn)[Pn * C:])
        return g_in, gw, gb, None


class PointwiseFn(torch.autograd.Function):
    """1x1 conv + bias + activation (``models/submodules.py:16-113`` with kernel_size 1)."""

    @staticmethod
    def forward(ctx, x, weight, bias, act):
        _lib.require_device(x, "ConvLayer input")
        B, cin, H, W = x.shape
        cout = weight.shape[0]
        if cin > _lib.PW_MAX_CIN or cout > _lib.PW_MAX_COUT:
            raise NotImplementedError(f"1x1 ConvLayer {cin}->{cout}: at most {_lib.PW_MAX_CIN} -> {_lib.PW_MAX_COUT}")
        w = weight.detach().contiguous()
        out = torch.empty(B, cout, H, W, device=x.device)
        a = _lib.PointwiseArgs()
        a.B, a.H, a.W, a.cin, a.cout, a.act = B, H, W, cin, cout, _lib.ACT[act]
        a.x, a.w, a.b, a.out = ptr(x), ptr(w), ptr(bias), ptr(out)
        for i in range(4):
            a.xs[i] = x.stride(i)
        _lib.call("pointwise_fwd", lib.snnflow_pointwise_fwd, ctypes.byref(a), _lib.stream_ptr(x.device))
        ctx.act = act
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, w, out)
        return out

    @staticmethod
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        B, cin, H, W = x.shape
        cout = w.shape[0]
        dev = x.device
        g = g.float()
        gx = torch.empty(B, cin, H, W, device=dev) if ctx.needs_input_grad[0] else None
        gw = torch.empty(cout, cin, 1, 1, device=dev) if ctx.needs_input_grad[1] else None
        gb = torch.empty(cout, device=dev) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        if g.stride(3) != 1 or g.stride(2) != W:
            g = g.contiguous()
        a = _lib.PointwiseArgs()
        a.B, a.H, a.W, a.cin, a.cout, a.act = B, H, W, cin, cout, _lib.ACT[ctx.act]
        a.x, a.w, a.out, a.g_x = ptr(x), ptr(w), ptr(out), ptr(gx)
        for i in range(4):
            a.xs[i] = x.stride(i)
            a.gxs[i] = gx.stride(i) if gx is not None else 0
        scratch = _scratch(_lib.BN_PARTS * cout * (cin + 1), dev)
        _lib.call("pointwise_bwd", lib.snnflow_pointwise_bwd, ctypes.byref(a), ptr(g), g.stride(0), g.stride(1),
                  ptr(gw), ptr(gb), ptr(scratch), _lib.stream_ptr(dev))
        return gx, gw, gb, None
