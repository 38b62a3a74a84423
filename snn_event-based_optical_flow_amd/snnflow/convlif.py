"""U-Net neuron flavour with the reference's module API, running on the HIP kernels.

``ConvLIF`` / ``ConvLIFRecurrent`` mirror ``models/spiking_submodules.py:29-151`` /
``:154-300`` (fp32 branch): constructor signature, parameter/buffer names (``ff``, ``rec``,
``leak``, ``thresh``, ``act_width``), torch RNG draw order at construction, and
``forward(input_, prev_state[, residual]) -> (z + residual, stack([v, z]))``.
One call is one autograd node: forward = one kernel (conv [+ rec conv] + membrane +
spike, csrc/convlif.hip); backward = one kernel (surrogate + dgrad of both convs +
dL/dv_prev + threshold/leak sums), one deferred-weight-gradient launch, the slab
reduction and the parameter-gradient finalisation.

Two kernel paths: the fused one-kernel-per-cell path above for kernel 3, stride 1, arctanspike,
detach=True, hidden 4/8/16/32 and input sizes 1-5 or equal to the hidden size; every other
supported cell (odd kernel sizes, stride 2, hidden sizes up to 512 in multiples of 4, the four
surrogates of spiking_util.py, detach=False) runs on the implicit-GEMM kernels of csrc/unet.hip
(``snnflow.unet.ConvLIFCellFn``).  Quantization and norm='weight'/'group' raise.
"""
import ctypes
import math

import torch
import torch.nn as nn

from . import _lib
from ._lib import lib, ptr
from .engine import _ptr_t, _x_strides, as_nhwc_state, empty_state

_HIDDEN = (4, 8, 16, 32)
_SURROGATES = ("arctanspike", "superspike", "mgspike", "trianglespike")


def _check(input_size, hidden_size, kernel_size, stride, activation, detach, norm, quantization_config):
    if quantization_config is not None and quantization_config.get("enabled", False):
        raise NotImplementedError("quantized ConvLIF (brevitas) is not implemented on the HIP path")
    if kernel_size % 2 != 1 or stride not in (1, 2):
        raise NotImplementedError("ConvLIF: odd kernel sizes and strides 1, 2 are implemented")
    if activation not in _SURROGATES:
        raise NotImplementedError(f"ConvLIF: activation {activation!r}")
    if norm is not None:
        raise NotImplementedError("ConvLIF: norm='weight'/'group' is not implemented")
    if hidden_size % 4 != 0 or hidden_size > 512:
        raise NotImplementedError(f"ConvLIF: hidden size {hidden_size} (multiples of 4 up to 512)")


def _fixed_kernel(cell):
    """True when the one-kernel-per-cell ConvLIF path (csrc/convlif.hip) covers the cell; else the
    implicit-GEMM cell path of csrc/unet.hip runs (snnflow.unet.ConvLIFCellFn)."""
    k = cell.ff.kernel_size[0]
    return (k == 3 and cell.ff.stride[0] == 1 and cell.hidden_size in _HIDDEN and cell.activation == "arctanspike"
            and cell.detach and (1 <= cell.input_size <= 5 or cell.input_size == cell.hidden_size))


class _Cell(nn.Module):
    def _common(self, hidden_size, activation, act_width, leak, thresh, learn_leak, learn_thresh, hard_reset,
                detach):
        if learn_leak:
            self.leak = nn.Parameter(torch.randn(hidden_size, 1, 1) * leak[1] + leak[0])
        else:
            self.register_buffer("leak", torch.randn(hidden_size, 1, 1) * leak[1] + leak[0])
        if learn_thresh:
            self.thresh = nn.Parameter(torch.randn(hidden_size, 1, 1) * thresh[1] + thresh[0])
        else:
            self.register_buffer("thresh", torch.randn(hidden_size, 1, 1) * thresh[1] + thresh[0])

    def _finish(self, activation, act_width, hard_reset, detach):
        self.activation = activation
        self.register_buffer("act_width", torch.tensor(act_width))
        self.hard_reset = hard_reset
        self.detach = detach

    def _params(self):
        ps = [self.ff.weight]
        if self.recurrent:
            ps.append(self.rec.weight)
        return ps + [self.leak, self.thresh]

    def _run(self, input_, prev_state, residual):
        res = residual if torch.is_tensor(residual) else None
        if res is None and residual != 0:
            raise NotImplementedError("residual must be a tensor or 0")
        if res is not None:
            res = res.expand(input_.shape[0], self.hidden_size, input_.shape[2], input_.shape[3])
        prev = None if prev_state is None else as_nhwc_state(prev_state)
        if not _fixed_kernel(self):
            from .unet import ConvLIFCellFn
            return ConvLIFCellFn.apply(self, input_, prev, res, *self._params())
        return ConvLIFFn.apply(self, input_, prev, res, *self._params())


class ConvLIF(_Cell):
    """``models/spiking_submodules.py:29-151``."""

    def __init__(self, input_size, hidden_size, kernel_size, stride=1, activation="arctanspike", act_width=10.0,
                 leak=(-4.0, 0.1), thresh=(0.8, 0.0), learn_leak=True, learn_thresh=True, hard_reset=True,
                 detach=True, norm=None, quantization_config=None):
        super().__init__()
        _check(input_size, hidden_size, kernel_size, stride, activation, detach, norm, quantization_config)
        self.input_size, self.hidden_size, self.recurrent = input_size, hidden_size, False
        self.ff = nn.Conv2d(input_size, hidden_size, kernel_size, stride=stride, padding=kernel_size // 2, bias=False)
        self._common(hidden_size, activation, act_width, leak, thresh, learn_leak, learn_thresh, hard_reset, detach)
        w_scale = math.sqrt(1 / input_size)
        nn.init.uniform_(self.ff.weight, -w_scale, w_scale)
        self._finish(activation, act_width, hard_reset, detach)
        self.norm = None

    def forward(self, input_, prev_state, residual=0):
        return self._run(input_, prev_state, residual)


class ConvLIFRecurrent(_Cell):
    """``models/spiking_submodules.py:154-300``."""

    def __init__(self, input_size, hidden_size, kernel_size, activation="arctanspike", act_width=10.0,
                 leak=(-4.0, 0.1), thresh=(0.8, 0.0), learn_leak=True, learn_thresh=True, hard_reset=True,
                 detach=True, norm=None, quantization_config=None):
        super().__init__()
        _check(input_size, hidden_size, kernel_size, 1, activation, detach, norm, quantization_config)
        self.input_size, self.hidden_size, self.recurrent = input_size, hidden_size, True
        self.ff = nn.Conv2d(input_size, hidden_size, kernel_size, padding=kernel_size // 2, bias=False)
        self.rec = nn.Conv2d(hidden_size, hidden_size, kernel_size, padding=kernel_size // 2, bias=False)
        self._common(hidden_size, activation, act_width, leak, thresh, learn_leak, learn_thresh, hard_reset, detach)
        nn.init.uniform_(self.ff.weight, -math.sqrt(1 / input_size), math.sqrt(1 / input_size))
        nn.init.uniform_(self.rec.weight, -math.sqrt(1 / hidden_size), math.sqrt(1 / hidden_size))
        self._finish(activation, act_width, hard_reset, detach)
        self.norm_ff = self.norm_rec = None

    def forward(self, input_, prev_state):
        return self._run(input_, prev_state, 0)


def _prep(weights, stream):
    """Transposed copies of the conv weights (one batched launch, no threshold clamp)."""
    out, descs = [], []
    for w in weights:
        c, cin = w.shape[0], w.shape[1]
        fwd = torch.empty(w.numel(), device=w.device)
        bwd = torch.empty(w.numel(), device=w.device)
        descs.append(_lib.PrepDesc(ptr(w.contiguous()), c, cin, ptr(fwd), ptr(bwd), None, 0))
        out.append((fwd, bwd))
    _lib.call("prep_weights", lib.snnflow_prep_weights_batch, (_lib.PrepDesc * len(descs))(*descs), len(descs), stream)
    return out


def _params_struct(cell):
    return _lib.ConvLifParams(ptr(cell.leak), ptr(cell.thresh), float(cell.act_width), 1 if cell.hard_reset else 0)


class ConvLIFFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cell, x, prev, res, *params):
        _lib.require_device(x, "ConvLIF input")
        B, cin, H, W = x.shape
        C = cell.hidden_size
        dev = x.device
        s = _lib.stream_ptr(dev)
        prepped = _prep([p for p in params[:2 if cell.recurrent else 1]], s)
        out = torch.empty(B, C, H, W, device=dev, memory_format=torch.channels_last)
        state = empty_state(B, C, H, W, dev)
        cur = torch.empty(B, H, W, C, device=dev)
        a = _lib.ConvLifFwdArgs()
        a.B, a.H, a.W, a.cin, a.c = B, H, W, cin, C
        a.x = ptr(x)
        a.xs_b, a.xs_c, a.xs_h, a.xs_w = _x_strides(x)
        a.prev_state = _ptr_t(prev)
        a.wt_ff = ptr(prepped[0][0])
        a.wt_rec = ptr(prepped[1][0]) if cell.recurrent else None
        a.p = _params_struct(cell)
        if res is not None:
            a.residual = ptr(res)
            a.rs_b, a.rs_c, a.rs_h, a.rs_w = _x_strides(res)
        a.out, a.state, a.current = ptr(out), ptr(state), ptr(cur)
        _lib.call("convlif_fwd", lib.snnflow_convlif_fwd, ctypes.byref(a), s)
        ctx.cell = cell
        ctx.prepped = prepped
        ctx.has_prev, ctx.has_res = prev is not None, res is not None
        saved = [x, state, cur] + ([prev] if prev is not None else [])
        ctx.save_for_backward(*saved)
        ctx.set_materialize_grads(False)
        return out, state

    @staticmethod
    def backward(ctx, g_out, g_state):
        cell = ctx.cell
        x, state, cur = ctx.saved_tensors[:3]
        prev = ctx.saved_tensors[3] if ctx.has_prev else None
        B, cin, H, W = x.shape
        C = cell.hidden_size
        dev = x.device
        s = _lib.stream_ptr(dev)
        acc = torch.zeros(_lib.acc_storage(2 * C), dtype=torch.float64, device=dev)
        g_cur = torch.empty(B, H, W, C, device=dev)
        a = _lib.ConvLifBwdArgs()
        a.B, a.H, a.W, a.cin, a.c = B, H, W, cin, C
        if g_out is not None:
            g_out = g_out.float()
            a.g_out = ptr(g_out)
            a.gs_b, a.gs_c, a.gs_h, a.gs_w = _x_strides(g_out)
        gst = as_nhwc_state(g_state) if g_state is not None else None
        a.g_state, a.state, a.prev_state, a.current = _ptr_t(gst), ptr(state), _ptr_t(prev), ptr(cur)
        a.wt_bwd_ff = ptr(ctx.prepped[0][1])
        a.wt_bwd_rec = ptr(ctx.prepped[1][1]) if cell.recurrent else None
        a.p = _params_struct(cell)
        gx = None
        if ctx.needs_input_grad[1]:
            gx = torch.empty_like(x)
            a.g_x = ptr(gx)
            a.gxs_b, a.gxs_c, a.gxs_h, a.gxs_w = _x_strides(gx)
        g_prev = None
        if ctx.has_prev and ctx.needs_input_grad[2]:
            g_prev = empty_state(B, C, H, W, dev)
            a.g_prev = ptr(g_prev)
        a.g_current, a.acc = ptr(g_cur), ptr(acc)
        _lib.call("convlif_bwd", lib.snnflow_convlif_bwd, ctypes.byref(a), s)

        # weight gradients: snnflow_wgrad with one step and no BatchNorm (G = dL/dI)
        nblk = lib.snnflow_conv_blocks(B, H, W)
        slab_ff = torch.empty(nblk, C * cin * 9, device=dev)
        slab_rec = torch.empty(nblk, C * C * 9, device=dev) if cell.recurrent else None
        wa = _lib.WgradArgs()
        wa.B, wa.H, wa.W, wa.cin, wa.c, wa.nsteps, wa.accumulate = B, H, W, cin, C, 1, 0
        wa.rec = 1 if (cell.recurrent and prev is not None) else 0
        wa.slab_ff, wa.slab_rec = ptr(slab_ff), _ptr_t(slab_rec) if wa.rec else None
        st = wa.steps[0]
        st.g_cur, st.y = ptr(g_cur), ptr(g_cur)
        st.x = ptr(x)
        st.xs_b, st.xs_c, st.xs_h, st.xs_w = _x_strides(x)
        st.s_prev = ptr(prev) + 4 * B * H * W * C if wa.rec else None
        _lib.call("wgrad", lib.snnflow_wgrad, ctypes.byref(wa), s)
        g_wff = torch.empty_like(cell.ff.weight)
        descs = [_lib.SlabDesc(ptr(slab_ff), ptr(g_wff), g_wff.numel())]
        g_wrec = None
        if cell.recurrent:
            g_wrec = torch.zeros_like(cell.rec.weight)  # stays zero without a previous state
            if wa.rec:
                descs.append(_lib.SlabDesc(ptr(slab_rec), ptr(g_wrec), g_wrec.numel()))
        _lib.call("slab_reduce", lib.snnflow_slab_reduce, (_lib.SlabDesc * len(descs))(*descs), len(descs), nblk, s)
        g_leak = torch.empty_like(cell.leak)
        g_th = torch.empty_like(cell.thresh)
        _lib.call("convlif_param_grads", lib.snnflow_convlif_param_grads, ptr(acc), ptr(cell.leak), ptr(cell.thresh),
                  C, 0, ptr(g_leak), ptr(g_th), s)
        g_res = g_out if (ctx.has_res and ctx.needs_input_grad[3]) else None
        pg = [g_wff] + ([g_wrec] if cell.recurrent else []) + [g_leak, g_th]
        return (None, gx, g_prev, g_res, *pg)
