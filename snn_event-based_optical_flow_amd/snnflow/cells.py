"""Spiking cells with the reference's module API, running on the HIP kernels.

``SNNtorch_ConvLIF`` / ``SNNtorch_ConvLIFRecurrent`` mirror
``models/SNNtorch_spiking_submodules.py:124-322`` / ``:324-567`` (fp32 branch):
constructor signature, parameter/buffer names (``ff``, ``rec``, ``bn``,
``lif.beta``, ``lif.threshold``, ...), torch RNG draw order at construction, and
``forward(input_, prev_state, residual=0, timestep=None) -> (spk, stack([mem, spk]))``.
A standalone cell call is one autograd node (conv+stats kernel, LIF kernel; backward:
LIF-bwd kernel, BN-bwd+dgrad+wgrad kernel, slab reduction).  Inside ``LIFFireNet``
the cells are not called one by one: the whole time step is fused (engine.py).
"""
import ctypes
import math

import torch
import torch.nn as nn

from . import _lib
from ._lib import check, lib, ptr
from .engine import (Workspace, _ptr_t, _x_strides, as_nhwc_state, empty_state,
                     neuron_struct, theta_subtract)
from .norm import MPBN, TEBN, MPBNStateFn, PointwiseFn


class Leaky(nn.Module):
    """Parameter/state holder with the attribute layout of ``snntorch.Leaky`` 0.9.4 as the
    reference builds it (``SNNtorch_spiking_submodules.py:232-239``): learnable ``beta`` and
    ``threshold`` [C,1,1], buffers ``graded_spikes_factor`` and ``reset_mechanism_val``,
    a non-persistent membrane cache ``mem``.  Its arithmetic runs inside the fused cell
    kernels (csrc/snnflow_dev.h: lif_step / atan_sg)."""

    def __init__(self, beta, threshold, learn_beta=True, learn_threshold=True, reset_mechanism="zero",
                 reset_delay=False):
        super().__init__()
        if reset_delay:
            raise NotImplementedError("only reset_delay=False (the reference's setting) is implemented")
        if reset_mechanism not in ("zero", "subtract"):
            raise NotImplementedError(f"reset_mechanism={reset_mechanism!r}")
        beta = torch.as_tensor(beta, dtype=torch.float32).clone()
        threshold = torch.as_tensor(threshold, dtype=torch.float32).clone()
        if learn_beta:
            self.beta = nn.Parameter(beta)
        else:
            self.register_buffer("beta", beta)
        if learn_threshold:
            self.threshold = nn.Parameter(threshold)
        else:
            self.register_buffer("threshold", threshold)
        self.register_buffer("graded_spikes_factor", torch.as_tensor(1.0))
        self.register_buffer("reset_mechanism_val", torch.as_tensor(1 if reset_mechanism == "zero" else 0))
        self.reset_mechanism = reset_mechanism
        self.mem = None

    @property
    def mem(self):
        """Membrane cache (snntorch's ``Leaky.mem``).  The fused step leaves it as a lazy view spec
        (storage, shape, strides, offset) into its state buffer: built on first read."""
        lazy = self.__dict__.get("_mem_lazy")
        if lazy is not None:
            st, shape, stride, off = lazy
            self.__dict__["_mem"] = st.as_strided(shape, stride, off).detach()
            self.__dict__["_mem_lazy"] = None
        return self.__dict__.get("_mem")

    @mem.setter
    def mem(self, value):
        self.__dict__["_mem_lazy"] = None
        self.__dict__["_mem"] = value

    def detach_hidden(self):
        if self.mem is not None:
            self.mem = self.mem.detach()

    def reset_mem(self):
        if self.mem is not None:
            self.mem = torch.zeros_like(self.mem)
        return self.mem


def _check_supported(kernel_size, stride, quantization_config, tebn, mpbn, norm, detach, activation):
    if kernel_size != 3 or stride != 1:
        raise NotImplementedError("snnflow cells implement the reference's 3x3 / stride-1 convolutions")
    if quantization_config is not None and quantization_config.get("enabled", False):
        raise NotImplementedError("quantized (brevitas) cells are out of scope (DESIGN.md)")
    if norm not in (None, "weight"):
        # GroupNorm of the conv inputs (:277-279 / :506-509) would feed non-spike values into the
        # recurrent conv, whose kernels take spikes (0/1) there
        raise NotImplementedError("norm='group' is not implemented (norm=None and norm='weight' are)")


class _SnnTorchCellBase(nn.Module):
    recurrent = False

    def _build(self, input_size, hidden_size, kernel_size, leak, thresh, learn_leak, learn_thresh, hard_reset,
               stride=1, tebn=False, num_timesteps=4, mpbn=False, detach=True):
        self.input_size, self.hidden_size = input_size, hidden_size
        pad = kernel_size // 2
        beta_init = torch.empty(hidden_size, 1, 1).uniform_(leak[0], leak[1])
        threshold_init = torch.empty(hidden_size, 1, 1).uniform_(thresh[0], thresh[1])
        self.hard_reset = hard_reset
        self.ff = nn.Conv2d(input_size, hidden_size, kernel_size, stride=stride, padding=pad, bias=False)
        if self.recurrent:
            self.rec = nn.Conv2d(hidden_size, hidden_size, kernel_size, padding=pad, bias=False)
        self.lif = Leaky(beta_init, threshold_init, learn_leak, learn_thresh,
                         "zero" if hard_reset else "subtract", reset_delay=False)
        w_ff = math.sqrt(1 / input_size)
        nn.init.uniform_(self.ff.weight, -w_ff, w_ff)
        if self.recurrent:
            w_rec = math.sqrt(1 / hidden_size)
            nn.init.uniform_(self.rec.weight, -w_rec, w_rec)
        # :245-263 / :469-487 -- TEBN in place of the BatchNorm, MPBN of the membrane
        self.bn = TEBN(hidden_size, num_timesteps=num_timesteps, momentum=0.1, eps=1e-5) if tebn else \
            nn.BatchNorm2d(hidden_size, momentum=0.1, eps=1e-5)
        self.tebn_enabled = bool(tebn)
        self.num_timesteps = num_timesteps
        self.mpbn = MPBN(hidden_size, momentum=0.1, eps=1e-5) if mpbn else None
        self.mpbn_enabled = bool(mpbn)
        self.detach = bool(detach)
        self.exporting = False
        # norm="weight" (:274-276 / :500-504): nn.utils.weight_norm on the convolutions, as the reference
        # applies it (state-dict keys ff.weight_g / ff.weight_v); the effective weight g v / ||v|| is
        # formed per call (_params) and the cell kernels run on it, autograd taking its gradient to g, v
        self.weight_norm = False

    def _apply_weight_norm(self):
        import warnings
        with warnings.catch_warnings():  # (torch deprecates the hook-based form; its keys are the reference's)
            warnings.simplefilter("ignore", FutureWarning)
            self.ff = nn.utils.weight_norm(self.ff)
            if self.recurrent:
                self.rec = nn.utils.weight_norm(self.rec)
        self.weight_norm = True

    @staticmethod
    def _conv_weight(conv, normed):
        return torch._weight_norm(conv.weight_v, conv.weight_g, 0) if normed else conv.weight

    @property
    def batch_norm(self):
        """The nn.BatchNorm2d of the input current (TEBN's inner one when TEBN is on)."""
        return self.bn.bn if self.tebn_enabled else self.bn

    def forward(self, input_, prev_state, residual=0, timestep=None):
        if not self.detach and prev_state is None:
            # detach=False: snn.Leaky continues from its (non-detached) membrane cache, so the
            # gradient reaches the call that produced it; zero spikes as the recurrent input
            cache = self.lif.mem
            B, _, H, W = input_.shape
            if cache is not None and tuple(cache.shape) == (B, self.hidden_size, H, W) and cache.device == input_.device:
                prev_state = torch.stack([cache, torch.zeros_like(cache)])
        spk, state = CellFn.apply(self, input_, prev_state, *self._params(timestep))
        # SNNtorch_spiking_submodules.py:309-311: detach_hidden() + mem_out.detach() unless detach=False
        self.lif.mem = state[0].detach() if self.detach else state[0]
        if self.mpbn_enabled:  # :313-317 / :558-562 (after the detach: no gradient into the LIF)
            state = MPBNStateFn.apply(state, self.mpbn.bn.weight, self.mpbn.bn.bias, self.mpbn.bn)
        return spk, state

    def _params(self, timestep=None):
        ps = [self._conv_weight(self.ff, self.weight_norm)]
        if self.recurrent:
            ps.append(self._conv_weight(self.rec, self.weight_norm))
        if self.tebn_enabled:  # BN(x) * p_t == BN with (weight * p_t, bias * p_t)
            bw, bb = self.bn.affine(timestep)
        else:
            bw, bb = self.bn.weight, self.bn.bias
        return ps + [bw, bb, self.lif.beta, self.lif.threshold]


class SNNtorch_ConvLIF(_SnnTorchCellBase):
    """``models/SNNtorch_spiking_submodules.py:124-322`` (fp32 branch)."""

    recurrent = False

    def __init__(self, input_size, hidden_size, kernel_size, stride=1, activation="arctanspike", act_width=10.0,
                 leak=(0.0, 1.0), thresh=(0.0, 0.8), learn_leak=True, learn_thresh=True, hard_reset=True,
                 detach=True, norm=None, quantization_config=None, exporting=False, tebn=False, num_timesteps=4,
                 mpbn=False):
        super().__init__()
        _check_supported(kernel_size, stride, quantization_config, tebn, mpbn, norm, detach, activation)
        self._build(input_size, hidden_size, kernel_size, leak, thresh, learn_leak, learn_thresh, hard_reset, stride,
                    tebn, num_timesteps, mpbn, detach)
        if norm == "weight":
            self._apply_weight_norm()


class SNNtorch_ConvLIFRecurrent(_SnnTorchCellBase):
    """``models/SNNtorch_spiking_submodules.py:324-567`` (fp32 branch)."""

    recurrent = True

    def __init__(self, input_size, hidden_size, kernel_size, activation="arctanspike", act_width=10.0,
                 leak=(0.0, 1.0), thresh=(0.0, 0.8), learn_leak=True, learn_thresh=True, hard_reset=True,
                 detach=True, norm=None, quantization_config=None, exporting=False, tebn=False, num_timesteps=4,
                 mpbn=False):
        super().__init__()
        _check_supported(kernel_size, 1, quantization_config, tebn, mpbn, norm, detach, activation)
        if input_size != hidden_size and input_size not in (1, 2, 4, 5):
            raise NotImplementedError("recurrent cells take input_size == hidden_size or 1, 2, 4, 5 (event inputs)")
        self._build(input_size, hidden_size, kernel_size, leak, thresh, learn_leak, learn_thresh, hard_reset,
                    1, tebn, num_timesteps, mpbn, detach)
        if norm == "weight":
            self._apply_weight_norm()


class ConvLayer(nn.Module):
    """``models/submodules.py:ConvLayer`` (``:16-113``), fp32 branch, as used for
    LIFFireNet's ``pred`` (1x1, bias, tanh, ``w_scale`` init).  Inside LIFFireNet it
    is fused into the last cell's LIF kernel; a standalone call runs the HIP 1x1 kernel
    (csrc/norm.hip, ``snnflow_pointwise_fwd/bwd``)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, activation="relu", norm=None,
                 BN_momentum=0.1, w_scale=None, quantization_config=None, exporting=False):
        super().__init__()
        if quantization_config is not None and quantization_config.get("enabled", False):
            raise NotImplementedError("quantized ConvLayer is out of scope")
        bias = norm != "BN"
        self.conv2d = nn.Conv2d(in_channels, out_channels, kernel_size, stride, kernel_size // 2, bias=bias)
        if w_scale is not None:
            nn.init.uniform_(self.conv2d.weight, -w_scale, w_scale)
            if self.conv2d.bias is not None:
                nn.init.zeros_(self.conv2d.bias)
        self.activation = getattr(torch, activation) if activation is not None else None
        self.activation_name = activation
        self.norm = norm
        # the reference builds the norm layer (state-dict keys) but its forward never applies it:
        # the normalisation block is commented out (submodules.py:98-102)
        if norm == "BN":
            self.norm_layer = nn.BatchNorm2d(out_channels, momentum=BN_momentum)
        elif norm == "IN":
            self.norm_layer = nn.InstanceNorm2d(out_channels, track_running_stats=True)

    def forward(self, x):
        if self.conv2d.kernel_size != (1, 1) or self.conv2d.stride != (1, 1):
            raise NotImplementedError("ConvLayer: only the 1x1 prediction layer is implemented")
        if self.activation_name not in _lib.ACT:
            raise NotImplementedError(f"ConvLayer activation {self.activation_name!r}")
        return PointwiseFn.apply(x.float(), self.conv2d.weight, self.conv2d.bias, self.activation_name)


# ---------------------------------------------------------------------------
# Standalone cell call (one autograd node per call)
# ---------------------------------------------------------------------------
_WS = {}


def _cell_ws(B, H, W, C, dev):
    key = (B, H, W, C, dev)
    ws = _WS.get(key)
    if ws is None:
        ws = Workspace(B, H, W, C, 1, dev)
        _WS[key] = ws
    return ws


class _CellPrep:
    def __init__(self):
        self.fwd = self.bwd = None


def _prep(w, s):
    c, cin = w.shape[0], w.shape[1]
    fwd = torch.empty(9 * cin * c, device=w.device)
    bwd = torch.empty(9 * cin * c, device=w.device)
    _lib.call("prep_weights", lib.snnflow_prep_weights, ptr(w.detach().contiguous()), c, cin, ptr(fwd), ptr(bwd), None, s)
    return fwd, bwd


class CellFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cell, x, prev_state, *params):
        _lib.require_device(x, "cell input")
        B, cin, H, W = x.shape
        C = cell.hidden_size
        dev = x.device
        s = _lib.stream_ptr(dev)
        _lib.call("threshold clamp", lib.snnflow_prep_weights, None, C, 1, None, None, ptr(cell.lif.threshold), s)
        wff = _prep(params[0], s)  # the conv weights as passed (weight norm: the effective g v / ||v||)
        wrec = _prep(params[1], s) if cell.recurrent else (None, None)
        ws = _cell_ws(B, H, W, C, dev)
        if prev_state is None:
            cache = cell.lif.mem
            mem = cache if (cache is not None and tuple(cache.shape) == (B, C, H, W) and cache.device == dev) else None
            sp = None
            pn = None
        else:
            pn = as_nhwc_state(prev_state)
            mem, sp = pn[0], (pn[1] if cell.recurrent else None)
        n = neuron_struct(cell, params[-4], params[-3])
        y = torch.empty(B, H, W, C, device=dev)
        stats = torch.empty(2, C, device=dev)
        facc = ws.fwd_acc[0]
        facc.zero_()
        a = _lib.ConvFwdArgs()
        a.B, a.H, a.W, a.cin, a.c, a.lif_in = B, H, W, cin, C, 0
        a.x = ptr(x)
        a.xs_b, a.xs_c, a.xs_h, a.xs_w = _x_strides(x)
        a.wt_ff, a.wt_rec, a.s_prev = ptr(wff[0]), _ptr_t(wrec[0]), _ptr_t(sp)
        a.wt_ff_t, a.wt_rec_t = ptr(wff[1]), _ptr_t(wrec[1])
        a.y, a.acc = ptr(y), (ptr(facc) if n.bn_train else None)
        _lib.call("conv_fwd", lib.snnflow_conv_fwd, ctypes.byref(a), s)
        state = empty_state(B, C, H, W, dev)
        f = _lib.LifFwdArgs()
        f.B, f.H, f.W, f.c = B, H, W, C
        f.y, f.mem, f.acc, f.stats, f.n, f.state = ptr(y), _ptr_t(mem), ptr(facc), ptr(stats), n, ptr(state)
        _lib.call("lif_fwd", lib.snnflow_lif_fwd, ctypes.byref(f), s)
        spk = state[1].detach().clone()  # a separate output tensor (same values as state[1])
        ctx.cell = cell
        ctx.has_mem, ctx.has_sp = mem is not None, sp is not None
        ctx.has_prev = prev_state is not None
        ctx.wbwd = (wff[1], wrec[1])
        ctx.wfwd = (wff[0], wrec[0])
        ctx.bn_affine = (params[-4], params[-3])
        ctx.save_for_backward(x, y, stats, *(t for t in (mem, sp) if t is not None))
        ctx.set_materialize_grads(False)
        return spk, state

    @staticmethod
    def backward(ctx, g_spk, g_state):
        cell = ctx.cell
        saved = list(ctx.saved_tensors)
        x, y, stats = saved[:3]
        rest = saved[3:]
        mem = rest.pop(0) if ctx.has_mem else None
        sp = rest.pop(0) if ctx.has_sp else None
        B, cin, H, W = x.shape
        C = cell.hidden_size
        dev = x.device
        s = _lib.stream_ptr(dev)
        ws = _cell_ws(B, H, W, C, dev)
        n = neuron_struct(cell, *ctx.bn_affine)
        g_bw, g_bb = torch.empty(C, device=dev), torch.empty(C, device=dev)
        g_beta, g_th = torch.empty(C, device=dev), torch.empty(C, device=dev)
        ng = _lib.NeuronGrad(ptr(g_bw), ptr(g_bb), ptr(g_beta), ptr(g_th))
        g_cur = torch.empty(B, H, W, C, device=dev)
        bacc = ws.bwd_acc[0]
        bacc.zero_()
        b = _lib.LifBwdArgs()
        b.B, b.H, b.W, b.c = B, H, W, C
        b.y, b.mem, b.stats, b.n = ptr(y), _ptr_t(mem), ptr(stats), n
        gs = None
        if g_spk is not None:
            gs = g_spk.contiguous(memory_format=torch.channels_last).float()
            b.g_out = ptr(gs)
        gst = as_nhwc_state(g_state) if g_state is not None else None
        b.g_state = _ptr_t(gst)
        # detach=False: the membrane half of the state output carries gradient too
        b.mem_grad_in = 1 if (gst is not None and not cell.detach) else 0
        g_prev = None
        if ctx.has_prev and ctx.needs_input_grad[2]:
            g_prev = torch.zeros((2, B, C, H, W), device=dev).as_strided(
                (2, B, C, H, W), (B * H * W * C, H * W * C, 1, W * C, C))
            b.g_mem = ptr(g_prev)
        b.g_cur, b.acc = ptr(g_cur), ptr(bacc)
        _lib.call("lif_bwd", lib.snnflow_lif_bwd, ctypes.byref(b), s)

        slab_ff = torch.empty(ws.nblk, C * cin * 9, device=dev)
        slab_rec = torch.empty(ws.nblk, C * C * 9, device=dev) if cell.recurrent else None
        bnc = torch.empty(2, C, device=dev)
        a = _lib.LayerBwdArgs()
        a.B, a.H, a.W, a.cin, a.c, a.lif_in = B, H, W, cin, C, 0
        a.y, a.stats, a.g_cur, a.acc_in, a.n = ptr(y), ptr(stats), ptr(g_cur), ptr(bacc), n
        a.ng, a.accumulate, a.bnc_out = ng, 0, ptr(bnc)
        gx = None
        if ctx.needs_input_grad[1]:
            gx = torch.empty_like(x)
            a.wt_bwd_ff, a.wt_fwd_ff, a.g_x = ptr(ctx.wbwd[0]), ptr(ctx.wfwd[0]), ptr(gx)
            a.gxs_b, a.gxs_c, a.gxs_h, a.gxs_w = _x_strides(gx)
        if cell.recurrent:
            a.wt_bwd_rec, a.wt_fwd_rec = ptr(ctx.wbwd[1]), ptr(ctx.wfwd[1])
            if g_prev is not None:
                a.g_state_prev, a.zero_mem_half = ptr(g_prev), 0
        _lib.call("layer_bwd", lib.snnflow_layer_bwd, ctypes.byref(a), s)
        theta_subtract(cell, g_cur, mem, B * H * W, ptr(g_th), s)
        # weight gradients of this single step (snnflow_wgrad with one step)
        slab_ff = torch.empty(ws.nblk, C * cin * 9, device=dev)
        slab_rec = torch.empty(ws.nblk, C * C * 9, device=dev) if cell.recurrent else None
        wa = _lib.WgradArgs()
        wa.B, wa.H, wa.W, wa.cin, wa.c, wa.nsteps, wa.accumulate = B, H, W, cin, C, 1, 0
        wa.rec = 1 if cell.recurrent else 0
        wa.bn_weight, wa.slab_ff, wa.slab_rec = ptr(ctx.bn_affine[0]), ptr(slab_ff), _ptr_t(slab_rec)
        st = wa.steps[0]
        st.g_cur, st.y, st.stats, st.bnc = ptr(g_cur), ptr(y), ptr(stats), ptr(bnc)
        st.x = ptr(x)
        st.xs_b, st.xs_c, st.xs_h, st.xs_w = _x_strides(x)
        st.s_prev = _ptr_t(sp) if cell.recurrent else None
        _lib.call("wgrad", lib.snnflow_wgrad, ctypes.byref(wa), s)
        g_wff = torch.empty(cell.hidden_size, cin, 3, 3, device=dev)
        descs = [_lib.SlabDesc(ptr(slab_ff), ptr(g_wff), g_wff.numel())]
        g_wrec = None
        if cell.recurrent:
            g_wrec = torch.empty(C, C, 3, 3, device=dev)
            descs.append(_lib.SlabDesc(ptr(slab_rec), ptr(g_wrec), g_wrec.numel()))
        arr = (_lib.SlabDesc * len(descs))(*descs)
        _lib.call("slab_reduce", lib.snnflow_slab_reduce, arr, len(descs), ws.nblk, s)
        pg = [g_wff] + ([g_wrec] if cell.recurrent else [])
        pg += [g_bw, g_bb, g_beta.view(C, 1, 1), g_th.view(C, 1, 1)]
        return (None, gx, g_prev, *pg)
