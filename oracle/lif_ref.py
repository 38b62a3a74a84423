"""ORACLE (test infrastructure only) -- CPU fp32 restatement of the spiking cells
and the LIFFireNet family of the reference.

Every class cites the reference lines it restates.  Construction draws from the
torch RNG in the same order as the reference constructors, so
``torch.manual_seed(s)`` gives the same initial parameters as the reference.
"""
import math

import torch
import torch.nn as nn


# ---------------------------------------------------------------------------
# Surrogate-gradient Heavisides
# ---------------------------------------------------------------------------
class ATanHeaviside(torch.autograd.Function):
    """snntorch 0.9.4 ``surrogate.atan(alpha=2.0)`` (third-party, restated):
    forward ``x > 0``; backward ``alpha/2 / (1 + (pi/2*alpha*x)^2) * g``.
    Used by ``snn.Leaky`` in the reference cells
    (``models/SNNtorch_spiking_submodules.py:232-239, 454-461``).  PARITY UNPINNED.
    """

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return (x > 0).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        alpha = 2.0
        return alpha / 2 / (1 + (math.pi / 2 * alpha * x).pow(2)) * g


class WidthHeaviside(torch.autograd.Function):
    """``models/spiking_util.py:13-25`` forward (``x.gt(0)``) with the surrogate
    selected by ``kind`` (``:28-93``); no gradient to ``width``."""

    @staticmethod
    def forward(ctx, x, width, kind):
        ctx.save_for_backward(x, width)
        ctx.kind = kind
        # the reference's x.gt(0).float(): identical for its fp32 tensors; the dtype of x keeps an
        # fp64 run of the oracle in fp64 (tests/test_gpu_unet.py measures precision against one)
        return x.gt(0).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        x, width = ctx.saved_tensors
        if ctx.kind == "arctanspike":  # spiking_util.py:92
            sg = 1 / (1 + width * x * x)
        elif ctx.kind == "superspike":  # :41
            sg = 1 / (1 + width * x.abs()) ** 2
        elif ctx.kind == "trianglespike":  # :77
            sg = torch.relu(1 - width * x.abs())
        elif ctx.kind == "mgspike":  # :59-64, gaussian :6-10
            def gauss(mu, sigma):
                return torch.exp(-((x - mu) * (x - mu)) / (2 * sigma * sigma)) / (sigma * math.sqrt(2 * math.pi))

            sg = 1.15 * gauss(0.0, width) - 0.15 * gauss(width, 6 * width) - 0.15 * gauss(-width, 6 * width)
        else:
            raise NotImplementedError(ctx.kind)
        return g.clone() * sg, None, None


def width_spike(v, thresh, width, kind="arctanspike"):
    """``spiking_util.arctanspike`` and friends (``:96-109``): spike of ``v - thresh``."""
    return WidthHeaviside.apply(v - thresh, width, kind)


# ---------------------------------------------------------------------------
# snntorch.Leaky restated (third-party dependency absent from the reference tree)
# ---------------------------------------------------------------------------
class LeakyRef(nn.Module):
    """Restatement of ``snntorch.Leaky`` 0.9.4 as the reference constructs it
    (``SNNtorch_spiking_submodules.py:232-239``: learnable beta/threshold,
    ``reset_mechanism="zero"`` for ``hard_reset=True``, ``reset_delay=False``).

    Per step (input current I, stored membrane m):
        r  = H(m - theta)                 (detached)
        zero reset:     v = clamp(beta,0,1) * ((1 - r) * m) + I
        subtract reset: v = clamp(beta,0,1) * m + I - r * theta
        s  = H(v - theta)                 (ATan surrogate)
        zero reset:     m_out = v - (s - r) * v
        subtract reset: m_out = v - (s - r) * theta
    ``mem=None`` reuses the cached membrane when its shape matches (the
    stale-membrane quirk after ``reset_states``).  PARITY UNPINNED.
    """

    def __init__(self, beta, threshold, reset_mechanism="zero"):
        super().__init__()
        self.beta = nn.Parameter(beta.clone())
        self.threshold = nn.Parameter(threshold.clone())
        self.register_buffer("graded_spikes_factor", torch.as_tensor(1.0))
        self.register_buffer("reset_mechanism_val", torch.as_tensor(1 if reset_mechanism == "zero" else 0))
        self.register_buffer("mem", torch.zeros(0), persistent=False)
        self.zero_reset = reset_mechanism == "zero"

    def forward(self, current, mem=None):
        if mem is not None:
            self.mem = mem
        if self.mem.shape != current.shape:
            self.mem = torch.zeros_like(current)
        r = ATanHeaviside.apply(self.mem - self.threshold).clone().detach()
        b = self.beta.clamp(0, 1)
        if self.zero_reset:
            v = b * ((1 - r) * self.mem) + current
        else:
            v = b * self.mem + current - r * self.threshold
        self.last_v = v.detach()  # pre-reset membrane, kept for near-threshold parity checks
        s = ATanHeaviside.apply(v - self.threshold) * self.graded_spikes_factor
        do_reset = s / self.graded_spikes_factor - r
        out = v - do_reset * v if self.zero_reset else v - do_reset * self.threshold
        self.mem = out
        return s, out

    def detach_hidden(self):
        self.mem.detach_()


# ---------------------------------------------------------------------------
# TEBN / MPBN (models/SNNtorch_spiking_submodules.py:18-121)
# ---------------------------------------------------------------------------
class TEBNRef(nn.Module):
    """``TEBN`` (``:18-63``): ``BatchNorm2d(x) * p_t`` with ``p_t = p[t]`` for a valid step, else
    ``p.mean(0)`` (the reference's cells never pass a step, ``models/model.py:172-180``)."""

    def __init__(self, c, num_timesteps=4):
        super().__init__()
        self.bn = nn.BatchNorm2d(c, momentum=0.1, eps=1e-5)
        self.p = nn.Parameter(torch.ones(num_timesteps, c, 1, 1))
        self.num_timesteps = num_timesteps

    def forward(self, x, timestep=None):
        if timestep is not None and 0 <= timestep < self.num_timesteps:
            pt = self.p[timestep:timestep + 1]
        else:
            pt = self.p.mean(dim=0, keepdim=True)
        return self.bn(x) * pt


class MPBNRef(nn.Module):
    """``MPBN`` (``:66-95``): BatchNorm2d of the membrane."""

    def __init__(self, c):
        super().__init__()
        self.bn = nn.BatchNorm2d(c, momentum=0.1, eps=1e-5)

    def forward(self, mem):
        return self.bn(mem)


# ---------------------------------------------------------------------------
# Cells
# ---------------------------------------------------------------------------
class SnnTorchCellRef(nn.Module):
    """``SNNtorch_ConvLIF`` (``SNNtorch_spiking_submodules.py:124-322``) and, with
    ``recurrent=True``, ``SNNtorch_ConvLIFRecurrent`` (``:324-567``), fp32 branch:
    conv3x3 (no bias) [+ conv3x3 of previous spikes] -> BatchNorm2d -> Leaky;
    membrane detached (unless ``detach=False``, :309-311), state = stack([mem, spk]).  ``tebn``: TEBN in place of the BatchNorm
    (``:245-251``); ``mpbn``: state = stack([MPBN(mem), spk]) after the detach (``:313-317``)."""

    def __init__(self, cin, c, k=3, recurrent=False, leak=(0.0, 1.0), thresh=(0.0, 0.8), hard_reset=True,
                 tebn=False, num_timesteps=4, mpbn=False, detach=True):
        super().__init__()
        self.input_size, self.hidden_size, self.recurrent = cin, c, recurrent
        self.detach = detach
        beta0 = torch.empty(c, 1, 1).uniform_(leak[0], leak[1])
        th0 = torch.empty(c, 1, 1).uniform_(thresh[0], thresh[1])
        self.ff = nn.Conv2d(cin, c, k, padding=k // 2, bias=False)
        if recurrent:
            self.rec = nn.Conv2d(c, c, k, padding=k // 2, bias=False)
        self.lif = LeakyRef(beta0, th0, "zero" if hard_reset else "subtract")
        nn.init.uniform_(self.ff.weight, -math.sqrt(1 / cin), math.sqrt(1 / cin))
        if recurrent:
            nn.init.uniform_(self.rec.weight, -math.sqrt(1 / c), math.sqrt(1 / c))
        self.tebn = tebn
        self.bn = TEBNRef(c, num_timesteps) if tebn else nn.BatchNorm2d(c, momentum=0.1, eps=1e-5)
        self.mpbn = MPBNRef(c) if mpbn else None

    def forward(self, x, prev_state, residual=0, timestep=None):
        self.lif.threshold.data.clamp_(min=0.01)
        cur = self.ff(x)
        if self.recurrent:
            prev_spk = torch.zeros_like(cur) if prev_state is None else prev_state[1]
            cur = cur + self.rec(prev_spk)
        cur = self.bn(cur, timestep=timestep) if self.tebn else self.bn(cur)
        spk, mem = self.lif(cur, None if prev_state is None else prev_state[0])
        if self.detach:  # :309-311
            self.lif.detach_hidden()
            mem = mem.detach()
        if self.mpbn is not None:
            mem = self.mpbn(mem)
        return spk, torch.stack([mem, spk], dim=0)


class SpikingCellRef(nn.Module):
    """``ConvLIF`` / ``ConvLIFRecurrent`` of ``models/spiking_submodules.py:29-151,
    154-300`` (U-Net neuron flavour): sigmoid leak, clamp_min(thresh, 0.01),
    detached reset spikes, hard or soft reset, ``spiking_util`` surrogate."""

    def __init__(self, cin, c, k=3, recurrent=False, activation="arctanspike", act_width=10.0,
                 leak=(-4.0, 0.1), thresh=(0.8, 0.0), hard_reset=True, detach=True):
        super().__init__()
        self.recurrent = recurrent
        self.ff = nn.Conv2d(cin, c, k, padding=k // 2, bias=False)
        if recurrent:
            self.rec = nn.Conv2d(c, c, k, padding=k // 2, bias=False)
        self.leak = nn.Parameter(torch.randn(c, 1, 1) * leak[1] + leak[0])
        self.thresh = nn.Parameter(torch.randn(c, 1, 1) * thresh[1] + thresh[0])
        nn.init.uniform_(self.ff.weight, -math.sqrt(1 / cin), math.sqrt(1 / cin))
        if recurrent:
            nn.init.uniform_(self.rec.weight, -math.sqrt(1 / c), math.sqrt(1 / c))
        self.activation = activation
        self.register_buffer("act_width", torch.tensor(act_width))
        self.hard_reset, self.detach = hard_reset, detach

    def forward(self, x, prev_state, residual=0):
        cur = self.ff(x)
        if prev_state is None:
            prev_state = torch.zeros(2, *cur.shape, dtype=cur.dtype, device=cur.device)
        v, z = prev_state
        if self.recurrent:
            cur = cur + self.rec(z)
        th = self.thresh.clamp_min(0.01)
        lam = torch.sigmoid(self.leak)
        if self.detach:
            z = z.detach()
        if self.hard_reset:
            v_out = v * lam * (1 - z) + (1 - lam) * cur
        else:
            v_out = v * lam + (1 - lam) * cur - z * th
        z_out = width_spike(v_out, th, self.act_width, self.activation)
        return z_out + residual, torch.stack([v_out, z_out])


class ConvLayerRef(nn.Module):
    """``models/submodules.py:ConvLayer`` (``:16-113``) as used for ``pred``:
    conv (bias) -> activation; ``w_scale`` re-initialises weight U(+-w), bias 0."""

    def __init__(self, cin, cout, k, activation="tanh", w_scale=None):
        super().__init__()
        self.conv2d = nn.Conv2d(cin, cout, k, 1, k // 2, bias=True)
        if w_scale is not None:
            nn.init.uniform_(self.conv2d.weight, -w_scale, w_scale)
            nn.init.zeros_(self.conv2d.bias)
        self.activation = getattr(torch, activation) if activation is not None else None

    def forward(self, x):
        out = self.conv2d(x)
        return self.activation(out) if self.activation is not None else out


# ---------------------------------------------------------------------------
# LIFFireNet family (models/model.py)
# ---------------------------------------------------------------------------
# (name, input tag, recurrent) per cell; input tag = index of the producing cell
# (-1 = network input).  models/model.py:172-182 (LIFFireNet), :327-333 (_short),
# :519-529 (LIFFireFlowNet), :687-693 (LIFFireFlowNet_short).
FAMILY = {
    "LIFFireNet": [("head", False), ("G1", True), ("R1a", False), ("R1b", False),
                   ("G2", True), ("R2a", False), ("R2b", False)],
    "LIFFireNet_short": [("head", False), ("G1", True), ("R1a", False),
                         ("G2", True), ("R2a", False)],
    "LIFFireFlowNet": [("head", False), ("G1", False), ("R1a", False), ("R1b", False),
                       ("G2", False), ("R2a", False), ("R2b", False)],
    "LIFFireFlowNet_short": [("head", False), ("G1", False), ("R1a", False),
                             ("G2", False), ("R2a", False)],
}


class LIFFireNetRef(nn.Module):
    """``LIFFireNet`` (``models/model.py:29-207``) and its variants, built from
    ``SnnTorchCellRef`` cells chained in sequence + ``pred`` ConvLayer(C->2, 1x1, tanh,
    w_scale 0.01).  ``forward`` keeps the reference signature and return dict."""

    def __init__(self, unet_kwargs, name="LIFFireNet"):
        super().__init__()
        self.spec = FAMILY[name]
        self.num_bins = unet_kwargs["num_bins"]
        self.encoding = unet_kwargs["encoding"]
        self.norm_input = unet_kwargs.get("norm_input", False)
        self.mask = unet_kwargs["mask_output"]
        c = unet_kwargs["base_num_channels"]
        k = unet_kwargs["kernel_size"]
        tebn = unet_kwargs.get("tebn", {})  # models/model.py:74-81
        nts = tebn.get("num_timesteps", 4) if isinstance(tebn, dict) else 4
        tebn = tebn.get("enabled", False) if isinstance(tebn, dict) else bool(tebn)
        mpbn = unet_kwargs.get("mpbn", {})
        mpbn = mpbn.get("enabled", False) if isinstance(mpbn, dict) else bool(mpbn)
        for i, (cell, rec) in enumerate(self.spec):
            setattr(self, cell, SnnTorchCellRef(self.num_bins if i == 0 else c, c, k, recurrent=rec, tebn=tebn,
                                                num_timesteps=nts, mpbn=mpbn))
        self.pred = ConvLayerRef(c, 2, 1, activation="tanh", w_scale=0.01)
        self.num_recurrent_units = len(self.spec)
        self.reset_states()

    @property
    def states(self):
        if self._states[0] is None:
            return list(self._states)
        return [s.clone() for s in self._states]

    @states.setter
    def states(self, states):
        self._states = states

    def detach_states(self):
        self.states = [s.detach() for s in self.states]

    def reset_states(self):
        self._states = [None] * self.num_recurrent_units

    def forward(self, event_voxel=None, event_cnt=None, log=False, return_dict=True):
        if self.encoding == "voxel":
            x = event_voxel
        elif self.encoding == "cnt" and self.num_bins == 2:
            x = event_cnt
        else:
            raise AttributeError("incorrect input encoding")
        if self.norm_input:
            nz = x != 0
            mean, std = x[nz].mean(), x[nz].std()
            x[nz] = (x[nz] - mean) / std
        h = x
        for i, (cell, _) in enumerate(self.spec):
            h, self._states[i] = getattr(self, cell)(h, self._states[i])
        flow = self.pred(h)
        if not return_dict:
            return flow
        return {"flow": [flow], "activity": None}


def make_unet_kwargs(base_num_channels=8, num_bins=2, encoding="cnt", mask_output=True):
    """The ``model`` section of ``configs/train_SNN.yml:10-31`` with ``spiking_neuron``
    moved under ``model`` as ``configs/parser.py:123-125`` does."""
    return {
        "name": "LIFFireNet", "encoding": encoding, "round_encoding": False, "norm_input": False,
        "num_bins": num_bins, "base_num_channels": base_num_channels, "kernel_size": 3,
        "activations": ["arctanspike", "arctanspike"], "mask_output": mask_output,
        "quantization": {"enabled": False, "PTQ": False, "Conv_only": False},
        "tebn": {"enabled": False, "num_timesteps": 4}, "mpbn": {"enabled": False},
        "spiking_neuron": {"leak": [0.0, 1.0], "thresh": [0.0, 0.8], "learn_leak": True,
                           "learn_thresh": True, "hard_reset": True},
    }


# ---------------------------------------------------------------------------
# Export op
# ---------------------------------------------------------------------------
def lif_export_ref(x, mem, beta, threshold):
    """``SNN_implementation::LIF`` (``ONNX_LIF_operator/src/lif_op.cpp:8-55``), restated:
    per element of NCHW, ``m' = beta[c]*mem + x`` (two roundings, :41), spike on
    ``m' >= threshold[c]`` (:42, note ``>=`` and no beta clamp, unlike snntorch), reset
    to exactly 0 else keep ``m'`` (:43-48).  Pinned against the op itself
    (``oracle/_ref/lif_op.so``, fixture ``tests/golden/lif_export_case.npz``)."""
    C = x.shape[1]
    mp = beta.view(1, C, 1, 1) * mem + x
    spk = (mp >= threshold.view(1, C, 1, 1)).to(x.dtype)
    return spk, torch.where(spk > 0, torch.zeros_like(mp), mp)
