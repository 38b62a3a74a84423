"""SpikingRecEVFlowNet -- the spiking recurrent multi-resolution U-Net -- on the HIP kernels of
csrc/unet.hip, with the reference's module API:

* ``SpikingRecEVFlowNet(unet_kwargs)`` (``models/model.py:723-858``): ``.multires_unetrec``,
  ``states`` / ``reset_states`` / ``detach_states`` / ``init_cropping``, ``forward(event_voxel,
  event_cnt, log=False) -> {"flow": [4 x [B,2,H,W]], "activity": None}``.
* ``SpikingMultiResUNetRecurrent`` (``models/unet.py:310-461``) with ``encoders`` /
  ``resblocks`` / ``decoders`` / ``preds`` ModuleLists of ``SpikingRecurrentConvLayer``,
  ``SpikingResidualBlock``, ``SpikingUpsampleConvLayer`` (``models/spiking_submodules.py:303-417``)
  and ``ConvLayer`` -- same submodule and parameter names (reference checkpoints load unchanged),
  same torch RNG draw order at construction.

A model ``forward`` is ONE autograd node per time step (``UNetStep``): 16 ConvLIF cells as
implicit-GEMM matrix-core convolutions with the LIF update fused into the epilogue, decoder
inputs (bilinear x2 upsample of the concatenated skips and the previous prediction) materialised
once as bf16 operands, 4 prediction heads.  Its backward runs, per cell, the elementwise LIF
backward, the input-gradient GEMM and the weight-gradient GEMM; membranes back-propagate across
time steps (``ConvLIF`` does not detach ``v``), reset spikes are detached
(``spiking_submodules.py:138-140``).  Parameter gradients of a truncated-BPTT window are
accumulated on the device and returned by its first step.
"""
import ctypes
import math
import os

import torch
import torch.nn as nn

from . import _lib
from ._lib import lib, ptr
from .cells import ConvLayer
from .convlif import ConvLIF, ConvLIFRecurrent

BF16 = torch.bfloat16


def pad32(c):
    return (c + 31) // 32 * 32


def mpad(m):
    return (m + 127) // 128 * 128


def _stream(dev):
    return _lib.stream_ptr(dev)


# ---------------------------------------------------------------------------
# Modules (reference API)
# ---------------------------------------------------------------------------
class SpikingRecurrentConvLayer(nn.Module):
    """``models/spiking_submodules.py:303-346``: ConvLIF (strided) followed by ConvLIFRecurrent."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, recurrent_block_type="lif",
                 activation_ff="arctanspike", activation_rec="arctanspike", **kwargs):
        super().__init__()
        assert recurrent_block_type in ["lif", "alif", "plif", "xlif"]
        if recurrent_block_type != "lif":  # the reference defines blocks for "lif" only (NameError otherwise)
            raise NotImplementedError(f"recurrent_block_type {recurrent_block_type!r}")
        kwargs.pop("spiking_feedforward_block_type", None)
        self.conv = ConvLIF(in_channels, out_channels, kernel_size, stride, activation_ff, **kwargs)
        self.recurrent_block = ConvLIFRecurrent(out_channels, out_channels, kernel_size, activation=activation_rec,
                                                **kwargs)

    def forward(self, x, prev_state):
        if prev_state is None:
            prev_state = [None, None]
        ff, rec = prev_state
        x1, ff = self.conv(x, ff)
        x2, rec = self.recurrent_block(x1, rec)
        return x2, torch.stack([ff, rec])


class SpikingResidualBlock(nn.Module):
    """``models/spiking_submodules.py:349-385``: two ConvLIF, the block input added to the spikes."""

    def __init__(self, in_channels, out_channels, stride=1, spiking_feedforward_block_type="lif",
                 activation="arctanspike", **kwargs):
        super().__init__()
        assert spiking_feedforward_block_type in ["lif", "alif", "plif", "xlif"]
        if spiking_feedforward_block_type != "lif":
            raise NotImplementedError(f"spiking_feedforward_block_type {spiking_feedforward_block_type!r}")
        self.conv1 = ConvLIF(in_channels, out_channels, kernel_size=3, stride=stride, activation=activation, **kwargs)
        self.conv2 = ConvLIF(out_channels, out_channels, kernel_size=3, stride=1, activation=activation, **kwargs)

    def forward(self, x, prev_state):
        if prev_state is None:
            prev_state = [None, None]
        conv1, conv2 = prev_state
        residual = x
        x1, conv1 = self.conv1(x, conv1)
        x2, conv2 = self.conv2(x1, conv2, residual=residual)
        return x2, torch.stack([conv1, conv2])


class SpikingUpsampleConvLayer(nn.Module):
    """``models/spiking_submodules.py:388-417``: bilinear x2 upsample (align_corners=False) + ConvLIF."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, spiking_feedforward_block_type="lif",
                 activation="arctanspike", **kwargs):
        super().__init__()
        assert spiking_feedforward_block_type in ["lif", "alif", "plif", "xlif"]
        if spiking_feedforward_block_type != "lif":
            raise NotImplementedError(f"spiking_feedforward_block_type {spiking_feedforward_block_type!r}")
        self.conv2d = ConvLIF(in_channels, out_channels, kernel_size, stride=stride, activation=activation, **kwargs)

    def forward(self, x, prev_state):
        x_up = upsample_bilinear2x(x)
        return self.conv2d(x_up, prev_state)


class SpikingTransposedConvLayer(nn.Module):
    """``models/spiking_submodules.py:420-436``: raises, as in the reference."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError


class SpikingMultiResUNetRecurrent(nn.Module):
    """``models/unet.py:414-461`` (with ``MultiResUNetRecurrent.__init__`` :320-383 and
    ``BaseUNet.__init__`` :36-85): skip_type "concat", use_upsample_conv, spiking blocks."""

    w_scale_pred = 0.01

    def __init__(self, unet_kwargs):
        super().__init__()
        kw = dict(unet_kwargs)
        self.final_activation = kw.pop("final_activation", None)
        self.base_num_channels = kw["base_num_channels"]
        self.num_encoders = kw["num_encoders"]
        self.num_residual_blocks = kw["num_residual_blocks"]
        self.num_output_channels = kw["num_output_channels"]
        self.kernel_size = kw.get("kernel_size", 5)
        self.skip_type = kw["skip_type"]
        self.norm = kw.get("norm")
        self.num_bins = kw["num_bins"]
        self.recurrent_block_type = kw.get("recurrent_block_type")
        self.channel_multiplier = kw.get("channel_multiplier", 2)
        self.ff_act, self.rec_act = kw.get("activations", ["relu", None])
        if self.skip_type != "concat" or not kw.get("use_upsample_conv", True) or self.norm is not None:
            raise NotImplementedError("snnflow U-Net: skip_type 'concat', use_upsample_conv, norm None")
        self.spiking_kwargs = {}
        if kw.get("spiking_feedforward_block_type") is not None:
            self.spiking_kwargs["spiking_feedforward_block_type"] = kw["spiking_feedforward_block_type"]
        if type(kw.get("spiking_neuron")) is dict:
            self.spiking_kwargs.update(kw["spiking_neuron"])
        C, m = self.base_num_channels, self.channel_multiplier
        self.encoder_input_sizes = [int(C * pow(m, i)) for i in range(self.num_encoders)]
        self.encoder_output_sizes = [int(C * pow(m, i + 1)) for i in range(self.num_encoders)]
        self.max_num_channels = self.encoder_output_sizes[-1]

        self.encoders = nn.ModuleList()
        for i, (cin, cout) in enumerate(zip(self.encoder_input_sizes, self.encoder_output_sizes)):
            self.encoders.append(SpikingRecurrentConvLayer(
                self.num_bins if i == 0 else cin, cout, kernel_size=self.kernel_size, stride=2,
                recurrent_block_type=self.recurrent_block_type, activation_ff=self.ff_act,
                activation_rec=self.rec_act, norm=self.norm, **self.spiking_kwargs))
        self.resblocks = nn.ModuleList()
        for _ in range(self.num_residual_blocks):
            self.resblocks.append(SpikingResidualBlock(self.max_num_channels, self.max_num_channels,
                                                       activation=self.ff_act, norm=self.norm, **self.spiking_kwargs))
        self.decoders = nn.ModuleList()
        for i, (cin, cout) in enumerate(zip(reversed(self.encoder_output_sizes), reversed(self.encoder_input_sizes))):
            pc = 0 if i == 0 else self.num_output_channels
            self.decoders.append(SpikingUpsampleConvLayer(2 * cin + pc, cout, kernel_size=self.kernel_size,
                                                          activation=self.ff_act, norm=self.norm,
                                                          **self.spiking_kwargs))
        self.preds = nn.ModuleList()
        for cout in reversed(self.encoder_input_sizes):
            self.preds.append(ConvLayer(cout, self.num_output_channels, 1, activation=self.final_activation,
                                        norm=self.norm, w_scale=self.w_scale_pred))
        self.num_states = self.num_encoders * 2 + self.num_residual_blocks
        self.states = [None] * self.num_states


class SpikingRecEVFlowNet(nn.Module):
    """``models/model.py:723-858``."""

    unet_type = SpikingMultiResUNetRecurrent
    recurrent_block_type = "lif"
    spiking_feedforward_block_type = "lif"

    def __init__(self, unet_kwargs):
        super().__init__()
        norm = unet_kwargs.get("norm")
        use_upsample_conv = unet_kwargs.get("use_upsample_conv", True)
        rec_kwargs = {
            "base_num_channels": unet_kwargs["base_num_channels"], "num_encoders": 4, "num_residual_blocks": 2,
            "num_output_channels": 2, "skip_type": "concat", "norm": norm, "use_upsample_conv": use_upsample_conv,
            "kernel_size": unet_kwargs["kernel_size"], "channel_multiplier": 2,
            "recurrent_block_type": self.recurrent_block_type, "final_activation": "tanh",
            "spiking_feedforward_block_type": self.spiking_feedforward_block_type,
            "spiking_neuron": unet_kwargs["spiking_neuron"],
        }
        q = unet_kwargs.get("quantization")
        if isinstance(q, dict) and q.get("enabled", False):
            raise NotImplementedError("quantized U-Net (brevitas) is out of scope")
        self.crop = None
        self.mask = unet_kwargs["mask_output"]
        self.norm_input = unet_kwargs.get("norm_input", False)
        self.encoding = unet_kwargs["encoding"]
        self.num_bins = unet_kwargs["num_bins"]
        self.num_encoders = rec_kwargs["num_encoders"]
        kw = dict(rec_kwargs)
        kw["num_bins"] = self.num_bins
        kw["activations"] = unet_kwargs.get("activations", ["relu", None])
        self.multires_unetrec = self.unet_type(kw)
        self._engine = None

    @property
    def engine(self):
        if self._engine is None:
            object.__setattr__(self, "_engine", UNetEngine(self))
        return self._engine

    @property
    def states(self):
        st = self.multires_unetrec.states
        if st[0] is None:
            return list(st)
        return [s.clone() for s in st]

    @states.setter
    def states(self, states):
        self.multires_unetrec.states = states

    def detach_states(self):
        self.multires_unetrec.states = [s.detach() if s is not None else None for s in self.multires_unetrec.states]

    def reset_states(self):
        self.multires_unetrec.states = [None] * self.multires_unetrec.num_states

    def init_cropping(self, width, height, safety_margin=0):
        self.crop = CropParameters(width, height, self.num_encoders, safety_margin)

    def forward(self, event_voxel, event_cnt, log=False):
        if self.encoding == "voxel":
            x = event_voxel
        elif self.encoding == "cnt" and self.num_bins == 2:
            x = event_cnt
        else:
            print("Model error: Incorrect input encoding.")
            raise AttributeError
        if self.norm_input:
            nz = x != 0
            mean, std = x[nz].mean(), x[nz].std()
            x[nz] = (x[nz] - mean) / std
        x = x.float()
        if self.crop is not None:
            x = self.crop.pad(x)
        if log:
            raise NotImplementedError("Activity logging not implemented")  # as the reference (model.py:834-835)
        eng = self.engine
        u = self.multires_unetrec
        res = UNetStep.apply(eng, x, *u.states, *eng.params)
        flows = list(res[:4])
        u.states = list(res[4:])
        if self.crop is not None:
            flows = [f[:, :, self.crop.iy0:self.crop.iy1, self.crop.ix0:self.crop.ix1].contiguous() for f in flows]
        return {"flow": flows, "activity": None}


class CropParameters:
    """``models/model_util.py:41-79`` (zero padding to a multiple of 2**num_encoders, cropping back)."""

    def __init__(self, width, height, num_encoders, safety_margin=0):
        def crop_size(n):
            return int(pow(2, num_encoders) * math.ceil(n / pow(2, num_encoders))) + safety_margin * pow(2, num_encoders)

        self.height, self.width = height, width
        self.width_crop_size, self.height_crop_size = crop_size(width), crop_size(height)
        self.padding_top = math.ceil(0.5 * (self.height_crop_size - height))
        self.padding_bottom = math.floor(0.5 * (self.height_crop_size - height))
        self.padding_left = math.ceil(0.5 * (self.width_crop_size - width))
        self.padding_right = math.floor(0.5 * (self.width_crop_size - width))
        self.cx, self.cy = math.floor(self.width_crop_size / 2), math.floor(self.height_crop_size / 2)
        self.ix0, self.ix1 = self.cx - math.floor(width / 2), self.cx + math.ceil(width / 2)
        self.iy0, self.iy1 = self.cy - math.floor(height / 2), self.cy + math.ceil(height / 2)

    def pad(self, x):
        return torch.nn.functional.pad(x, (self.padding_left, self.padding_right, self.padding_top, self.padding_bottom))

    def crop(self, img):
        return img[..., self.iy0:self.iy1, self.ix0:self.ix1]


# ---------------------------------------------------------------------------
# kmaps: act position -> reference input channel
# ---------------------------------------------------------------------------
def kmap_identity(c, pitch):
    return [k if k < c else -1 for k in range(pitch)], [[k, -1, -1] for k in range(c)]


def kmap_split(c, pitch):
    km = [k % c if k < 3 * c else -1 for k in range(pitch)]
    return km, [[k, c + k, 2 * c + k] for k in range(c)]


def kmap_decoder(cx, cb, has_pred, pitch):
    """Decoder input act [x (cx) | block (cb) | pred hi0 hi1 mid0 mid1 lo0 lo1 | 0] against the
    reference concat order cat([pred (2), x, block]) (unet.py:455-457)."""
    o = 2 if has_pred else 0
    km, inv = [], []
    for k in range(pitch):
        if k < cx + cb:
            km.append(o + k)
        elif has_pred and k < cx + cb + 6:
            km.append((k - cx - cb) % 2)
        else:
            km.append(-1)
    if has_pred:
        inv = [[cx + cb + c, cx + cb + 2 + c, cx + cb + 4 + c] for c in range(2)]
    inv += [[k, -1, -1] for k in range(cx + cb)]
    return km, inv


class _Seg:
    """One GEMM input segment of a cell: the reference weight it multiplies, its act layout."""

    def __init__(self, weight, kmap, inv, pitch, mode, kc0, dev):
        self.weight = weight
        self.kmap = torch.tensor(kmap, dtype=torch.int32, device=dev)
        self.inv = torch.tensor(inv, dtype=torch.int32, device=dev)
        self.pitch, self.mode, self.kc0 = pitch, mode, kc0
        self.k0 = kc0 * 32
        self.wd = None  # input-gradient weight operand (made on demand)


class _CellPlan:
    """Device-side bookkeeping of one ConvLIF cell of the U-Net."""

    def __init__(self, mod, segs, dev):
        self.mod = mod
        self.C = mod.hidden_size
        self.ks = mod.ff.kernel_size[0]
        self.taps = self.ks * self.ks
        self.segs = segs
        self.kct = sum(s.pitch // 32 for s in segs)
        self.mp = mpad(self.C)
        self.gp = pad32(self.C)
        self.wf = torch.zeros(3 * self.taps * self.kct * self.mp * 32, dtype=BF16, device=dev)
        self.ktot = self.kct * 32
        self.dwk = torch.zeros(self.taps * self.ktot * self.C, device=dev)
        self.acc = torch.zeros(2 * self.C, dtype=torch.float64, device=dev)
        self.sg = _lib.SURROGATES.get(mod.activation)
        if self.sg is None:
            raise NotImplementedError(f"activation {mod.activation!r}")

    def prep(self, s):
        if not torch.cuda.is_current_stream_capturing():  # host copy of the act_width buffer (no read in a capture)
            self.width = float(self.mod.act_width)
        for sg in self.segs:
            w = sg.weight.detach()
            cin = w.shape[1]
            _lib.call("unet_prep_weights", lib.snnflow_unet_prep_weights, ptr(w), self.C, cin, self.ks, ptr(sg.kmap),
                      0, 0, 0, sg.kc0, sg.pitch // 32, self.kct, self.mp, ptr(self.wf), s)

    def prep_dgrad(self, sg, mvalid, s):
        w = sg.weight.detach()
        mp = mpad(mvalid)
        if sg.wd is None or sg.wd.numel() != 3 * self.taps * (self.gp // 32) * mp * 32:
            sg.wd = torch.zeros(3 * self.taps * (self.gp // 32) * mp * 32, dtype=BF16, device=w.device)
        _lib.call("unet_prep_weights(dgrad)", lib.snnflow_unet_prep_weights, ptr(w), self.C, w.shape[1], self.ks,
                  ptr(sg.kmap), 1, 1 if sg.mode == _lib.UNET_MODE_S1 else 0, mvalid, 0, self.gp // 32, self.gp // 32,
                  mp, ptr(sg.wd), s)
        sg.wd_mp = mp


def _unet_seg(act, mode, kc0, nparts=3):
    B, H, W, pitch = act.shape
    return _lib.UNetSeg(ptr(act), H, W, pitch, mode, kc0, nparts)


_PARTIAL = {}
_SHAPES = os.environ.get("SNNFLOW_UNET_SHAPES") == "1"  # profiling: kernel names carry the GEMM shape
# Tests: set to a list to record every GEMM launch's split plan as (kind, M, K, P, plan) -- plan is the
# split-K factor of a conv / input gradient, the partial-sum floats (pixel-split plan) of a weight gradient
PLAN_LOG = None
# Tests: an upper bound on the split-K factor of convs and input gradients (1: none), so that runs at
# different batch sizes sum every conv in the same order (split-K partitions K, not pixels)
KSPLIT_MAX = None


def _name(kind, M, K, P):
    return f"{kind}[M{M} K{K} P{P}]" if _SHAPES else kind


def _workspace(n, dev):
    buf = _PARTIAL.get(dev)
    if buf is None or buf.numel() < n:
        buf = torch.empty(n, device=dev)
        _PARTIAL[dev] = buf
    return buf


def _split_k(a, P, dev):
    """Split-K of a launch (library's choice) with the shared partial-sum workspace (stream-ordered
    reuse; sized by the largest request, which the eager warm-up steps make before any graph capture)."""
    ks = lib.snnflow_unet_conv_ksplit(ctypes.byref(a))
    if KSPLIT_MAX is not None:
        ks = min(ks, KSPLIT_MAX)
    if PLAN_LOG is not None:
        PLAN_LOG.append(("dgrad" if a.xparts == 3 else "conv", a.M, sum(a.seg[i].cpitch for i in range(a.nseg)), P, ks))
    if ks <= 1:
        a.ksplit, a.partial = 1, None
        return
    a.ksplit, a.partial = ks, _workspace(ks * P * a.M, dev).data_ptr()


def conv_lif(plan, B, Ho, Wo, acts, prev_state, residual, state, current, act_out, s):
    """Forward of one cell: implicit GEMM over its segments + the LIF epilogue."""
    a = _lib.UNetConvArgs()
    a.B, a.Ho, a.Wo, a.M, a.ksize = B, Ho, Wo, plan.C, plan.ks
    n = 0
    for sg, act in zip(plan.segs, acts):
        if act is None:
            continue
        a.seg[n] = _unet_seg(act, sg.mode, sg.kc0)
        n += 1
    a.nseg, a.xparts, a.pclass = n, 1, -1
    a.w, a.kct, a.mpad, a.epi = ptr(plan.wf), plan.kct, plan.mp, _lib.UNET_EPI_LIF
    m = plan.mod
    a.leak, a.thresh, a.hard_reset = ptr(m.leak), ptr(m.thresh), 1 if m.hard_reset else 0
    a.prev_state = ptr(prev_state)
    if residual is not None:
        a.residual, a.res_pitch = ptr(residual), residual.shape[-1]
    a.state, a.current, a.act, a.act_pitch = ptr(state), ptr(current), ptr(act_out), act_out.shape[-1]
    _split_k(a, B * Ho * Wo, state.device)
    _lib.call(_name("unet_conv", a.M, sum(a.seg[i].cpitch for i in range(n)), B * Ho * Wo), lib.snnflow_unet_conv,
              ctypes.byref(a), s, work=_conv_flops(plan, B * Ho * Wo, acts))


def _conv_flops(plan, P_out, acts=None):
    """Algorithmic FLOPs of a cell's convolution(s) (the reference's fp32 conv: 2 * output pixels *
    output channels * input channels * k^2), for the segments that take part."""
    cin = sum(sg.weight.shape[1] for sg, a in zip(plan.segs, acts or [True] * len(plan.segs)) if a is not None)
    return 2.0 * P_out * plan.C * cin * plan.taps


def conv_dgrad(plan, sg, g3, B, Hi, Wi, out, ld, mvalid, accumulate, s):
    """Input gradient of segment sg of a cell: transposed conv of the gradient held as hi/mid/lo
    bf16 planes (xparts 3) into out [B*Hi*Wi][ld] (fp32).  A stride-2 segment's transposed conv
    runs as four launches, one per output parity class, each over the taps that reach it."""
    a = _lib.UNetConvArgs()
    a.B, a.Ho, a.Wo, a.M, a.ksize = B, Hi, Wi, mvalid, plan.ks
    t2 = sg.mode == _lib.UNET_MODE_S2
    a.seg[0] = _unet_seg(g3[0], _lib.UNET_MODE_T2 if t2 else _lib.UNET_MODE_S1, 0, 3)
    a.nseg, a.xparts, a.xpart = 1, 3, g3[0].numel()
    a.w, a.kct, a.mpad, a.epi = ptr(sg.wd), plan.gp // 32, sg.wd_mp, _lib.UNET_EPI_STORE
    a.out, a.ld, a.accumulate = ptr(out), ld, 1 if accumulate else 0
    Ho, Wo = g3.shape[2], g3.shape[3]
    work = 2.0 * B * Ho * Wo * plan.C * sg.weight.shape[1] * plan.taps
    for cls in (range(4) if t2 else (-1,)):
        a.pclass = cls
        P = B * ((Hi - (cls >> 1) + 1) // 2) * ((Wi - (cls & 1) + 1) // 2) if t2 else B * Hi * Wi
        _split_k(a, P, out.device)
        _lib.call(_name("unet_dgrad", a.M, a.seg[0].cpitch, P), lib.snnflow_unet_conv, ctypes.byref(a), s,
                  work=work / 4 if t2 else work)


def wgrad(plan, sg, g3, B, Ho, Wo, act, s):
    a = _lib.UNetWgradArgs()
    a.B, a.Ho, a.Wo, a.M, a.ksize = B, Ho, Wo, plan.C, plan.ks
    a.g3, a.gpitch, a.gpart = ptr(g3), g3.shape[-1], g3[0].numel()
    a.seg = _unet_seg(act, sg.mode, sg.kc0)
    a.k0, a.ktot, a.dwk = sg.k0, plan.ktot, ptr(plan.dwk)
    n = lib.snnflow_unet_wgrad_partial_floats(ctypes.byref(a))  # deterministic split sums
    if PLAN_LOG is not None:
        PLAN_LOG.append(("wgrad", a.M, a.seg.cpitch, B * Ho * Wo, int(n)))
    a.partial = _workspace(n, plan.dwk.device).data_ptr() if n > 0 else None
    _lib.call(_name("unet_wgrad", plan.C, a.seg.cpitch, B * Ho * Wo), lib.snnflow_unet_wgrad, ctypes.byref(a), s,
              work=2.0 * B * Ho * Wo * plan.C * sg.weight.shape[1] * plan.taps)


def lif_bwd(plan, P, g_out, g_state, state, prev_state, current, g3, g_prev, g_res, s, res_assign=False):
    m = plan.mod
    a = _lib.UNetLifBwdArgs()
    a.P, a.C = P, plan.C
    a.leak, a.thresh, a.width = ptr(m.leak), ptr(m.thresh), plan.width
    a.hard_reset, a.detach, a.surrogate = 1 if m.hard_reset else 0, 1 if m.detach else 0, plan.sg
    if g_out is not None:
        a.g_out, a.g_pitch = ptr(g_out), g_out.shape[-1]
    a.g_state, a.state, a.prev_state, a.current = ptr(g_state), ptr(state), ptr(prev_state), ptr(current)
    a.g_cur3, a.gc_pitch, a.gc_part = ptr(g3), g3.shape[-1], g3[0].numel()
    a.g_prev = ptr(g_prev)
    if g_res is not None:
        a.g_res, a.gres_pitch = ptr(g_res), g_res.shape[-1]
        a.res_assign = 1 if res_assign else 0
    a.acc = ptr(plan.acc)
    # per-block sums reduced in block order (deterministic; no fp64 atomic contention on 2C addresses)
    n = int(lib.snnflow_unet_lif_bwd_partial_doubles(P, plan.C, a.gc_pitch))
    part = plan.__dict__.get("lif_part")
    if part is None or part.numel() < n or part.device != plan.acc.device:
        part = torch.empty(n, dtype=torch.float64, device=plan.acc.device)
        plan.lif_part = part
    a.partial = ptr(part)
    _lib.call("unet_lif_bwd", lib.snnflow_unet_lif_bwd, ctypes.byref(a), s)


def pack(src, split, pitch, s, out=None):
    """fp32 [B,C,H,W] (any strides) -> act [B,H,W,pitch] (bf16; split: hi|mid|lo channels)."""
    B, C, H, W = src.shape
    if out is None:
        out = torch.empty(B, H, W, pitch, dtype=BF16, device=src.device)
    sb, sc, sh, sw = src.stride()
    _lib.call("unet_pack", lib.snnflow_unet_pack, ptr(src), B, H, W, C, sb, sc, sh, sw, 1 if split else 0, ptr(out),
              pitch, s)
    return out


def nhwc_state(P, C, dev, cells=1):
    return torch.empty(cells, 2, P, C, device=dev)


def state_view(buf, B, C, H, W):
    """[cells][2][P][C] storage -> [2,B,C,H,W] (one cell) or [cells,2,B,C,H,W] view."""
    cells = buf.shape[0]
    P = B * H * W
    st = (P * C, H * W * C, 1, W * C, C)
    if cells == 1:
        return buf.as_strided((2, B, C, H, W), st)
    return buf.as_strided((cells, 2, B, C, H, W), (2 * P * C,) + st)


def as_cell_state(t, B, C, H, W):
    """Any [2,B,C,H,W] (or None) -> contiguous [2][P][C] fp32 storage (no copy if already)."""
    if t is None:
        return None
    if t.dtype == torch.float32 and t.stride() == (B * H * W * C, H * W * C, 1, W * C, C):
        return t
    out = torch.empty(2, B, H, W, C, device=t.device)
    out.copy_(t.permute(0, 1, 3, 4, 2))
    return out.as_strided((2, B, C, H, W), (B * H * W * C, H * W * C, 1, W * C, C))


# ---------------------------------------------------------------------------
# Engine
# ---------------------------------------------------------------------------
class UNetEngine:
    """Cell plans (weight operands, gradient accumulators) of one SpikingRecEVFlowNet."""

    def __init__(self, model):
        u = model.multires_unetrec
        self.model = model
        self.u = u
        self.params = list(model.parameters())
        self.dev = self.params[0].device
        self.base = u.base_num_channels
        if self.base % 4 != 0:
            raise NotImplementedError("snnflow U-Net: base_num_channels must be a multiple of 4")
        if u.num_encoders != 4 or u.num_output_channels != 2:
            raise NotImplementedError("snnflow U-Net: 4 encoders, 2 output channels")
        self.nb = u.num_bins
        if 3 * self.nb > 32:
            raise NotImplementedError("snnflow U-Net: num_bins <= 10")
        self.bwd_open = False
        self.pending_root = None
        self.prep_key = None
        self.prep_stale = True
        self._build()

    def _build(self):
        u, dev = self.u, self.dev
        S1, S2 = _lib.UNET_MODE_S1, _lib.UNET_MODE_S2
        self.enc = []
        in_pitch = 32
        in_map = kmap_split(self.nb, 32)
        for i, e in enumerate(u.encoders):
            c = e.conv.hidden_size
            cp = pad32(c)
            km, inv = in_map if i == 0 else kmap_identity(e.conv.input_size, in_pitch)
            pc = _CellPlan(e.conv, [_Seg(e.conv.ff.weight, km, inv, in_pitch, S2, 0, dev)], dev)
            kmi = kmap_identity(c, cp)
            pr = _CellPlan(e.recurrent_block, [_Seg(e.recurrent_block.ff.weight, *kmi, cp, S1, 0, dev),
                                               _Seg(e.recurrent_block.rec.weight, *kmi, cp, S1, cp // 32, dev)], dev)
            self.enc.append((pc, pr))
            in_pitch = cp
        self.res = []
        cm = u.max_num_channels
        for r in u.resblocks:
            kmi = kmap_identity(cm, pad32(cm))
            pa = _CellPlan(r.conv1, [_Seg(r.conv1.ff.weight, *kmi, pad32(cm), S1, 0, dev)], dev)
            pb = _CellPlan(r.conv2, [_Seg(r.conv2.ff.weight, *kmi, pad32(cm), S1, 0, dev)], dev)
            self.res.append((pa, pb))
        self.dec = []
        for i, d in enumerate(u.decoders):
            cx = u.encoder_output_sizes[3 - i]
            has_pred = i > 0
            pitch = pad32(2 * cx + (6 if has_pred else 0))
            km, inv = kmap_decoder(cx, cx, has_pred, pitch)
            pl = _CellPlan(d.conv2d, [_Seg(d.conv2d.ff.weight, km, inv, pitch, S1, 0, dev)], dev)
            pl.cx, pl.has_pred = cx, has_pred
            self.dec.append(pl)
        self.preds = [p.conv2d for p in u.preds]
        self.pred_acc = [torch.zeros(2 * p.weight.shape[1] + 2, dtype=torch.float64, device=dev) for p in self.preds]
        self.cells = [c for pair in self.enc for c in pair] + [c for pair in self.res for c in pair] + self.dec

    def prep_weights(self, s):
        key = tuple((p.data_ptr(), p._version) for p in self.params)
        if not self.prep_stale and key == self.prep_key:
            return
        self.prep_key = key
        self.prep_stale = False
        for c in self.cells:
            c.prep(s)
        # input-gradient operands (the encoder-0 input gets no gradient)
        for i, (pc, pr) in enumerate(self.enc):
            if i > 0:
                pc.prep_dgrad(pc.segs[0], pc.segs[0].pitch, s)
            pr.prep_dgrad(pr.segs[0], pr.segs[0].pitch, s)
            pr.prep_dgrad(pr.segs[1], pr.C, s)
        for pa, pb in self.res:
            pa.prep_dgrad(pa.segs[0], pa.segs[0].pitch, s)
            pb.prep_dgrad(pb.segs[0], pb.segs[0].pitch, s)
        for d in self.dec:
            d.prep_dgrad(d.segs[0], d.segs[0].pitch, s)

    def open_window(self):
        for c in self.cells:
            c.dwk.zero_()
            c.acc.zero_()
        for a in self.pred_acc:
            a.zero_()
        self.bwd_open = True

    def finalize(self, s):
        """Parameter gradients of the window, in self.params order, as views of ONE flat buffer
        (a single all-reduce / clip over it, snnflow.dp)."""
        total = sum(p.numel() for p in self.params)
        flat = torch.empty(total, device=self.dev)
        views, off = {}, 0
        for p in self.params:
            views[id(p)] = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        for c in self.cells:
            m = c.mod
            for sg in c.segs:
                w = sg.weight
                _lib.call("unet_wgrad_finalize", lib.snnflow_unet_wgrad_finalize, ptr(c.dwk), c.ktot, ptr(sg.inv),
                          sg.k0, sg.pitch, c.C, w.shape[1], c.ks, 0, ptr(views[id(w)]), s)
            _lib.call("unet_cell_param_grads", lib.snnflow_unet_cell_param_grads, ptr(c.acc), ptr(m.leak),
                      ptr(m.thresh), c.C, 0, ptr(views[id(m.leak)]), ptr(views[id(m.thresh)]), s)
        for p, acc in zip(self.preds, self.pred_acc):
            _lib.call("unet_pred_param_grads", lib.snnflow_unet_pred_param_grads, ptr(acc), p.weight.shape[1], 0,
                      ptr(views[id(p.weight)]), ptr(views[id(p.bias)]), s)
        self.last_flat = flat
        off, out = 0, []
        for p in self.params:  # fresh views: AccumulateGrad adopts them as .grad
            out.append(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        return out


class _StepCtx:
    pass


class UNetStep(torch.autograd.Function):
    """One time step of SpikingMultiResUNetRecurrent (unet.py:433-461) + the flow upsampling of
    SpikingRecEVFlowNet.forward (model.py:839-850).  Inputs: eng, x [B,nb,H,W], 10 states,
    parameters.  Outputs: 4 flows [B,2,H,W], 10 states."""

    @staticmethod
    def forward(ctx, eng, x, *rest):
        u = eng.u
        ns = u.num_states
        prev = list(rest[:ns])
        _lib.require_device(x, "event tensor")
        B, nb, H, W = x.shape
        if H % 16 or W % 16:
            raise _lib.SnnflowError("U-Net input must be a multiple of 16 (use init_cropping)")
        dev = x.device
        s = _stream(dev)
        eng.prep_weights(s)
        S = _StepCtx()
        S.B, S.H, S.W = B, H, W
        root = True
        for p in prev:
            if p is not None and p.requires_grad and getattr(p.grad_fn, "eng", None) is eng:
                root = False
        S.ext = [p is not None and p.requires_grad and getattr(p.grad_fn, "eng", None) is not eng for p in prev]

        # input act: hi / mid / lo bf16 channels of the event tensor (pack zero-fills the padding)
        a_in = pack(x, True, 32, s)
        S.acts = {"in": a_in}
        S.states, S.prev, S.cur = [], [], []
        out_states = []
        # encoders
        h, w = H, W
        xin = a_in
        for i, (pc, pr) in enumerate(eng.enc):
            h2, w2 = (h + 1) // 2, (w + 1) // 2
            P = B * h2 * w2
            C = pc.C
            st = nhwc_state(P, C, dev, cells=2)
            pv = prev[i]
            pv_c = pv_r = None
            if pv is not None:
                pv_c = as_cell_state(pv[0], B, C, h2, w2)
                pv_r = as_cell_state(pv[1], B, C, h2, w2)
            cur_c, cur_r = torch.empty(P, C, device=dev), torch.empty(P, C, device=dev)
            act_c = _act(B, h2, w2, C, dev)
            conv_lif(pc, B, h2, w2, [xin], pv_c, None, st[0], cur_c, act_c, s)
            zp = pack(pv_r[1], False, pad32(C), s) if pv_r is not None else None
            act_r = _act(B, h2, w2, C, dev)
            conv_lif(pr, B, h2, w2, [act_c, zp], pv_r, None, st[1], cur_r, act_r, s)
            S.acts[f"e{i}c"], S.acts[f"e{i}r"], S.acts[f"e{i}z"] = act_c, act_r, zp
            S.acts[f"e{i}in"] = xin
            S.states.append(st)
            S.prev.append((pv_c, pv_r))
            S.cur.append((cur_c, cur_r))
            out_states.append(state_view(st, B, C, h2, w2))
            xin, h, w = act_r, h2, w2
        # residual blocks
        for j, (pa, pb) in enumerate(eng.res):
            P, C = B * h * w, pa.C
            st = nhwc_state(P, C, dev, cells=2)
            pv = prev[4 + j]
            pv_a = pv_b = None
            if pv is not None:
                pv_a, pv_b = as_cell_state(pv[0], B, C, h, w), as_cell_state(pv[1], B, C, h, w)
            cur_a, cur_b = torch.empty(P, C, device=dev), torch.empty(P, C, device=dev)
            act_a, act_b = _act(B, h, w, C, dev), _act(B, h, w, C, dev)
            conv_lif(pa, B, h, w, [xin], pv_a, None, st[0], cur_a, act_a, s)
            conv_lif(pb, B, h, w, [act_a], pv_b, xin, st[1], cur_b, act_b, s)
            S.acts[f"r{j}in"], S.acts[f"r{j}a"], S.acts[f"r{j}b"] = xin, act_a, act_b
            S.states.append(st)
            S.prev.append((pv_a, pv_b))
            S.cur.append((cur_a, cur_b))
            out_states.append(state_view(st, B, C, h, w))
            xin = act_b
        # decoders + predictions
        flows_lo, flows = [], []
        pred = None
        for i, d in enumerate(eng.dec):
            h2, w2 = 2 * h, 2 * w
            P, C = B * h2 * w2, d.C
            din = torch.empty(B, h2, w2, d.segs[0].pitch, dtype=BF16, device=dev)
            blk = S.acts[f"e{3 - i}r"]
            _lib.call("unet_dec_in", lib.snnflow_unet_dec_in, ptr(xin), d.cx, xin.shape[-1], ptr(blk), d.cx,
                      blk.shape[-1], ptr(pred) if d.has_pred else None, B, h, w, ptr(din), din.shape[-1], s)
            st = nhwc_state(P, C, dev, cells=1)
            pv = as_cell_state(prev[6 + i], B, C, h2, w2)
            cur = torch.empty(P, C, device=dev)
            act = _act(B, h2, w2, C, dev)
            conv_lif(d, B, h2, w2, [din], pv, None, st[0], cur, act, s)
            pw = eng.preds[i]
            flo = torch.empty(B, 2, h2, w2, device=dev)
            ffull = torch.empty(B, 2, H, W, device=dev)
            _lib.call("unet_pred_fwd", lib.snnflow_unet_pred_fwd, ptr(act), act.shape[-1], C, ptr(pw.weight),
                      ptr(pw.bias), B, h2, w2, H // h2, ptr(flo), ptr(ffull), s)
            S.acts[f"d{i}in"], S.acts[f"d{i}"] = din, act
            S.states.append(st)
            S.prev.append((pv,))
            S.cur.append((cur,))
            flows_lo.append(flo)
            flows.append(ffull)
            out_states.append(state_view(st, B, C, h2, w2))
            xin, h, w, pred = act, h2, w2, flo
        S.flows_lo = flows_lo
        ctx.eng, ctx.S, ctx.root = eng, S, root
        ctx.set_materialize_grads(False)
        return (*flows, *out_states)

    @staticmethod
    def backward(ctx, *grads):
        eng, S = ctx.eng, ctx.S
        B, H, W = S.B, S.H, S.W
        g_flows = list(grads[:4])
        g_states = list(grads[4:])
        dev = eng.dev
        s = _stream(dev)
        if not eng.bwd_open:
            eng.open_window()
        keys = [f"e{i}{c}" for i in range(4) for c in "cr"] + [f"r{j}{c}" for j in range(len(eng.res)) for c in "ab"]
        keys += [f"d{i}" for i in range(4)]
        # dL/d act (fp32, act layout), not zero-filled: each buffer's first contribution is written
        # (assign / accumulate=False), the later ones added
        gacts = {k: torch.empty(S.acts[k].shape, device=dev) for k in keys}
        g_prev_out = [None] * len(g_states)

        def gstate_cell(i, cell, C, h, w):
            g = g_states[i]
            if g is None:
                return None
            gi = g[cell] if g.dim() == 6 else g
            return as_cell_state(gi, B, C, h, w)

        def g3_buf(P, C):
            return torch.empty(3, P, pad32(C), dtype=BF16, device=dev)

        # decoders, last first
        g_extra = None
        hs = [H // 8, H // 4, H // 2, H]
        ws = [W // 8, W // 4, W // 2, W]
        for i in range(3, -1, -1):
            d = eng.dec[i]
            h2, w2 = hs[i], ws[i]
            h, w = h2 // 2, w2 // 2
            P, C = B * h2 * w2, d.C
            act = S.acts[f"d{i}"]
            pw = eng.preds[i]
            gpre = torch.empty(B, 2, h2, w2, device=dev)
            gf = g_flows[i]
            if gf is not None:
                gf = gf.float().contiguous()
            npart = int(lib.snnflow_unet_pred_bwd_partial_doubles(B, h2, w2, C))
            part = d.__dict__.get("pred_part")
            if part is None or part.numel() < npart or part.device != dev:
                part = d.pred_part = torch.empty(npart, dtype=torch.float64, device=dev)
            _lib.call("unet_pred_bwd", lib.snnflow_unet_pred_bwd, ptr(act), act.shape[-1], C, ptr(pw.weight),
                      ptr(S.flows_lo[i]), ptr(gf), ptr(g_extra), B, h2, w2, H // h2, ptr(gpre), ptr(gacts[f"d{i}"]),
                      gacts[f"d{i}"].shape[-1], ptr(eng.pred_acc[i]), 1 if i == 3 else 0, ptr(part), s)
            g3 = g3_buf(P, C)
            gp = torch.empty(1, 2, P, C, device=dev)
            st = S.states[6 + i]
            lif_bwd(d, P, gacts[f"d{i}"], gstate_cell(6 + i, 0, C, h2, w2), st[0], S.prev[6 + i][0], S.cur[6 + i][0],
                    g3, gp[0], None, s)
            g_prev_out[6 + i] = state_view(gp, B, C, h2, w2)
            din = S.acts[f"d{i}in"]
            wgrad(d, d.segs[0], g3, B, h2, w2, din, s)
            gup = torch.empty(P, din.shape[-1], device=dev)
            conv_dgrad(d, d.segs[0], g3.view(3, B, h2, w2, -1), B, h2, w2, gup, din.shape[-1], din.shape[-1], False, s)
            gx = gacts["r1b"] if i == 0 else gacts[f"d{i - 1}"]
            gb = gacts[f"e{3 - i}r"]
            g_extra = torch.empty(B, 2, h, w, device=dev) if d.has_pred else None
            _lib.call("unet_dec_in_bwd", lib.snnflow_unet_dec_in_bwd, ptr(gup), din.shape[-1], d.cx, d.cx,
                      1 if d.has_pred else 0, B, h, w, ptr(gx), gx.shape[-1], ptr(gb), gb.shape[-1], ptr(g_extra), 3, s)
        # residual blocks, last first
        h, w = H // 16, W // 16
        for j in range(len(eng.res) - 1, -1, -1):
            pa, pb = eng.res[j]
            P, C = B * h * w, pa.C
            st = S.states[4 + j]
            gp = torch.empty(2, 2, P, C, device=dev)
            xin_key = "r0b" if j == 1 else "e3r"
            g3 = g3_buf(P, C)
            lif_bwd(pb, P, gacts[f"r{j}b"], gstate_cell(4 + j, 1, C, h, w), st[1], S.prev[4 + j][1], S.cur[4 + j][1],
                    g3, gp[1], gacts[xin_key], s, res_assign=xin_key != "e3r")
            wgrad(pb, pb.segs[0], g3, B, h, w, S.acts[f"r{j}a"], s)
            conv_dgrad(pb, pb.segs[0], g3.view(3, B, h, w, -1), B, h, w, gacts[f"r{j}a"], pad32(C), pad32(C), False, s)
            g3 = g3_buf(P, C)
            lif_bwd(pa, P, gacts[f"r{j}a"], gstate_cell(4 + j, 0, C, h, w), st[0], S.prev[4 + j][0], S.cur[4 + j][0],
                    g3, gp[0], None, s)
            wgrad(pa, pa.segs[0], g3, B, h, w, S.acts[f"r{j}in"], s)
            conv_dgrad(pa, pa.segs[0], g3.view(3, B, h, w, -1), B, h, w, gacts[xin_key], pad32(C), pad32(C), True, s)
            g_prev_out[4 + j] = state_view(gp, B, C, h, w)
        # encoders, last first
        for i in range(3, -1, -1):
            pc, pr = eng.enc[i]
            h, w = H >> (i + 1), W >> (i + 1)
            P, C = B * h * w, pc.C
            st = S.states[i]
            gp = torch.empty(2, 2, P, C, device=dev)
            g3 = g3_buf(P, C)
            lif_bwd(pr, P, gacts[f"e{i}r"], gstate_cell(i, 1, C, h, w), st[1], S.prev[i][1], S.cur[i][1], g3, gp[1],
                    None, s)
            wgrad(pr, pr.segs[0], g3, B, h, w, S.acts[f"e{i}c"], s)
            zp = S.acts[f"e{i}z"]
            if zp is not None:
                wgrad(pr, pr.segs[1], g3, B, h, w, zp, s)
                # previous spikes feed the recurrent conv before the reset detach (spiking_submodules.py:279, 288-289)
                conv_dgrad(pr, pr.segs[1], g3.view(3, B, h, w, -1), B, h, w, gp[1, 1], C, C, True, s)
            conv_dgrad(pr, pr.segs[0], g3.view(3, B, h, w, -1), B, h, w, gacts[f"e{i}c"], pad32(C), pad32(C), False, s)
            g3 = g3_buf(P, C)
            lif_bwd(pc, P, gacts[f"e{i}c"], gstate_cell(i, 0, C, h, w), st[0], S.prev[i][0], S.cur[i][0], g3, gp[0],
                    None, s)
            wgrad(pc, pc.segs[0], g3, B, h, w, S.acts[f"e{i}in"], s)
            if i > 0:
                gx = gacts[f"e{i - 1}r"]
                conv_dgrad(pc, pc.segs[0], g3.view(3, B, h, w, -1), B, 2 * h, 2 * w, gx, gx.shape[-1], gx.shape[-1],
                           True, s)
            g_prev_out[i] = state_view(gp, B, C, h, w)
        # gradients into the previous states: only where a previous state was given
        outs = []
        for k in range(len(g_prev_out)):
            pv = S.prev[k]
            outs.append(g_prev_out[k] if pv[0] is not None else None)
        pgrads = [None] * len(eng.params)
        if ctx.root:
            pgrads = eng.finalize(s)
            eng.bwd_open = False
            eng.prep_stale = True
        return (None, None, *outs, *pgrads)


def _act(B, H, W, C, dev):
    p = pad32(C)
    if p == C:
        return torch.empty(B, H, W, p, dtype=BF16, device=dev)
    return torch.zeros(B, H, W, p, dtype=BF16, device=dev)


def upsample_bilinear2x(x):
    """F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False) for a standalone
    SpikingUpsampleConvLayer call (the network path fuses it into the decoder input)."""
    return torch.nn.functional.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)


# ---------------------------------------------------------------------------
# Standalone cell call (ConvLIF / ConvLIFRecurrent outside the fused network step)
# ---------------------------------------------------------------------------
def _cell_plan(cell, cin, dev):
    """Implicit-GEMM plan of a standalone cell: the input (and previous spikes) packed as hi/mid/lo
    bf16 channels, so any fp32 input is exact (kmap_split)."""
    key = (cin, str(dev))
    plan = getattr(cell, "_unet_plan", None)
    if plan is not None and plan.key == key:
        return plan
    k = cell.ff.kernel_size[0]
    stride = cell.ff.stride[0]
    px = pad32(3 * cin)
    segs = [_Seg(cell.ff.weight, *kmap_split(cin, px), px, _lib.UNET_MODE_S2 if stride == 2 else _lib.UNET_MODE_S1,
                 0, dev)]
    if cell.recurrent:
        pz = pad32(3 * cell.hidden_size)
        segs.append(_Seg(cell.rec.weight, *kmap_split(cell.hidden_size, pz), pz, _lib.UNET_MODE_S1, px // 32, dev))
    plan = _CellPlan(cell, segs, dev)
    plan.key, plan.k, plan.stride = key, k, stride
    object.__setattr__(cell, "_unet_plan", plan)
    return plan


class ConvLIFCellFn(torch.autograd.Function):
    """One ConvLIF / ConvLIFRecurrent call (spiking_submodules.py:121-151 / 265-300) on the
    implicit-GEMM kernels: forward = pack + conv with the LIF epilogue; backward = LIF backward,
    weight gradients, input gradient and (recurrent) previous-spike gradient."""

    @staticmethod
    def forward(ctx, cell, x, prev, res, *params):
        _lib.require_device(x, "ConvLIF input")
        B, cin, H, W = x.shape
        dev = x.device
        s = _stream(dev)
        plan = _cell_plan(cell, cin, dev)
        C, k, st_ = plan.C, plan.k, plan.stride
        Ho, Wo = (H + 2 * (k // 2) - k) // st_ + 1, (W + 2 * (k // 2) - k) // st_ + 1
        if st_ == 2 and (Ho * 2 != H or Wo * 2 != W):
            raise _lib.SnnflowError("ConvLIF stride 2: even input sizes")
        P = B * Ho * Wo
        plan.prep(s)
        act_x = pack(x, True, plan.segs[0].pitch, s)
        act_z = None
        if cell.recurrent and prev is not None:
            act_z = pack(prev[1], True, plan.segs[1].pitch, s)
        state = torch.empty(1, 2, P, C, device=dev)
        cur = torch.empty(P, C, device=dev)
        act = _act(B, Ho, Wo, C, dev)
        conv_lif(plan, B, Ho, Wo, [act_x, act_z], prev, None, state[0], cur, act, s)
        sv = state_view(state, B, C, Ho, Wo)
        out = sv[1] + res if res is not None else sv[1].clone()
        ctx.plan, ctx.dims = plan, (B, cin, H, W, Ho, Wo)
        ctx.has_prev, ctx.has_res = prev is not None, res is not None
        ctx.act_x, ctx.act_z, ctx.cur = act_x, act_z, cur
        ctx.save_for_backward(state, *([prev] if prev is not None else []))
        ctx.set_materialize_grads(False)
        return out, sv

    @staticmethod
    def backward(ctx, g_out, g_state):
        plan = ctx.plan
        cell = plan.mod
        B, cin, H, W, Ho, Wo = ctx.dims
        state = ctx.saved_tensors[0]
        prev = ctx.saved_tensors[1] if ctx.has_prev else None
        dev = state.device
        s = _stream(dev)
        C, P = plan.C, B * Ho * Wo
        go = None
        if g_out is not None:
            go = g_out.float().permute(0, 2, 3, 1).contiguous()  # NHWC [P][C]
        gs = as_cell_state(g_state, B, C, Ho, Wo) if g_state is not None else None
        g3 = torch.empty(3, P, pad32(C), dtype=BF16, device=dev)
        g_prev = None
        if ctx.has_prev and ctx.needs_input_grad[2]:
            g_prev = torch.empty(1, 2, P, C, device=dev)
        plan.dwk.zero_()
        plan.acc.zero_()
        lif_bwd(plan, P, go, gs, state[0], prev, ctx.cur, g3, g_prev[0] if g_prev is not None else None, None, s)
        g3v = g3.view(3, B, Ho, Wo, -1)
        wgrad(plan, plan.segs[0], g3, B, Ho, Wo, ctx.act_x, s)
        if ctx.act_z is not None:
            wgrad(plan, plan.segs[1], g3, B, Ho, Wo, ctx.act_z, s)
        gx = None
        if ctx.needs_input_grad[1]:
            ld = (cin + 3) // 4 * 4
            plan.prep_dgrad(plan.segs[0], cin, s)
            gbuf = torch.empty(B, H, W, ld, device=dev)
            conv_dgrad(plan, plan.segs[0], g3v, B, H, W, gbuf, ld, cin, False, s)
            gx = gbuf[..., :cin].permute(0, 3, 1, 2)
        if g_prev is not None and ctx.act_z is not None:
            plan.prep_dgrad(plan.segs[1], C, s)
            conv_dgrad(plan, plan.segs[1], g3v, B, Ho, Wo, g_prev[0, 1], C, C, True, s)
        grads = []
        for sg in plan.segs:
            gw = torch.zeros_like(sg.weight)
            if sg is plan.segs[0] or ctx.act_z is not None:
                _lib.call("unet_wgrad_finalize", lib.snnflow_unet_wgrad_finalize, ptr(plan.dwk), plan.ktot, ptr(sg.inv),
                          sg.k0, sg.pitch, C, sg.weight.shape[1], plan.ks, 0, ptr(gw), s)
            grads.append(gw)
        gl, gt = torch.empty_like(cell.leak), torch.empty_like(cell.thresh)
        _lib.call("unet_cell_param_grads", lib.snnflow_unet_cell_param_grads, ptr(plan.acc), ptr(cell.leak),
                  ptr(cell.thresh), C, 0, ptr(gl), ptr(gt), s)
        g_res = g_out if (ctx.has_res and ctx.needs_input_grad[3]) else None
        gp = state_view(g_prev, B, C, Ho, Wo) if g_prev is not None else None
        return (None, gx, gp, g_res, *grads, gl, gt)
