"""The LIFFireNet family with the reference's module API (``models/model.py``).

Same class names, constructor (``unet_kwargs`` dict of ``configs/train_SNN.yml``'s
``model`` section), submodule names (head, G1, R1a, R1b, G2, R2a, R2b, pred),
``states`` / ``reset_states`` / ``detach_states`` / ``mask`` / ``init_cropping`` and
``forward(event_voxel, event_cnt, log, return_dict) -> {"flow": [B,2,H,W], "activity"}``.
A forward call is one fused time step on the GPU (engine.FireNetStep).  If forward
hooks are registered on a cell, or the cells carry TEBN / MPBN normalisation
(``unet_kwargs["tebn"|"mpbn"]``, ``models/model.py:74-83``), the cells are called one by one
instead (hooks see the reference's ``(spk, state)`` outputs).
"""
import copy
import ctypes

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .cells import ConvLayer, SNNtorch_ConvLIF, SNNtorch_ConvLIFRecurrent
from .engine import FireNetEngine, FireNetSequence, FireNetStep, eval_fused_ok, eval_sequence


class BaseModel(nn.Module):
    """``models/base.py:10-31``."""

    def __str__(self):
        n = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return super().__str__() + "\nTrainable parameters: {}".format(n)


def copy_states(states):
    """``models/model_util.py:96-102``: deepcopy a list of Nones, else clone."""
    if states[0] is None:
        return copy.deepcopy(states)
    return [s.clone() if hasattr(s, "clone") else type(s)(t.clone() for t in s) for s in states]


def _dense(t):
    """True when t's elements fill one contiguous memory span (any dimension order)."""
    dims = sorted((st, n) for st, n in zip(t.stride(), t.shape) if n > 1)
    expect = 1
    for st, n in dims:
        if st != expect:
            return False
        expect *= n
    return True


def activity_log(names, tensors):
    """``models/model.py:188-205``: ``{name: l.detach().ne(0).float().mean().item()}`` for every
    layer output of the step, as ONE ``snnflow_count_nonzero`` launch (wavefront ballots) and one
    read-back instead of a reduction and a host sync per tensor.  The counts are exact; the mean
    is the fp32 quotient count / numel, as torch's fp32 mean of 0/1 values below 2**24."""
    ts = [t.detach() for t in tensors]
    ts = [t if _dense(t) else t.contiguous() for t in ts]
    for t, n in zip(ts, names):
        _lib.require_device(t, n)
    counts = torch.empty(len(ts), dtype=torch.int64, device=ts[0].device)
    res = {}
    for i0 in range(0, len(ts), _lib.MAX_COUNT_TENSORS):
        chunk = ts[i0:i0 + _lib.MAX_COUNT_TENSORS]
        ptrs = (ctypes.c_void_p * len(chunk))(*[t.data_ptr() for t in chunk])
        sizes = (ctypes.c_int64 * len(chunk))(*[t.numel() for t in chunk])
        _lib.call("count_nonzero", _lib.lib.snnflow_count_nonzero, ptrs, sizes, len(chunk),
                  counts[i0:].data_ptr(), _lib.stream_ptr(ts[0].device))
    host = counts.cpu().numpy()
    for n, t, c in zip(names, ts, host):
        res[n] = float(np.float32(c) / np.float32(t.numel())) if t.numel() else float("nan")
    return res


class _FireNetBase(BaseModel):
    head_neuron = SNNtorch_ConvLIF
    ff_neuron = SNNtorch_ConvLIF
    rec_neuron = SNNtorch_ConvLIFRecurrent
    residual = False
    w_scale_pred = 0.01
    # (cell name, uses rec_neuron)
    layer_names = ()

    def __init__(self, unet_kwargs):
        super().__init__()
        self.num_bins = unet_kwargs["num_bins"]
        self.encoding = unet_kwargs["encoding"]
        self.norm_input = unet_kwargs.get("norm_input", False)
        self.mask = unet_kwargs["mask_output"]
        self.exporting = unet_kwargs.get("exporting", False)
        self.kwargs = [dict() for _ in range(self.num_recurrent_units)]
        if isinstance(unet_kwargs.get("spiking_neuron"), dict):
            for kw in self.kwargs:  # stored but, as in the reference, not passed to the cells
                kw.update(unet_kwargs["spiking_neuron"])
        C = unet_kwargs["base_num_channels"]
        k = unet_kwargs["kernel_size"]
        q = unet_kwargs.get("quantization", {})
        tebn = unet_kwargs.get("tebn", {})
        tebn = tebn.get("enabled", False) if isinstance(tebn, dict) else bool(tebn)
        mpbn = unet_kwargs.get("mpbn", {})
        mpbn = mpbn.get("enabled", False) if isinstance(mpbn, dict) else bool(mpbn)
        spec = []
        for i, (name, is_rec) in enumerate(self.layer_names):
            cls = self.head_neuron if i == 0 else (self.rec_neuron if is_rec else self.ff_neuron)
            cin = self.num_bins if i == 0 else C
            setattr(self, name, cls(cin, C, k, quantization_config=q, tebn=tebn, mpbn=mpbn))
            spec.append((name, cls is SNNtorch_ConvLIFRecurrent))
        self.layer_spec = spec
        self.pred = ConvLayer(C, out_channels=2, kernel_size=1, activation="tanh", w_scale=self.w_scale_pred,
                              quantization_config=q)
        self._engine = None
        self.reset_states()

    @property
    def num_recurrent_units(self):
        return len(self.layer_names)

    @property
    def engine(self):
        if self._engine is None:
            object.__setattr__(self, "_engine", FireNetEngine(self))
        return self._engine

    @property
    def states(self):
        return copy_states(self._states)

    @states.setter
    def states(self, states):
        self._states = states

    def detach_states(self):
        # models/model.py:126-130 detaches copies of the states; the kernels never write a state in
        # place (every step's states are new buffers), so detaching the states themselves gives the
        # same values without one clone launch per state
        self._states = [s.detach() if s is not None else None for s in self._states]

    def reset_states(self):
        self._states = [None] * self.num_recurrent_units

    def init_cropping(self, width, height):
        pass

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        if self._engine is not None:  # tensors moved or replaced: drop cached pointers
            self._engine.invalidate()
        return out

    def _mods(self):
        """The cells + pred (cached module list; submodules are not re-assigned)."""
        m = self.__dict__.get("_mods_cache")
        if m is None:
            m = [getattr(self, n) for n, _ in self.layer_spec] + [self.pred]
            self.__dict__["_mods_cache"] = m
        return m

    def _hooked(self):
        return any(m._forward_hooks or m._forward_pre_hooks for m in self._mods())

    def _cellwise(self):
        """Cells called one by one (each an autograd node on the HIP cell kernels): forward hooks
        registered, TEBN / MPBN cells (their extra normalisation sits between the fused kernels), or
        weight-normalised convolutions (the effective weights are formed per call)."""
        return self._hooked() or any(c.tebn_enabled or c.mpbn_enabled or getattr(c, "weight_norm", False)
                                     for c in self._mods()[:-1])

    def _input(self, event_voxel, event_cnt):
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
        return x.float()

    def forward_sequence(self, event_voxels=None, event_cnts=None, log=False):
        """T consecutive time steps in one call (not in the reference; its training loop calls
        ``forward`` once per window, ``train_flow.py:232-279``).  Same results, states and
        ``lif.mem`` caches as T ``forward`` calls -- returns their T result dicts -- with the
        steps' kernels issued as wavefront launches (engine.FireNetSequence).  In eval mode without
        autograd (eval_flow.py's loop under torch.no_grad()) at C = 8 the fused evaluation launches
        run instead (engine.eval_sequence: conv + BatchNorm + LIF per task, T + L - 1 launches).  With
        ``log`` the T activity dicts come from one count launch per 16 tensors and one read-back.
        Falls back to T ``forward`` calls where those launches do not apply (hooks, TEBN/MPBN,
        C = 4)."""
        seq = event_voxels if self.encoding == "voxel" else event_cnts
        T = len(seq)
        none = [None] * T
        pairs = list(zip(event_voxels if event_voxels is not None else none, event_cnts if event_cnts is not None else none))
        if T == 0:
            return []
        xs = [self._input(v, c) for v, c in pairs]
        eng = self.engine
        if T == 1 or self._cellwise() or not xs[0].is_cuda or not eng.sequence_ok(xs[0].shape[1]):
            outs = []
            for x in xs:  # already encoded / normalised: feed through the per-step path
                outs.append(self._step(x, log))
            return outs
        logging = isinstance(log, bool) and log and not self.exporting
        eng.keep_seq_states = logging or eng.capture_states
        try:
            if eval_fused_ok(eng, xs, self._states):  # eval mode, no autograd: conv + BN + LIF fused per task
                flows, fin = eval_sequence(eng, xs, list(self._states))
                res = list(flows) + list(fin)
            else:
                res = FireNetSequence.apply(eng, T, *xs, *self._states, *eng.param_list())
        finally:
            eng.keep_seq_states = False
        self._states = list(res[T:])
        outs = [{"flow": [f], "activity": None} for f in res[:T]]
        if logging:
            names = self._activity_names()
            sts, eng.seq_states = eng.seq_states, None
            tensors = [[x] + [st[1] for st in sts[t]] + [res[t]] for t, x in enumerate(xs)]
            keyed = [f"{t}/{n}" for t in range(T) for n in names]
            act = activity_log(keyed, [u for ts in tensors for u in ts])
            for t in range(T):
                outs[t]["activity"] = {n: act[f"{t}/{n}"] for n in names}
        return outs

    def _activity_names(self):
        names = ["0:input"] + [f"{i + 1}:{n}" for i, (n, _) in enumerate(self.layer_spec)]
        return names + [f"{len(self.layer_spec) + 1}:pred"]

    def forward(self, event_voxel=None, event_cnt=None, log=False, return_dict=True):
        out = self._step(self._input(event_voxel, event_cnt), log)
        return out if return_dict else out["flow"][0]

    def _step(self, x, log):
        if self._cellwise():
            h, outs = x, []
            for i, (name, _) in enumerate(self.layer_spec):
                h, self._states[i] = getattr(self, name)(h, self._states[i])
                outs.append(h)
            flow = self.pred(h)
        else:
            eng = self.engine
            res = FireNetStep.apply(eng, x, *self._states, eng.anchor(self._states))
            flow, new_states = res[0], list(res[1:])
            self.__dict__["_states"] = new_states  # (plain attribute; skips Module.__setattr__)
            outs = None
        activity = None
        if isinstance(log, bool) and log and not self.exporting:
            if outs is None:
                outs = [st[1] for st in new_states]
            activity = activity_log(self._activity_names(), [x] + outs + [flow])
        return {"flow": [flow], "activity": activity}


class LIFFireNet(_FireNetBase):
    """``models/model.py:29-207``."""

    layer_names = (("head", False), ("G1", True), ("R1a", False), ("R1b", False),
                   ("G2", True), ("R2a", False), ("R2b", False))


class LIFFireNet_short(_FireNetBase):
    """``models/model.py:210-384`` (R1b and R2b removed)."""

    layer_names = (("head", False), ("G1", True), ("R1a", False), ("G2", True), ("R2a", False))


class LIFFireFlowNet(_FireNetBase):
    """``models/model.py:387-554`` (feed-forward cells everywhere)."""

    rec_neuron = SNNtorch_ConvLIF
    layer_names = LIFFireNet.layer_names


class LIFFireFlowNet_short(_FireNetBase):
    """``models/model.py:557-720``."""

    rec_neuron = SNNtorch_ConvLIF
    layer_names = LIFFireNet_short.layer_names
