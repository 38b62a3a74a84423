"""Contrast-maximisation loss with the reference's ``EventWarping`` API
(``loss/flow.py:28-303``) running on the HIP IWE kernels (csrc/iwe_loss.hip).

``event_flow_association`` only records the per-window tensors; ``forward`` runs
two kernels (warp + bilinear splat of all events of all windows into the 8 IWEs
-- forward/backward warp x {count, timestamp} x polarity -- then per-pixel loss
terms, Charbonnier smoothness and the batch reduction); its backward runs two
more (per-pixel image gradients + smoothness gradient, then per-event gradient
gathered from the 4 corners of both warps and scattered onto the flow maps).
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib, ptr


class _Scratch:
    def __init__(self):
        self.key = None

    def get(self, B, H, W, device):
        key = (B, H, W, device)
        if self.key != key:
            self.acc = torch.zeros(6 * B + 5, dtype=torch.float64, device=device)
            self.key = key
        return self


def _fill_args(meta, events, pol, masks, flows, images, persample, smooth, loss, scr):
    a = _lib.IweLossArgs()
    B, M = events.shape[0], events.shape[1]
    a.B, a.M, a.T, a.H, a.W, a.tf = B, M, meta["T"], meta["H"], meta["W"], flows.shape[1]
    a.events, a.pol, a.flows, a.masks = ptr(events), ptr(pol), ptr(flows), ptr(masks)
    for i, o in enumerate(meta["off"]):
        a.off[i] = o
    a.flow_scaling, a.weight = float(meta["flow_scaling"]), float(meta["weight"])
    a.smoothing_mask = 1 if meta["smoothing_mask"] else 0
    a.overwrite_intermediate = 1 if meta["overwrite_intermediate"] else 0
    a.loss_scaling = 1 if meta["loss_scaling"] else 0
    a.images, a.acc, a.persample, a.smooth, a.loss = ptr(images), ptr(scr.acc), ptr(persample), ptr(smooth), ptr(loss)
    return a


class EventWarpingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, scr, events, pol, masks, *flows):
        dev = events.device
        s = _lib.stream_ptr(dev)
        flows_all = torch.stack([f.float() for f in flows], dim=1).contiguous()  # [B, Tf, 2, H, W]
        B, H, W = events.shape[0], meta["H"], meta["W"]
        scr = scr.get(B, H, W, dev)
        images = torch.empty(8 * B * H * W, device=dev)
        persample = torch.empty(2 * B * 4, device=dev)
        smooth = torch.empty(8, device=dev)
        loss = torch.empty((), device=dev)
        a = _fill_args(meta, events, pol, masks, flows_all, images, persample, smooth, loss, scr)
        _lib.call("iwe_loss_fwd", lib.snnflow_iwe_loss_fwd, ctypes.byref(a), s)
        ctx.meta, ctx.scr = meta, scr
        ctx.save_for_backward(events, pol, masks, flows_all, images, persample, smooth)
        ctx.nflows = len(flows)
        return loss

    @staticmethod
    def backward(ctx, g):
        events, pol, masks, flows_all, images, persample, smooth = ctx.saved_tensors
        dev = events.device
        s = _lib.stream_ptr(dev)
        loss = torch.empty((), device=dev)
        a = _fill_args(ctx.meta, events, pol, masks, flows_all, images, persample, smooth, loss, ctx.scr)
        g = g.contiguous().float()
        gimg = torch.empty_like(images)
        g_flows = torch.empty_like(flows_all)
        _lib.call("iwe_loss_bwd", lib.snnflow_iwe_loss_bwd, ctypes.byref(a), ptr(g), ptr(gimg), ptr(g_flows), s)
        return (None, None, None, None, None, *g_flows.unbind(1))


class EventWarping(torch.nn.Module):
    """``loss/flow.py:EventWarping``: contrast maximisation (Zhu et al., CVPR'19) with
    forward and backward warps, loss scaling by the number of non-zero IWE pixels and
    Charbonnier smoothness (``flow_regul_weight``)."""

    def __init__(self, config, device, flow_scaling=None, loss_scaling=True):
        super().__init__()
        self.loss_scaling = loss_scaling
        self.res = config["loader"]["resolution"]
        self.flow_scaling = flow_scaling if flow_scaling is not None else max(config["loader"]["resolution"])
        self.weight = config["loss"]["flow_regul_weight"]
        self.smoothing_mask = config["model"].get("mask_output", False)
        self.overwrite_intermediate = config["loss"].get("overwrite_intermediate", False)
        self.device = device
        self._scratch = _Scratch()
        self.reset()

    def reset(self):
        self._passes = 0
        self._events, self._pols, self._masks, self._flows = [], [], [], []
        self._final_flow = None

    @property
    def num_events(self):
        return sum(e.shape[1] for e in self._events)

    @property
    def event_mask(self):
        m = torch.cat(self._masks, dim=1)
        if self.overwrite_intermediate:
            return self._overwritten_mask()
        return m[:, -1:, :, :]

    def event_flow_association(self, flow_list, event_list, pol_mask, event_mask):
        """Records one window (``loss/flow.py:58-121``).  The pass index is added to the
        timestamps inside the kernels (``:92``); the caller's ``event_list`` is not
        modified in place."""
        self._events.append(event_list.float().contiguous())
        self._pols.append(pol_mask.float().contiguous())
        self._masks.append(event_mask.float())
        self._flows.append(list(flow_list))
        self._passes += 1

    def overwrite_intermediate_flow(self, flow_list):
        """``loss/flow.py:123-150``: every window uses the final flow estimate."""
        self._final_flow = list(flow_list)

    def _overwritten_mask(self):
        m = torch.cat(self._masks, dim=1).sum(dim=1, keepdim=True)
        m[m > 1] = 1
        return m

    def forward(self):
        T = self._passes
        events = torch.cat(self._events, dim=1)
        pol = torch.cat(self._pols, dim=1)
        off = [0]
        for e in self._events:
            off.append(off[-1] + e.shape[1])
        H, W = int(self.res[0]), int(self.res[1])
        nflow = len(self._flows[0])
        if self.overwrite_intermediate and self._final_flow is not None:
            masks = self._overwritten_mask().reshape(events.shape[0], 1, H, W).contiguous()
        else:
            masks = torch.cat(self._masks, dim=1).reshape(events.shape[0], T, H, W).contiguous()
        meta = {"T": T, "H": H, "W": W, "off": off, "flow_scaling": self.flow_scaling, "weight": self.weight,
                "smoothing_mask": self.smoothing_mask, "overwrite_intermediate": self.overwrite_intermediate,
                "loss_scaling": self.loss_scaling}
        losses = []
        for i in range(nflow):
            if self.overwrite_intermediate and self._final_flow is not None:
                flows = [self._final_flow[i]]
            else:
                flows = [fl[i] for fl in self._flows]
            losses.append(EventWarpingFn.apply(meta, self._scratch, events, pol, masks, *flows))
        if nflow == 1:
            return losses[0]  # loss /= len(flow_list) with one flow map is the identity
        return sum(losses) / nflow
