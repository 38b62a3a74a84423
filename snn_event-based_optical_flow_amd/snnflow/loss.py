"""Contrast-maximisation loss with the reference's ``EventWarping`` API
(``loss/flow.py:28-303``) running on the HIP IWE kernels (csrc/iwe_loss.hip).

``event_flow_association`` only records the per-window tensors, which the kernels read
in place through per-window pointer tables (nothing is concatenated).  ``forward`` runs
four kernels (include/snnflow.h snnflow_iwe_loss_fwd): k_iwe_wbin bins every event of a
(sample, window) by the 1024-pixel band of its warped corners (and, with one flow per window,
by the 512-pixel band of its own pixel for the backward); k_iwe_splat splats each band's
records into the 8 IWEs (forward/backward warp x {count, timestamp} x polarity) in exact
two-word fixed point; k_iwe_loss reduces the per (pixel, window) loss and Charbonnier
smoothness terms to per-block rows; k_iwe_finalize sums the rows in a fixed fp64 order.
The backward (snnflow_iwe_loss_bwd) is ONE kernel, k_iwe_bwd_band -- or two when the flows
are fewer than the windows (tf != T: k_iwe_bin forms the own-pixel binning first): per
(sample, flow window, band) the smoothness gradient of its pixels and each binned event's
flow gradient, formed at the 4 corners of both warps from the IWE values there and summed
onto its pixel's flow in exact fixed point.  The images scratch therefore holds the IWEs
AND both event binnings, and must be kept from the forward to the backward.  A corrupted
bin table is skipped and flagged (snnflow.check_device_errors), never read out of bounds.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib, ptr


class _Scratch:
    def __init__(self):
        self.key = None

    def get(self, B, H, W, tf, device):
        key = (B, H, W, tf, device)
        if self.key != key:
            self.acc = torch.empty(lib.snnflow_iwe_acc_doubles(B, H, W, tf), dtype=torch.float64, device=device)
            self.dummy = torch.zeros(8, device=device)  # pointer for empty event windows (never read)
            self.key = key
        return self


def _fill_args(meta, windows, flows, images, persample, smooth, loss, scr):
    """windows: (events [B,N_k,4], pols [B,N_k,2], masks [B,1,H,W]) per window, read in place."""
    evs, pols, masks = windows
    a = _lib.IweLossArgs()
    B = evs[0].shape[0]
    a.B, a.M, a.T, a.H, a.W, a.tf = B, meta["off"][-1], meta["T"], meta["H"], meta["W"], len(flows)
    for k, (e, p) in enumerate(zip(evs, pols)):
        a.events[k] = ptr(e) if e.numel() else ptr(scr.dummy)
        a.pol[k] = ptr(p) if p.numel() else ptr(scr.dummy)
    for t, (f, m) in enumerate(zip(flows, masks)):
        a.flows[t], a.masks[t] = ptr(f), ptr(m)
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
    def forward(ctx, meta, scr, windows, *flows):
        evs = windows[0]
        dev = evs[0].device
        s = _lib.stream_ptr(dev)
        if len(evs) > _lib.MAX_WINDOWS:
            raise _lib.SnnflowError(f"EventWarping: at most {_lib.MAX_WINDOWS} windows per loss")
        flows_c = [f.float().contiguous() for f in flows]  # [B, 2, H, W] each, no copy when already so
        B, H, W = evs[0].shape[0], meta["H"], meta["W"]
        # the kernels index every tensor by (B, H, W): a mis-shaped one would be read out of bounds
        for f in flows_c:
            _lib.require_device(f, "flow")
            if tuple(f.shape) != (B, 2, H, W):
                raise _lib.SnnflowError(f"EventWarping: flow of shape {tuple(f.shape)}, expected {(B, 2, H, W)} "
                                        "(event_flow_association takes a list of flow maps)")
        for e, p in zip(evs, windows[1]):
            if e.dim() != 3 or e.shape[0] != B or e.shape[2] != 4 or tuple(p.shape) != (B, e.shape[1], 2):
                raise _lib.SnnflowError(f"EventWarping: events {tuple(e.shape)} / polarity masks {tuple(p.shape)}, "
                                        f"expected [{B}, N, 4] / [{B}, N, 2]")
        for m in windows[2]:
            if tuple(m.shape) != (B, 1, H, W):
                raise _lib.SnnflowError(f"EventWarping: mask of shape {tuple(m.shape)}, expected {(B, 1, H, W)}")
        scr = scr.get(B, H, W, len(flows_c), dev)
        images = torch.empty(lib.snnflow_iwe_scratch_floats(B, meta["off"][-1], meta["T"], len(flows_c), H, W), device=dev)
        persample = torch.empty(2 * B * 4, device=dev)
        smooth = torch.empty(8, device=dev)
        loss = torch.empty((), device=dev)
        a = _fill_args(meta, windows, flows_c, images, persample, smooth, loss, scr)
        _lib.call("iwe_loss_fwd", lib.snnflow_iwe_loss_fwd, ctypes.byref(a), s)
        ctx.meta, ctx.scr, ctx.windows = meta, scr, windows
        ctx.save_for_backward(images, persample, smooth, *flows_c)
        return loss

    @staticmethod
    def backward(ctx, g):
        images, persample, smooth = ctx.saved_tensors[:3]
        flows_c = list(ctx.saved_tensors[3:])
        dev = images.device
        s = _lib.stream_ptr(dev)
        loss = torch.empty((), device=dev)
        a = _fill_args(ctx.meta, ctx.windows, flows_c, images, persample, smooth, loss, ctx.scr)
        g = g.contiguous().float()
        B, H, W = flows_c[0].shape[0], ctx.meta["H"], ctx.meta["W"]
        g_flows = torch.empty(B, len(flows_c), 2, H, W, device=dev)
        # (the events binned by pixel band in the images scratch; per band the flow gradients summed per
        # pixel in fixed point: bit-reproducible g_flows)
        _lib.call("iwe_loss_bwd", lib.snnflow_iwe_loss_bwd, ctypes.byref(a), ptr(g), ptr(g_flows), s)
        return (None, None, None, *g_flows.unbind(1))


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
        d = self.__dict__  # plain attributes (Module.__setattr__ skipped: once per window matters)
        d["_passes"] = 0
        d["_events"], d["_pols"], d["_masks"], d["_flows"] = [], [], [], []
        d["_final_flow"] = None

    @property
    def num_events(self):
        return sum(e.shape[1] for e in self._events)

    @property
    def event_mask(self):
        """``loss/flow.py:170-176``: with ``overwrite_intermediate`` the stacked [B,T,H,W] masks
        of the window, collapsed to [B,1,H,W] once ``overwrite_intermediate_flow`` ran
        (``:151-152``); otherwise the mask of the last pass."""
        m = torch.cat(self._masks, dim=1)
        if self.overwrite_intermediate:
            return self._overwritten_mask() if self._final_flow is not None else m
        return m[:, -1:, :, :]

    def event_flow_association(self, flow_list, event_list, pol_mask, event_mask):
        """Records one window (``loss/flow.py:58-121``).  The pass index is added to the
        timestamps inside the kernels (``:92``); the caller's ``event_list`` is not
        modified in place."""
        self._events.append(event_list.float().contiguous())
        self._pols.append(pol_mask.float().contiguous())
        self._masks.append(event_mask.float())
        self._flows.append(list(flow_list))
        self.__dict__["_passes"] += 1

    def overwrite_intermediate_flow(self, flow_list):
        """``loss/flow.py:123-150``: every window uses the final flow estimate."""
        self._final_flow = list(flow_list)

    def _overwritten_mask(self):
        m = torch.cat(self._masks, dim=1).sum(dim=1, keepdim=True)
        m[m > 1] = 1
        return m

    def forward(self):
        T = self._passes
        off = [0]
        for e in self._events:
            off.append(off[-1] + e.shape[1])
        H, W = int(self.res[0]), int(self.res[1])
        nflow = len(self._flows[0])
        overwrite = self.overwrite_intermediate and self._final_flow is not None
        if overwrite:
            masks = [self._overwritten_mask().reshape(-1, 1, H, W).contiguous()]
        else:
            masks = [m.reshape(-1, 1, H, W).contiguous() for m in self._masks]
        meta = {"T": T, "H": H, "W": W, "off": off, "flow_scaling": self.flow_scaling, "weight": self.weight,
                "smoothing_mask": self.smoothing_mask, "overwrite_intermediate": self.overwrite_intermediate,
                "loss_scaling": self.loss_scaling}
        windows = (list(self._events), list(self._pols), masks)
        losses = []
        for i in range(nflow):
            if overwrite:
                flows = [self._final_flow[i]]
            else:
                flows = [fl[i] for fl in self._flows]
            losses.append(EventWarpingFn.apply(meta, self._scratch, windows, *flows))
        if nflow == 1:
            return losses[0]  # loss /= len(flow_list) with one flow map is the identity
        return sum(losses) / nflow
