"""``utils/iwe.py`` API on the HIP kernels.

``get_interpolation`` returns float-valued flat indices [B, K*M, 1] and weights
[B, K*M, 1] exactly like the reference (K = 4 bilinear corners, corner-major; K = 1
with ``round_idx``); the integer corner computation is bit-exact with the reference
(oracle/iwe_ref.py:warp_corners_np).  As in the reference, the bilinear weights carry
gradient back to the per-event flow (``utils/iwe.py:59, 65``) and ``interpolate``'s image
back to the weights (``:85, 91``): both are autograd Functions whose backward runs
``snnflow_iwe_corners_bwd`` / ``snnflow_iwe_interpolate_bwd``.  (The training loss does
not go through these: EventWarping fuses the whole chain, loss.py.)
"""
import torch

from . import _lib
from ._lib import check, lib, ptr


class _Corners(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ev, fl, tref, res, flow_scaling, round_idx):
        B, M = ev.shape[0], ev.shape[1]
        K = 1 if round_idx else 4
        idx = torch.empty(B, K * M, dtype=torch.int32, device=ev.device)
        w = torch.empty(B, K * M, device=ev.device)
        check(lib.snnflow_iwe_corners(ptr(ev), ptr(fl), B, M, float(tref), int(res[0]), int(res[1]),
                                      float(flow_scaling), int(bool(round_idx)), ptr(idx), ptr(w),
                                      _lib.stream_ptr(ev.device)), "iwe_corners")
        ctx.save_for_backward(ev, fl)
        ctx.args = (float(tref), int(res[0]), int(res[1]), float(flow_scaling))
        ctx.mark_non_differentiable(idx)
        return idx, w

    @staticmethod
    def backward(ctx, g_idx, g_w):
        ev, fl = ctx.saved_tensors
        if g_w is None or not ctx.needs_input_grad[1]:
            return None, None, None, None, None, None
        tref, H, W, s = ctx.args
        B, M = ev.shape[0], ev.shape[1]
        g_fl = torch.empty(B, M, 2, device=ev.device)
        gw = g_w.float().contiguous()
        check(lib.snnflow_iwe_corners_bwd(ptr(ev), ptr(fl), B, M, tref, H, W, s, ptr(gw), ptr(g_fl),
                                          _lib.stream_ptr(ev.device)), "iwe_corners_bwd")
        return None, g_fl, None, None, None, None


def get_interpolation(events, flow, tref, res, flow_scaling, round_idx=False):
    """``utils/iwe.py:20-71`` (includes ``purge_unfeasible``, ``:4-17``).  The weights are
    differentiable w.r.t. ``flow`` for the bilinear case (rounded weights are constant ones,
    as in the reference)."""
    _lib.require_device(events, "events")
    ev = events.detach().float().contiguous()
    fl = flow.float().contiguous()
    if round_idx:
        fl = fl.detach()
    idx, w = _Corners.apply(ev, fl, tref, res, flow_scaling, bool(round_idx))
    return idx.float().unsqueeze(-1), w.unsqueeze(-1)


def purge_unfeasible(x, res):
    """``utils/iwe.py:4-17`` on [B, N, 2] (y, x) locations."""
    bad = (x[:, :, 0:1] < 0) | (x[:, :, 0:1] >= res[0]) | (x[:, :, 1:2] < 0) | (x[:, :, 1:2] >= res[1])
    mask = (~bad).to(x.dtype)
    return x * mask, mask


class _Interpolate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ii, ww, pol, pol_sb, H, W):
        B, K = ii.shape
        img = torch.empty(B, 1, H, W, device=ww.device)
        check(lib.snnflow_iwe_interpolate(ptr(ii), ptr(ww), ptr(pol), pol_sb, B, K, H, W, ptr(img),
                                          _lib.stream_ptr(ww.device)), "iwe_interpolate")
        ctx.save_for_backward(ii, pol)
        ctx.dims = (pol_sb, H, W, pol is not None)
        return img

    @staticmethod
    def backward(ctx, g_img):
        ii, pol = ctx.saved_tensors
        pol_sb, H, W, has_pol = ctx.dims
        if g_img is None or not ctx.needs_input_grad[1]:
            return None, None, None, None, None, None
        B, K = ii.shape
        g = g_img.float().contiguous()
        g_w = torch.empty(B, K, device=g.device)
        check(lib.snnflow_iwe_interpolate_bwd(ptr(ii), ptr(pol) if has_pol else None, pol_sb, B, K, H, W, ptr(g),
                                              ptr(g_w), _lib.stream_ptr(g.device)), "iwe_interpolate_bwd")
        return None, g_w, None, None, None, None


def interpolate(idx, weights, res, polarity_mask=None):
    """``utils/iwe.py:74-93``: image of warped events [B, 1, H, W] (scatter-add), differentiable
    w.r.t. ``weights`` (the backward gathers the image gradient at each index)."""
    B, K = idx.shape[0], idx.shape[1]
    H, W = int(res[0]), int(res[1])
    ii = idx.detach().reshape(B, K).to(torch.int32).contiguous()
    if not (bool((ii >= 0).all()) and bool((ii < H * W).all())):  # utils/iwe.py:87-89 (host sync, as there)
        raise ValueError(f"Invalid idx values detected in interpolate: min={int(ii.min())}, max={int(ii.max())}")
    ww = weights.reshape(B, K).float().contiguous()
    pol = None
    pol_sb = 0
    if polarity_mask is not None:
        pol = polarity_mask.detach().reshape(B, K).float().contiguous()
        pol_sb = K
    return _Interpolate.apply(ii, ww, pol, pol_sb, H, W)


def _pol_iwe(flow, event_list, res, masks, flow_scaling, round_idx, tref=1.0):
    _lib.require_device(event_list, "event_list")
    ev = event_list.float().contiguous()
    fl = flow.float().contiguous()
    B, N = ev.shape[0], ev.shape[1]
    H, W = int(res[0]), int(res[1])
    if fl.shape[2] * fl.shape[3] != H * W:
        raise ValueError("flow map and resolution disagree")
    pol, stride, nimg = None, 0, 1
    if masks is not None:
        m0 = masks[0]
        if (len(masks) == 2 and all(m.dtype == torch.float32 and m.device == ev.device and tuple(m.shape) == (B, N, 1)
                                    and m.stride()[:2] == (2 * N, 2) for m in masks)
                and masks[1].data_ptr() == m0.data_ptr() + 4):
            pol, stride, nimg = m0, 2, 2  # the two columns of one [B][N][2] mask tensor: read in place
        else:
            pol = torch.cat([m.reshape(B, N, 1).float() for m in masks], dim=2).contiguous()
            stride, nimg = pol.shape[2], pol.shape[2]
    out = torch.empty(B, nimg, H, W, device=ev.device)
    check(lib.snnflow_pol_iwe(ptr(ev), ptr(fl), ptr(pol), stride, nimg, B, N, H, W, float(tref), float(flow_scaling),
                              int(bool(round_idx)), ptr(out), _lib.stream_ptr(ev.device)), "pol_iwe")
    return out


def deblur_events(flow, event_list, res, flow_scaling=128, round_idx=True, polarity_mask=None):
    """``utils/iwe.py:96-131``: image of the events warped to t=1 by the flow map [B,1,H,W]."""
    return _pol_iwe(flow, event_list, res, None if polarity_mask is None else [polarity_mask], flow_scaling,
                    round_idx)


def compute_pol_iwe(flow, event_list, res, pos_mask, neg_mask, flow_scaling=128, round_idx=True):
    """``utils/iwe.py:134-150``: per-polarity images of warped events [B,2,H,W] (one launch)."""
    return _pol_iwe(flow, event_list, res, [pos_mask, neg_mask], flow_scaling, round_idx)


def upsample_flow(flow, target_height, target_width):
    """``utils/iwe.py:153-171``: nearest-neighbour upsampling of a flow map."""
    return torch.nn.functional.interpolate(flow, size=(target_height, target_width), mode="nearest")
