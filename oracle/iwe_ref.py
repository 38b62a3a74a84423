"""ORACLE (test infrastructure only) -- event warping, bilinear IWE splatting and
the contrast-maximisation loss of the reference, restated on the CPU.

Two restatements:
  * ``warp_corners_np``: plain numpy float32 arithmetic in the reference's exact
    operation order (no fused multiply-add) -> the bit-exact oracle for the
    integer corner indices / in-bounds masks and for the corner weights
    (``utils/iwe.py:20-71``).
  * ``get_interpolation_t`` / ``interpolate_t`` / ``EventWarpingRef``: torch fp32
    restatements with autograd, the oracle for IWE images, the loss value and
    dL/dflow (``utils/iwe.py:4-93``, ``loss/flow.py:28-303``); ``deblur_events_t`` /
    ``compute_pol_iwe_t`` the evaluation images (``utils/iwe.py:96-154``).
"""
import numpy as np
import torch

F32 = np.float32


# ---------------------------------------------------------------------------
# numpy bit-exact corner computation
# ---------------------------------------------------------------------------
def warp_corners_np(events, flow_ev, tref, res, flow_scaling, round_idx=False):
    """events [B,M,4] (ts,y,x,p) f32, flow_ev [B,M,2] (fy,fx) f32.

    Returns (idx [B,K*M] int64, weights [B,K*M] f32, inb [B,K*M] bool) with
    corners concatenated corner-major (K=4: TL, TR, BL, BR; K=1 for round_idx),
    matching ``utils/iwe.py:37-69``:
        w     = pos + ((tref - ts) * f) * s
        y0 = floor(wy), y1 = floor(wy + 1), x0 = floor(wx), x1 = floor(wx + 1)
        wt    = max(0, 1-|wy-cy|) * max(0, 1-|wx-cx|) * inb
        idx   = (cy*inb)*W + cx*inb       (computed in f32, exact below 2^24)
    """
    events = np.asarray(events, dtype=F32)
    flow_ev = np.asarray(flow_ev, dtype=F32)
    H, W = int(res[0]), int(res[1])
    ts = events[:, :, 0:1]
    dt = (F32(tref) - ts).astype(F32)
    warped = (events[:, :, 1:3] + ((dt * flow_ev).astype(F32) * F32(flow_scaling)).astype(F32)).astype(F32)
    wy, wx = warped[:, :, 0], warped[:, :, 1]
    if round_idx:
        corners = [(np.round(wy).astype(F32), np.round(wx).astype(F32))]  # half-to-even like torch.round
        wts = [np.ones_like(wy)]
    else:
        y0 = np.floor(wy).astype(F32)
        y1 = np.floor((wy + F32(1)).astype(F32)).astype(F32)
        x0 = np.floor(wx).astype(F32)
        x1 = np.floor((wx + F32(1)).astype(F32)).astype(F32)
        corners = [(y0, x0), (y0, x1), (y1, x0), (y1, x1)]

        def tri(w, c):
            return np.maximum(F32(0), (F32(1) - np.abs((w - c).astype(F32))).astype(F32)).astype(F32)

        wts = [(tri(wy, cy) * tri(wx, cx)).astype(F32) for cy, cx in corners]
    idx_l, wt_l, inb_l = [], [], []
    for (cy, cx), wt in zip(corners, wts):
        inb = (cy >= 0) & (cy < H) & (cx >= 0) & (cx < W)
        m = inb.astype(F32)
        idx = ((cy * m).astype(F32) * F32(W) + (cx * m).astype(F32)).astype(F32)
        idx_l.append(idx.astype(np.int64))
        wt_l.append((wt * m).astype(F32))
        inb_l.append(inb)
    return np.concatenate(idx_l, 1), np.concatenate(wt_l, 1), np.concatenate(inb_l, 1)


def event_pixel_index_np(events, res):
    """``loss/flow.py:66-69``: per-event flat pixel index y*W + x (f32 then long)."""
    e = np.asarray(events, dtype=F32)
    return ((e[:, :, 1] * F32(res[1])).astype(F32) + e[:, :, 2]).astype(F32).astype(np.int64)


# ---------------------------------------------------------------------------
# torch restatements (autograd-capable)
# ---------------------------------------------------------------------------
def purge_unfeasible_t(x, res):
    """``utils/iwe.py:4-17``."""
    bad = (x[:, :, 0:1] < 0) | (x[:, :, 0:1] >= res[0]) | (x[:, :, 1:2] < 0) | (x[:, :, 1:2] >= res[1])
    mask = (~bad).to(x.dtype)
    return x * mask, mask


def get_interpolation_t(events, flow, tref, res, flow_scaling, round_idx=False):
    """``utils/iwe.py:20-71`` -> (idx [B,K*M,1] f32-valued, weights [B,K*M,1])."""
    warped = events[:, :, 1:3] + (tref - events[:, :, 0:1]) * flow * flow_scaling
    if round_idx:
        idx = torch.round(warped)
        weights = torch.ones(idx.shape, dtype=warped.dtype)
    else:
        wy, wx = warped[:, :, 0:1], warped[:, :, 1:2]
        y0, y1 = torch.floor(wy), torch.floor(wy + 1)
        x0, x1 = torch.floor(wx), torch.floor(wx + 1)
        idx = torch.cat([torch.cat(c, dim=2) for c in ((y0, x0), (y0, x1), (y1, x0), (y1, x1))], dim=1)
        rep = torch.cat([warped] * 4, dim=1)
        weights = torch.max(torch.zeros(rep.shape, dtype=rep.dtype), 1 - torch.abs(rep - idx))
    idx, mask = purge_unfeasible_t(idx, res)
    weights = torch.prod(weights, dim=-1, keepdim=True) * mask
    flat = idx[:, :, 0:1] * res[1] + idx[:, :, 1:2]
    return flat, weights


def interpolate_t(idx, weights, res, polarity_mask=None):
    """``utils/iwe.py:74-93`` (scatter_add of weights into [B,1,H,W])."""
    if polarity_mask is not None:
        weights = weights * polarity_mask
    if not (bool((idx >= 0).all()) and bool((idx < res[0] * res[1]).all())):
        raise ValueError("Invalid idx values detected in interpolate")
    img = torch.zeros((idx.shape[0], res[0] * res[1], 1), dtype=weights.dtype)
    img = img.scatter_add_(1, idx.long(), weights)
    return img.view(idx.shape[0], 1, res[0], res[1])


def deblur_events_t(flow, event_list, res, flow_scaling=128, round_idx=True, polarity_mask=None):
    """``utils/iwe.py:96-130``: the flow vector at each event's pixel (gather; channel 1 = y,
    channel 0 = x), events warped to tref = 1, splatted into [B,1,H,W]."""
    B = flow.shape[0]
    pix = (event_list[:, :, 1] * res[1] + event_list[:, :, 2]).long()
    fl = flow.reshape(B, 2, -1)
    ev_flow = torch.stack([torch.gather(fl[:, 1], 1, pix), torch.gather(fl[:, 0], 1, pix)], dim=2)
    idx, w = get_interpolation_t(event_list, ev_flow, 1, res, flow_scaling, round_idx=round_idx)
    if not round_idx and polarity_mask is not None:
        polarity_mask = torch.cat([polarity_mask] * 4, dim=1)
    return interpolate_t(idx, w, res, polarity_mask)


def compute_pol_iwe_t(flow, event_list, res, pos_mask, neg_mask, flow_scaling=128, round_idx=True):
    """``utils/iwe.py:133-154``: [B,2,H,W] per-polarity images of warped events."""
    return torch.cat([deblur_events_t(flow, event_list, res, flow_scaling, round_idx, m) for m in (pos_mask, neg_mask)],
                     dim=1)


def _charbonnier(d):
    return torch.sqrt(d ** 2 + 1e-6)


class EventWarpingRef:
    """``loss/flow.py:EventWarping`` restated (association ``:58-121``, loss ``:178-303``).

    Differences kept on purpose: none in arithmetic.  ``event_flow_association``
    does not mutate the caller's ``event_list`` (the reference adds the pass index to
    its timestamps in place, ``:92``); the shifted copy is identical in value.
    """

    def __init__(self, res, flow_scaling=None, weight=0.001, smoothing_mask=True,
                 overwrite_intermediate=False, loss_scaling=True):
        self.res = list(res)
        self.flow_scaling = flow_scaling if flow_scaling is not None else max(res)
        self.weight = weight
        self.smoothing_mask = smoothing_mask
        self.overwrite_intermediate = overwrite_intermediate
        self.loss_scaling = loss_scaling
        self.reset()

    def reset(self):
        self._passes = 0
        self.events, self.flows_ev, self.pols, self.masks, self.maps = [], [], [], [], []

    @property
    def num_events(self):
        return sum(e.shape[1] for e in self.events)

    def event_flow_association(self, flow_list, event_list, pol_mask, event_mask):
        flow = flow_list[-1]
        B = flow.shape[0]
        pix = (event_list[:, :, 1] * self.res[1] + event_list[:, :, 2]).long()
        f = flow.reshape(B, 2, -1)
        fy = torch.gather(f[:, 1, :], 1, pix)
        fx = torch.gather(f[:, 0, :], 1, pix)
        self.flows_ev.append(torch.stack([fy, fx], dim=2))
        ev = event_list.clone()
        if self._passes > 0:
            ev[:, :, 0:1] += self._passes
        self.events.append(ev)
        self.pols.append(pol_mask)
        self.masks.append(event_mask)
        self.maps.append(flow)
        self._passes += 1

    def _iwe_term(self, events, flow_ev, pol4, tsw, tref):
        idx, w = get_interpolation_t(events, flow_ev, tref, self.res, self.flow_scaling)
        cnt_p = interpolate_t(idx, w, self.res, pol4[:, :, 0:1])
        cnt_n = interpolate_t(idx, w, self.res, pol4[:, :, 1:2])
        ts_p = interpolate_t(idx, w * tsw, self.res, pol4[:, :, 0:1])
        ts_n = interpolate_t(idx, w * tsw, self.res, pol4[:, :, 1:2])
        T = self._passes
        a = (ts_p / (cnt_p + 1e-9) / T).reshape(events.shape[0], -1)
        b = (ts_n / (cnt_n + 1e-9) / T).reshape(events.shape[0], -1)
        per_sample = torch.sum(a ** 2, dim=1) + torch.sum(b ** 2, dim=1)
        if self.loss_scaling:
            nz = (cnt_p + cnt_n).clone()
            nz[nz > 0] = 1
            per_sample = per_sample / torch.sum(nz.reshape(events.shape[0], -1), dim=1)
        return torch.sum(per_sample)

    def overwrite_intermediate_flow(self, flow_list):
        """``loss/flow.py:123-150``: re-gather every event's flow from the final map,
        keep a single flow map and a single (clipped) event mask."""
        flow = flow_list[-1]
        B = flow.shape[0]
        events = torch.cat(self.events, dim=1)
        pix = (events[:, :, 1] * self.res[1] + events[:, :, 2]).long()
        f = flow.reshape(B, 2, -1)
        self.flows_ev = [torch.stack([torch.gather(f[:, 1, :], 1, pix), torch.gather(f[:, 0, :], 1, pix)], dim=2)]
        self.events = [events]
        self.pols = [torch.cat(self.pols, dim=1)]
        m = torch.cat(self.masks, dim=1).sum(dim=1, keepdim=True)
        m[m > 1] = 1
        self.masks = [m]
        self.maps = [flow]

    def __call__(self):
        T = self._passes
        events = torch.cat(self.events, dim=1)
        flow_ev = torch.cat(self.flows_ev, dim=1)
        pol4 = torch.cat([torch.cat(self.pols, dim=1)] * 4, dim=1)
        ts4 = torch.cat([events[:, :, 0:1]] * 4, dim=1)
        fw = self._iwe_term(events, flow_ev, pol4, ts4, T)
        bw = self._iwe_term(events, flow_ev, pol4, T - ts4, 0)

        fx = torch.cat([m[:, 0:1] for m in self.maps], dim=1)
        fy = torch.cat([m[:, 1:2] for m in self.maps], dim=1)
        em = torch.cat(self.masks, dim=1)

        def pair(t, a, b):
            return t[a] - t[b]

        sl = slice(None)
        shifts = {
            "dx": ((sl, sl, sl, slice(None, -1)), (sl, sl, sl, slice(1, None))),
            "dy": ((sl, sl, slice(None, -1), sl), (sl, sl, slice(1, None), sl)),
            "dr": ((sl, sl, slice(None, -1), slice(None, -1)), (sl, sl, slice(1, None), slice(1, None))),
            "ur": ((sl, sl, slice(1, None), slice(None, -1)), (sl, sl, slice(None, -1), slice(1, None))),
            "dt": ((sl, slice(None, -1), sl, sl), (sl, slice(1, None), sl, sl)),
        }
        terms = []
        for key, (a, b) in shifts.items():
            if key == "dt" and self.overwrite_intermediate:
                continue
            d = _charbonnier(pair(fx, a, b) + pair(fy, a, b))
            if self.smoothing_mask:
                d = (em[a] * em[b]) * d
            terms.append(d)
        smooth = terms[0].sum()
        for t in terms[1:]:
            smooth = smooth + t.sum()
        smooth = smooth / len(terms) / fx.shape[1]  # flow_dx.shape[1]: number of flow maps (flow.py:293)
        return fw + bw + self.weight * smooth
