"""Validation metrics with the reference's API (``loss/flow.py:306-937``: BaseValidationLoss,
AEE, NEE, AAE, NAAE, AE_ofMeans, AAE_Weighted, AAE_Filtered), the evaluation counterpart of
the training loss.

``AEE.forward`` runs the HIP kernels of csrc/eval.hip (per-pixel endpoint error,
validity, outliers, per-sample reduction); the other metrics share one pass
(``snnflow_flow_metrics``: every per-pixel term of every metric, per-block rows, a
fixed-order reduction), each class returning its own columns with the reference's
formulas and quirks (AAE's inverted cosine, batch-total outlier counts of AEE/NEE,
the unmasked numerator of AAE_Weighted).  The association bookkeeping is the
reference's (last flow map, event masks, ground truth, time scaling).  Error heatmap
accumulation for visualisation (``accumulate_error_heatmap`` and friends) is not part of
this path; ``get_error_map`` returns None.

Difference, documented: the reference multiplies the flow by ``dt_gt / dt_input`` with
plain broadcasting, which is only per-sample for a batch of one; here the ratio is applied
per sample for any batch size (identical for B = 1 and for scalar dt).
"""
import collections
import ctypes

import torch

from . import _lib
from ._lib import lib, ptr
from .iwe import compute_pol_iwe

_AEE_SCRATCH_STREAMS = 8  # AEE scratch buffers kept per metric object (one per stream, LRU)


class BaseValidationLoss(torch.nn.Module):
    """``loss/flow.py:306-475`` bookkeeping."""

    def __init__(self, config, device, flow_scaling=128):
        super().__init__()
        self.res = config["loader"]["resolution"]
        self.flow_scaling = flow_scaling
        self.overwrite_intermediate = config["loss"].get("overwrite_intermediate", False)
        self.device = device
        self.reset()

    def reset(self):
        self._passes = 0
        self._event_list = None
        self._pol_mask_list = None
        self._flow_map = None
        self._event_mask = None
        self._gtflow = None

    @property
    def num_events(self):
        return 0 if self._event_list is None else self._event_list.shape[1]

    def event_flow_association(self, flow_list, inputs):
        event_list = inputs["event_list"].to(self.device)
        pol_mask = inputs["event_list_pol_mask"].to(self.device)
        event_mask = inputs["event_mask"].to(self.device)
        gtflow = inputs["gtflow"].to(self.device) if "gtflow" in inputs else None
        flow = flow_list[-1]
        if self._event_list is None:
            self._event_list = event_list
            self._pol_mask_list = pol_mask
            self._event_mask = event_mask
            self._flow_map = []
        else:
            event_list = event_list.clone()
            event_list[:, :, 0:1] += self._passes
            self._event_list = torch.cat([self._event_list, event_list], dim=1)
            self._pol_mask_list = torch.cat([self._pol_mask_list, pol_mask], dim=1)
            self._event_mask = torch.cat([self._event_mask, event_mask], dim=1)
        self._flow_map.append(flow.reshape(flow.shape[0], 2, self.res[0], self.res[1]))
        self._gtflow = gtflow
        self._dt_input = inputs["dt_input"]
        self._dt_gt = inputs["dt_gt"]
        self._passes += 1

    def overwrite_intermediate_flow(self, flow_list):
        flow = flow_list[-1]
        self._flow_map = [flow.reshape(flow.shape[0], 2, self.res[0], self.res[1])]
        m = torch.sum(self._event_mask, dim=1, keepdim=True)
        m[m > 1] = 1
        self._event_mask = m

    def get_error_map(self):
        return None

    def compute_window_iwe(self, round_idx=True):
        """Per-polarity image of all window events warped with their window's flow (``:476-487``);
        uses the last flow map for every event (the reference's per-event flow list)."""
        pol = self._pol_mask_list
        return compute_pol_iwe(self._flow_map[-1], self._event_list, self.res, pol[:, :, 0:1], pol[:, :, 1:2],
                               flow_scaling=self.flow_scaling, round_idx=round_idx)


class AEE(BaseValidationLoss):
    """``loss/flow.py:597-649``: average endpoint error and outlier percentage per sample."""

    @property
    def num_events(self):
        return float("inf")

    def forward(self):
        flow = self._flow_map[-1].float().contiguous()
        B, _, H, W = flow.shape
        gt = self._gtflow.float().contiguous()
        mask = self._event_mask[:, -1, :, :].float().contiguous()
        # dt_gt / dt_input (one value for the batch, or B) divided in the kernel
        dtg = torch.as_tensor(self._dt_gt, dtype=torch.float32, device=flow.device).reshape(-1).contiguous()
        dti = torch.as_tensor(self._dt_input, dtype=torch.float32, device=flow.device).reshape(-1).contiguous()
        n = lib.snnflow_aee_acc_doubles(B, H, W)
        # the scratch carries the kernel's completion counter acc[0] (zero between calls: the last
        # block resets it), so it must never be shared by launches that can overlap: one scratch per
        # stream (a graph replays on the stream it was captured on, in order with eager calls there)
        # (a stream handle may be reused after its stream is destroyed: harmless, the counter is zero
        # between calls).  At most _AEE_SCRATCH_STREAMS streams are kept, least recently used dropped.
        stream = _lib.stream_ptr(flow.device)
        scratch = self.__dict__.setdefault("_aee_acc", collections.OrderedDict())
        key = (flow.device, stream)
        acc = scratch.pop(key, None)
        if acc is None or acc.numel() < n:
            acc = torch.zeros(n, dtype=torch.float64, device=flow.device)  # counter acc[0]: zero, kept zero
        scratch[key] = acc  # most recently used last
        while len(scratch) > _AEE_SCRATCH_STREAMS:
            scratch.popitem(last=False)
        aee = torch.empty(B, device=flow.device)
        pct = torch.empty(B, device=flow.device)
        a = _lib.AeeArgs()
        a.B, a.H, a.W = B, H, W
        a.flow, a.gtflow, a.event_mask, a.dt_ratio = ptr(flow), ptr(gt), ptr(mask), None
        a.dt_gt, a.dt_input, a.dt_gt_n, a.dt_input_n = ptr(dtg), ptr(dti), dtg.numel(), dti.numel()
        a.flow_scaling = float(self.flow_scaling)
        a.acc, a.aee, a.percent = ptr(acc), ptr(aee), ptr(pct)
        try:
            _lib.call("aee", lib.snnflow_aee, ctypes.byref(a), stream)
        except Exception:
            scratch.pop(key, None)  # a refused or failed launch may leave the counter nonzero: fresh scratch next time
            raise
        return aee, pct


def _flow_metrics(m, mag_threshold=0.5):
    """All SNNFLOW_M_* columns for the current association state of metric object m."""
    flow = m._flow_map[-1].float().contiguous()
    B, _, H, W = flow.shape
    gt = m._gtflow.float().contiguous()
    mask = m._event_mask[:, -1, :, :].float().contiguous()
    ratio = torch.as_tensor(m._dt_gt, dtype=torch.float32, device=flow.device) / torch.as_tensor(
        m._dt_input, dtype=torch.float32, device=flow.device)
    ratio = ratio.reshape(-1).expand(B).contiguous() if ratio.numel() == 1 else ratio.reshape(B).contiguous()
    rows = torch.empty(lib.snnflow_flow_metrics_rows(B, H, W), dtype=torch.float64, device=flow.device)
    out = torch.empty(B, len(_lib.METRICS), device=flow.device)
    a = _lib.FlowMetricsArgs()
    a.B, a.H, a.W = B, H, W
    a.flow, a.gtflow, a.event_mask, a.dt_ratio = ptr(flow), ptr(gt), ptr(mask), ptr(ratio)
    a.flow_scaling, a.mag_threshold = float(m.flow_scaling), float(mag_threshold)
    a.rows, a.out = ptr(rows), ptr(out)
    _lib.call("flow_metrics", lib.snnflow_flow_metrics, ctypes.byref(a), _lib.stream_ptr(flow.device))
    return {k: out[:, i] for i, k in enumerate(_lib.METRICS)}


class NEE(BaseValidationLoss):
    """``loss/flow.py:651-701``: normalised endpoint error |f-g| / (min(|f|,|g|) + 0.01) and
    the share of outliers (> 0.5), the latter counted over the whole batch as the reference does."""

    @property
    def num_events(self):
        return float("inf")

    def forward(self):
        r = _flow_metrics(self)
        return r["nee"], r["nee_pct"]


class AAE(BaseValidationLoss):
    """``loss/flow.py:703-762``: angular error with the reference's cosine
    (|f||g| / (f.g + 0.01), clamped) and the per-sample share of errors above pi/6."""

    @property
    def num_events(self):
        return float("inf")

    def forward(self):
        r = _flow_metrics(self)
        return r["aae"], r["aae_pct"]


class NAAE(BaseValidationLoss):
    """``loss/flow.py:764-820``: angular error divided by the predicted flow magnitude."""

    @property
    def num_events(self):
        return float("inf")

    def forward(self):
        return _flow_metrics(self)["naae"]


class AE_ofMeans(BaseValidationLoss):
    """``loss/flow.py:822-883``: angle between the masked mean flow and mean ground truth."""

    @property
    def num_events(self):
        return float("inf")

    def forward(self):
        return _flow_metrics(self)["ae_of_means"]


class AAE_Weighted(BaseValidationLoss):
    """``loss/flow.py:885-909``: magnitude-weighted angular error (numerator over all pixels,
    as in the reference)."""

    def forward(self):
        return _flow_metrics(self)["aae_weighted"]


class AAE_Filtered(BaseValidationLoss):
    """``loss/flow.py:911-937``: angular error over valid pixels with |f| >= mag_threshold."""

    def __init__(self, config, device, flow_scaling=128, mag_threshold=0.5):
        super().__init__(config, device, flow_scaling)
        self.mag_threshold = mag_threshold

    def forward(self):
        return _flow_metrics(self, self.mag_threshold)["aae_filtered"]
