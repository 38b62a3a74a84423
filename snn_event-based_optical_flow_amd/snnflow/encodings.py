"""Event encodings on the device with the reference's function API
(``dataloader/encodings.py:30-85``, ``dataloader/base.py`` create_*_encoding /
create_polarity_mask), running on the HIP encoder (csrc/encode.hip).

The reference encodes one window on the CPU inside the data loader; here whole
batches [B, N] are encoded by one launch on the GPU.  Inputs must be device tensors
(there is no CPU path); outputs are fresh fp32 tensors.
"""
import ctypes

import torch

from . import _lib
from ._lib import lib, ptr


def _field(t):
    _lib.require_device(t, "event field")
    return t


def _run(B, N, H, W, ts, ys, xs, ps, ev_stride, batch_stride, num_bins=0, round_ts=False, accumulate=True,
         want=()):
    dev = ps.device
    a = _lib.EncodeArgs()
    a.B, a.N, a.H, a.W = B, N, H, W
    a.ts, a.ys, a.xs, a.ps = ptr(ts), ptr(ys), ptr(xs), ptr(ps)
    a.ev_stride, a.batch_stride = ev_stride, batch_stride
    a.num_bins, a.round_ts, a.accumulate = num_bins, 1 if round_ts else 0, 1 if accumulate else 0
    out = {}
    if "cnt" in want:
        out["cnt"] = torch.empty(B, 2, H, W, device=dev)
        a.cnt = ptr(out["cnt"])
    if "voxel" in want:
        out["voxel"] = torch.empty(B, num_bins, H, W, device=dev)
        a.voxel = ptr(out["voxel"])
    if "image" in want:
        out["image"] = torch.empty(B, H, W, device=dev)
        a.image = ptr(out["image"])
    if "mask" in want:
        out["mask"] = torch.empty(B, 1, H, W, device=dev)
        a.mask = ptr(out["mask"])
    if "pol" in want:
        out["pol"] = torch.empty(B, N, 2, device=dev)
        a.pol_mask = ptr(out["pol"])
    _lib.call("encode_events", lib.snnflow_encode_events, ctypes.byref(a), _lib.stream_ptr(dev))
    return out


def _flat(*ts):
    return [_field(t.float().contiguous()) for t in ts]


def events_to_image(xs, ys, ps, sensor_size=(180, 240), accumulate=True):
    """``encodings.py:30-45``: index_put_ of ps at (ys, xs) into an [H, W] image."""
    xs, ys, ps = _flat(xs, ys, ps)
    H, W = int(sensor_size[0]), int(sensor_size[1])
    return _run(1, ps.numel(), H, W, None, ys, xs, ps, 1, 0, accumulate=accumulate, want=("image",))["image"][0]


def events_to_voxel(xs, ys, ts, ps, num_bins, sensor_size=(180, 240), round_ts=False):
    """``encodings.py:48-67``: temporal bilinear voxel grid [num_bins, H, W]."""
    xs, ys, ts, ps = _flat(xs, ys, ts, ps)
    H, W = int(sensor_size[0]), int(sensor_size[1])
    return _run(1, ps.numel(), H, W, ts, ys, xs, ps, 1, 0, num_bins=num_bins, round_ts=round_ts,
                want=("voxel",))["voxel"][0]


def events_to_channels(xs, ys, ps, sensor_size=(180, 240)):
    """``encodings.py:70-85``: per-polarity event counts [2, H, W]."""
    xs, ys, ps = _flat(xs, ys, ps)
    H, W = int(sensor_size[0]), int(sensor_size[1])
    return _run(1, ps.numel(), H, W, None, ys, xs, ps, 1, 0, want=("cnt",))["cnt"][0]


def create_mask_encoding(xs, ys, ps, sensor_size=(180, 240)):
    """``base.py:create_mask_encoding``: [1, H, W] image of |p| (accumulate=False)."""
    xs, ys, ps = _flat(xs, ys, ps)
    H, W = int(sensor_size[0]), int(sensor_size[1])
    return _run(1, ps.numel(), H, W, None, ys, xs, ps, 1, 0, want=("mask",))["mask"][0]


def create_polarity_mask(ps):
    """``base.py:create_polarity_mask``: [2, N] (positive, negative) masks."""
    (ps,) = _flat(ps)
    n = ps.numel()
    return _run(1, n, 1, 1, None, ps, ps, ps, 1, 0, want=("pol",))["pol"][0].t()


def encode_batch(event_list, resolution, num_bins=2, round_ts=False, voxel=True):
    """All network inputs of a batch of windows from its event list [B, N, 4] (ts, y, x, p),
    in the loader's collate layout: event_cnt [B,2,H,W], event_voxel [B,bins,H,W],
    event_mask [B,1,H,W], event_list_pol_mask [B,N,2] -- one launch."""
    ev = _field(event_list.float().contiguous())
    B, N, _ = ev.shape
    H, W = int(resolution[0]), int(resolution[1])
    base = ev.view(-1)
    want = ("cnt", "mask", "pol") + (("voxel",) if voxel else ())
    out = _run(B, N, H, W, base[0:], base[1:], base[2:], base[3:], 4, 4 * N, num_bins=num_bins, round_ts=round_ts,
               want=want)
    res = {"event_cnt": out["cnt"], "event_mask": out["mask"], "event_list_pol_mask": out["pol"]}
    if voxel:
        res["event_voxel"] = out["voxel"]
    return res
