"""HIP kernel behind the reference's one native operator, ``torch.ops.SNN_implementation.LIF``.

Reference: schema and CPU/Meta registrations in ``ONNX_LIF_operator/src/lif_op.cpp:70-82``
(arithmetic ``:33-52``: ``m' = beta[c]*mem + x``; ``spk = m' >= thr[c]``; ``mem_out = spk ? 0 : m'``),
loaded with ``torch.ops.load_library`` (``Model_export.py:37-38``) and called by the export-mode
cells (``models/SNNtorch_spiking_submodules.py:651, 662, 782, 795``, ``models/model.py:892, 988``).

``register_lif_op()`` adds a HIP (``CUDA`` dispatch key under ROCm) implementation of that op that
launches ``snnflow_lif_export``; callers keep calling ``torch.ops.SNN_implementation.LIF(...)`` and
device tensors now run on the GPU.  When the reference's own library is loaded first, its schema,
CPU and Meta kernels stay as they are and only the HIP kernel is added; otherwise the schema and a
Meta kernel are defined here.  There is no CPU kernel from this package: a host-tensor call without
the reference library fails in the dispatcher, as the product path does everywhere.
Load the reference library BEFORE calling ``register_lif_op()`` if both are wanted (its
``TORCH_LIBRARY`` block refuses a namespace whose op is already defined).
"""
import torch

from . import _lib

NAMESPACE = "SNN_implementation"
SCHEMA = "LIF(Tensor input, Tensor mem, Tensor beta, Tensor threshold) -> (Tensor, Tensor)"

_registered = None


def _op_defined():
    try:
        getattr(getattr(torch.ops, NAMESPACE), "LIF")
        return True
    except (AttributeError, RuntimeError):
        return False


def lif_hip(input, mem, beta, threshold):
    """One LIF export step on the GPU: (spike, mem_out), fresh [N, C, H, W] fp32 tensors."""
    if input.dim() != 4:
        raise RuntimeError(f"SNN_implementation::LIF: input must be [N, C, H, W] (got {tuple(input.shape)})")
    N, C, H, W = input.shape
    if tuple(mem.shape) != tuple(input.shape):
        raise RuntimeError("SNN_implementation::LIF: mem must have the input's shape")
    if beta.numel() != C or threshold.numel() != C:
        raise RuntimeError("SNN_implementation::LIF: beta and threshold need one value per channel")
    x, m, b, t = (u.contiguous() for u in (input, mem, beta, threshold))
    for u, n in ((x, "input"), (m, "mem"), (b, "beta"), (t, "threshold")):
        _lib.require_device(u, n)
    spk = torch.empty_like(x)
    mem_out = torch.empty_like(x)
    _lib.call("lif_export", _lib.lib.snnflow_lif_export, x.data_ptr(), m.data_ptr(), b.data_ptr(), t.data_ptr(),
              N, C, H * W, spk.data_ptr(), mem_out.data_ptr(), _lib.stream_ptr(x.device))
    return spk, mem_out


def _lif_meta(input, mem, beta, threshold):
    return torch.empty_like(input), torch.empty_like(input)


def register_lif_op():
    """Register the HIP kernel of ``SNN_implementation::LIF`` (idempotent); returns the op."""
    global _registered
    if _registered is None:
        lib = torch.library.Library(NAMESPACE, "FRAGMENT")
        if not _op_defined():
            lib.define(SCHEMA)
            lib.impl("LIF", _lif_meta, "Meta")
        lib.impl("LIF", lif_hip, "CUDA")
        _registered = lib
    return torch.ops.SNN_implementation.LIF
