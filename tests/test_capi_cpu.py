"""CPU-side checks of the C-ABI boundary (no GPU compute): the library loads, exports
every entry point include/snnflow.h declares, the ctypes mirrors have the C layout
(checked against gcc's sizeof/offsetof), and argument validation fails loudly before
any device work."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "snnflow.h")


def _declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(snnflow_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from snnflow import _lib

    names = _declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(_lib.lib, n), n
        assert n in _lib.EXPORTS, f"{n} has no ctypes prototype"
    assert _lib.lib.snnflow_abi_version() == _lib.ABI_VERSION


def test_struct_layouts_match_c(tmp_path):
    from snnflow import _lib

    structs = {
        "snnflow_neuron": _lib.Neuron, "snnflow_neuron_grad": _lib.NeuronGrad,
        "snnflow_conv_fwd_args": _lib.ConvFwdArgs, "snnflow_lif_fwd_args": _lib.LifFwdArgs,
        "snnflow_lif_bwd_args": _lib.LifBwdArgs, "snnflow_layer_bwd_args": _lib.LayerBwdArgs,
        "snnflow_slab_desc": _lib.SlabDesc, "snnflow_prep_desc": _lib.PrepDesc,
        "snnflow_wgrad_step": _lib.WgradStep, "snnflow_aee_args": _lib.AeeArgs, "snnflow_encode_args": _lib.EncodeArgs, "snnflow_convlif_params": _lib.ConvLifParams,
        "snnflow_convlif_fwd_args": _lib.ConvLifFwdArgs, "snnflow_convlif_bwd_args": _lib.ConvLifBwdArgs, "snnflow_wgrad_args": _lib.WgradArgs, "snnflow_iwe_loss_args": _lib.IweLossArgs,
        "snnflow_flow_metrics_args": _lib.FlowMetricsArgs,
        "snnflow_adam_tensor": _lib.AdamTensor, "snnflow_clip_adam_args": _lib.ClipAdamArgs,
        "snnflow_eval_fwd_args": _lib.EvalFwdArgs,
        "snnflow_unet_seg": _lib.UNetSeg, "snnflow_unet_conv_args": _lib.UNetConvArgs,
        "snnflow_unet_wgrad_args": _lib.UNetWgradArgs, "snnflow_unet_lif_bwd_args": _lib.UNetLifBwdArgs,
        "snnflow_bn_fwd_args": _lib.BnFwdArgs, "snnflow_bn_bwd_args": _lib.BnBwdArgs,
        "snnflow_pointwise_args": _lib.PointwiseArgs,
        "snnflow_firenet_plan": _lib.FireNetPlan, "snnflow_firenet_fwd_io": _lib.FireNetFwdIo,
        "snnflow_firenet_bwd_io": _lib.FireNetBwdIo, "snnflow_firenet_wgrad_step": _lib.FireNetWgradStep,
    }
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    for c_ in (4, 8, 16, 32):  # accumulator sizing macros vs the Python mirror
        lines.append(f'printf("acc_fwd_{c_} %d\\n", SNNFLOW_ACC_LEN(2 * {c_}));')
        lines.append(f'printf("acc_bwd_{c_} %d\\n", SNNFLOW_ACC_LEN(SNNFLOW_BWD_ACC({c_})));')
    lines.append(f'printf("abi %d\\n", SNNFLOW_ABI_VERSION);')
    lines.append(f'printf("theta_scratch %d\\n", SNNFLOW_THETA_SCRATCH);')
    lines.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(line.rsplit(" ", 1) for line in out if line)
    for c_ in (4, 8, 16, 32):
        assert int(got[f"acc_fwd_{c_}"]) == _lib.acc_storage(2 * c_)
        assert int(got[f"acc_bwd_{c_}"]) == _lib.acc_storage(_lib.bwd_acc_len(c_))
    assert int(got["abi"]) == _lib.ABI_VERSION
    assert int(got["theta_scratch"]) == _lib.THETA_SCRATCH
    for cname, py in structs.items():
        assert int(got[f"{cname} size"]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, f"{cname}.{fname}"


def test_argument_validation_without_gpu():
    from snnflow import _lib

    lib = _lib.lib
    a = _lib.ConvFwdArgs()
    assert lib.snnflow_conv_fwd(ctypes.byref(a), None) == -1
    assert b"conv_fwd" in lib.snnflow_last_error()
    a.B, a.H, a.W, a.c, a.cin = 1, 8, 8, 7, 2
    a.wt_ff = a.y = a.stats = a.x = 1
    assert lib.snnflow_conv_fwd(ctypes.byref(a), None) == -2  # no kernel for c=7
    e = _lib.IweLossArgs()
    assert lib.snnflow_iwe_loss_fwd(ctypes.byref(e), None) == -1
    assert lib.snnflow_conv_blocks(8, 128, 128) == 8 * 16 * 4
    assert lib.snnflow_slab_reduce(None, 1, 1, None) == -1
    ptrs, sizes = (ctypes.c_void_p * 17)(), (ctypes.c_int64 * 17)()
    assert lib.snnflow_count_nonzero(ptrs, sizes, 0, 1, None) == -1    # no tensor
    assert lib.snnflow_count_nonzero(ptrs, sizes, 17, 1, None) == -1   # > SNNFLOW_MAX_COUNT_TENSORS
    sizes[0] = 4
    assert lib.snnflow_count_nonzero(ptrs, sizes, 1, 1, None) == -1    # NULL data, non-empty
    assert b"count_nonzero" in lib.snnflow_last_error()
    ca = _lib.ClipAdamArgs()
    assert lib.snnflow_clip_adam(ctypes.byref(ca), None) == -1          # NULL buffers
    ca.grad = ca.exp_avg = ca.exp_avg_sq = ca.step = 1
    ca.n, ca.ntensors = 16, 1
    ca.t[0].param, ca.t[0].offset, ca.t[0].numel = 1, 8, 9             # range past n
    assert lib.snnflow_clip_adam(ctypes.byref(ca), None) == -1
    assert b"clip_adam" in lib.snnflow_last_error()
    ev = (_lib.EvalFwdArgs * 1)()
    assert lib.snnflow_eval_slot(ev, 0, None) == -1                    # no task
    ev[0].B, ev[0].H, ev[0].W, ev[0].c, ev[0].cin = 1, 8, 8, 8, 8
    ev[0].n.bn_train = 1
    assert lib.snnflow_eval_slot(ev, 1, None) == -1                    # train-mode BatchNorm refused
    assert b"eval_slot" in lib.snnflow_last_error()


def test_product_path_refuses_cpu_tensors():
    import torch

    import snnflow
    from oracle import lif_ref

    model = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=8))
    with pytest.raises(snnflow._lib.SnnflowError):
        model(None, torch.zeros(1, 2, 16, 16))


def test_wavefront_slots_respect_dependencies():
    """Every (kernel k, step t) task appears once; its inputs (k-1, t), (k, t-1), (k+1, t-1)
    run in strictly earlier launches; a launch never holds more than SNNFLOW_MAX_SLOT_TASKS."""
    from snnflow import _lib
    from snnflow.engine import wavefront_slots

    for T in (1, 2, 5, 10):
        for K in (6, 8):
            slots = wavefront_slots(T, K)
            where = {}
            for i, tasks in enumerate(slots):
                assert 0 < len(tasks) <= _lib.MAX_SLOT_TASKS
                for task in tasks:
                    assert task not in where
                    where[task] = i
            assert len(where) == T * K
            for (k, t), i in where.items():
                for dep in ((k - 1, t), (k, t - 1), (k + 1, t - 1)):
                    if dep in where:
                        assert where[dep] < i, (T, K, k, t, dep)


def test_slot_and_fragment_entry_points_validate_without_gpu():
    """snnflow_fwd_slot / snnflow_bwd_slot refuse bad task lists before any launch; the
    fragment size query matches the kernels' operand geometry (chunks x n-tiles x 3 x 512)."""
    from snnflow import _lib

    lib = _lib.lib
    assert lib.snnflow_slot_supported(8, 2) == 1 and lib.snnflow_slot_supported(32, 2) == 1
    assert lib.snnflow_slot_supported(16, 4) == 1 and lib.snnflow_slot_supported(12, 2) == 0
    assert lib.snnflow_slot_supported(8, 5) == 0
    conv = (_lib.ConvFwdArgs * 5)()
    assert lib.snnflow_fwd_slot(conv, 5, None, None) == -1          # more than 4 tasks
    assert lib.snnflow_fwd_slot(conv, 0, None, None) == -1          # no task
    for i in range(2):
        c = conv[i]
        c.B, c.H, c.W, c.c, c.cin, c.lif_in = 1, 8, 8, 8, 2, 0
        c.wt_ff = c.y = c.x = 1
    conv[1].H = 16
    assert lib.snnflow_fwd_slot(conv, 2, None, None) == -1          # tasks of different shapes
    assert b"shapes" in lib.snnflow_last_error()
    conv[0].c = conv[1].c = 12
    assert lib.snnflow_fwd_slot(conv, 1, None, None) == -2          # c not 8, 16 or 32
    conv[0].c = conv[0].cin = 32
    conv[0].wt_ff_t = 1
    assert lib.snnflow_fwd_slot(conv, 1, None, None) == -2          # c = 32: LIFFireNet task kinds only (no plain conv)
    assert b"task kinds" in lib.snnflow_last_error()
    layer = (_lib.LayerBwdArgs * 1)()
    assert lib.snnflow_bwd_slot(layer, 1, None, None) == -2         # c = 0
    layer[0].c = 8
    assert lib.snnflow_bwd_slot(layer, 1, None, None) == -1         # missing buffers
    assert lib.snnflow_frag_halfs(8, 8) == 3 * 1 * 3 * 512          # 3 K chunks (4 taps each)
    assert lib.snnflow_frag_halfs(16, 16) == 5 * 1 * 3 * 512
    assert lib.snnflow_frag_halfs(32, 32) == 9 * 2 * 3 * 512
    assert lib.snnflow_frag_halfs(32, 2) == 0 and lib.snnflow_frag_halfs(12, 12) == 0


_EXPORT_OP_PROBE = r"""
import os, sys, torch
sys.path.insert(0, os.path.join({repo!r}, "snn_event-based_optical_flow_amd"))
so = os.path.join({repo!r}, "oracle", "_ref", "lif_op.so")
if {ref_first} and os.path.exists(so):
    torch.ops.load_library(so)
from snnflow.export_op import register_lif_op
op = register_lif_op()
assert register_lif_op() is op
assert torch._C._dispatch_has_kernel_for_dispatch_key("SNN_implementation::LIF", "CUDA")
x = torch.empty(2, 3, 4, 5, device="meta")
s, m = op(x, x, torch.empty(3, device="meta"), torch.empty(3, device="meta"))
assert s.shape == x.shape and m.shape == x.shape and s.device.type == "meta"
xc = torch.ones(1, 2, 2, 2)
try:
    s, m = op(xc, torch.zeros_like(xc), torch.ones(2), torch.ones(2))
    print("cpu", int(s.sum().item()))
except NotImplementedError:
    print("cpu refused")
"""


@pytest.mark.parametrize("ref_first", [False, True])
def test_export_op_registration(ref_first):
    """snnflow.export_op registers the HIP kernel of torch.ops.SNN_implementation.LIF (the
    reference's op, ONNX_LIF_operator/src/lif_op.cpp:70-82): schema + Meta when the reference
    library is absent (host tensors refused: no CPU fallback), only the HIP kernel beside the
    reference's CPU/Meta kernels when its library was loaded first.  Fresh interpreter each:
    an op registry is per process."""
    import sys

    code = _EXPORT_OP_PROBE.format(repo=REPO, ref_first=ref_first)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    ref_loaded = ref_first and os.path.exists(os.path.join(REPO, "oracle", "_ref", "lif_op.so"))
    assert out.stdout.strip().splitlines()[-1] == ("cpu 8" if ref_loaded else "cpu refused")


def test_activity_dense_regions():
    """The activity log hands a tensor to snnflow_count_nonzero as one memory span only when
    its elements fill that span in some dimension order (else it is made contiguous first)."""
    import torch

    from snnflow.model import _dense

    x = torch.zeros(2, 3, 5, 4)
    assert _dense(x) and _dense(x.permute(0, 2, 3, 1)) and _dense(x[1]) and _dense(torch.zeros(0))
    st = torch.zeros(2, 4, 6, 7, 8).permute(0, 1, 4, 2, 3)  # [2,B,C,H,W] state over NHWC memory
    assert _dense(st) and _dense(st[1])
    assert not _dense(x[:, :2]) and not _dense(x[..., ::2]) and not _dense(x.expand(2, 3, 5, 4)[:, :, :1].expand(2, 3, 5, 4))


def test_event_warping_event_mask_shapes():
    """loss/flow.py:170-176: with overwrite_intermediate the property returns the stacked
    [B,T,H,W] masks until overwrite_intermediate_flow() collapses them to [B,1,H,W]; without it,
    the mask of the last pass.  (Bookkeeping only: no kernel runs.)"""
    import torch

    import snnflow

    B, T, H, W = 2, 3, 6, 7
    for overwrite in (False, True):
        cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001,
                                                          "overwrite_intermediate": overwrite},
               "model": {"mask_output": True}}
        ew = snnflow.EventWarping(cfg, "cpu")
        masks = [(torch.rand(B, 1, H, W) < 0.5).float() for _ in range(T)]
        flows = [torch.zeros(B, 2, H, W) for _ in range(T)]
        for t in range(T):
            ew.event_flow_association([flows[t]], torch.zeros(B, 4, 4), torch.zeros(B, 4, 2), masks[t])
        if overwrite:
            assert tuple(ew.event_mask.shape) == (B, T, H, W)
            assert torch.equal(ew.event_mask, torch.cat(masks, 1))
            ew.overwrite_intermediate_flow([flows[-1]])
            want = torch.cat(masks, 1).sum(1, keepdim=True).clamp(max=1)
            assert torch.equal(ew.event_mask, want)
        else:
            assert torch.equal(ew.event_mask, masks[-1])


def test_tebn_mpbn_model_loads_reference_state_dict_strict():
    """LIFFireNet with TEBN + MPBN cells has the reference's parameter/buffer names
    (bn.p, bn.bn.*, mpbn.bn.*): the reference model's state dict loads strict."""
    import numpy as np
    import torch
    import snnflow
    from oracle import lif_ref

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "liffirenet_norm_case.npz"))
    kw = lif_ref.make_unet_kwargs(base_num_channels=int(g["C"]))
    kw["tebn"], kw["mpbn"] = {"enabled": True, "num_timesteps": 4}, {"enabled": True}
    model = snnflow.LIFFireNet(kw)
    model.load_state_dict({k[3:]: torch.from_numpy(np.asarray(v)) for k, v in g.items() if k.startswith("p0.")},
                          strict=True)
    assert model.G1.tebn_enabled and model.G1.mpbn_enabled and model._cellwise()


def test_clip_adam_state_dict_loads_into_torch_adam():
    """ClipAdam keeps ONE device step counter for all parameters internally; its state dict must
    still be torch.optim.Adam's form (one step tensor per parameter), so that the reference's
    optimizer continues correctly from a saved optimizer_state_dict (train_flow.py:131-150):
    after one torch Adam step every parameter's step is n + 1 (a shared tensor would be n + P)."""
    import torch

    import snnflow

    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(s)) for s in ((3, 4), (5,), (2, 2, 3))]
    opt = snnflow.ClipAdam(params, lr=1e-3, max_norm=1.0)
    _, ea, es, step, _ = opt._state(params)  # the persistent flat moments (no kernel runs)
    ea.normal_()
    es.uniform_(0.1, 1.0)
    step.fill_(4.0)
    sd = opt.state_dict()
    steps = [sd["state"][i]["step"] for i in range(len(params))]
    assert all(s.device.type == "cpu" and s.dtype == torch.float32 and float(s) == 4.0 for s in steps)
    assert len({id(s) for s in steps}) == len(params)
    assert float(step) == 4.0 and opt.state[params[0]]["step"] is step  # the internal counter untouched
    twin = [torch.nn.Parameter(p.detach().clone()) for p in params]
    topt = torch.optim.Adam(twin, lr=1e-3, foreach=False)
    topt.load_state_dict(sd)
    for t in twin:
        t.grad = torch.ones_like(t)
    topt.step()
    assert [float(topt.state[t]["step"]) for t in twin] == [5.0] * len(params)
    # and back: a fresh ClipAdam picks the counter up from the per-parameter entries
    opt2 = snnflow.ClipAdam(params, lr=1e-3, max_norm=1.0)
    opt2.load_state_dict(topt.state_dict())
    m = opt2._state(params)
    assert float(m[3]) == 5.0
    assert torch.equal(m[1][:12], topt.state[twin[0]]["exp_avg"].reshape(-1))


def test_cell_constructor_options():
    """SNNtorch_ConvLIF(Recurrent) constructor options (SNNtorch_spiking_submodules.py:124-567):
    norm="weight" registers nn.utils.weight_norm's weight_g / weight_v (the reference's state-dict
    keys) and the cell's conv weights are the effective g v / ||v||; detach=False with MPBN builds;
    norm="group" and stride 2 raise NotImplementedError (not silently ignored)."""
    import torch

    import snnflow

    for cls in (snnflow.SNNtorch_ConvLIF, snnflow.SNNtorch_ConvLIFRecurrent):
        c = cls(8, 8, 3, norm="weight")
        keys = set(c.state_dict())
        assert {"ff.weight_g", "ff.weight_v"} <= keys and "ff.weight" not in keys
        assert (("rec.weight_g" in keys) == cls.recurrent)
        w = c._params()[0]
        assert torch.allclose(w, torch._weight_norm(c.ff.weight_v, c.ff.weight_g, 0))
        assert w.requires_grad  # the gradient reaches weight_g / weight_v through the reparametrisation
        cls(8, 8, 3, detach=False, mpbn=True)
        with pytest.raises(NotImplementedError):
            cls(8, 8, 3, norm="group")
    with pytest.raises(NotImplementedError):
        snnflow.SNNtorch_ConvLIF(8, 8, 3, stride=2)
    snnflow.SNNtorch_ConvLIFRecurrent(2, 8, 3)  # narrow event input into a recurrent cell
    with pytest.raises(NotImplementedError):
        snnflow.SNNtorch_ConvLIFRecurrent(3, 8, 3)
