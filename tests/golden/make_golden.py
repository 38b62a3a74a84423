"""Generate the golden fixtures under tests/golden/ by running the REFERENCE code.

Run in the build container only (the reference tree does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

The reference's fp32 path imports third-party packages that are absent here
(snntorch, brevitas).  They are replaced by *import-only* stubs inserted into
``sys.modules``; the only stub that executes arithmetic is ``snntorch.Leaky``,
which is the oracle's restatement (``oracle.lif_ref.LeakyRef``) -- so fixtures
that go through ``SNNtorch_ConvLIF*`` / ``LIFFireNet`` pin the reference's conv,
BatchNorm, state and model wiring but NOT snntorch's LIF arithmetic (parity
unpinned for that piece).  Fixtures for ``utils/iwe.py``, ``loss/flow.py``,
``models/spiking_submodules.py`` and ``models/submodules.py:ConvLayer`` are
produced by reference code end to end.

Outputs are small .npz files (inputs + expected outputs), nothing else.
"""
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.lif_ref import LeakyRef  # noqa: E402


def install_stubs():
    class _Unavailable:
        def __init__(self, *a, **k):
            raise RuntimeError("quantized path is not part of the fixtures")

    snn = types.ModuleType("snntorch")

    class Leaky(LeakyRef):
        def __init__(self, beta, threshold=1.0, learn_beta=False, learn_threshold=False,
                     reset_mechanism="subtract", reset_delay=True, state_quant=False, **_):
            assert reset_delay is False and not state_quant
            super().__init__(torch.as_tensor(beta), torch.as_tensor(threshold), reset_mechanism)

    snn.Leaky = Leaky
    func = types.ModuleType("snntorch.functional")
    func.quant = types.SimpleNamespace(state_quant=_Unavailable)
    snn.functional = func
    sys.modules["snntorch"] = snn
    sys.modules["snntorch.functional"] = func
    bre = types.ModuleType("brevitas")
    bnn = types.ModuleType("brevitas.nn")
    for n in ("QuantConv2d", "QuantIdentity", "QuantTanh", "QuantReLU"):
        setattr(bnn, n, _Unavailable)
    bq = types.ModuleType("brevitas.quant")
    for n in ("Int8WeightPerTensorFloat", "Int8ActPerTensorFloat", "Int8Bias"):
        setattr(bq, n, object)
    bql = types.ModuleType("brevitas.nn.quant_layer")
    bql.QuantLayerMixin = object
    bcore = types.ModuleType("brevitas.core")
    bcq = types.ModuleType("brevitas.core.quant")
    bcq.QuantType = object
    bre.nn, bre.quant, bre.core = bnn, bq, bcore
    for name, mod in {"brevitas": bre, "brevitas.nn": bnn, "brevitas.quant": bq,
                      "brevitas.nn.quant_layer": bql, "brevitas.core": bcore,
                      "brevitas.core.quant": bcq}.items():
        sys.modules[name] = mod


def synth_events(gen, B, N, H, W):
    """Synthetic window in the reference's list layout [B,N,4] = (ts, y, x, p)."""
    ys = torch.randint(0, H, (B, N), generator=gen).float()
    xs = torch.randint(0, W, (B, N), generator=gen).float()
    ts = torch.sort(torch.rand(B, N, generator=gen), dim=1).values
    ts = (ts - ts[:, :1]) / (ts[:, -1:] - ts[:, :1])
    ps = torch.randint(0, 2, (B, N), generator=gen).float() * 2 - 1
    ev = torch.stack([ts, ys, xs, ps], dim=2)
    pol = torch.stack([(ps > 0).float(), (ps < 0).float()], dim=2)
    cnt = torch.zeros(B, 2, H, W)
    mask = torch.zeros(B, 1, H, W)
    for b in range(B):
        pos = ps[b] > 0
        cnt[b, 0].index_put_((ys[b][pos].long(), xs[b][pos].long()), torch.ones(int(pos.sum())), accumulate=True)
        cnt[b, 1].index_put_((ys[b][~pos].long(), xs[b][~pos].long()), torch.ones(int((~pos).sum())), accumulate=True)
        mask[b, 0, ys[b].long(), xs[b].long()] = 1
    return ev, pol, cnt, mask


def iwe_case(ref_iwe, out):
    """utils/iwe.py get_interpolation / interpolate incl. edge cases."""
    gen = torch.Generator().manual_seed(11)
    H, W, B, M = 12, 20, 2, 160
    ev, pol, _, _ = synth_events(gen, B, M, H, W)
    flow = (torch.rand(B, M, 2, generator=gen) - 0.5) * 0.3
    # edge cases: zero flow (exact-integer warps), exact half/integer displacements,
    # boundary pixels, far out-of-range warps, values that straddle floor(w + 1).
    flow[:, :8] = 0.0
    ev[:, 8:16, 0] = 0.5
    flow[:, 8:16, 0] = torch.tensor([2.0, -2.0, 1.0, -1.0, 0.25, -0.25, 4.0, -4.0]) / 20.0
    flow[:, 8:16, 1] = torch.tensor([-4.0, 4.0, 0.5, -0.5, 2.0, -2.0, 1.0, -1.0]) / 20.0
    ev[:, 16:20, 1] = torch.tensor([0.0, H - 1.0, 0.0, H - 1.0])
    ev[:, 16:20, 2] = torch.tensor([0.0, 0.0, W - 1.0, W - 1.0])
    flow[:, 20:24] = torch.tensor([[3.0, 3.0], [-3.0, -3.0], [3.0, -3.0], [-3.0, 3.0]])
    ev[:, 24, 1] = 3.0
    ev[:, 24, 0] = 1.0 - 2.0 ** -24
    flow[:, 24, 0] = -1e-8
    res = [H, W]
    rec = {"events": ev.numpy(), "flow_ev": flow.numpy(), "pol": pol.numpy(), "res": np.array(res)}
    for name, tref in (("fw", 3), ("bw", 0)):
        evk = ev.clone()
        evk[:, :, 0] += 1.0  # a second-pass window (ts + pass index)
        idx, w = ref_iwe.get_interpolation(evk, flow, tref, res, 20)
        pol4 = torch.cat([pol] * 4, dim=1)
        img_p = ref_iwe.interpolate(idx.long(), w, res, polarity_mask=pol4[:, :, 0:1])
        img_n = ref_iwe.interpolate(idx.long(), w, res, polarity_mask=pol4[:, :, 1:2])
        rec[f"{name}_idx"] = idx.long().numpy()[:, :, 0]
        rec[f"{name}_w"] = w.numpy()[:, :, 0]
        rec[f"{name}_iwe_pos"] = img_p.numpy()
        rec[f"{name}_iwe_neg"] = img_n.numpy()
    ridx, rw = ref_iwe.get_interpolation(ev, flow, 1, res, 20, round_idx=True)
    rec["round_idx"] = ridx.long().numpy()[:, :, 0]
    rec["round_w"] = rw.numpy()[:, :, 0]
    np.savez_compressed(os.path.join(out, "iwe_case.npz"), **rec)


def loss_case(ref_flow, out, overwrite=False, name="loss_case.npz"):
    """loss/flow.py EventWarping: value and dL/dflow over T windows."""
    gen = torch.Generator().manual_seed(12)
    H, W, B, N, T = 12, 20, 2, 96, 3
    config = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001,
              "overwrite_intermediate": overwrite}, "model": {"mask_output": True}}
    lossf = ref_flow.EventWarping(config, "cpu")
    flows, rec = [], {"res": np.array([H, W]), "T": T}
    for t in range(T):
        ev, pol, cnt, mask = synth_events(gen, B, N, H, W)
        f = ((torch.rand(B, 2, H, W, generator=gen) - 0.5) * 0.2).requires_grad_(True)
        if t == 1:
            with torch.no_grad():
                f[:, :, :3] = 0.0  # exact-integer warps on some rows
        flows.append(f)
        rec[f"events_{t}"] = ev.numpy().copy()
        rec[f"pol_{t}"] = pol.numpy()
        rec[f"mask_{t}"] = mask.numpy()
        rec[f"flow_{t}"] = f.detach().numpy().copy()
        lossf.event_flow_association([f], ev, pol, mask)
    if overwrite:
        lossf.overwrite_intermediate_flow([flows[-1]])
    loss = lossf()
    loss.backward()
    rec["loss"] = np.array(loss.item(), dtype=np.float32)
    for t in range(T):
        g = flows[t].grad
        rec[f"grad_{t}"] = g.numpy() if g is not None else np.zeros_like(rec[f"flow_{t}"])
    np.savez_compressed(os.path.join(out, name), **rec)


def spiking_cells_case(ref_sub, out):
    """models/spiking_submodules.py ConvLIF / ConvLIFRecurrent (U-Net flavour)."""
    torch.manual_seed(13)
    B, Cin, C, H, W, T = 2, 3, 4, 9, 11, 3
    rec = {}
    for tag, cls in (("ff", ref_sub.ConvLIF), ("rec", ref_sub.ConvLIFRecurrent)):
        cell = cls(Cin, C, 3, leak=(0.0, 1.0), thresh=(0.8, 0.1))
        xs = [(torch.rand(B, Cin, H, W) < 0.4).float() * 2.0 for _ in range(T)]
        state, outs, loss = None, [], 0
        for t in range(T):
            z, state = cell(xs[t], state)
            outs.append(z)
            loss = loss + (z * torch.linspace(-1, 1, z.numel()).view_as(z)).sum() + 0.3 * state[0].sum()
        loss.backward()
        for k, v in cell.state_dict().items():
            rec[f"{tag}.p.{k}"] = v.numpy()
        for n, p in cell.named_parameters():
            rec[f"{tag}.g.{n}"] = p.grad.numpy()
        for t in range(T):
            rec[f"{tag}.x_{t}"] = xs[t].numpy()
            rec[f"{tag}.z_{t}"] = outs[t].detach().numpy()
        rec[f"{tag}.v_last"] = state[0].detach().numpy()
    np.savez_compressed(os.path.join(out, "spiking_cells_case.npz"), **rec)


# the cell options outside spiking_cells_case (other surrogates, soft reset, detach=False, stride 2)
CELL_VARIANTS = [tuple(v) for v in json.load(open(os.path.join(HERE, "cell_variants.json")))["variants"]]


def spiking_cell_variants_case(ref_sub, out):
    """models/spiking_submodules.py ConvLIF / ConvLIFRecurrent for CELL_VARIANTS: 2 steps from a
    random initial state; spikes, states and the gradients of the inputs, the initial state and
    every parameter of loss = sum(z * wz) + 0.3 * sum(v) per step."""
    rec = {}
    for i, (tag, recurrent, stride, cin, C, act, width, hard, detach) in enumerate(CELL_VARIANTS):
        torch.manual_seed(60 + i)
        kw = dict(activation=act, act_width=width, leak=(0.0, 1.0), thresh=(0.5, 0.2), hard_reset=hard, detach=detach)
        cell = (ref_sub.ConvLIFRecurrent(cin, C, 3, **kw) if recurrent
                else ref_sub.ConvLIF(cin, C, 3, stride=stride, **kw))
        gen = torch.Generator().manual_seed(70 + i)
        B, H, W = 2, 8, 12
        Ho, Wo = H // stride, W // stride
        s0 = torch.randn(2, B, C, Ho, Wo, generator=gen) * 0.5
        s0[1] = (s0[1] > 0).float()
        s0.requires_grad_(True)
        xs = [((torch.rand(B, cin, H, W, generator=gen) < 0.5).float() * 1.5).requires_grad_(True) for _ in range(2)]
        state, loss = s0, 0
        for t in range(2):
            z, state = cell(xs[t], state)
            wz = torch.randn(B, C, Ho, Wo, generator=gen)
            loss = loss + (z * wz).sum() + 0.3 * state[0].sum()
            rec[f"{tag}.x_{t}"] = xs[t].detach().numpy()
            rec[f"{tag}.wz_{t}"] = wz.numpy()
            rec[f"{tag}.z_{t}"] = z.detach().numpy()
            rec[f"{tag}.state_{t}"] = state.detach().numpy()
        loss.backward()
        rec[f"{tag}.s0"] = s0.detach().numpy()
        rec[f"{tag}.gs0"] = s0.grad.numpy()
        for t in range(2):
            rec[f"{tag}.gx_{t}"] = xs[t].grad.numpy()
        for k, v in cell.state_dict().items():
            rec[f"{tag}.p.{k}"] = v.numpy()
        for n, p in cell.named_parameters():
            rec[f"{tag}.g.{n}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(out, "spiking_cell_variants_case.npz"), **rec)


def liffirenet_case(ref_model, ref_flow, out, name="LIFFireNet", C=4, fname=None, norm=False):
    """models/model.py LIFFireNet (reference wiring, conv, BN, states) with the
    restated Leaky; T forwards + EventWarping + backward, train mode.  norm: TEBN and MPBN
    enabled (models/model.py:74-83) with their parameters perturbed from the ones/zeros init."""
    sys.path.insert(0, REPO)
    from oracle.lif_ref import make_unet_kwargs

    torch.manual_seed(14)
    gen = torch.Generator().manual_seed(15)
    H, W, B, N, T = 16, 16, 2, 128, 3
    kw = make_unet_kwargs(base_num_channels=C)
    kw["name"] = name
    if norm:
        kw["tebn"] = {"enabled": True, "num_timesteps": 4}
        kw["mpbn"] = {"enabled": True}
    model = getattr(ref_model, name)(dict(kw))
    if norm:
        pg = torch.Generator().manual_seed(16)
        with torch.no_grad():
            for n, p in model.named_parameters():
                if n.endswith("bn.p") or ".mpbn.bn.weight" in n:
                    p.copy_(0.5 + torch.rand(p.shape, generator=pg))
                elif ".mpbn.bn.bias" in n:
                    p.copy_(0.4 * torch.rand(p.shape, generator=pg) - 0.2)
    model.train()
    config = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001,
              "overwrite_intermediate": False}, "model": {"mask_output": True}}
    lossf = ref_flow.EventWarping(config, "cpu")
    rec = {"res": np.array([H, W]), "T": T, "C": C}
    for k, v in model.state_dict().items():
        rec[f"p0.{k}"] = v.numpy().copy()
    for t in range(T):
        ev, pol, cnt, mask = synth_events(gen, B, N, H, W)
        x = model(None, cnt)
        lossf.event_flow_association(x["flow"], ev.clone(), pol, mask)
        rec[f"cnt_{t}"] = cnt.numpy()
        rec[f"events_{t}"] = ev.numpy()
        rec[f"pol_{t}"] = pol.numpy()
        rec[f"mask_{t}"] = mask.numpy()
        rec[f"flow_{t}"] = x["flow"][0].detach().numpy()
        for i, s in enumerate(model._states):
            rec[f"state_{t}_{i}"] = s.detach().numpy()
    loss = lossf()
    loss.backward()
    rec["loss"] = np.array(loss.item(), dtype=np.float32)
    for n, p in model.named_parameters():
        rec[f"g.{n}"] = p.grad.numpy()
    for k, v in model.state_dict().items():
        rec[f"p1.{k}"] = v.numpy().copy()
    np.savez_compressed(os.path.join(out, fname or f"{name.lower()}_case.npz"), **rec)


def convlayer_case(ref_sub, out):
    torch.manual_seed(16)
    layer = ref_sub.ConvLayer(6, 2, 1, activation="tanh", w_scale=0.3)
    with torch.no_grad():
        layer.conv2d.bias.uniform_(-0.2, 0.2)
    x = (torch.rand(2, 6, 5, 7) < 0.5).float()
    y = layer(x)
    (y * torch.arange(y.numel()).view_as(y).float()).sum().backward()
    np.savez_compressed(os.path.join(out, "convlayer_case.npz"), x=x.numpy(), y=y.detach().numpy(),
                        w=layer.conv2d.weight.detach().numpy(), b=layer.conv2d.bias.detach().numpy(),
                        gw=layer.conv2d.weight.grad.numpy(), gb=layer.conv2d.bias.grad.numpy())


def encodings_case(ref_enc, ref_base, out):
    """dataloader/encodings.py events_to_image / events_to_voxel / events_to_channels and
    dataloader/base.py create_mask_encoding / create_polarity_mask on a window with
    repeated pixels, both polarities and ts at bin edges."""
    gen = torch.Generator().manual_seed(31)
    H, W, N = 13, 17, 600
    xs = torch.randint(0, W, (N,), generator=gen).float()
    ys = torch.randint(0, H, (N,), generator=gen).float()
    ts = torch.sort(torch.rand(N, generator=gen)).values
    ts[:5] = torch.tensor([0.0, 0.25, 0.5, 0.75, 1.0])
    ps = (torch.rand(N, generator=gen) < 0.5).float() * 2 - 1
    rec = {"xs": xs.numpy(), "ys": ys.numpy(), "ts": ts.numpy(), "ps": ps.numpy(), "res": np.array([H, W])}
    rec["cnt"] = ref_enc.events_to_channels(xs, ys, ps, sensor_size=(H, W)).numpy()
    rec["image_acc"] = ref_enc.events_to_image(xs, ys, ps, sensor_size=(H, W)).numpy()
    for nb in (2, 5):
        for rnd in (False, True):
            rec[f"voxel_{nb}_{int(rnd)}"] = ref_enc.events_to_voxel(xs, ys, ts, ps, nb, sensor_size=(H, W),
                                                                    round_ts=rnd).numpy()
    loader = ref_base.BaseDataLoader.__new__(ref_base.BaseDataLoader)
    loader.resolution = (H, W)
    rec["mask"] = ref_base.BaseDataLoader.create_mask_encoding(loader, xs, ys, ps).numpy()
    rec["pol_mask"] = ref_base.BaseDataLoader.create_polarity_mask(ps).numpy()
    np.savez_compressed(os.path.join(out, "encodings_case.npz"), **rec)


def eval_case(ref_flow, ref_iwe, out):
    """loss/flow.py AEE (B=1 with tensor dt, B=2 with scalar dt) and utils/iwe.py
    compute_pol_iwe (rounded and bilinear) / deblur_events on synthetic windows."""
    gen = torch.Generator().manual_seed(41)
    H, W, N = 20, 24, 400
    rec = {"res": np.array([H, W])}
    for B in (1, 2):
        flow = (torch.rand(B, 2, H, W, generator=gen) - 0.5) * 0.1
        gt = (torch.rand(B, 2, H, W, generator=gen) - 0.5) * 12
        gt[:, :, :3, :] = 0.0  # invalid ground truth rows
        mask = (torch.rand(B, 1, H, W, generator=gen) < 0.6).float()
        ys = torch.randint(0, H, (B, N), generator=gen).float()
        xs = torch.randint(0, W, (B, N), generator=gen).float()
        ts = torch.sort(torch.rand(B, N, generator=gen), dim=1).values
        ps = (torch.rand(B, N, generator=gen) < 0.5).float() * 2 - 1
        ev = torch.stack([ts, ys, xs, ps], dim=2)
        pol = torch.stack([(ps > 0).float(), (ps < 0).float()], dim=2)
        dt_in, dt_gt = (torch.tensor([0.5]), torch.tensor([1.25])) if B == 1 else (torch.tensor(0.5), torch.tensor(0.8))
        cfg = {"loader": {"resolution": [H, W]}, "loss": {"overwrite_intermediate": False}}
        aee = ref_flow.AEE(cfg, "cpu", flow_scaling=128)
        aee.event_flow_association([flow], {"event_list": ev, "event_list_pol_mask": pol, "event_mask": mask,
                                            "gtflow": gt, "dt_input": dt_in, "dt_gt": dt_gt})
        v, pct = aee()
        # the other flow metrics of loss/flow.py on the same association (no randomness drawn)
        for name in ("NEE", "AAE", "NAAE", "AE_ofMeans", "AAE_Weighted", "AAE_Filtered"):
            mobj = getattr(ref_flow, name)(cfg, "cpu", flow_scaling=128)
            mobj.event_flow_association([flow], {"event_list": ev, "event_list_pol_mask": pol, "event_mask": mask,
                                                 "gtflow": gt, "dt_input": dt_in, "dt_gt": dt_gt})
            try:
                res = mobj()
            except RuntimeError as err:  # NEE broadcasts [B,H,W] / [B,1,H,W]: the reference raises for B > 1
                print(f"reference {name} fails for B={B}: {err}")
                continue
            res = res if isinstance(res, tuple) else (res,)
            for j, r in enumerate(res):
                rec[f"b{B}_{name}_{j}"] = r.detach().reshape(-1).numpy()
        rec.update({f"b{B}_flow": flow.numpy(), f"b{B}_gt": gt.numpy(), f"b{B}_mask": mask.numpy(),
                    f"b{B}_ev": ev.numpy(), f"b{B}_pol": pol.numpy(), f"b{B}_dt_in": dt_in.numpy(),
                    f"b{B}_dt_gt": dt_gt.numpy(), f"b{B}_aee": v.numpy(), f"b{B}_pct": pct.numpy()})
        for rnd in (True, False):
            iwe = ref_iwe.compute_pol_iwe(flow, ev, [H, W], pol[:, :, 0:1], pol[:, :, 1:2], flow_scaling=128,
                                          round_idx=rnd)
            rec[f"b{B}_poliwe_{int(rnd)}"] = iwe.numpy()
        rec[f"b{B}_deblur"] = ref_iwe.deblur_events(flow, ev, [H, W], flow_scaling=128, round_idx=True).numpy()
    np.savez_compressed(os.path.join(out, "eval_case.npz"), **rec)


def lif_export_case(out):
    """SNN_implementation::LIF (ONNX_LIF_operator/src/lif_op.cpp:8-55), the reference's own
    compiled CPU op built from its source by oracle/Makefile into oracle/_ref/lif_op.so.
    Ties of m' == threshold are planted (the op spikes on >=)."""
    so = os.path.join(REPO, "oracle", "_ref", "lif_op.so")
    if not os.path.exists(so):
        raise SystemExit("build oracle/_ref first: make -C oracle")
    torch.ops.load_library(so)
    gen = torch.Generator().manual_seed(11)
    N, C, H, W = 3, 5, 7, 9
    x = torch.randn(N, C, H, W, generator=gen)
    mem = torch.randn(N, C, H, W, generator=gen)
    beta = torch.rand(C, generator=gen) * 1.2 - 0.1  # no clamp in the op: include beta < 0, > 1
    thr = torch.rand(C, generator=gen)
    x[0, :, 0, 0] = thr - 0.5 * mem[0, :, 0, 0]
    beta[:] = torch.where(torch.arange(C) == 0, torch.tensor(0.5), beta)
    x[0, 0, 0, 0] = thr[0] - 0.5 * mem[0, 0, 0, 0]  # exact tie only where the products are exact
    mem[1, 0, 0, 0], x[1, 0, 0, 0] = 0.0, thr[0]      # m' == thr exactly -> spike
    spk, mo = torch.ops.SNN_implementation.LIF(x, mem, beta, thr)
    np.savez_compressed(os.path.join(out, "lif_export_case.npz"), x=x.numpy(), mem=mem.numpy(), beta=beta.numpy(),
                        threshold=thr.numpy(), spk=spk.numpy(), mem_out=mo.numpy())


def unet_kwargs_ref(base=4, activations=("arctanspike", "arctanspike")):
    """The train_SNN.yml model section for SpikingRecEVFlowNet, minus the keys the reference's
    BaseUNet constructor rejects (quantization / tebn / mpbn: SURVEY f3)."""
    return {"name": "SpikingRecEVFlowNet", "encoding": "cnt", "round_encoding": False, "norm_input": False,
            "num_bins": 2, "base_num_channels": base, "kernel_size": 3, "activations": list(activations),
            "mask_output": True,
            "spiking_neuron": {"leak": [0.0, 1.0], "thresh": [0.0, 0.8], "learn_leak": True, "learn_thresh": True,
                               "hard_reset": True}}


def unet_case(ref_model, ref_flow, out, base=4, fname="unet_case.npz"):
    """models/model.py SpikingRecEVFlowNet (SpikingMultiResUNetRecurrent of ConvLIF cells, reference
    code end to end): T forwards with carried states, EventWarping over the 4 flow maps, backward."""
    torch.manual_seed(17)
    gen = torch.Generator().manual_seed(18)
    H, W, B, N, T = 32, 32, 2, 200, 3
    model = ref_model.SpikingRecEVFlowNet(unet_kwargs_ref(base))
    config = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001,
              "overwrite_intermediate": False}, "model": {"mask_output": True}}
    lossf = ref_flow.EventWarping(config, "cpu")
    rec = {"res": np.array([H, W]), "T": T, "base": base}
    for k, v in model.state_dict().items():
        rec[f"p0.{k}"] = v.numpy().copy()
    for t in range(T):
        ev, pol, cnt, mask = synth_events(gen, B, N, H, W)
        cnt = cnt * 1.0
        x = model(None, cnt)
        lossf.event_flow_association(x["flow"], ev.clone(), pol, mask)
        rec[f"cnt_{t}"] = cnt.numpy()
        rec[f"events_{t}"] = ev.numpy()
        rec[f"pol_{t}"] = pol.numpy()
        rec[f"mask_{t}"] = mask.numpy()
        for i, f in enumerate(x["flow"]):
            rec[f"flow_{t}_{i}"] = f.detach().numpy()
        for i, st in enumerate(model.states):
            rec[f"state_{t}_{i}"] = st.detach().numpy()
    loss = lossf()
    loss.backward()
    rec["loss"] = np.array(loss.item(), dtype=np.float32)
    for n, p in model.named_parameters():
        rec[f"g.{n}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(out, fname), **rec)


def import_dataloader(ref_root):
    """dataloader/__init__.py imports h5py (absent): register the package without running
    it, then import the two pure-torch modules."""
    pkg = types.ModuleType("dataloader")
    pkg.__path__ = [os.path.join(ref_root, "dataloader")]
    sys.modules["dataloader"] = pkg
    import dataloader.base as ref_base
    import dataloader.encodings as ref_enc
    return ref_enc, ref_base


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--only=")]
    only = [a[len("--only="):] for a in sys.argv[1:] if a.startswith("--only=")]
    ref_root = args[0] if args else "/root/reference"
    install_stubs()
    sys.path.insert(0, ref_root)
    if only == ["encodings"]:
        ref_enc, ref_base = import_dataloader(ref_root)
        encodings_case(ref_enc, ref_base, HERE)
        print("encodings fixture written")
        return
    if only == ["lif_export"]:
        lif_export_case(HERE)
        print("lif_export fixture written")
        return
    if only == ["liffirenet_c8"]:  # C = 8 (the width of the wavefront launches)
        import loss.flow as ref_flow
        import models.model as ref_model
        torch.set_num_threads(1)
        liffirenet_case(ref_model, ref_flow, HERE, "LIFFireNet", 8, "liffirenet_c8_case.npz")
        print("liffirenet_c8 fixture written")
        return
    if only == ["liffirenet_norm"]:  # TEBN + MPBN cells
        import loss.flow as ref_flow
        import models.model as ref_model
        torch.set_num_threads(1)
        liffirenet_case(ref_model, ref_flow, HERE, "LIFFireNet", 8, "liffirenet_norm_case.npz", norm=True)
        print("liffirenet_norm fixture written")
        return
    if only == ["cell_variants"]:
        import models.spiking_submodules as ref_sub_sp
        torch.set_num_threads(1)
        spiking_cell_variants_case(ref_sub_sp, HERE)
        print("cell variants fixture written")
        return
    if only == ["unet"]:
        import loss.flow as ref_flow
        import models.model as ref_model
        torch.set_num_threads(1)
        unet_case(ref_model, ref_flow, HERE)
        print("unet fixture written")
        return
    if only == ["eval"]:
        import loss.flow as ref_flow
        import utils.iwe as ref_iwe
        eval_case(ref_flow, ref_iwe, HERE)
        print("eval fixture written")
        return
    import loss.flow as ref_flow
    import models.model as ref_model
    import models.spiking_submodules as ref_sub_sp
    import models.submodules as ref_sub
    import utils.iwe as ref_iwe

    out = HERE
    torch.set_num_threads(1)
    iwe_case(ref_iwe, out)
    loss_case(ref_flow, out)
    loss_case(ref_flow, out, overwrite=True, name="loss_case_overwrite.npz")
    spiking_cells_case(ref_sub_sp, out)
    spiking_cell_variants_case(ref_sub_sp, out)
    convlayer_case(ref_sub, out)
    liffirenet_case(ref_model, ref_flow, out, "LIFFireNet", 4)
    liffirenet_case(ref_model, ref_flow, out, "LIFFireNet_short", 4)
    liffirenet_case(ref_model, ref_flow, out, "LIFFireNet", 8, "liffirenet_c8_case.npz")
    liffirenet_case(ref_model, ref_flow, out, "LIFFireNet", 8, "liffirenet_norm_case.npz", norm=True)
    ref_enc, ref_base = import_dataloader(ref_root)
    encodings_case(ref_enc, ref_base, out)
    eval_case(ref_flow, ref_iwe, out)
    unet_case(ref_model, ref_flow, out)
    lif_export_case(out)
    print("golden fixtures written to", out)


if __name__ == "__main__":
    main()
