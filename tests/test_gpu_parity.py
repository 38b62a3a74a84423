"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the
reference-generated golden vectors.

Tolerances (fp32, stated per north_star): loss values rtol 1e-5..1e-4, per-step
membranes / flows rtol 1e-4, parameter gradients relative-L2 4e-6 vs the reference fixtures and
1e-5 vs the oracle (GOLDEN_GRAD_TOL / ORACLE_GRAD_TOL below; summation order differs: oneDNN conv
vs tile-ordered MFMA chains, atomics in the IWE scatter).  Integer IWE
corner indices: bit-exact.  Spikes: identical except where |v - theta| < 1e-4
(SURVEY finding 4: the recurrence is chaotic, so end-to-end comparisons use
teacher forcing or configurations verified to have no flips).
"""
import numpy as np
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

# Parameter-gradient bounds (relative L2) where the spikes agree; ~2x the worst case measured on
# MI355X (printed by _grad_check; DESIGN.md section 3 lists the figures).
GOLDEN_GRAD_TOL = 4e-6   # vs the reference-generated fixtures (fp32 CPU, oneDNN summation order);
                         # measured worst 1.5e-6 (head.lif.threshold, C=8)
ORACLE_GRAD_TOL = 1e-5   # vs the CPU oracle on fresh inputs; measured worst 4.4e-6 (cell C=8 recurrent, ff.weight)
NORM_GRAD_TOL = 1e-5     # TEBN + MPBN cells one by one vs their fixture; measured worst 4.2e-6 (G1.lif.beta)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _grad_check(tag, pairs, tol):
    """Relative-L2 error of every (name, ours, reference) gradient: printed (the measured figures
    behind the tolerances), then asserted against tol."""
    errs = {n: _rel(a, b) for n, a, b in pairs}
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"\n[{tag}] grad rel-L2 worst {worst[0]} {worst[1]:.2e}: " + ", ".join(f"{k}={v:.1e}" for k, v in errs.items()))
    for n, v in errs.items():
        assert v < tol, (tag, n, v)


def _sd(rec, prefix, dev):
    return {k[len(prefix):]: torch.from_numpy(v).to(dev) for k, v in rec.items() if k.startswith(prefix)}


# ---------------------------------------------------------------------------
# IWE / loss
# ---------------------------------------------------------------------------
def test_iwe_corners_bit_exact_vs_golden(golden, dev):
    import snnflow.iwe as siwe
    from oracle import iwe_ref

    g = golden("iwe_case.npz")
    ev = g["events"].copy()
    ev[:, :, 0] += np.float32(1.0)
    for name, tref in (("fw", 3), ("bw", 0)):
        idx, w = siwe.get_interpolation(torch.from_numpy(ev).to(dev), torch.from_numpy(g["flow_ev"]).to(dev),
                                        tref, list(g["res"]), 20)
        np.testing.assert_array_equal(idx[:, :, 0].long().cpu().numpy(), g[f"{name}_idx"])
        np.testing.assert_array_equal(w[:, :, 0].cpu().numpy(), g[f"{name}_w"])
        pol4 = torch.cat([torch.from_numpy(g["pol"]).to(dev)] * 4, dim=1)
        img = siwe.interpolate(idx, w, list(g["res"]), pol4[:, :, 0:1])
        np.testing.assert_allclose(img.cpu().numpy(), g[f"{name}_iwe_pos"], rtol=1e-6, atol=1e-6)
    ridx, rw = siwe.get_interpolation(torch.from_numpy(g["events"]).to(dev), torch.from_numpy(g["flow_ev"]).to(dev),
                                      1, list(g["res"]), 20, round_idx=True)
    np.testing.assert_array_equal(ridx[:, :, 0].long().cpu().numpy(), g["round_idx"])
    # random large case vs the numpy oracle
    gen = torch.Generator().manual_seed(5)
    B, M, H, W = 3, 20000, 96, 160
    evr = torch.stack([torch.rand(B, M, generator=gen) * 4, torch.randint(0, H, (B, M), generator=gen).float(),
                       torch.randint(0, W, (B, M), generator=gen).float(), torch.ones(B, M)], 2)
    flr = (torch.rand(B, M, 2, generator=gen) - 0.5) * 0.4
    idx, w = siwe.get_interpolation(evr.to(dev), flr.to(dev), 5, [H, W], 160)
    oi, ow, _ = iwe_ref.warp_corners_np(evr.numpy(), flr.numpy(), 5, [H, W], 160)
    np.testing.assert_array_equal(idx[:, :, 0].long().cpu().numpy(), oi)
    np.testing.assert_array_equal(w[:, :, 0].cpu().numpy(), ow)


@pytest.mark.parametrize("case,overwrite", [("loss_case.npz", False), ("loss_case_overwrite.npz", True)])
def test_event_warping_vs_golden(golden, dev, case, overwrite):
    import snnflow

    g = golden(case)
    T, (H, W) = int(g["T"]), list(g["res"])
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": overwrite},
           "model": {"mask_output": True}}
    ew = snnflow.EventWarping(cfg, dev)
    flows = []
    for t in range(T):
        f = torch.from_numpy(g[f"flow_{t}"]).to(dev).requires_grad_(True)
        flows.append(f)
        ew.event_flow_association([f], torch.from_numpy(g[f"events_{t}"]).to(dev),
                                  torch.from_numpy(g[f"pol_{t}"]).to(dev), torch.from_numpy(g[f"mask_{t}"]).to(dev))
    assert ew.num_events == sum(g[f"events_{t}"].shape[1] for t in range(T))
    if overwrite:
        ew.overwrite_intermediate_flow([flows[-1]])
    loss = ew()
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=2e-5)
    for t in range(T):
        gr = flows[t].grad
        if not g[f"grad_{t}"].any():
            assert gr is None or float(gr.abs().max()) == 0.0
            continue
        assert _rel(gr.cpu().numpy(), g[f"grad_{t}"]) < 1e-4, t


def test_event_warping_vs_oracle_random(dev):
    import snnflow
    from oracle import iwe_ref
    from snnflow.synthetic import make_window

    H, W, B, N, T = 40, 56, 3, 500, 4
    gen = torch.Generator(device=dev).manual_seed(3)
    for overwrite in (False, True):
        cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.01, "overwrite_intermediate": overwrite},
               "model": {"mask_output": True}}
        ew = snnflow.EventWarping(cfg, dev)
        ref = iwe_ref.EventWarpingRef([H, W], weight=0.01, overwrite_intermediate=overwrite)
        fl_d, fl_c = [], []
        for t in range(T):
            w = make_window(B, N, H, W, gen, dev)
            f = ((torch.rand(B, 2, H, W, generator=gen, device=dev) - 0.5) * 0.1).requires_grad_(True)
            fc = f.detach().cpu().requires_grad_(True)
            fl_d.append(f)
            fl_c.append(fc)
            ew.event_flow_association([f], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            ref.event_flow_association([fc], w["event_list"].cpu(), w["event_list_pol_mask"].cpu(), w["event_mask"].cpu())
        if overwrite:
            ew.overwrite_intermediate_flow([fl_d[-1]])
            ref.overwrite_intermediate_flow([fl_c[-1]])
        ref_loss = ref()
        loss = ew()
        loss.backward()
        ref_loss.backward()
        np.testing.assert_allclose(loss.item(), ref_loss.item(), rtol=2e-5)
        for t in range(T):
            gd = fl_d[t].grad
            gc = fl_c[t].grad
            if gc is None:
                assert gd is None or float(gd.abs().max()) == 0.0
                continue
            assert _rel(gd.cpu().numpy(), gc.numpy()) < 1e-4, (overwrite, t)


# ---------------------------------------------------------------------------
# Cells and the fused network
# ---------------------------------------------------------------------------
def _spike_mismatch_ok(ours, ref, v, theta, tol=1e-4):
    """spikes must agree except where the membrane sits within tol of threshold."""
    bad = ours != ref
    if not bad.any():
        return True
    near = (v - theta).abs() < tol
    return bool((bad & ~near).sum() == 0)


@pytest.mark.parametrize("recurrent", [False, True])
@pytest.mark.parametrize("C", [8, 16, 32])
def test_cell_teacher_forced(dev, recurrent, C):
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(2)
    cin = C if recurrent else 2
    cls = snnflow.SNNtorch_ConvLIFRecurrent if recurrent else snnflow.SNNtorch_ConvLIF
    cell = cls(cin, C, 3).to(dev).train()
    ref = lif_ref.SnnTorchCellRef(cin, C, 3, recurrent=recurrent).train()
    ref.load_state_dict({k: v.cpu() for k, v in cell.state_dict().items()})
    B, H, W = 2, 24, 40  # W not a multiple of the 32-wide tile: exercises partial tiles
    gen = torch.Generator().manual_seed(7)
    x = (torch.rand(B, cin, H, W, generator=gen) < 0.3).float() * (2.0 if not recurrent else 1.0)
    prev = torch.stack([torch.randn(B, C, H, W, generator=gen) * 0.5,
                        (torch.rand(B, C, H, W, generator=gen) < 0.2).float()])
    xd = x.to(dev).requires_grad_(True)
    xc = x.clone().requires_grad_(True)
    pd = prev.to(dev).requires_grad_(True)
    pc = prev.clone().requires_grad_(True)
    spk, st = cell(xd, pd)
    rspk, rst = ref(xc, pc)
    v_ref = rst[0]
    np.testing.assert_allclose(cell.bn.running_mean.cpu().numpy(), ref.bn.running_mean.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(cell.bn.running_var.cpu().numpy(), ref.bn.running_var.numpy(), rtol=1e-5, atol=1e-6)
    assert _spike_mismatch_ok(spk.detach().cpu(), rspk.detach(), v_ref.detach(), ref.lif.threshold.detach())
    assert _rel(st[0].detach().cpu().numpy(), rst[0].detach().numpy()) < 1e-5
    wgt = torch.linspace(-1, 1, spk.numel()).view_as(spk)
    (spk * wgt.to(dev)).sum().backward()
    (rspk * wgt).sum().backward()
    if (spk.detach().cpu() == rspk.detach()).all():
        pairs = [(n, p.grad.cpu().numpy(), q.grad.numpy())
                 for (n, p), (_, q) in zip(cell.named_parameters(), ref.named_parameters())]
        pairs.append(("input", xd.grad.cpu().numpy(), xc.grad.numpy()))
        if recurrent:
            pairs.append(("prev_state", pd.grad.cpu().numpy(), pc.grad.numpy()))
        _grad_check(f"cell C={C} rec={recurrent}", pairs, ORACLE_GRAD_TOL)


def _run_golden_firenet(g, name, dev, seq=False, norm=False, tol=GOLDEN_GRAD_TOL):
    """seq: the T windows through model.forward_sequence (wavefront launches; only the final
    step's states are observable there) instead of T model() calls.  norm: TEBN + MPBN cells."""
    import snnflow
    from oracle import lif_ref

    T, C = int(g["T"]), int(g["C"])
    H, W = list(g["res"])
    kw = lif_ref.make_unet_kwargs(base_num_channels=C)
    if norm:
        kw["tebn"], kw["mpbn"] = {"enabled": True, "num_timesteps": 4}, {"enabled": True}
    model = getattr(snnflow, name)(kw).to(dev).train()
    model.load_state_dict(_sd(g, "p0.", dev))
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ew = snnflow.EventWarping(cfg, dev)
    cnts = [torch.from_numpy(g[f"cnt_{t}"]).to(dev) for t in range(T)]
    outs = model.forward_sequence(None, cnts) if seq else None
    for t in range(T):
        out = outs[t] if seq else model(None, cnts[t])
        np.testing.assert_allclose(out["flow"][0].detach().cpu().numpy(), g[f"flow_{t}"], rtol=1e-4, atol=1e-6)
        if not seq or t == T - 1:
            for i, s in enumerate(model._states):
                ref_s = g[f"state_{t}_{i}"]
                np.testing.assert_array_equal(s[1].detach().cpu().numpy(), ref_s[1])  # spikes
                np.testing.assert_allclose(s[0].detach().cpu().numpy(), ref_s[0], rtol=1e-4, atol=1e-5)
        ew.event_flow_association(out["flow"], torch.from_numpy(g[f"events_{t}"]).to(dev),
                                  torch.from_numpy(g[f"pol_{t}"]).to(dev), torch.from_numpy(g[f"mask_{t}"]).to(dev))
    loss = ew()
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-4)
    for n, p in model.named_parameters():
        assert p.grad is not None, n
    _grad_check(f"golden {name} C={C} seq={seq}", [(n, p.grad.cpu().numpy(), g[f"g.{n}"])
                                                   for n, p in model.named_parameters()], tol)
    for k, v in model.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), g[f"p1.{k}"], rtol=1e-5, atol=1e-6, err_msg=k)


def test_liffirenet_vs_golden(golden, dev):
    _run_golden_firenet(golden("liffirenet_case.npz"), "LIFFireNet", dev)


def test_liffirenet_short_vs_golden(golden, dev):
    _run_golden_firenet(golden("liffirenet_short_case.npz"), "LIFFireNet_short", dev)


def test_liffirenet_c8_vs_golden(golden, dev):
    _run_golden_firenet(golden("liffirenet_c8_case.npz"), "LIFFireNet", dev)


def test_liffirenet_tebn_mpbn_vs_golden(golden, dev):
    """TEBN + MPBN cells (SNNtorch_spiking_submodules.py:18-121; reference-generated fixture with
    perturbed p and MPBN affine parameters): the cells run one by one on the HIP cell kernels with
    the temporal weight folded into the BatchNorm affine and MPBN on the standalone BatchNorm kernel;
    forward_sequence takes the same path."""
    _run_golden_firenet(golden("liffirenet_norm_case.npz"), "LIFFireNet", dev, norm=True, tol=NORM_GRAD_TOL)
    _run_golden_firenet(golden("liffirenet_norm_case.npz"), "LIFFireNet", dev, seq=True, norm=True, tol=NORM_GRAD_TOL)


@pytest.mark.parametrize("C,train,affine", [(8, True, True), (32, True, True), (16, False, True), (4, True, False)])
def test_batchnorm_rows_vs_torch(dev, C, train, affine):
    """The standalone BatchNorm kernel (csrc/norm.hip) against torch.nn.BatchNorm2d in fp64 on the
    same data: output, running statistics, num_batches_tracked and all gradients."""
    from snnflow.norm import batch_norm_nchw

    gen = torch.Generator().manual_seed(C)
    x = torch.randn(3, C, 17, 23, generator=gen) * 2 + 0.5
    gy = torch.randn(3, C, 17, 23, generator=gen)
    bn = torch.nn.BatchNorm2d(C, affine=affine).to(dev)
    ref = torch.nn.BatchNorm2d(C, affine=affine).double()
    if affine:
        with torch.no_grad():
            w, b = torch.rand(C, generator=gen) + 0.5, torch.randn(C, generator=gen) * 0.1
            bn.weight.copy_(w), bn.bias.copy_(b), ref.weight.copy_(w.double()), ref.bias.copy_(b.double())
    with torch.no_grad():
        rm, rv = torch.randn(C, generator=gen) * 0.1, torch.rand(C, generator=gen) + 0.5
        bn.running_mean.copy_(rm), bn.running_var.copy_(rv), ref.running_mean.copy_(rm.double()), ref.running_var.copy_(rv.double())
    bn.train(train)
    ref.train(train)
    xd = x.to(dev).requires_grad_(True)
    xr = x.double().requires_grad_(True)
    y = batch_norm_nchw(xd, bn)
    yr = ref(xr)
    np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=1e-5)
    (y * gy.to(dev)).sum().backward()
    (yr * gy.double()).sum().backward()
    np.testing.assert_allclose(xd.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-4, atol=1e-5)
    if affine:
        np.testing.assert_allclose(bn.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(bn.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(bn.running_mean.cpu().numpy(), ref.running_mean.numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(bn.running_var.cpu().numpy(), ref.running_var.numpy(), rtol=1e-6, atol=1e-7)
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked)


def test_tebn_timestep_and_mpbn_threshold(dev):
    """TEBN with an explicit time step (p[t], :56-57) and without (p.mean(0)), and MPBN's
    get_effective_threshold in eval mode (:97-121), against the oracle restatement."""
    import snnflow
    from oracle.lif_ref import TEBNRef

    gen = torch.Generator().manual_seed(3)
    x = torch.randn(2, 8, 9, 10, generator=gen)
    m = snnflow.TEBN(8, num_timesteps=4).to(dev)
    r = TEBNRef(8, 4)
    with torch.no_grad():
        p = torch.rand(4, 8, 1, 1, generator=gen) + 0.5
        m.p.copy_(p), r.p.copy_(p)
    for t in (None, 2, 7):
        m.zero_grad(), r.zero_grad()
        y, yr = m(x.to(dev), timestep=t), r(x, timestep=t)
        np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=1e-5)
        (y * y).sum().backward()
        (yr * yr).sum().backward()
        np.testing.assert_allclose(m.p.grad.cpu().numpy(), r.p.grad.numpy(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(m.bn.weight.grad.cpu().numpy(), r.bn.weight.grad.numpy(), rtol=1e-4, atol=1e-5)
    mp = snnflow.MPBN(8).to(dev).eval()
    th = torch.rand(8, 1, 1, device=dev)
    with torch.no_grad():
        mp.bn.running_var.fill_(4.0), mp.bn.running_mean.fill_(0.5)
    eff = mp.get_effective_threshold(th)
    np.testing.assert_allclose(eff.cpu().numpy(), (th.view(1, 8, 1, 1) * np.sqrt(4.0 + 1e-5) + 0.5).cpu().numpy(), rtol=1e-6)


def test_convlayer_pointwise_vs_golden(golden, dev):
    """ConvLayer called as a module (1x1 + bias + tanh) on the HIP pointwise kernels against the
    reference-generated fixture (models/submodules.py:16-113)."""
    import snnflow

    g = golden("convlayer_case.npz")
    layer = snnflow.ConvLayer(6, 2, 1, activation="tanh", w_scale=0.3).to(dev)
    with torch.no_grad():
        layer.conv2d.weight.copy_(torch.from_numpy(g["w"]))
        layer.conv2d.bias.copy_(torch.from_numpy(g["b"]))
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    y = layer(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["y"], rtol=1e-6, atol=1e-7)
    (y * torch.arange(y.numel(), device=dev).view_as(y).float()).sum().backward()
    np.testing.assert_allclose(layer.conv2d.weight.grad.cpu().numpy(), g["gw"], rtol=1e-5)
    np.testing.assert_allclose(layer.conv2d.bias.grad.cpu().numpy(), g["gb"], rtol=1e-5)
    assert x.grad is not None and torch.isfinite(x.grad).all()


@pytest.mark.parametrize("cin,act,norm", [(256, "tanh", None), (128, None, None), (64, "tanh", "BN")])
def test_convlayer_wide_unet_preds_vs_torch(dev, cin, act, norm):
    """The U-Net's multires prediction layers called standalone (models/unet.py:255-262: ConvLayer
    (base*2^k -> 2, 1x1, final activation), cin up to 256 at base 32) on the HIP pointwise kernels
    against a torch fp32 1x1 conv; norm="BN" drops the bias and, as in the reference
    (submodules.py:98-102), is never applied."""
    import snnflow

    torch.manual_seed(cin)
    layer = snnflow.ConvLayer(cin, 2, 1, activation=act, norm=norm).to(dev)
    assert (layer.conv2d.bias is None) == (norm == "BN")
    if norm == "BN":
        assert isinstance(layer.norm_layer, torch.nn.BatchNorm2d)
    x = torch.randn(2, cin, 24, 40, device=dev, requires_grad=True)
    y = layer(x)
    xr = x.detach().double().requires_grad_(True)
    wr = layer.conv2d.weight.detach().double().requires_grad_(True)
    br = layer.conv2d.bias.detach().double().requires_grad_(True) if layer.conv2d.bias is not None else None
    yr = torch.nn.functional.conv2d(xr, wr, br)
    if act is not None:
        yr = getattr(torch, act)(yr)
    np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().cpu().numpy(), rtol=1e-5, atol=1e-5)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    (yr * gy.double()).sum().backward()
    assert _rel(x.grad.cpu().numpy(), xr.grad.cpu().numpy()) < 1e-6
    assert _rel(layer.conv2d.weight.grad.cpu().numpy(), wr.grad.cpu().numpy()) < 1e-6
    if br is not None:
        assert _rel(layer.conv2d.bias.grad.cpu().numpy(), br.grad.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("case,name", [("liffirenet_c8_case.npz", "LIFFireNet"),
                                       ("liffirenet_case.npz", "LIFFireNet"),
                                       ("liffirenet_short_case.npz", "LIFFireNet_short")])
def test_forward_sequence_vs_golden(golden, dev, case, name):
    """The reference-generated fixtures through forward_sequence: the wavefront launches at C = 8,
    the per-step fallback at C = 4."""
    _run_golden_firenet(golden(case), name, dev, seq=True)


@pytest.mark.parametrize("C", [8, 16, 32])
def test_liffirenet_layerwise_teacher_forced_128(dev, C):
    """Every layer of the fused time step at the benchmark size (128x128, B=2, 3 steps),
    teacher-forced layer by layer: the oracle cell gets OUR previous layer's spikes and
    OUR previous state, so a near-threshold flip cannot cascade."""
    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(0)
    kw = lif_ref.make_unet_kwargs(base_num_channels=C)
    model = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    ref = lif_ref.LIFFireNetRef(dict(kw), "LIFFireNet").train()
    ref.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    gen = torch.Generator(device=dev).manual_seed(4)
    total_flips, worst_mem = 0, 0.0
    for t in range(3):
        w = make_window(2, 1000, 128, 128, gen, dev)
        prev = [None] * 7 if t == 0 else [s.detach().cpu() for s in model._states]
        out = model(w["event_voxel"], w["event_cnt"])
        x_in = w["event_cnt"].cpu()
        for i, (name, _) in enumerate(model.layer_spec):
            rcell = getattr(ref, name)
            with torch.no_grad():
                rs, rst = rcell(x_in, prev[i])
            ours = model._states[i].detach().cpu()
            v = rcell.lif.last_v
            theta = rcell.lif.threshold.detach()
            assert _spike_mismatch_ok(ours[1], rs, v, theta), (t, name)
            total_flips += int((ours[1] != rs).sum())
            agree = ours[1] == rs
            worst_mem = max(worst_mem, _rel(ours[0][agree].numpy(), rst[0][agree].numpy()))
            x_in = ours[1]
        with torch.no_grad():
            rflow = ref.pred(x_in)
        np.testing.assert_allclose(out["flow"][0].detach().cpu().numpy(), rflow.numpy(), rtol=1e-4, atol=1e-6)
    for (n, a), (_, b) in zip(model.state_dict().items(), ref.state_dict().items()):
        if "running" in n:
            np.testing.assert_allclose(a.cpu().numpy(), b.numpy(), rtol=1e-4, atol=1e-6, err_msg=n)
    assert worst_mem < 1e-5, worst_mem
    print(f"C={C}: near-threshold flips {total_flips}, worst membrane rel err {worst_mem:.2e}")


def test_state_api_and_eval_mode(dev):
    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(1)
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    model = snnflow.LIFFireNet(dict(kw)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(9)
    w = make_window(2, 300, 32, 32, gen, dev)
    model.train()
    model(None, w["event_cnt"])
    st = model.states
    assert len(st) == 7 and tuple(st[0].shape) == (2, 2, 8, 32, 32)
    model.detach_states()
    assert not any(s.requires_grad for s in model._states)
    model.reset_states()
    assert model._states == [None] * 7
    # eval mode: running statistics, no running-stat updates
    model.eval()
    rm = model.head.bn.running_mean.clone()
    ref = lif_ref.LIFFireNetRef(dict(kw), "LIFFireNet").eval()
    ref.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    for i, (n, _) in enumerate(model.layer_spec):  # identical stale membranes (Leaky cache quirk)
        getattr(ref, n).lif.mem = getattr(model, n).lif.mem.detach().cpu()
    with torch.no_grad():
        out = model(None, w["event_cnt"])
        ro = ref(None, w["event_cnt"].cpu())
    assert torch.equal(model.head.bn.running_mean, rm)
    np.testing.assert_allclose(out["flow"][0].cpu().numpy(), ro["flow"][0].numpy(), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("sequence", [False, True])
def test_replaced_parameters_after_forward(dev, sequence):
    """Neuron parameters and BatchNorm buffers replaced (not edited in place) after the engine has
    cached its neuron structs and step-driver plan: the next forward must read the new tensors.
    Checked bit for bit against a fresh model loaded with the same state."""
    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(3)
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    model = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(4)
    ws = [make_window(2, 300, 32, 32, gen, dev) for _ in range(2)]

    def run(m):
        m.reset_states()
        for c in m.engine.cells:
            c.lif.mem = None
        if sequence:
            outs = m.forward_sequence([w["event_voxel"] for w in ws], [w["event_cnt"] for w in ws])
        else:
            outs = [m(w["event_voxel"], w["event_cnt"]) for w in ws]
        loss = sum((o["flow"][0] ** 2).sum() for o in outs)
        loss.backward()
        return torch.stack([o["flow"][0].detach() for o in outs])

    run(model)  # caches neuron structs, the plan, prepared weights
    with torch.no_grad():
        model.head.bn.weight = torch.nn.Parameter(model.head.bn.weight * 1.5)
        model.G1.lif.threshold = torch.nn.Parameter(model.G1.lif.threshold + 0.05)
        model.R1a.lif.beta = torch.nn.Parameter(model.R1a.lif.beta * 0.5)
        model.R2b.bn.running_mean = torch.full_like(model.R2b.bn.running_mean, 0.25)
    model.R1b.bn.momentum = 0.3
    model.zero_grad(set_to_none=True)
    fresh = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    fresh.load_state_dict(model.state_dict())  # the replaced tensors' values, before the next step
    fresh.R1b.bn.momentum = 0.3
    got = run(model)
    want = run(fresh)
    assert torch.equal(got, want)
    assert torch.equal(model.R1b.bn.running_mean, fresh.R1b.bn.running_mean)
    assert torch.equal(model.R2b.bn.running_mean, fresh.R2b.bn.running_mean)
    for (n, a), (_, b) in zip(model.named_parameters(), fresh.named_parameters()):
        assert a.grad is not None and torch.allclose(a.grad, b.grad, rtol=1e-5, atol=1e-7), n


def test_lif_export_op(dev):
    from snnflow import _lib
    from snnflow._lib import lib, ptr

    gen = torch.Generator().manual_seed(0)
    N, C, H, W = 2, 3, 4, 5
    x = torch.randn(N, C, H, W, generator=gen)
    m = torch.randn(N, C, H, W, generator=gen)
    beta = torch.rand(C, generator=gen)
    thr = torch.rand(C, generator=gen)
    x[0, 0, 0, 0], m[0, 0, 0, 0], thr[0], beta[0] = 1.0, 0.0, 1.0, 0.5  # m' == thr -> spike (>=)
    xd, md, bd, td = (t.to(dev) for t in (x, m, beta, thr))
    spk, mo = torch.empty_like(xd), torch.empty_like(xd)
    _lib.check(lib.snnflow_lif_export(ptr(xd), ptr(md), ptr(bd), ptr(td), N, C, H * W, ptr(spk), ptr(mo),
                                      _lib.stream_ptr(dev)), "lif_export")
    mp = beta.view(1, C, 1, 1) * m + x
    s_ref = (mp >= thr.view(1, C, 1, 1)).float()
    np.testing.assert_array_equal(spk.cpu().numpy(), s_ref.numpy())
    np.testing.assert_array_equal(mo.cpu().numpy(), torch.where(s_ref > 0, torch.zeros_like(mp), mp).numpy())
    assert spk[0, 0, 0, 0].item() == 1.0


def test_lif_export_op_vs_reference_op(golden, dev):
    """snnflow_lif_export bit-exact against the reference's own compiled CPU op
    (ONNX_LIF_operator/src/lif_op.cpp via oracle/_ref/lif_op.so): its committed fixture,
    and the .so itself on fresh random inputs when it was shipped with the tree."""
    import os

    from snnflow import _lib
    from snnflow._lib import lib, ptr

    def run(x, m, b, th):
        N, C, H, W = x.shape
        xd, md, bd, td = (t.contiguous().to(dev) for t in (x, m, b, th))
        spk, mo = torch.empty_like(xd), torch.empty_like(xd)
        _lib.check(lib.snnflow_lif_export(ptr(xd), ptr(md), ptr(bd), ptr(td), N, C, H * W, ptr(spk), ptr(mo),
                                          _lib.stream_ptr(dev)), "lif_export")
        return spk.cpu(), mo.cpu()

    g = golden("lif_export_case.npz")
    spk, mo = run(*(torch.from_numpy(g[k]) for k in ("x", "mem", "beta", "threshold")))
    np.testing.assert_array_equal(spk.numpy(), g["spk"])
    np.testing.assert_array_equal(mo.numpy(), g["mem_out"])
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "lif_op.so")
    if os.path.exists(so):
        torch.ops.load_library(so)
        gen = torch.Generator().manual_seed(7)
        x, m = torch.randn(4, 16, 33, 17, generator=gen), torch.randn(4, 16, 33, 17, generator=gen)
        b, th = torch.rand(16, generator=gen), torch.rand(16, generator=gen)
        rs, rm = torch.ops.SNN_implementation.LIF(x, m, b, th)
        s2, m2 = run(x, m, b, th)
        assert torch.equal(rs, s2) and torch.equal(rm, m2)


def test_training_steps_fused_adam_vs_oracle(dev):
    """Three optimizer steps (T=2 windows each, truncated BPTT) with torch's fused Adam,
    which updates parameters without bumping their version counters: the engine must
    re-read the weights at every forward.  Before every step the oracle is re-synced to
    OUR parameters and states (Adam amplifies last-bit gradient differences of
    near-zero gradients, so parameters are not compared across steps); flows, loss and
    gradients of every step must then match."""
    import snnflow
    from oracle import iwe_ref, lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(3)
    H = W = 32
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    model = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    ref = lif_ref.LIFFireNetRef(dict(kw), "LIFFireNet").train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, fused=True)
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ew = snnflow.EventWarping(cfg, dev)
    rew = iwe_ref.EventWarpingRef([H, W], weight=0.001)
    gen = torch.Generator(device=dev).manual_seed(11)
    for step in range(3):
        ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
        ref._states = [None if s is None else s.detach().cpu() for s in model._states]
        for n, _ in model.layer_spec:
            m = getattr(model, n).lif.mem
            if m is not None:
                getattr(ref, n).lif.mem = m.detach().cpu()
        for t in range(2):
            w = make_window(2, 400, H, W, gen, dev)
            out = model(w["event_voxel"], w["event_cnt"])
            rout = ref(None, w["event_cnt"].cpu())
            np.testing.assert_allclose(out["flow"][0].detach().cpu().numpy(), rout["flow"][0].detach().numpy(),
                                       rtol=1e-3, atol=1e-5, err_msg=f"step {step} window {t}")
            ew.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            rew.event_flow_association(rout["flow"], w["event_list"].cpu(), w["event_list_pol_mask"].cpu(),
                                       w["event_mask"].cpu())
        loss, rloss = ew(), rew()
        opt.zero_grad(set_to_none=True)
        ref.zero_grad(set_to_none=True)
        loss.backward()
        rloss.backward()
        np.testing.assert_allclose(loss.item(), rloss.item(), rtol=1e-4)
        _grad_check(f"fused adam step {step}", [(n, a.grad.cpu().numpy(), b.grad.numpy()) for (n, a), (_, b)
                                                 in zip(model.named_parameters(), ref.named_parameters())],
                    ORACLE_GRAD_TOL)
        opt.step()
        model.detach_states()
        ew.reset()
        rew.reset()


# ---------------------------------------------------------------------------
# U-Net neuron flavour: ConvLIF / ConvLIFRecurrent (models/spiking_submodules.py)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("tag", ["ff", "rec"])
def test_convlif_vs_golden(golden, dev, tag):
    """Reference-generated fixture: 3 steps, loss = sum z*linspace + 0.3*sum v each step
    (tests/golden/make_golden.py:spiking_cells_case); spikes, last membrane and every
    parameter gradient (BPTT through the membrane)."""
    import snnflow

    g = golden("spiking_cells_case.npz")
    cls = snnflow.ConvLIF if tag == "ff" else snnflow.ConvLIFRecurrent
    cell = cls(3, 4, 3, leak=(0.0, 1.0), thresh=(0.8, 0.1)).to(dev)
    cell.load_state_dict({k[len(tag) + 3:]: torch.from_numpy(v).to(dev) for k, v in g.items()
                          if k.startswith(f"{tag}.p.")})
    state, loss = None, 0
    for t in range(3):
        x = torch.from_numpy(g[f"{tag}.x_{t}"]).to(dev)
        z, state = cell(x, state)
        np.testing.assert_array_equal(z.detach().cpu().numpy(), g[f"{tag}.z_{t}"])
        lin = torch.linspace(-1, 1, z.numel(), device=dev).view_as(z)
        loss = loss + (z * lin).sum() + 0.3 * state[0].sum()
    np.testing.assert_allclose(state[0].detach().cpu().numpy(), g[f"{tag}.v_last"], rtol=1e-5, atol=1e-6)
    loss.backward()
    for n, p in cell.named_parameters():
        ref = g[f"{tag}.g.{n}"]
        assert _rel(p.grad.cpu().numpy(), ref) < 1e-4, (n, _rel(p.grad.cpu().numpy(), ref))


@pytest.mark.parametrize("recurrent", [False, True])
@pytest.mark.parametrize("C,cin,hard", [(8, 8, True), (8, 2, False), (16, 16, True), (32, 32, False)])
def test_convlif_vs_oracle_random(dev, recurrent, C, cin, hard):
    """Random cells and inputs, 3 steps with a residual on the ff cell: outputs, states and
    gradients of inputs, initial state and parameters against the oracle (steps run
    teacher-forced on OUR spikes/state so a near-threshold flip cannot cascade)."""
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(21 + C)
    B, H, W, T = 2, 20, 37, 3
    if recurrent:
        cell = snnflow.ConvLIFRecurrent(cin, C, 3, leak=(0.0, 1.0), thresh=(0.5, 0.2), hard_reset=hard).to(dev)
    else:
        cell = snnflow.ConvLIF(cin, C, 3, leak=(0.0, 1.0), thresh=(0.5, 0.2), hard_reset=hard).to(dev)
    ref = lif_ref.SpikingCellRef(cin, C, 3, recurrent=recurrent, hard_reset=hard)
    ref.load_state_dict({k: v.cpu() for k, v in cell.state_dict().items()})
    gen = torch.Generator().manual_seed(5)
    s0 = torch.randn(2, B, C, H, W, generator=gen) * 0.5
    s0[1] = (s0[1] > 0).float()
    state_d = s0.to(dev).requires_grad_(True)
    state_c = s0.clone().requires_grad_(True)
    for t in range(T):
        x = (torch.rand(B, cin, H, W, generator=gen) < 0.5).float()
        xd, xc = x.to(dev).requires_grad_(True), x.clone().requires_grad_(True)
        res = torch.randn(B, C, H, W, generator=gen) if not recurrent else None
        if recurrent:
            zd, sd = cell(xd, state_d)
            zc, sc = ref(xc, state_c)
        else:
            zd, sd = cell(xd, state_d, res.to(dev))
            zc, sc = ref(xc, state_c, res)
        v = sc[0].detach()
        th = ref.thresh.detach().clamp_min(0.01)
        assert _spike_mismatch_ok(sd[1].detach().cpu(), sc[1].detach(), v, th), t
        np.testing.assert_allclose(sd[0].detach().cpu().numpy(), sc[0].detach().numpy(), rtol=1e-5, atol=1e-5)
        wz = torch.randn(B, C, H, W, generator=gen)
        wv = torch.randn(B, C, H, W, generator=gen)
        ((zd * wz.to(dev)).sum() + (sd[0] * wv.to(dev)).sum()).backward()
        ((zc * wz).sum() + (sc[0] * wv).sum()).backward()
        if (sd[1].detach().cpu() == sc[1].detach()).all():
            assert _rel(xd.grad.cpu().numpy(), xc.grad.numpy()) < 1e-4, t
            assert _rel(state_d.grad.cpu().numpy(), state_c.grad.numpy()) < 1e-4, t
            for (n, p), (_, q) in zip(cell.named_parameters(), ref.named_parameters()):
                assert _rel(p.grad.cpu().numpy(), q.grad.numpy()) < 1e-4, (t, n)
        cell.zero_grad()
        ref.zero_grad()
        # next step from OUR state (teacher forcing), fresh leaves
        state_d = sd.detach().clone().requires_grad_(True)
        state_c = sd.detach().cpu().clone().requires_grad_(True)


# ---------------------------------------------------------------------------
# On-device event encodings (dataloader/encodings.py, dataloader/base.py)
# ---------------------------------------------------------------------------
def test_encodings_vs_golden(golden, dev):
    """Counts, masks and polarity masks bit-exact; voxel grids exact with rounded
    timestamps (0/1 weights) and within fp32 summation-order error otherwise."""
    from snnflow import encodings as E

    g = golden("encodings_case.npz")
    xs, ys, ts, ps = (torch.from_numpy(g[k]).to(dev) for k in ("xs", "ys", "ts", "ps"))
    res = tuple(int(v) for v in g["res"])
    np.testing.assert_array_equal(E.events_to_channels(xs, ys, ps, res).cpu().numpy(), g["cnt"])
    np.testing.assert_array_equal(E.events_to_image(xs, ys, ps, res).cpu().numpy(), g["image_acc"])
    for nb in (2, 5):
        for rnd in (0, 1):
            v = E.events_to_voxel(xs, ys, ts, ps, nb, res, bool(rnd)).cpu().numpy()
            if rnd:
                np.testing.assert_array_equal(v, g[f"voxel_{nb}_{rnd}"])
            else:
                np.testing.assert_allclose(v, g[f"voxel_{nb}_{rnd}"], rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(E.create_mask_encoding(xs, ys, ps, res).cpu().numpy(), g["mask"])
    np.testing.assert_array_equal(E.create_polarity_mask(ps).cpu().numpy(), g["pol_mask"])


def test_encode_batch_vs_oracle(dev):
    """One launch for a whole batch (B=4, 128x128, 3000 events each, duplicates) against the
    per-sample oracle; and the synthetic loader's own counts."""
    from oracle import encodings_ref as E
    from snnflow import encodings
    from snnflow.synthetic import make_window

    gen = torch.Generator(device=dev).manual_seed(7)
    w = make_window(4, 3000, 128, 128, gen, dev)
    out = encodings.encode_batch(w["event_list"], (128, 128), num_bins=5, round_ts=False)
    ev = w["event_list"].cpu()
    for b in range(4):
        ts, ys, xs, ps = ev[b, :, 0], ev[b, :, 1], ev[b, :, 2], ev[b, :, 3]
        np.testing.assert_array_equal(out["event_cnt"][b].cpu().numpy(),
                                      E.events_to_channels(xs, ys, ps, (128, 128)).numpy())
        np.testing.assert_allclose(out["event_voxel"][b].cpu().numpy(),
                                   E.events_to_voxel(xs, ys, ts, ps, 5, (128, 128)).numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(out["event_mask"][b].cpu().numpy(),
                                      E.create_mask_encoding(xs, ys, ps, (128, 128)).numpy())
        np.testing.assert_array_equal(out["event_list_pol_mask"][b].cpu().numpy(),
                                      E.create_polarity_mask(ps).t().numpy())
    np.testing.assert_array_equal(out["event_cnt"].cpu().numpy(), w["event_cnt"].cpu().numpy())


# ---------------------------------------------------------------------------
# Evaluation path (utils/iwe.py deblur / compute_pol_iwe, loss/flow.py AEE)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("B", [1, 2])
def test_eval_vs_golden(golden, dev, B):
    """Rounded IWEs bit-exact (integer counts), bilinear IWEs within fp32 atomic-order error,
    AEE and outlier percentage within 1e-5 relative (north_star: AEE within 1e-4)."""
    import snnflow
    from snnflow import iwe

    g = golden("eval_case.npz")
    H, W = (int(v) for v in g["res"])
    t = {k: torch.from_numpy(g[f"b{B}_{k}"]).to(dev) for k in ("flow", "gt", "mask", "ev", "pol")}
    for rnd in (1, 0):
        out = iwe.compute_pol_iwe(t["flow"], t["ev"], [H, W], t["pol"][:, :, 0:1], t["pol"][:, :, 1:2],
                                  flow_scaling=128, round_idx=bool(rnd)).cpu().numpy()
        if rnd:
            np.testing.assert_array_equal(out, g[f"b{B}_poliwe_{rnd}"])
        else:
            np.testing.assert_allclose(out, g[f"b{B}_poliwe_{rnd}"], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(iwe.deblur_events(t["flow"], t["ev"], [H, W], flow_scaling=128).cpu().numpy(),
                                  g[f"b{B}_deblur"])
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"overwrite_intermediate": False}}
    m = snnflow.AEE(cfg, dev, flow_scaling=128)
    m.event_flow_association([t["flow"]], {"event_list": t["ev"], "event_list_pol_mask": t["pol"],
                                           "event_mask": t["mask"], "gtflow": t["gt"],
                                           "dt_input": torch.from_numpy(g[f"b{B}_dt_in"]),
                                           "dt_gt": torch.from_numpy(g[f"b{B}_dt_gt"])})
    aee, pct = m()
    np.testing.assert_allclose(aee.cpu().numpy(), g[f"b{B}_aee"], rtol=1e-5)
    np.testing.assert_allclose(pct.cpu().numpy(), g[f"b{B}_pct"], rtol=1e-6)
    # one launch with a self-resetting completion counter and fixed-order sums: repeated calls on
    # the same scratch give the same bits
    for _ in range(3):
        a2, p2 = m()
        assert torch.equal(a2, aee) and torch.equal(p2, pct)


_METRIC_CLASSES = {"NEE": ("nee", "nee_pct"), "AAE": ("aae", "aae_pct"), "NAAE": ("naae",),
                   "AE_ofMeans": ("ae_of_means",), "AAE_Weighted": ("aae_weighted",),
                   "AAE_Filtered": ("aae_filtered",)}


@pytest.mark.parametrize("B", [1, 2])
def test_flow_metrics_vs_golden(golden, dev, B):
    """NEE/AAE/NAAE/AE_ofMeans/AAE_Weighted/AAE_Filtered through the reference's class API
    against the values the reference classes produced (rtol 1e-5; NEE and AAE exist for
    B = 1 only: the reference raises for B > 1)."""
    import snnflow

    g = golden("eval_case.npz")
    H, W = (int(v) for v in g["res"])
    t = {k: torch.from_numpy(g[f"b{B}_{k}"]).to(dev) for k in ("flow", "gt", "mask", "ev", "pol")}
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"overwrite_intermediate": False}}
    n = 0
    for name in _METRIC_CLASSES:
        m = getattr(snnflow, name)(cfg, dev, flow_scaling=128)
        m.event_flow_association([t["flow"]], {"event_list": t["ev"], "event_list_pol_mask": t["pol"],
                                               "event_mask": t["mask"], "gtflow": t["gt"],
                                               "dt_input": torch.from_numpy(g[f"b{B}_dt_in"]),
                                               "dt_gt": torch.from_numpy(g[f"b{B}_dt_gt"])})
        res = m()
        res = res if isinstance(res, tuple) else (res,)
        for j, r in enumerate(res):
            key = f"b{B}_{name}_{j}"
            if key in g:
                np.testing.assert_allclose(r.cpu().numpy().reshape(-1), g[key], rtol=1e-5, err_msg=key)
                n += 1
    assert n == (8 if B == 1 else 4)


def test_flow_metrics_vs_oracle_random(dev):
    """Every metric column vs the CPU oracle on a ragged random case (B=3, 37x53: partial
    pixel chunks; per-sample dt ratios; zero-gt rows; tiny flows near the magnitude filter)."""
    from snnflow import _lib, metrics
    from oracle.metrics_ref import flow_metrics_ref

    gen = torch.Generator().manual_seed(17)
    B, H, W = 3, 37, 53
    flow = (torch.rand(B, 2, H, W, generator=gen) - 0.5) * 0.08
    gt = (torch.rand(B, 2, H, W, generator=gen) - 0.5) * 10
    gt[:, :, :4] = 0.0
    mask = (torch.rand(B, 1, H, W, generator=gen) < 0.5).float()
    dt_in, dt_gt = torch.tensor([0.5, 0.25, 1.0]), torch.tensor([1.0, 1.0, 0.5])

    class _M:
        pass

    m = _M()
    m._flow_map, m._gtflow, m._event_mask = [flow.to(dev)], gt.to(dev), mask.to(dev)
    m._dt_input, m._dt_gt, m.flow_scaling = dt_in, dt_gt, 128
    ours = metrics._flow_metrics(m, mag_threshold=0.5)
    ref = flow_metrics_ref(flow, gt, mask, dt_in, dt_gt, 128, 0.5)
    for k in _lib.METRICS:
        np.testing.assert_allclose(ours[k].cpu().numpy(), ref[k].numpy(), rtol=2e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("scale", [1e-3, 10.0])
def test_clip_grad_norm_flat_vs_torch(dev, scale):
    """snnflow_clip_grad_norm (one launch over the engine's flat gradient buffer) against
    torch.nn.utils.clip_grad_norm_ on the same gradients (no clipping / clipping)."""
    from snnflow import dp

    gen = torch.Generator().manual_seed(9)
    shapes = [(8, 2, 3, 3), (8,), (8, 8, 3, 3), (2, 8, 1, 1), (2,)]
    vals = [torch.randn(s, generator=gen) * scale for s in shapes]
    flat = torch.cat([v.reshape(-1) for v in vals]).to(dev)
    ps, ref = [], []
    off = 0
    for v in vals:
        p = torch.nn.Parameter(torch.zeros_like(v, device=dev))
        p.grad = flat[off:off + v.numel()].view(v.shape)
        off += v.numel()
        ps.append(p)
        q = torch.nn.Parameter(torch.zeros_like(v))
        q.grad = v.clone()
        ref.append(q)
    total = dp.clip_grad_norm_(ps, 1.0)
    rtotal = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    np.testing.assert_allclose(total.item(), rtotal.item(), rtol=1e-5)
    for p, q in zip(ps, ref):
        np.testing.assert_allclose(p.grad.cpu().numpy(), q.grad.numpy(), rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("H,W,Ns", [(256, 256, (3000, 2500, 3000)), (100, 130, (700, 0, 500)),
                                    (48, 640, (800, 600))])
def test_event_warping_bands_and_empty_windows_vs_oracle(dev, H, W, Ns):
    """The binned IWE splat and the banded backward at 256x256 (64 splat bands of 1024 pixels), a
    ragged image (100x130: partial last band and pixel chunk), an empty event window (N_k = 0) and a
    wide image (48x640: warps up to +-16 pixels, corners in a neighbouring band, the backward's LDS
    neighbourhood of 2 W + 2 extra pixels) against the CPU oracle: loss rtol 2e-5, per-window flow
    gradients relative-L2 1e-4."""
    import snnflow
    from oracle import iwe_ref
    from snnflow.synthetic import make_window

    B = 2
    gen = torch.Generator(device=dev).manual_seed(21)
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ew = snnflow.EventWarping(cfg, dev)
    ref = iwe_ref.EventWarpingRef([H, W])
    fl_d, fl_c = [], []
    for n in Ns:
        if n:
            w = make_window(B, n, H, W, gen, dev)
        else:
            w = {"event_list": torch.zeros(B, 0, 4, device=dev), "event_list_pol_mask": torch.zeros(B, 0, 2, device=dev),
                 "event_mask": torch.zeros(B, 1, H, W, device=dev)}
        f = ((torch.rand(B, 2, H, W, generator=gen, device=dev) - 0.5) * 0.05).requires_grad_(True)
        fc = f.detach().cpu().requires_grad_(True)
        fl_d.append(f)
        fl_c.append(fc)
        ew.event_flow_association([f], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        ref.event_flow_association([fc], w["event_list"].cpu(), w["event_list_pol_mask"].cpu(), w["event_mask"].cpu())
    loss = ew()
    rl = ref()
    loss.backward()
    rl.backward()
    np.testing.assert_allclose(loss.item(), rl.item(), rtol=2e-5)
    for t in range(len(Ns)):
        gc = fl_c[t].grad
        gd = fl_d[t].grad
        if gc is None or not gc.abs().max() > 0:
            assert gd is None or float(gd.abs().max()) == 0.0
            continue
        assert _rel(gd.cpu().numpy(), gc.numpy()) < 1e-4, t


# ---------------------------------------------------------------------------
# Wavefront sequence path (forward_sequence) against the per-step path
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("H,W,T,name", [(64, 64, 5, "LIFFireNet"), (40, 72, 3, "LIFFireNet"),
                                         (64, 64, 5, "LIFFireNet_short"), (48, 64, 4, "LIFFireFlowNet"),
                                         (40, 56, 3, "LIFFireFlowNet_short")])
def test_forward_sequence_matches_per_step(dev, H, W, T, name):
    _check_sequence_vs_per_step(dev, H, W, T, name, B=2, N=300, iters=2)


@pytest.mark.parametrize("H,B", [(128, 8), (256, 4)])
def test_forward_sequence_matches_per_step_full_size(dev, H, B):
    """BASELINE cfg2 (128x128, B=8) and cfg3 (256x256, B=4) at full size, T=10 windows of 1000
    events, C=8: the bench's wavefront train step against the reference loop's per-step calls
    (size-independent property: two launch orders of the same arithmetic agree near-exactly),
    plus spikes exactly 0/1 and every gradient finite."""
    mb = _check_sequence_vs_per_step(dev, H, H, 10, "LIFFireNet", B=B, N=1000, iters=1)
    for st in mb.states:
        s = st[1].detach()
        assert torch.equal(s, (s > 0.5).float())
    assert all(torch.isfinite(p.grad).all() for p in mb.parameters())


@pytest.mark.parametrize("C", [16, 32])
def test_forward_sequence_matches_per_step_wide(dev, C):
    """C = 16 / 32 wavefront launches (LIFFireNet task kinds in k_fwd_slot / k_bwd_slot, the top
    LIF in the quad layout, bf16 six-product input gradients from global fragments) against the
    per-step calls: flows, loss, gradients, states, running statistics over two windows."""
    _check_sequence_vs_per_step(dev, 48, 64, 3, "LIFFireNet", B=2, N=300, iters=2, C=C)


def _check_sequence_vs_per_step(dev, H, W, T, name, B, N, iters, C=8):
    """T steps through model.forward_sequence (wavefront launches, FireNetSequence) against T
    model.forward calls (FireNetStep) of an identical copy: flows, loss, every parameter
    gradient, final states, lif.mem caches and BatchNorm running statistics, over two
    truncated-BPTT windows (the second starts from the first's detached states).  The
    per-(layer, step) arithmetic is the same code; only fp64 batch-sum atomics may add in
    another order, so the tolerances are near-exact."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(5)
    kw = lif_ref.make_unet_kwargs(base_num_channels=C)
    ma = getattr(snnflow, name)(dict(kw)).to(dev).train()
    mb = copy.deepcopy(ma)
    assert mb.engine.sequence_ok(2)  # the wavefront path runs
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ea, eb = snnflow.EventWarping(cfg, dev), snnflow.EventWarping(cfg, dev)
    gen = torch.Generator(device=dev).manual_seed(13)
    for it in range(iters):
        wins = [make_window(B, N, H, W, gen, dev) for _ in range(T)]
        fa = [ma(w["event_voxel"], w["event_cnt"])["flow"][0] for w in wins]
        outs = mb.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
        assert len(outs) == T
        for t, w in enumerate(wins):
            ea.event_flow_association([fa[t]], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            eb.event_flow_association(outs[t]["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            np.testing.assert_allclose(outs[t]["flow"][0].detach().cpu().numpy(), fa[t].detach().cpu().numpy(),
                                       rtol=1e-5, atol=1e-7, err_msg=f"flow it {it} t {t}")
        la, lb = ea(), eb()
        ma.zero_grad(set_to_none=True)
        mb.zero_grad(set_to_none=True)
        la.backward()
        lb.backward()
        np.testing.assert_allclose(lb.item(), la.item(), rtol=1e-6)
        for (n, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
            assert _rel(b.grad.cpu().numpy(), a.grad.cpu().numpy()) < 1e-5, (it, n)
        for sa, sb in zip(ma.states, mb.states):
            np.testing.assert_allclose(sb.detach().cpu().numpy(), sa.detach().cpu().numpy(), rtol=1e-5, atol=1e-6)
        for (n, a), (_, b) in zip(ma.named_buffers(), mb.named_buffers()):
            np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-5, atol=1e-7, err_msg=n)
        for n, _ in ma.layer_spec:
            np.testing.assert_allclose(getattr(mb, n).lif.mem.cpu().numpy(), getattr(ma, n).lif.mem.cpu().numpy(),
                                       rtol=1e-5, atol=1e-6)
        ma.detach_states()
        mb.detach_states()
        ea.reset()
        eb.reset()
    return mb


def test_forward_sequence_input_and_state_grads(dev):
    """Gradients into the sequence's inputs and into initial states that did not come from the
    engine (the 'external state' path) match the per-step path."""
    import copy

    import snnflow
    from oracle import lif_ref

    torch.manual_seed(6)
    H = W = 32
    T, B, C = 3, 2, 8
    kw = lif_ref.make_unet_kwargs(base_num_channels=C)
    ma = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    mb = copy.deepcopy(ma)
    gen = torch.Generator(device=dev).manual_seed(2)
    xs = [(torch.rand(B, 2, H, W, generator=gen, device=dev) < 0.2).float() * 3 for _ in range(T)]
    st0 = [(torch.rand(2, B, C, H, W, generator=gen, device=dev) * 0.8) for _ in range(7)]
    for s in st0:
        s[1] = (s[1] > 0.5).float()
    wts = [torch.randn(B, 2, H, W, generator=gen, device=dev) for _ in range(T)]
    res = {}
    for tag, m in (("step", ma), ("seq", mb)):
        xg = [x.clone().requires_grad_(True) for x in xs]
        sg = [s.clone().requires_grad_(True) for s in st0]
        m.states = sg
        if tag == "step":
            flows = [m(None, x)["flow"][0] for x in xg]
        else:
            flows = [o["flow"][0] for o in m.forward_sequence(None, xg)]
        loss = sum((f * w).sum() for f, w in zip(flows, wts))
        loss.backward()
        res[tag] = ([x.grad.cpu().numpy() for x in xg], [None if s.grad is None else s.grad.cpu().numpy() for s in sg],
                    [p.grad.cpu().numpy() for p in m.parameters()])
    for a, b in zip(res["step"][0], res["seq"][0]):
        assert _rel(b, a) < 1e-5
    for a, b in zip(res["step"][1], res["seq"][1]):
        assert (a is None) == (b is None)
        if a is not None:
            assert _rel(b, a) < 1e-5
    for a, b in zip(res["step"][2], res["seq"][2]):
        assert _rel(b, a) < 1e-5


def test_forward_sequence_final_state_out(dev):
    """FireNetEngine.final_state_out (the bench's copy-free state hand-over): two chained train
    sequences with the final states written into alternating caller buffers give the same flows,
    parameter gradients and states, bit for bit, as fresh allocations + detach; the returned states
    are views into the buffer; a buffer aliasing the initial states is refused."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow import _lib

    torch.manual_seed(8)
    H = W = 32
    T, B, C = 3, 2, 8
    ma = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=C)).to(dev).train()
    mb = copy.deepcopy(ma)
    gen = torch.Generator(device=dev).manual_seed(4)
    xs = [(torch.rand(B, 2, H, W, generator=gen, device=dev) < 0.2).float() * 3 for _ in range(2 * T)]
    n = mb.engine.L * 2 * B * C * H * W
    bufs = [torch.full((n,), float("nan"), device=dev), torch.full((n,), float("nan"), device=dev)]
    out = {}
    for tag, m in (("alloc", ma), ("buf", mb)):
        flows, grads = [], []
        for k in range(2):
            if tag == "buf":
                m.engine.final_state_out = bufs[k % 2]
            outs = m.forward_sequence(None, xs[k * T:(k + 1) * T])
            if tag == "buf":
                base = bufs[k % 2].data_ptr()
                assert all(base <= s.data_ptr() < base + 4 * n for s in m._states)
            sum(o["flow"][0].square().sum() for o in outs).backward()
            flows += [o["flow"][0].detach().cpu() for o in outs]
            grads.append([p.grad.detach().cpu().clone() for p in m.parameters()])
            m.zero_grad(set_to_none=True)
            m.detach_states()
        out[tag] = (flows, grads, [s.detach().cpu() for s in m._states])
    for a, b in zip(out["alloc"][0], out["buf"][0]):
        assert torch.equal(a, b)
    for ga, gb in zip(out["alloc"][1], out["buf"][1]):
        for a, b in zip(ga, gb):
            assert torch.equal(a, b)
    for a, b in zip(out["alloc"][2], out["buf"][2]):
        assert torch.equal(a, b)
    with torch.no_grad():
        mb.engine.final_state_out = bufs[0]
        mb.forward_sequence(None, xs[:T])  # mb's states are now views of bufs[0]
        mb.engine.final_state_out = bufs[0]
        with pytest.raises(_lib.SnnflowError):
            mb.forward_sequence(None, xs[:T])


def test_forward_sequence_unread_state_writes(dev):
    """The window leaves out the spike half of the feed-forward layers' intermediate states
    (state_spk_skip, C = 8) and the membrane half of the internal state gradients; a run that keeps
    every step's states (capture_states: nothing skipped) gives the same flows, parameter gradients
    and final states bit for bit, and its per-step states are complete (finite) everywhere."""
    import copy

    import snnflow
    from oracle import lif_ref

    torch.manual_seed(9)
    H = W = 32
    T, B, C = 4, 2, 8
    ma = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=C)).to(dev).train()
    mb = copy.deepcopy(ma)
    mb.engine.capture_states = True
    gen = torch.Generator(device=dev).manual_seed(5)
    xs = [(torch.rand(B, 2, H, W, generator=gen, device=dev) < 0.2).float() * 3 for _ in range(2 * T)]
    out = {}
    for tag, m in (("skip", ma), ("keep", mb)):
        flows, grads = [], []
        for k in range(2):
            outs = m.forward_sequence(None, xs[k * T:(k + 1) * T])
            if tag == "keep":
                for sts in m.engine.seq_states:
                    assert all(bool(torch.isfinite(s).all()) for s in sts)
                m.engine.seq_states = None
            sum(o["flow"][0].square().sum() for o in outs).backward()
            flows += [o["flow"][0].detach().cpu() for o in outs]
            grads.append([p.grad.detach().cpu().clone() for p in m.parameters()])
            m.zero_grad(set_to_none=True)
            m.detach_states()
        out[tag] = (flows, grads, [s.detach().cpu() for s in m._states])
    for a, b in zip(out["skip"][0], out["keep"][0]):
        assert torch.equal(a, b)
    for ga, gb in zip(out["skip"][1], out["keep"][1]):
        for a, b in zip(ga, gb):
            assert torch.equal(a, b)
    for a, b in zip(out["skip"][2], out["keep"][2]):
        assert torch.equal(a, b)


def test_forward_sequence_eval_mode_and_fallbacks(dev):
    """Eval mode (running statistics, no running-stat update) through the wavefront launches
    matches per-step eval; T = 1 and log=True take the per-step path with the same results."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(8)
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    ma = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(3)
    wins = [make_window(2, 300, 48, 64, gen, dev) for _ in range(4)]
    for w in wins[:2]:  # populate running statistics and the lif.mem caches
        ma(w["event_voxel"], w["event_cnt"])
    ma.eval()
    ma.detach_states()
    mb = copy.deepcopy(ma)
    rm = ma.G1.bn.running_mean.clone()
    with torch.no_grad():
        fa = [ma(w["event_voxel"], w["event_cnt"])["flow"][0] for w in wins]
        fb = [o["flow"][0] for o in mb.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])]
    assert torch.equal(mb.G1.bn.running_mean, rm)
    for a, b in zip(fa, fb):
        np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-5, atol=1e-7)
    for sa, sb in zip(ma.states, mb.states):
        np.testing.assert_allclose(sb.cpu().numpy(), sa.cpu().numpy(), rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        one = mb.forward_sequence(None, [wins[0]["event_cnt"]])
        logged = mb.forward_sequence(None, [w["event_cnt"] for w in wins[:2]], log=True)
    assert len(one) == 1 and len(logged) == 2 and logged[0]["activity"] is not None


@pytest.mark.parametrize("C", [16, 32])
def test_engine_gradients_wide_vs_oracle(dev, C):
    """C = 16 / 32 through the engine (pre-split weight fragments from the prep kernel: forward
    spike convs and the bf16 six-product input gradients read them from L2) against the oracle:
    flows, loss and every parameter gradient of a T = 2 window."""
    import snnflow
    from oracle import iwe_ref, lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(12)
    H = W = 32
    kw = lif_ref.make_unet_kwargs(base_num_channels=C)
    model = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    ref = lif_ref.LIFFireNetRef(dict(kw), "LIFFireNet").train()
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ew = snnflow.EventWarping(cfg, dev)
    rew = iwe_ref.EventWarpingRef([H, W], weight=0.001)
    gen = torch.Generator(device=dev).manual_seed(17)
    for t in range(2):
        w = make_window(2, 400, H, W, gen, dev)
        out = model(w["event_voxel"], w["event_cnt"])
        rout = ref(None, w["event_cnt"].cpu())
        a, b = out["flow"][0].detach().cpu().numpy(), rout["flow"][0].detach().numpy()
        print(f"\n[engine C={C}] step {t}: flow max |d| {np.abs(a - b).max():.2e}")
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
        ew.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        rew.event_flow_association(rout["flow"], w["event_list"].cpu(), w["event_list_pol_mask"].cpu(),
                                   w["event_mask"].cpu())
    loss, rloss = ew(), rew()
    loss.backward()
    rloss.backward()
    np.testing.assert_allclose(loss.item(), rloss.item(), rtol=1e-5)
    assert model.engine.prep.frag.get(1) is not None  # the fragment path ran
    _grad_check(f"engine C={C}", [(n, a.grad.cpu().numpy(), b.grad.numpy()) for (n, a), (_, b)
                                   in zip(model.named_parameters(), ref.named_parameters())], ORACLE_GRAD_TOL)


@pytest.mark.parametrize("recurrent", [False, True])
def test_subtract_reset_cell_vs_oracle(dev, recurrent):
    """A standalone SNNtorch_ConvLIF(Recurrent) cell with hard_reset=False (snn.Leaky reset_mechanism
    "subtract", SNNtorch_spiking_submodules.py:171; reachable through the cell constructors only:
    LIFFireNet does not pass spiking_neuron to its cells, models/model.py:53-56, 83-107) over 3
    calls against SnnTorchCellRef: spikes, states and every parameter gradient.  The threshold's
    gradient includes -sum r * dL/dv through v = beta*m + I - r*theta (snnflow_lif_theta_subtract)."""
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(31)
    C, B, H, W = 8, 2, 24, 40
    cls = snnflow.SNNtorch_ConvLIFRecurrent if recurrent else snnflow.SNNtorch_ConvLIF
    cell = cls(C, C, 3, hard_reset=False, thresh=(0.2, 0.4)).to(dev).train()
    ref = lif_ref.SnnTorchCellRef(C, C, 3, recurrent=recurrent, hard_reset=False).train()
    ref.load_state_dict({k: v.detach().cpu() for k, v in cell.state_dict().items()}, strict=False)
    gen = torch.Generator().manual_seed(37)
    xs = [(torch.rand(B, C, H, W, generator=gen) * 2.0) for _ in range(3)]
    st, rst = None, None
    loss = rloss = 0.0
    for x in xs:
        spk, st = cell(x.to(dev), st)
        rspk, rst = ref(x, rst)
        np.testing.assert_array_equal(spk.detach().cpu().numpy(), rspk.detach().numpy())
        # (the subtract-reset membrane is not reset to 0: values up to ~3 carry fp32 rounding)
        np.testing.assert_allclose(st.detach().cpu().numpy(), rst.detach().numpy(), rtol=1e-5, atol=1e-5)
        wgt = torch.linspace(0.5, 1.5, C).view(1, C, 1, 1)
        loss = loss + (spk * wgt.to(dev)).sum()
        rloss = rloss + (rspk * wgt).sum()
    loss.backward()
    rloss.backward()
    rp = dict(ref.named_parameters())
    _grad_check(f"subtract cell rec={recurrent}", [(n, a.grad.cpu().numpy(), rp[n].grad.numpy())
                                                   for n, a in cell.named_parameters()], ORACLE_GRAD_TOL)


@pytest.mark.parametrize("recurrent,hard,mpbn", [(False, True, False), (True, True, False), (False, False, False),
                                                (True, False, False), (False, True, True), (True, True, True)])
def test_detach_false_cell_vs_oracle(dev, recurrent, hard, mpbn):
    """SNNtorch_ConvLIF(Recurrent)(detach=False) (SNNtorch_spiking_submodules.py:309-311: the
    membrane output keeps its graph, BPTT through the membrane): 4 calls, the first two chained
    through prev_state, the third with prev_state=None (snn.Leaky continues from its non-detached
    membrane cache), the fourth chained again; the loss uses spikes AND final membranes, so the
    membrane-output gradient path (mem_grad_in) and its threshold part are exercised.  With ``mpbn``
    the state's membrane is MPBN(mem_out) (:313-317), whose gradient reaches the LIF through the
    non-detached membrane.  Every parameter gradient and the input gradients against SnnTorchCellRef."""
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(41)
    C, B, H, W = 8, 2, 24, 40
    cls = snnflow.SNNtorch_ConvLIFRecurrent if recurrent else snnflow.SNNtorch_ConvLIF
    cell = cls(C, C, 3, hard_reset=hard, detach=False, thresh=(0.2, 0.4), mpbn=mpbn).to(dev).train()
    ref = lif_ref.SnnTorchCellRef(C, C, 3, recurrent=recurrent, hard_reset=hard, detach=False, mpbn=mpbn).train()
    ref.load_state_dict({k: v.detach().cpu() for k, v in cell.state_dict().items()}, strict=False)
    gen = torch.Generator().manual_seed(43)
    xs = [(torch.rand(B, C, H, W, generator=gen) * 2.0).requires_grad_(True) for _ in range(4)]
    xd = [x.detach().to(dev).requires_grad_(True) for x in xs]
    st = rst = None
    loss = rloss = 0.0
    wgt = torch.linspace(0.5, 1.5, C).view(1, C, 1, 1)
    for i, (x, xg) in enumerate(zip(xs, xd)):
        if i == 2:
            st = rst = None
        spk, st = cell(xg, st)
        rspk, rst = ref(x, rst)
        np.testing.assert_array_equal(spk.detach().cpu().numpy(), rspk.detach().numpy())
        np.testing.assert_allclose(st.detach().cpu().numpy(), rst.detach().numpy(), rtol=1e-5, atol=1e-5)
        loss = loss + (spk * wgt.to(dev)).sum() + 0.1 * (st[0] * wgt.to(dev)).sum()
        rloss = rloss + (rspk * wgt).sum() + 0.1 * (rst[0] * wgt).sum()
    loss.backward()
    rloss.backward()
    rp = dict(ref.named_parameters())
    pairs = [(n, a.grad.cpu().numpy(), rp[n].grad.numpy()) for n, a in cell.named_parameters()]
    pairs += [(f"x{i}", a.grad.cpu().numpy(), b.grad.numpy()) for i, (a, b) in enumerate(zip(xd, xs))]
    _grad_check(f"detach=False rec={recurrent} hard={hard}", pairs, ORACLE_GRAD_TOL)


def test_forward_sequence_chained_without_detach(dev):
    """Two forward_sequence calls whose states are not detached in between (one BPTT window of
    2T steps): the second call's backward must hand its state gradients to the first (non-root
    node, deferred weight gradients flushed once by the first) -- against 2T model() calls."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(21)
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    ma = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    mb = copy.deepcopy(ma)
    H = W = 48
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ea, eb = snnflow.EventWarping(cfg, dev), snnflow.EventWarping(cfg, dev)
    gen = torch.Generator(device=dev).manual_seed(22)
    wins = [make_window(2, 300, H, W, gen, dev) for _ in range(6)]
    fa = [ma(w["event_voxel"], w["event_cnt"])["flow"][0] for w in wins]
    outs = (mb.forward_sequence([w["event_voxel"] for w in wins[:3]], [w["event_cnt"] for w in wins[:3]]) +
            mb.forward_sequence([w["event_voxel"] for w in wins[3:]], [w["event_cnt"] for w in wins[3:]]))
    for t, w in enumerate(wins):
        ea.event_flow_association([fa[t]], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        eb.event_flow_association(outs[t]["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
    la, lb = ea(), eb()
    la.backward()
    lb.backward()
    np.testing.assert_allclose(lb.item(), la.item(), rtol=1e-6)
    for (n, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
        assert _rel(b.grad.cpu().numpy(), a.grad.cpu().numpy()) < 1e-5, n


# ---------------------------------------------------------------------------
# Activity log (models/model.py:188-205)
# ---------------------------------------------------------------------------
def test_count_nonzero_exact_on_edge_cases(dev):
    """snnflow_count_nonzero against torch's count: ragged sizes (not multiples of 4 or of a
    block), an unaligned start, -0.0 (not counted), NaN and inf (counted), empty and all-zero
    regions, a permuted dense view (the [2,B,C,H,W] state over NHWC memory) -- exact against the
    CPU reduction (fp32 sum / numel; torch's HIP mean multiplies by 1/numel and can differ by
    one ulp)."""
    from snnflow.model import activity_log

    g = torch.Generator(device=dev).manual_seed(5)
    base = (torch.rand(1 << 20, generator=g, device=dev) < 0.3).float()
    special = torch.tensor([0.0, -0.0, float("nan"), float("inf"), -1e-38, 1e-45], device=dev)
    nhwc = (torch.rand(2, 3, 17, 19, 8, generator=g, device=dev) < 0.5).float()
    tensors = [base, base[:1], base[:3], base[:5], base[1:100003], base[3:], special,
               torch.zeros(777, device=dev), torch.empty(0, device=dev),
               nhwc.permute(0, 1, 4, 2, 3)[1], (torch.rand(4, 2, 33, 65, generator=g, device=dev) - 0.5)]
    names = [str(i) for i in range(len(tensors))]
    got = activity_log(names, tensors)
    for n, t in zip(names, tensors):
        want = t.cpu().ne(0).float().mean().item()
        if t.numel() == 0:
            assert np.isnan(got[n]) and np.isnan(want)
        else:
            assert got[n] == want, (n, got[n], want)
    assert got["6"] == float(np.float32(4) / np.float32(6))  # subnormals count, as on the CPU


def test_liffirenet_log_activity_matches_torch_reduction(dev):
    """forward(log=True) returns the reference's activity dict (names and values) for every
    layer output, equal to `l.detach().ne(0).float().mean().item()` on the same tensors (CPU
    reduction, the reference's platform)."""
    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(2)
    m = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=8)).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(4)
    names = ["0:input", "1:head", "2:G1", "3:R1a", "4:R1b", "5:G2", "6:R2a", "7:R2b", "8:pred"]
    for _ in range(3):
        w = make_window(2, 500, 48, 64, gen, dev)
        out = m(w["event_voxel"], w["event_cnt"], log=True)
        act = out["activity"]
        assert list(act) == names
        tensors = [w["event_cnt"]] + [s[1] for s in m.states] + [out["flow"][0]]
        for n, t in zip(names, tensors):
            assert act[n] == t.detach().cpu().ne(0).float().mean().item(), n
        assert 0.0 < act["0:input"] < 1.0 and act["8:pred"] > 0.0


def test_forward_sequence_log_activity(dev):
    """forward_sequence(log=True) keeps the wavefront launches and returns every step's activity
    dict: the last step equal to the CPU reduction of its returned tensors, every step within a
    few spike flips (1e-4) of T per-step forward(log=True) calls on a copy of the model."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(6)
    ma = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=8)).to(dev).train()
    mb = copy.deepcopy(ma)
    gen = torch.Generator(device=dev).manual_seed(9)
    wins = [make_window(2, 400, 48, 64, gen, dev) for _ in range(4)]
    with torch.no_grad():
        seq = mb.forward_sequence(None, [w["event_cnt"] for w in wins], log=True)
        per = [ma(None, w["event_cnt"], log=True) for w in wins]
    assert mb.engine.seq_states is None and not mb.engine.keep_seq_states
    names = list(per[0]["activity"])
    last = [wins[-1]["event_cnt"]] + [s[1] for s in mb.states] + [seq[-1]["flow"][0]]
    for n, t in zip(names, last):
        assert seq[-1]["activity"][n] == t.detach().cpu().ne(0).float().mean().item(), n
    for a, b in zip(per, seq):
        assert list(b["activity"]) == names
        for n in names:
            assert abs(a["activity"][n] - b["activity"][n]) <= 1e-4, n


def test_export_op_dispatches_to_hip(golden, dev):
    """torch.ops.SNN_implementation.LIF on device tensors runs snnflow_lif_export (registered by
    snnflow.export_op): bit-exact against the reference op's fixture; beside the reference's CPU
    kernel when its library is loaded (test_lif_export_op_vs_reference_op loads it first)."""
    from snnflow.export_op import register_lif_op

    op = register_lif_op()
    g = golden("lif_export_case.npz")
    args = [torch.from_numpy(g[k]) for k in ("x", "mem", "beta", "threshold")]
    spk, mo = op(*(a.to(dev) for a in args))
    assert spk.device.type == "cuda"
    np.testing.assert_array_equal(spk.cpu().numpy(), g["spk"])
    np.testing.assert_array_equal(mo.cpu().numpy(), g["mem_out"])
    gen = torch.Generator().manual_seed(11)
    x, m = torch.randn(3, 8, 20, 24, generator=gen), torch.randn(3, 8, 20, 24, generator=gen)
    b, th = torch.rand(8, 1, 1, generator=gen), torch.rand(8, 1, 1, generator=gen)  # [C,1,1] as the cells hold them
    s2, m2 = op(x.to(dev), m.to(dev), b.to(dev), th.to(dev))
    if torch._C._dispatch_has_kernel_for_dispatch_key("SNN_implementation::LIF", "CPU"):
        rs, rm = op(x, m, b, th)
        assert torch.equal(rs, s2.cpu()) and torch.equal(rm, m2.cpu())
    with pytest.raises(RuntimeError):
        op(x.to(dev), m[:, :4].to(dev), b.to(dev), th.to(dev))


def test_log_activity_with_forward_hooks(dev):
    """With a forward hook on a cell (analyze_voltage_dynamics.py:80-96 style) the cells run one by
    one; the activity log of that path equals the fused path's on an identical copy."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(3)
    ma = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=8)).to(dev).eval()
    mb = copy.deepcopy(ma)
    seen = []
    mb.G1.register_forward_hook(lambda m, i, o: seen.append(o[0].detach().ne(0).float().mean().item()))
    gen = torch.Generator(device=dev).manual_seed(12)
    with torch.no_grad():
        for _ in range(2):
            w = make_window(2, 500, 40, 48, gen, dev)
            a = ma(None, w["event_cnt"], log=True)["activity"]
            b = mb(None, w["event_cnt"], log=True)["activity"]
            assert list(a) == list(b)
            for n in a:
                assert abs(a[n] - b[n]) <= 1e-4, n
    assert len(seen) == 2


@pytest.mark.parametrize("name,B,H,W,T,tf", [("LIFFireNet", 8, 32, 32, 5, 2), ("LIFFireNet", 8, 64, 32, 2, 1),
                                              ("LIFFireNet", 8, 32, 48, 6, 3), ("LIFFireNet", 3, 40, 72, 4, 2),
                                              ("LIFFireNet_short", 8, 32, 32, 4, 4), ("LIFFireFlowNet", 8, 32, 32, 3, 2)])
def test_pipelined_slots_match_one_tile_slots(dev, name, B, H, W, T, tf):
    """The C = 8 forward tile pipeline of the wavefront launches (fwd_lif8_pipe: several tiles per
    block, the next tile's halos by LDS-DMA, swapped-operand convs packed by permlane32_swap, the batch
    sums accumulated over a block's tiles) against the one-tile-per-block bodies (snnflow_set_pipe(0,
    0)) on the same window: flows, every state, the lif.mem caches, BatchNorm running statistics and
    num_batches_tracked, and the backward's gradients.  tf: tiles per block of the forward pipeline.
    Shapes include partial tiles (W = 48, 40 x 72), a batch that is not a multiple of 8 and blocks with
    1-4 tiles.  Same per-(layer, step) arithmetic; the batch sums add in another order (fp32 per lane
    over a block's tiles, fp64 atomics), so spikes may only differ where the membrane lies within
    rounding of the threshold."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow import _lib
    from snnflow.synthetic import make_window

    torch.manual_seed(21)
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    ma = getattr(snnflow, name)(dict(kw)).to(dev).train()
    mb = copy.deepcopy(ma)
    gen = torch.Generator(device=dev).manual_seed(22)
    wins = [make_window(B, 500, H, W, gen, dev) for _ in range(T)]
    res = {}
    old = (_lib.lib.snnflow_get_pipe(0), _lib.lib.snnflow_get_pipe(1))
    try:
        for tag, m, fwd in (("pipe", ma, tf), ("one", mb, 0)):
            assert _lib.lib.snnflow_set_pipe(fwd, 0) == 0
            outs = m.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
            loss = sum(((o["flow"][0] * (t + 1)) ** 2).sum() for t, o in enumerate(outs))
            loss.backward()
            torch.cuda.synchronize()
            res[tag] = outs
    finally:
        _lib.lib.snnflow_set_pipe(*old)
    for t in range(T):
        np.testing.assert_allclose(res["pipe"][t]["flow"][0].detach().cpu().numpy(),
                                   res["one"][t]["flow"][0].detach().cpu().numpy(), rtol=1e-5, atol=1e-6)
    for sa, sb in zip(ma.states, mb.states):
        np.testing.assert_allclose(sa.detach().cpu().numpy(), sb.detach().cpu().numpy(), rtol=1e-5, atol=1e-5)
    for (n, a), (_, b) in zip(ma.named_buffers(), mb.named_buffers()):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, atol=1e-7, err_msg=n)
    for n, _ in ma.layer_spec:
        np.testing.assert_allclose(getattr(ma, n).lif.mem.cpu().numpy(), getattr(mb, n).lif.mem.cpu().numpy(),
                                   rtol=1e-5, atol=1e-5)
    for (n, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
        assert _rel(a.grad.cpu().numpy(), b.grad.cpu().numpy()) < 1e-5, n


def test_pipelined_forward_nonbinary_state(dev):
    """Initial states whose spike half is not 0/1 (a caller-provided state): the recurrent conv of the
    pipelined forward detects s_prev values that are not exact in bf16 and computes that tile's
    recurrent conv on the vector ALU in f32; flows and states equal the one-tile bodies' (which
    take the f32 matrix-core path there)."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow import _lib
    from snnflow.synthetic import make_window

    B, H, W, T = 8, 32, 32, 2
    torch.manual_seed(5)
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    ma = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    mb = copy.deepcopy(ma)
    gen = torch.Generator(device=dev).manual_seed(6)
    wins = [make_window(B, 500, H, W, gen, dev) for _ in range(T)]
    states = [torch.rand(2, B, 8, H, W, generator=gen, device=dev) for _ in range(ma.engine.L)]
    res = {}
    old = (_lib.lib.snnflow_get_pipe(0), _lib.lib.snnflow_get_pipe(1))
    try:
        for tag, m, fwd in (("pipe", ma, 2), ("one", mb, 0)):
            _lib.lib.snnflow_set_pipe(fwd, 0)
            m.states = [s.clone() for s in states]
            with torch.no_grad():
                outs = m.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
            torch.cuda.synchronize()
            res[tag] = outs
    finally:
        _lib.lib.snnflow_set_pipe(*old)
    for t in range(T):
        np.testing.assert_allclose(res["pipe"][t]["flow"][0].cpu().numpy(), res["one"][t]["flow"][0].cpu().numpy(),
                                   rtol=1e-5, atol=1e-6)
    for sa, sb in zip(ma.states, mb.states):
        np.testing.assert_allclose(sa.cpu().numpy(), sb.cpu().numpy(), rtol=1e-5, atol=1e-5)


def test_iwe_loss_bit_reproducible(dev):
    """The IWE splat accumulates in 64-bit fixed point (csrc/iwe_loss.hip, SNNFLOW_SPLAT_FIXED), and so
    do the per-pixel sums of the per-event flow gradients: the loss and dL/dflow are the same bits on
    every run even where hundreds of events pile onto a few pixels
    (LDS atomics landing in a different order each run), and matches the oracle (fp32 sequential
    index_put_, loss/flow.py:178-303) to rtol 1e-5."""
    import snnflow
    from oracle import iwe_ref

    H, W, B, N, T = 64, 64, 4, 6000, 3
    gen = torch.Generator().manual_seed(77)
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    wins = []
    for t in range(T):
        # events crowded onto a 6x6 patch: ~40 events and up to 4 corners per pixel per window
        ys = torch.randint(20, 26, (B, N), generator=gen).float()
        xs = torch.randint(30, 36, (B, N), generator=gen).float()
        ts = torch.sort(torch.rand(B, N, generator=gen), dim=1).values
        ps = torch.randint(0, 2, (B, N), generator=gen).float() * 2 - 1
        ev = torch.stack([ts, ys, xs, ps], dim=2)
        pol = torch.stack([(ps > 0).float(), (ps < 0).float()], dim=2)
        mask = torch.zeros(B, 1, H, W)
        mask[:, :, 20:26, 30:36] = 1
        flow = (torch.rand(B, 2, H, W, generator=gen) - 0.5) * 0.05
        wins.append((ev, pol, mask, flow))
    losses, grads = [], []
    for rep in range(5):
        lf = snnflow.EventWarping(cfg, dev)
        fl = [flow.to(dev).requires_grad_() for _, _, _, flow in wins]
        for (ev, pol, mask, _), f in zip(wins, fl):
            lf.event_flow_association([f], ev.to(dev), pol.to(dev), mask.to(dev))
        loss = lf()
        loss.backward()
        losses.append(loss.item())
        grads.append(torch.cat([f.grad.flatten() for f in fl]).cpu())
    assert all(v == losses[0] for v in losses), losses
    # the flow gradients too: the ~40 events per pixel are summed in fixed point (k_iwe_bwd_band)
    for g in grads[1:]:
        assert torch.equal(g, grads[0])
    rl = iwe_ref.EventWarpingRef([H, W])
    for ev, pol, mask, flow in wins:
        rl.event_flow_association([flow], ev, pol, mask)
    np.testing.assert_allclose(losses[0], rl().item(), rtol=1e-5)


def _eval_model(C=8, seed=0):
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(seed)
    m = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=C))
    g = torch.Generator().manual_seed(seed + 3)
    for mod in m.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            mod.running_mean.copy_(0.2 * torch.randn(mod.running_mean.shape, generator=g))
            mod.running_var.copy_(0.5 + torch.rand(mod.running_var.shape, generator=g))
    return m


@pytest.mark.parametrize("B,H,W,T", [(2, 40, 72, 4), (8, 128, 128, 10)])
def test_eval_fused_matches_split(dev, monkeypatch, B, H, W, T):
    """The fused evaluation launches (engine.eval_sequence: conv + BN + LIF per task, T + L - 1
    launches) against the train-path split launches in eval mode (SNNFLOW_EVAL_FUSED=0), two chained
    calls (states carried), on a ragged shape (tiles past the image edge) and at cfg2's size: flows
    within 1e-5, spikes identical except where the membrane lies within 1e-4 of the threshold,
    membranes within 1e-5; the final states and every lif.mem cache likewise."""
    import copy

    from snnflow.synthetic import make_window

    ma = _eval_model().to(dev).eval()
    mb = copy.deepcopy(ma)
    ma.engine.capture_states = mb.engine.capture_states = True
    gen = torch.Generator(device=dev).manual_seed(9)
    wins = [make_window(B, 600, H, W, gen, dev) for _ in range(2 * T)]
    out = {}
    for tag, m, fused in (("split", ma, "0"), ("fused", mb, "1")):
        monkeypatch.setenv("SNNFLOW_EVAL_FUSED", fused)
        flows, sts = [], []
        with torch.no_grad():
            for k in range(2):
                o = m.forward_sequence(None, [w["event_cnt"] for w in wins[k * T:(k + 1) * T]])
                flows += [x["flow"][0].cpu() for x in o]
                sts += [[s.cpu() for s in st] for st in m.engine.seq_states]
        out[tag] = (flows, sts, [s.cpu() for s in m._states], [c.lif.mem.cpu() for c in m.engine.cells])
    worst = max(float((a - b).abs().max()) for a, b in zip(out["split"][0], out["fused"][0]))
    flips = 0
    for sa, sb in zip(out["split"][1], out["fused"][1]):
        for a, b in zip(sa, sb):
            d = (a[1] != b[1])
            flips += int(d.sum())
            assert float((a[0] - b[0]).abs()[~d].max()) <= 1e-5
    print(f"\n[eval fused {B}x{H}x{W} T={T}] max|dflow| {worst:.2e}, spike flips {flips}")
    assert worst <= 1e-5 or flips > 0
    assert flips <= 4
    for a, b in zip(out["split"][2] + out["split"][3], out["fused"][2] + out["fused"][3]):
        assert float((a - b).abs().max()) <= 1e-5 or flips > 0


def test_eval_fused_nonbinary_state_and_final_out(dev, monkeypatch):
    """Initial states with non-binary spike halves (the recurrent conv's vector-ALU fallback) and
    FireNetEngine.final_state_out on the fused evaluation path, against the split launches."""
    import copy

    ma = _eval_model(seed=2).to(dev).eval()
    mb = copy.deepcopy(ma)
    B, H, W, T, C = 2, 24, 40, 3, 8
    gen = torch.Generator(device=dev).manual_seed(5)
    xs = [(torch.rand(B, 2, H, W, generator=gen, device=dev) < 0.2).float() * 2 for _ in range(T)]
    st0 = [torch.rand(2, B, C, H, W, generator=gen, device=dev) * 0.7 for _ in range(7)]
    n = mb.engine.L * 2 * B * C * H * W
    fin = torch.full((n,), float("nan"), device=dev)
    res = {}
    for tag, m, fused in (("split", ma, "0"), ("fused", mb, "1")):
        monkeypatch.setenv("SNNFLOW_EVAL_FUSED", fused)
        m.states = [s.clone() for s in st0]
        if fused == "1":
            m.engine.final_state_out = fin
        with torch.no_grad():
            o = m.forward_sequence(None, xs)
        res[tag] = ([x["flow"][0].cpu() for x in o], [s.cpu() for s in m._states])
    if True:
        base = fin.data_ptr()
        assert all(base <= s.data_ptr() < base + 4 * n for s in mb._states)
    for a, b in zip(res["split"][0] + res["split"][1], res["fused"][0] + res["fused"][1]):
        assert float((a - b).abs().max()) <= 1e-5


@pytest.mark.parametrize("case", ["all_flows", "partial_loss", "state_grad", "two_windows"])
def test_per_step_chain_backward_batched(dev, case):
    """The reference loop's per-window calls (train_flow.py:232-262: T model() calls, one
    loss.backward()) are T autograd nodes; with FireNetEngine.defer_backward the later nodes only record
    their inputs and the chain's first step issues every step's backward as wavefront launches
    (snnflow_firenet_bwd_seq).  Against the same loop with every node running its own step
    (defer_backward = False), same weights and windows: flows identical (same forward), loss
    identical, parameter gradients within rel-L2 1e-5 (fp64 batch-sum atomics and the fused weight
    gradients sum in another order).  Cases: every flow in the loss; a loss on the first half of the
    windows only (the later nodes are never called); an extra loss term on an intermediate state
    (external state gradient: the chain falls back to the steps one after the other); two windows
    with a detach between them (two chains in two backward calls)."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(21)
    B, H, W, T = 2, 64, 96, 5
    base = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=8)).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(4)
    wins = [make_window(B, 600, H, W, gen, dev) for _ in range(2 * T)]
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    res = {}
    for defer in (False, True):
        m = copy.deepcopy(base)
        m.engine.defer_backward = defer
        lf = snnflow.EventWarping(cfg, dev)
        flows, losses, grads = [], [], []
        for k in range(2 if case == "two_windows" else 1):
            lf.reset()
            extra = 0.0
            for t in range(T):
                w = wins[k * T + t]
                out = m(w["event_voxel"], w["event_cnt"])
                flows.append(out["flow"][0].detach().cpu())
                if case != "partial_loss" or t < T // 2 + 1:
                    lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
                if case == "state_grad" and t == 2:
                    extra = m._states[1][1].sum() * 1e-3 + m._states[4][0].square().sum() * 1e-4
            loss = lf() + extra
            loss.backward()
            losses.append(loss.item())
            grads.append([p.grad.detach().cpu().clone() for p in m.parameters()])
            m.zero_grad(set_to_none=True)
            m.detach_states()
        res[defer] = (flows, losses, grads)
    for a, b in zip(res[False][0], res[True][0]):
        assert torch.equal(a, b)
    assert res[False][1] == res[True][1]
    names = [n for n, _ in base.named_parameters()]
    worst = 0.0
    for ga, gb in zip(res[False][2], res[True][2]):
        for n, a, b in zip(names, ga, gb):
            e = float((a - b).double().norm() / max(float(b.double().norm()), 1e-30))
            worst = max(worst, e)
            assert e <= 1e-5, (case, n, e)
    print(f"\n[{case}] batched chain backward vs per-node: worst gradient rel-L2 {worst:.2e}")


def test_per_step_chain_intermediate_state_gradients(dev):
    """Reading the gradient of an intermediate recurrent state of the per-window loop (retain_grad, a
    tensor hook, torch.autograd.grad with that state as the input) gives the same values whether the
    engine defers the chain's backward to its first step (defer_backward, the default) or runs every
    node itself: a node whose incoming state is read, or a pass that will not reach the chain's parameter
    anchor, runs its backward at once.  A full backward after such a partial pass gives the parameter
    gradients of a fresh run (the partial pass's open chain is dropped, not added in)."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(22)
    B, H, W, T = 2, 48, 64, 5
    base = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=8)).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(6)
    wins = [make_window(B, 500, H, W, gen, dev) for _ in range(T)]
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}

    def run(m, mode):
        m.reset_states()
        lf = snnflow.EventWarping(cfg, dev)
        kept, hooked = None, []
        for t in range(T):
            w = wins[t]
            out = m(w["event_voxel"], w["event_cnt"])
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            if t == 2:
                kept = m._states[1]  # G1 (recurrent) after step 2
                if mode == "retain":
                    kept.retain_grad()
                    m._states[4].register_hook(lambda g: hooked.append(g.detach().clone()))
        loss = lf()
        if mode == "autograd_grad":
            (g,) = torch.autograd.grad(loss, [kept], retain_graph=True)
            loss.backward()  # and then the full pass
            return g.detach().cpu(), [p.grad.detach().cpu().clone() for p in m.parameters()]
        loss.backward()
        return (kept.grad.detach().cpu(), hooked[0].cpu()), [p.grad.detach().cpu().clone() for p in m.parameters()]

    res = {}
    for defer in (False, True):
        for mode in ("retain", "autograd_grad"):
            m = copy.deepcopy(base)
            m.engine.defer_backward = defer
            res[(defer, mode)] = run(m, mode)

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    (sg_ref, hk_ref), g_ref = res[(False, "retain")]
    (sg, hk), g = res[(True, "retain")]
    assert sg_ref.abs().sum() > 0 and hk_ref.abs().sum() > 0
    e_state, e_hook = rel(sg, sg_ref), rel(hk, hk_ref)
    e_par = max(rel(a, b) for a, b in zip(g, g_ref))
    ga_ref, gp_ref = res[(False, "autograd_grad")]
    ga, gp = res[(True, "autograd_grad")]
    e_ag = rel(ga, ga_ref)
    e_ag_state = rel(ga_ref, sg_ref)
    e_after = max(rel(a, b) for a, b in zip(gp, g_ref))
    e_after_ref = max(rel(a, b) for a, b in zip(gp_ref, g_ref))
    print(f"\n[intermediate state grads] retain_grad {e_state:.2e}, hook {e_hook:.2e}, params {e_par:.2e}; "
          f"autograd.grad {e_ag:.2e} (vs retain_grad {e_ag_state:.2e}); full pass after it {e_after:.2e} "
          f"(per-node engine {e_after_ref:.2e})")
    assert e_state <= 1e-5 and e_hook <= 1e-5 and e_par <= 1e-5
    assert e_ag <= 1e-5 and e_ag_state <= 1e-5
    assert e_after <= 1e-5 and e_after_ref <= 1e-5


def test_iwe_loss_rejects_misshaped_inputs(dev):
    """EventWarping validates what its kernels index by (B, H, W): a flow tensor passed where the
    reference takes a list of flow maps (``list(tensor)`` splits it into per-sample [2, H, W] maps),
    events / polarity masks of another batch, a mask of another resolution -- each raises instead of
    being read out of bounds."""
    import snnflow
    from snnflow import _lib

    H, W, B, N = 32, 32, 2, 100
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    gen = torch.Generator().manual_seed(5)
    ev = torch.stack([torch.rand(B, N, generator=gen), torch.randint(0, H, (B, N), generator=gen).float(),
                      torch.randint(0, W, (B, N), generator=gen).float(), torch.ones(B, N)], dim=2).to(dev)
    pol = torch.stack([torch.ones(B, N), torch.zeros(B, N)], dim=2).to(dev)
    mask = torch.ones(B, 1, H, W, device=dev)
    flow = torch.zeros(B, 2, H, W, device=dev, requires_grad=True)
    cases = [(flow, ev, pol, mask),                                 # bare tensor: B maps of [2, H, W]
             ([flow], ev[:1], pol[:1], mask),                       # events of another batch
             ([flow], ev, pol[:, :, :1], mask),                     # one polarity column
             ([flow], ev, pol, torch.ones(B, 1, H, 2 * W, device=dev))]  # mask of another resolution
    for fl, e, p, m in cases:
        lf = snnflow.EventWarping(cfg, dev)
        lf.event_flow_association(fl, e, p, m)
        with pytest.raises(_lib.SnnflowError):
            lf()
    lf = snnflow.EventWarping(cfg, dev)  # and the well-formed call still runs
    lf.event_flow_association([flow], ev, pol, mask)
    lf().backward()
    assert flow.grad is not None and bool(torch.isfinite(flow.grad).all())


_FAULT_SCRIPT = r"""
import sys, torch
sys.path[:0] = [REPO, PKG]
import snnflow
dev = torch.device("cuda:0")
H, W, B, N, T = 64, 64, 2, 500, 3
cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
       "model": {"mask_output": True}}
gen = torch.Generator().manual_seed(5)
lf = snnflow.EventWarping(cfg, dev)
flows = []
for t in range(T):
    ev = torch.stack([torch.rand(B, N, generator=gen), torch.randint(0, H, (B, N), generator=gen).float(),
                      torch.randint(0, W, (B, N), generator=gen).float(), torch.ones(B, N)], dim=2).to(dev)
    pol = torch.stack([torch.ones(B, N), torch.zeros(B, N)], dim=2).to(dev)
    f = (0.3 * torch.randn(B, 2, H, W, generator=gen)).to(dev).requires_grad_()
    flows.append(f)
    lf.event_flow_association([f], ev, pol, torch.ones(B, 1, H, W, device=dev))
loss = lf()
loss.backward()
try:
    snnflow.check_device_errors()
    print("NO-ERROR")
except snnflow.SnnflowError as e:
    print("SNNFLOW-ERROR", e)
snnflow.check_device_errors()  # cleared: a second check is clean
print("finite", bool(torch.isfinite(loss).item()), all(bool(torch.isfinite(f.grad).all()) for f in flows))
"""


@pytest.mark.parametrize("where", [1, 2], ids=["forward_bins", "backward_bins"])
def test_iwe_loss_corrupted_bin_table_is_flagged(where):
    """A corrupted bin table in the loss scratch (the cause of a round-5 probe's device fault: a timing
    variant of the bin kernel that left its table unwritten) is bounded inside k_iwe_splat /
    k_iwe_bwd_band: the segment is skipped, the library's device error flag is set, and
    snnflow.check_device_errors() raises a clean SnnflowError -- no out-of-bounds access, the process and
    the GPU stay healthy.  The library's fault-injection hook (SNNFLOW_FAULT_INJECT, read at load)
    overwrites one entry of the forward's (1) or the backward's (2) table, in a fresh process."""
    import subprocess
    import sys as _sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"REPO, PKG = {repo!r}, {os.path.join(repo, 'snn_event-based_optical_flow_amd')!r}\n" + _FAULT_SCRIPT
    env = dict(os.environ, SNNFLOW_FAULT_INJECT=str(where))
    r = subprocess.run([_sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "SNNFLOW-ERROR" in r.stdout, r.stdout + r.stderr
    want = "k_iwe_splat" if where == 1 else "k_iwe_bwd_band"
    assert want in r.stdout, r.stdout
    assert "finite True True" in r.stdout, r.stdout
    # without the hook the same script is clean
    env.pop("SNNFLOW_FAULT_INJECT")
    r = subprocess.run([_sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "NO-ERROR" in r.stdout, r.stdout + r.stderr
    print(f"\n[fault {where}] {r.stdout.strip().splitlines()[0]}")


@pytest.mark.parametrize("recurrent", [False, True])
def test_weight_norm_cell_vs_oracle(dev, recurrent):
    """SNNtorch_ConvLIF(Recurrent)(norm="weight") (SNNtorch_spiking_submodules.py:274-276 / :500-504:
    nn.utils.weight_norm on ff (and rec), parameters weight_g / weight_v): 3 chained calls against
    SnnTorchCellRef running on the effective weights g v / ||v||; spikes and states match, and the
    weight_g / weight_v gradients equal the reference's weight gradient taken through the same
    reparametrisation (torch._weight_norm on the CPU, the checker side); an optimizer-style in-place
    update of weight_v between calls is seen by the next call."""
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(47)
    C, B, H, W = 8, 2, 24, 40
    cls = snnflow.SNNtorch_ConvLIFRecurrent if recurrent else snnflow.SNNtorch_ConvLIF
    cell = cls(C, C, 3, thresh=(0.2, 0.4), norm="weight").to(dev).train()
    keys = set(cell.state_dict())
    assert {"ff.weight_g", "ff.weight_v"} <= keys and "ff.weight" not in keys
    if recurrent:
        assert {"rec.weight_g", "rec.weight_v"} <= keys
    with torch.no_grad():
        cell.ff.weight_v.mul_(1.3)  # moves ||v|| away from g: the normalisation is not the identity
        cell.ff.weight_g.mul_(0.9)
    convs = ["ff"] + (["rec"] if recurrent else [])
    gv = {c: (getattr(cell, c).weight_g.detach().cpu().clone().requires_grad_(True),
              getattr(cell, c).weight_v.detach().cpu().clone().requires_grad_(True)) for c in convs}
    ref = lif_ref.SnnTorchCellRef(C, C, 3, recurrent=recurrent).train()
    sd = {k: v.detach().cpu() for k, v in cell.state_dict().items() if "weight_g" not in k and "weight_v" not in k}
    ref.load_state_dict(sd, strict=False)
    eff = {c: torch._weight_norm(gv[c][1], gv[c][0], 0) for c in convs}
    with torch.no_grad():
        for c in convs:
            getattr(ref, c).weight.copy_(eff[c])
    gen = torch.Generator().manual_seed(53)
    xs = [(torch.rand(B, C, H, W, generator=gen) * 2.0) for _ in range(3)]
    st = rst = None
    loss = rloss = 0.0
    wgt = torch.linspace(0.5, 1.5, C).view(1, C, 1, 1)
    for x in xs:
        spk, st = cell(x.to(dev), st)
        rspk, rst = ref(x, rst)
        np.testing.assert_array_equal(spk.detach().cpu().numpy(), rspk.detach().numpy())
        np.testing.assert_allclose(st.detach().cpu().numpy(), rst.detach().numpy(), rtol=1e-5, atol=1e-5)
        loss = loss + (spk * wgt.to(dev)).sum()
        rloss = rloss + (rspk * wgt).sum()
    loss.backward()
    rloss.backward()
    pairs = []
    for c in convs:
        g_w = getattr(ref, c).weight.grad
        g_ref, v_ref = torch.autograd.grad(eff[c], gv[c], g_w)
        pairs.append((f"{c}.weight_v", getattr(cell, c).weight_v.grad.cpu().numpy(), v_ref.numpy()))
        # dL/dg is the projection of dL/dw on v / ||v||, ~0 here: the train-mode BatchNorm after the conv
        # is invariant to an output channel's weight scale, so g only sees rounding -- compared on the
        # scale of dL/dw instead of its own
        d = (getattr(cell, c).weight_g.grad.cpu() - g_ref).norm() / g_w.norm()
        print(f"[weight norm rec={recurrent}] {c}.weight_g |d| / |dL/dw| = {d:.2e}")
        assert d < ORACLE_GRAD_TOL, (c, float(d))
    rp = dict(ref.named_parameters())
    pairs += [(n, a.grad.cpu().numpy(), rp[n].grad.numpy()) for n, a in cell.named_parameters()
              if "weight_g" not in n and "weight_v" not in n]
    _grad_check(f"weight norm rec={recurrent}", pairs, ORACLE_GRAD_TOL)
    # a weight update between calls is picked up (the effective weight is formed per call)
    x0 = xs[0].to(dev)
    with torch.no_grad():
        cell.lif.mem = None
        s_a, _ = cell(x0, None)
        cell.ff.weight_v.mul_(-1.0)
        cell.lif.mem = None
        s_b, _ = cell(x0, None)
    assert not torch.equal(s_a, s_b)


@pytest.mark.parametrize("cin,C", [(2, 8), (4, 16), (1, 4), (5, 32)])
def test_recurrent_cell_narrow_input_vs_oracle(dev, cin, C):
    """SNNtorch_ConvLIFRecurrent with input_size != hidden_size (SNNtorch_spiking_submodules.py:452-453:
    ff is input_size -> hidden_size, rec hidden_size -> hidden_size), the event-input widths 1, 2, 4, 5:
    3 calls chained through prev_state (the recurrent conv on the previous spikes) against
    SnnTorchCellRef -- spikes, states, every parameter gradient and the input gradients."""
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(59)
    B, H, W = 2, 24, 40
    cell = snnflow.SNNtorch_ConvLIFRecurrent(cin, C, 3, thresh=(0.2, 0.4)).to(dev).train()
    ref = lif_ref.SnnTorchCellRef(cin, C, 3, recurrent=True).train()
    ref.load_state_dict({k: v.detach().cpu() for k, v in cell.state_dict().items()}, strict=False)
    gen = torch.Generator().manual_seed(61)
    xs = [(torch.rand(B, cin, H, W, generator=gen) * 3.0).requires_grad_(True) for _ in range(3)]
    xd = [x.detach().to(dev).requires_grad_(True) for x in xs]
    st = rst = None
    loss = rloss = 0.0
    wgt = torch.linspace(0.5, 1.5, C).view(1, C, 1, 1)
    for x, xg in zip(xs, xd):
        spk, st = cell(xg, st)
        rspk, rst = ref(x, rst)
        np.testing.assert_array_equal(spk.detach().cpu().numpy(), rspk.detach().numpy())
        np.testing.assert_allclose(st.detach().cpu().numpy(), rst.detach().numpy(), rtol=1e-5, atol=1e-5)
        loss = loss + (spk * wgt.to(dev)).sum()
        rloss = rloss + (rspk * wgt).sum()
    assert float(torch.stack([s.detach().float().mean() for s in (spk,)]).sum()) > 0.0  # spikes happen
    loss.backward()
    rloss.backward()
    rp = dict(ref.named_parameters())
    pairs = [(n, a.grad.cpu().numpy(), rp[n].grad.numpy()) for n, a in cell.named_parameters()]
    pairs += [(f"x{i}", a.grad.cpu().numpy(), b.grad.numpy()) for i, (a, b) in enumerate(zip(xd, xs))]
    _grad_check(f"rec cell cin={cin} C={C}", pairs, ORACLE_GRAD_TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("C", [8, 32])
def test_fused_head_weight_gradient_matches_deferred(dev, C):
    """ABI 40: the head's weight gradient added inside its wavefront backward tasks (fuse_head) against
    the deferred snnflow_wgrad form, two BPTT windows: every other gradient equal up to the fp64 batch-sum
    atomics' order, the head's conv weight up to the order of the fp32 sums over the steps (per step into
    the slab row vs across the steps in registers)."""
    import copy

    import snnflow
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    torch.manual_seed(11)
    kw = lif_ref.make_unet_kwargs(base_num_channels=C)
    ma = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    mb = copy.deepcopy(ma)
    ma.engine.fuse_head, mb.engine.fuse_head = False, True
    H, W, B, T = 64, 72, 2, 4
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ea, eb = snnflow.EventWarping(cfg, dev), snnflow.EventWarping(cfg, dev)
    gen = torch.Generator(device=dev).manual_seed(3)
    for it in range(2):
        wins = [make_window(B, 400, H, W, gen, dev) for _ in range(T)]
        for m, e in ((ma, ea), (mb, eb)):
            outs = m.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
            for o, w in zip(outs, wins):
                e.event_flow_association(o["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            m.zero_grad(set_to_none=True)
            e().backward()
        for (n, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
            if n == "head.ff.weight":
                r = _rel(b.grad.cpu().numpy(), a.grad.cpu().numpy())
                print(f"[fuse_head C={C} it {it}] head.ff.weight rel {r:.3e}")
                assert r < 1e-6, (it, n, r)
            else:  # the same kernels; only the fp64 batch-sum atomics may add in another order
                assert _rel(b.grad.cpu().numpy(), a.grad.cpu().numpy()) < 1e-6, (it, n)
        ma.detach_states()
        mb.detach_states()
        ea.reset()
        eb.reset()


def _slab_reduce_order(slab):
    """k_slab_reduce's fp64 order per element (16 row groups g; in each, rows g, g+16, ... into four
    interleaved accumulators, (s0 + s1) + (s2 + s3); the groups added in order), cast to fp32."""
    nblk, _ = slab.shape
    x = slab.astype(np.float64)
    tot = np.zeros(slab.shape[1])
    for g in range(16):
        s = [np.zeros(slab.shape[1]) for _ in range(4)]
        b = g
        while b + 48 < nblk:
            for k in range(4):
                s[k] = s[k] + x[b + 16 * k]
            b += 64
        while b < nblk:
            s[0] = s[0] + x[b]
            b += 16
        tot = tot + ((s[0] + s[1]) + (s[2] + s[3]))
    return tot.astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("elems,nblk", [(144, 512), (9216, 512), (72, 37), (1152, 100), (45, 130)])
def test_slab_reduce_fixed_order(dev, elems, nblk):
    """snnflow_slab_reduce equals the documented fixed fp64 order bit for bit (several slabs in one call,
    row counts with and without a remainder group).  A 16-B-load form of the kernel (4 elements per thread)
    passed this too but ran slower (C = 8 7.8 -> 16 us: a quarter of the blocks), so the scalar one stays."""
    from snnflow import _lib

    gen = torch.Generator().manual_seed(elems * 7 + nblk)
    slabs = [torch.randn(nblk, elems, generator=gen) * (10.0 ** k) for k in (-3, 0)]
    d_slabs = [s.to(dev) for s in slabs]
    outs = [torch.empty(elems, device=dev) for _ in slabs]
    descs = (_lib.SlabDesc * 2)(*[_lib.SlabDesc(s.data_ptr(), o.data_ptr(), elems) for s, o in zip(d_slabs, outs)])
    _lib.call("slab_reduce", _lib.lib.snnflow_slab_reduce, descs, 2, nblk, _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    for s, o in zip(slabs, outs):
        np.testing.assert_array_equal(o.cpu().numpy(), _slab_reduce_order(s.numpy()))
