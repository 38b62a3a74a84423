"""GPU parity at the headline configuration and measured precision bounds.

* ``test_cfg2_train_step_vs_oracle``: BASELINE cfg2 (LIFFireNet, 128x128, B=8, T=10 windows of
  1000 events, C=8), cfg3 (256x256, B=4) and the C=32 width at the cfg2 shape -- the north star's claim "AEE within 1e-4 of reference" -- through the
  bench's wavefront path (``forward_sequence``) and the reference loop's per-step path, against
  the CPU oracle (oracle/lif_ref.py + oracle/iwe_ref.py, the reference's PyTorch path restated
  and pinned by the golden fixtures).  Two oracle runs on the same windows and initial weights:
  (1) FREE-RUNNING -- spike flips counted per layer and step, reported with the loss, flow, AEE
  and gradient differences; the flip rate is asserted below 1e-6 per spike (measured: one flip in
  7.3e7 spikes, a near-threshold membrane; the spiking recurrence is chaotic, SURVEY finding 4,
  and an early-layer flip cascades through the step); (2) FLIP-CORRECTED -- the oracle adopts our
  spike (straight-through, its graph kept) wherever it differs AND its membrane lies within 1e-4
  of the threshold; any other differing spike fails the test.  The whole train step must then
  match: loss rtol 1e-5, flows within 1e-4, AEE of a synthetic ground truth within 1e-4 px, every
  parameter gradient within GRAD_TOL.
* ``test_input_gradient_bf16x6_error_vs_fp64``: the input-gradient convolutions of C = 8 run on
  the matrix cores with both operands split into three bf16 parts and the three smallest cross
  products dropped (``mfma_dgrad_bf6``).  Measured against an fp64 oracle next to the error of the
  fp32 CPU oracle itself.
* get_interpolation / interpolate autograd against the oracle's torch restatement.
"""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# relative-L2 bound on every parameter gradient of the train step when the spikes agree: ~2x the
# worst case measured on MI355X (profiles/r03/gpu_tests_*.txt).  cfg2: 2.9e-6
# (G1.bn.weight).  cfg3 sums 2x the pixels per channel and its oracle's own fp32 sums round more:
# 7.7e-6 (head.bn.bias).  C=32: 2.3e-5 (pred.conv2d.bias: two sums over 1.3 M pixel-steps of terms
# of both signs; the conv weights 3-4e-6).
GRAD_TOL = {"cfg2": 6e-6, "cfg3": 1.6e-5, "cfg2-C32": 5e-5, "cfg1": 1e-5}


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _cfg(H, W):
    return {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
            "model": {"mask_output": True}}


def _aee_pair(flow_ours, flow_ref, gt, mask, dev):
    """AEE of our flow through snnflow.AEE (HIP) and of the oracle's flow through the oracle's
    metric restatement (oracle/metrics_ref.py, pinned by eval_case.npz)."""
    import snnflow
    from oracle.metrics_ref import flow_metrics_ref

    B, _, H, W = flow_ours.shape
    m = snnflow.AEE(_cfg(H, W), dev, flow_scaling=128)
    ev = torch.zeros(B, 1, 4, device=dev)
    one = torch.ones(1)
    m.event_flow_association([flow_ours], {"event_list": ev, "event_list_pol_mask": torch.zeros(B, 1, 2, device=dev),
                                           "event_mask": mask.to(dev), "gtflow": gt.to(dev),
                                           "dt_input": one, "dt_gt": one})
    aee, _ = m()
    ref = flow_metrics_ref(flow_ref, gt, mask, one, one, 128)["aee"]
    return aee.cpu().numpy().astype(np.float64), ref.numpy().astype(np.float64)


def _oracle_step(ref, x, ours, eps):
    """One oracle time step, layer by layer (oracle/lif_ref.py LIFFireNetRef.forward).  Every
    oracle spike that differs from ours (``ours``: our [2,B,C,H,W] states of this step) is
    counted; if ``eps`` is set, a differing spike whose pre-reset membrane lies within eps of the
    threshold (fp32-ill-conditioned) is replaced by ours, straight-through (value ours, the
    oracle's graph and surrogate kept), with our reset membrane.  Returns (flow, flips per layer,
    flips NOT within eps of the threshold)."""
    h, flips, hard = x, [], 0
    for i, (name, _) in enumerate(ref.spec):
        cell = getattr(ref, name)
        spk, st = cell(h, ref._states[i])
        diff = spk.detach() != ours[i][1]
        n = int(diff.sum())
        flips.append(n)
        if n:
            near = (cell.lif.last_v - cell.lif.threshold.detach()).abs() <= (eps or 0.0)
            hard += int((diff & ~near).sum())
            if eps:
                spk = spk + (ours[i][1] - spk).detach()
                st = torch.stack([torch.where(diff, ours[i][0], st[0]), spk])
        ref._states[i] = st
        h = spk
    return ref.pred(h), flips, hard


def _new_model(C):
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(0)
    return snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=C))


def _gpu_run(dev, path, wins, C):
    """The train step's forward + loss + backward on the GPU; returns (model, initial state dict,
    flows, loss, per-step CPU copies of the 7 states)."""
    import snnflow

    model = _new_model(C).to(dev).train()
    init = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    B, _, H, W = wins[0]["event_cnt"].shape
    ew = snnflow.EventWarping(_cfg(H, W), dev)
    states = []
    if path == "sequence":
        model.engine.capture_states = True
        outs = model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
        flows = [o["flow"][0] for o in outs]
        states = [[s.detach().cpu() for s in sts] for sts in model.engine.seq_states]
        model.engine.seq_states = None
    else:
        flows = []
        for w in wins:
            flows.append(model(w["event_voxel"], w["event_cnt"])["flow"][0])
            states.append([s.detach().cpu() for s in model._states])
    for t, w in enumerate(wins):
        ew.event_flow_association([flows[t]], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
    loss = ew()
    loss.backward()
    return model, init, flows, loss.item(), states


def _oracle_run(init, C, cpu_wins, ours_states, eps):
    from oracle import iwe_ref, lif_ref

    B, _, H, W = cpu_wins[0]["event_cnt"].shape
    ref = lif_ref.LIFFireNetRef(lif_ref.make_unet_kwargs(base_num_channels=C), "LIFFireNet").train()
    ref.load_state_dict(init)
    rew = iwe_ref.EventWarpingRef([H, W], weight=0.001)
    flows, flips, hard = [], [], 0
    for t, w in enumerate(cpu_wins):
        f, fl, hd = _oracle_step(ref, w["event_cnt"], ours_states[t], eps)
        flows.append(f)
        flips.append(fl)
        hard += hd
        rew.event_flow_association([f], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
    loss = rew()
    loss.backward()
    return ref, flows, loss.item(), np.array(flips), hard


def _compare(tag, model, flows, loss, ref, rflows, rloss, flips, cpu_wins):
    B, _, H, W = cpu_wins[0]["event_cnt"].shape
    r = {"flips": flips, "loss": (loss, rloss),
         "flow_rel": [_rel(f.detach().cpu().numpy(), q.detach().numpy()) for f, q in zip(flows, rflows)],
         "flow_maxabs": max(float((f.detach().cpu() - q.detach()).abs().max()) for f, q in zip(flows, rflows)),
         "grad_rel": {n: _rel(a.grad.cpu().numpy(), b.grad.numpy())
                      for (n, a), (_, b) in zip(model.named_parameters(), ref.named_parameters())}}
    gtg = torch.Generator().manual_seed(2)
    gt = (torch.rand(B, 2, H, W, generator=gtg) - 0.5) * 8.0
    r["aee"] = _aee_pair(flows[-1].detach(), rflows[-1].detach(), gt, cpu_wins[-1]["event_mask"],
                         flows[-1].device)
    _report(tag, r, B * model.engine.C * H * W)
    return r


def _report(tag, r, per_layer):
    print(f"\n[{tag}] spike flips per step x layer (of {per_layer} each):\n{r['flips']}")
    print(f"[{tag}] loss ours {r['loss'][0]:.9g} oracle {r['loss'][1]:.9g} "
          f"rel {abs(r['loss'][0] - r['loss'][1]) / abs(r['loss'][1]):.3e}")
    print(f"[{tag}] flow rel-L2 per step {['%.2e' % v for v in r['flow_rel']]} max|d| {r['flow_maxabs']:.3e}")
    print(f"[{tag}] AEE ours {np.round(r['aee'][0], 6).tolist()} oracle {np.round(r['aee'][1], 6).tolist()} "
          f"max|dAEE| {np.abs(r['aee'][0] - r['aee'][1]).max():.3e}")
    worst = max(r["grad_rel"].items(), key=lambda kv: kv[1])
    print(f"[{tag}] grad rel-L2 worst {worst[0]} {worst[1]:.3e}; all: "
          + ", ".join(f"{k}={v:.1e}" for k, v in r["grad_rel"].items()))


# (tag, batch, resolution, base_num_channels, windows): BASELINE cfg2; cfg3 (256x256, B=4); the README /
# default-checkpoint width C=32 at the cfg2 shape; BASELINE configs[0] (cfg1: 128x128, T=5, batch 1 --
# the degenerate case of the batch statistics: one sequence per BatchNorm batch)
HEADLINE = [("cfg2", 8, 128, 8, 10), ("cfg3", 4, 256, 8, 10), ("cfg2-C32", 8, 128, 32, 10), ("cfg1", 1, 128, 8, 5)]


@pytest.mark.parametrize("path", ["sequence", "per_step"])
@pytest.mark.parametrize("tag,B,H,C,T", HEADLINE, ids=[h[0] for h in HEADLINE])
def test_cfg2_train_step_vs_oracle(dev, path, tag, B, H, C, T):
    from snnflow.synthetic import make_window

    N = 1000
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, N, H, H, gen, dev) for _ in range(T)]
    cpu_wins = [{k: v.cpu() for k, v in w.items()} for w in wins]
    model, init, flows, loss, states = _gpu_run(dev, path, wins, C)

    # 1. free-running oracle: the reference path's own trajectory; flips counted and reported.  At
    #    C = 8 the trajectory stays put (asserted); at C = 32 one near-threshold flip cascades
    #    through the recurrence (SURVEY finding 4: two fp32 CPU runs of the reference itself that
    #    differ only in conv summation order diverge the same way), so there the flip-corrected
    #    leg below is the assertion and the free-running figures are reported only.
    ref, rflows, rloss, flips, _ = _oracle_run(init, C, cpu_wins, states, eps=None)
    free = _compare(f"{tag} {path} free-running", model, flows, loss, ref, rflows, rloss, flips, cpu_wins)
    rate = flips.sum() / (flips.size * B * C * H * H)
    print(f"[{tag} {path}] free-running flips {int(flips.sum())}, rate {rate:.2e} per spike")
    if C == 8:
        assert rate < 1e-6, rate

    # 2. near-threshold flips adopted (|v - theta| <= 1e-4): every other spike must agree, and
    #    then the whole train step matches at the north star's tolerances
    ref, rflows, rloss, flips, hard = _oracle_run(init, C, cpu_wins, states, eps=1e-4)
    r = _compare(f"{tag} {path} flip-corrected", model, flows, loss, ref, rflows, rloss, flips, cpu_wins)
    assert hard == 0, f"{hard} spikes differ away from the threshold"
    assert abs(r["loss"][0] - r["loss"][1]) <= 1e-5 * abs(r["loss"][1]), r["loss"]
    assert max(r["flow_rel"]) <= 1e-4 and r["flow_maxabs"] <= 1e-4, (r["flow_rel"], r["flow_maxabs"])
    assert np.abs(r["aee"][0] - r["aee"][1]).max() <= 1e-4, r["aee"]
    for n, v in r["grad_rel"].items():
        assert v <= GRAD_TOL[tag], (n, v)
    if int(free["flips"].sum()) == 0:  # nothing was adopted: the free-running run IS the comparison
        assert np.abs(free["aee"][0] - free["aee"][1]).max() <= 1e-4


@pytest.mark.parametrize("recurrent", [False, True])
def test_input_gradient_bf16x6_error_vs_fp64(dev, recurrent):
    """Cell input gradient (and, for the recurrent cell, the previous-spike gradient through the
    recurrent conv) at C = 8: the HIP path (bf16x6 matrix-core dgrad) and the fp32 CPU oracle,
    both against the same oracle in fp64 on identical inputs."""
    import snnflow
    from oracle import lif_ref

    torch.manual_seed(3)
    C, B, H, W = 8, 4, 64, 96
    cls = snnflow.SNNtorch_ConvLIFRecurrent if recurrent else snnflow.SNNtorch_ConvLIF
    cell = cls(C, C, 3).to(dev).train()
    ref32 = lif_ref.SnnTorchCellRef(C, C, 3, recurrent=recurrent).train()
    ref32.load_state_dict({k: v.cpu() for k, v in cell.state_dict().items()})
    ref64 = copy.deepcopy(ref32).double()
    gen = torch.Generator().manual_seed(8)
    x = (torch.rand(B, C, H, W, generator=gen) < 0.3).float()
    prev = torch.stack([torch.randn(B, C, H, W, generator=gen) * 0.5, (torch.rand(B, C, H, W, generator=gen) < 0.2).float()])
    wgt = torch.randn(B, C, H, W, generator=gen)
    res = {}
    for tag, m, d, dt in (("hip", cell, dev, torch.float32), ("cpu32", ref32, "cpu", torch.float32),
                          ("fp64", ref64, "cpu", torch.float64)):
        xi = x.to(d, dt).clone().requires_grad_(True)
        pi = prev.to(d, dt).clone().requires_grad_(True)
        spk, _ = m(xi, pi)
        (spk * wgt.to(d, dt)).sum().backward()
        res[tag] = (spk.detach().cpu().double(), xi.grad.cpu().double(), pi.grad[1].cpu().double())
    assert torch.equal(res["hip"][0], res["fp64"][0]) and torch.equal(res["cpu32"][0], res["fp64"][0]), \
        "near-threshold flip in the fixture: change the seed"
    e = {t: (_rel(res[t][1], res["fp64"][1]), _rel(res[t][2], res["fp64"][2])) for t in ("hip", "cpu32")}
    print(f"\nrecurrent={recurrent}: input-grad rel-L2 vs fp64: hip {e['hip'][0]:.2e} cpu32 {e['cpu32'][0]:.2e}; "
          f"prev-spike grad: hip {e['hip'][1]:.2e} cpu32 {e['cpu32'][1]:.2e}")
    # bf16x6 drops terms below 2^-24 relative: the HIP gradients are fp32-accurate
    assert e["hip"][0] <= max(4 * e["cpu32"][0], 1e-6), e
    if recurrent:
        assert e["hip"][1] <= max(4 * e["cpu32"][1], 1e-6), e


def test_iwe_api_gradients_vs_oracle(dev):
    """snnflow.iwe.get_interpolation / interpolate carry the reference's gradients
    (utils/iwe.py:59, 65, 91): flow gradient of a weighted sum of per-polarity IWEs against the
    oracle's torch restatement; indices and weights bit-exact; round_idx has no flow gradient."""
    import snnflow.iwe as siwe
    from oracle import iwe_ref

    gen = torch.Generator().manual_seed(5)
    B, M, H, W, s = 3, 5000, 40, 56, 56
    ev = torch.stack([torch.rand(B, M, generator=gen) * 3, torch.randint(0, H, (B, M), generator=gen).float(),
                      torch.randint(0, W, (B, M), generator=gen).float(), torch.ones(B, M)], 2)
    fl = (torch.rand(B, M, 2, generator=gen) - 0.5) * 0.05
    fl[:, :50] = 0.0  # exact-integer warps (weight kinks)
    pol = (torch.rand(B, 4 * M, 1, generator=gen) < 0.5).float()
    img_w = torch.randn(B, 1, H, W, generator=gen)
    fd = fl.to(dev).requires_grad_(True)
    fc = fl.clone().requires_grad_(True)
    for tref in (3.0, 0.0):
        idx, w = siwe.get_interpolation(ev.to(dev), fd, tref, [H, W], s)
        ridx, rw = iwe_ref.get_interpolation_t(ev, fc, tref, [H, W], s)
        np.testing.assert_array_equal(idx.cpu().numpy(), ridx.detach().numpy())
        np.testing.assert_array_equal(w.detach().cpu().numpy(), rw.detach().numpy())
        img = siwe.interpolate(idx, w * 1.5, [H, W], pol.to(dev))
        rimg = iwe_ref.interpolate_t(ridx, rw * 1.5, [H, W], pol)
        np.testing.assert_allclose(img.detach().cpu().numpy(), rimg.detach().numpy(), rtol=1e-5, atol=1e-5)
        (img * img_w.to(dev)).sum().backward()
        (rimg * img_w).sum().backward()
    assert _rel(fd.grad.cpu().numpy(), fc.grad.numpy()) < 1e-5
    f2 = fl.to(dev).requires_grad_(True)
    _, wr = siwe.get_interpolation(ev.to(dev), f2, 1.0, [H, W], s, round_idx=True)
    assert not wr.requires_grad


def test_clip_grad_norm_large_vs_torch(dev):
    """The grid-wide clip (snnflow_clip_grad_norm_large, taken above 2^20 gradient floats: the U-Net's
    ~20 M parameters) against the fp64 norm of the same gradients and torch.nn.utils.clip_grad_norm_.
    The kernel sums squares in fp64, so it is compared with the fp64 truth at rtol 1e-6; torch's fp32
    CPU norm of these 3.4 M floats is itself 3e-5 low (measured), hence rtol 1e-4 against torch."""
    from snnflow import dp

    gen = torch.Generator().manual_seed(10)
    shapes = [(512, 512, 3, 3), (77,), (1000, 1001), (2, 3)]
    vals = [torch.randn(s, generator=gen) * 0.01 for s in shapes]
    flat = torch.cat([v.reshape(-1) for v in vals]).to(dev)
    truth = float(torch.cat([v.reshape(-1) for v in vals]).double().pow(2).sum().sqrt())
    ps, ref, off = [], [], 0
    for v in vals:
        p = torch.nn.Parameter(torch.zeros_like(v, device=dev))
        p.grad = flat[off:off + v.numel()].view(v.shape)
        off += v.numel()
        ps.append(p)
        q = torch.nn.Parameter(torch.zeros_like(v))
        q.grad = v.clone()
        ref.append(q)
    assert flat.numel() > (1 << 20)
    total = dp.clip_grad_norm_(ps, 1.0)
    rtotal = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    np.testing.assert_allclose(total.item(), truth, rtol=1e-6)
    np.testing.assert_allclose(total.item(), rtotal.item(), rtol=1e-4)
    coef = np.float32(1.0) / (np.float32(total.item()) + np.float32(1e-6))
    for p, v in zip(ps, vals):
        np.testing.assert_allclose(p.grad.cpu().numpy(), v.numpy() * coef, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("tag,B,T", [("cfg2", 8, 10), ("cfg1", 1, 5)], ids=["cfg2", "cfg1"])
def test_cfg2_eval_vs_oracle(dev, tag, B, T):
    """The evaluation path at cfg2's shape (eval_flow.py:208-338: model.eval(), BatchNorm on its
    running statistics, forward only, AEE per window): T = 10 windows of 1000 events at 128 x 128,
    B = 8, through forward_sequence (the wavefront launches the bench's --eval line times) against
    the oracle in eval mode, flip-corrected like the train step (a differing spike must lie within
    1e-4 of the threshold).  Running statistics are perturbed away from (0, 1) so that the eval
    BatchNorm is not the identity.  Flows within 1e-4, AEE of a synthetic ground truth per window
    within 1e-4 (north star).  Also at BASELINE configs[0] (T = 5 windows, batch 1)."""
    from oracle import lif_ref
    from snnflow.synthetic import make_window

    H, N, C = 128, 1000, 8
    gen = torch.Generator(device=dev).manual_seed(7)
    wins = [make_window(B, N, H, H, gen, dev) for _ in range(T)]
    cpu_wins = [{k: v.cpu() for k, v in w.items()} for w in wins]
    model = _new_model(C)
    g = torch.Generator().manual_seed(3)
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.running_mean.copy_(0.2 * torch.randn(m.running_mean.shape, generator=g))
            m.running_var.copy_(0.5 + torch.rand(m.running_var.shape, generator=g))
    init = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model = model.to(dev).eval()
    model.engine.capture_states = True
    with torch.no_grad():
        outs = model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
    flows = [o["flow"][0].detach() for o in outs]
    states = [[s.detach().cpu() for s in sts] for sts in model.engine.seq_states]
    model.engine.seq_states = None

    ref = lif_ref.LIFFireNetRef(lif_ref.make_unet_kwargs(base_num_channels=C), "LIFFireNet").eval()
    ref.load_state_dict(init)
    rflows, flips, hard = [], 0, 0
    with torch.no_grad():
        for t, w in enumerate(cpu_wins):
            f, fl, hd = _oracle_step(ref, w["event_cnt"], states[t], 1e-4)
            rflows.append(f)
            flips += sum(fl)
            hard += hd
    gtg = torch.Generator().manual_seed(2)
    worst_flow, worst_aee = 0.0, 0.0
    for t in range(T):
        worst_flow = max(worst_flow, float((flows[t].cpu() - rflows[t]).abs().max()))
        gt = (torch.rand(B, 2, H, H, generator=gtg) - 0.5) * 8.0
        ours, theirs = _aee_pair(flows[t], rflows[t], gt, cpu_wins[t]["event_mask"], dev)
        worst_aee = max(worst_aee, float(np.abs(ours - theirs).max()))
    print(f"\n[{tag} eval] spike flips {flips} (away from the threshold: {hard}); max|dflow| {worst_flow:.2e}; "
          f"max|dAEE| over {T} windows {worst_aee:.2e}")
    assert hard == 0
    assert worst_flow <= 1e-4 and worst_aee <= 1e-4


@pytest.mark.parametrize("C", [8, 32])
def test_clip_adam_matches_torch(dev, C):
    """snnflow.ClipAdam (one launch: clip_grad_norm_ + Adam, train_flow.py:265-267) against the
    reference's pair -- torch.nn.utils.clip_grad_norm_ + torch.optim.Adam (single-tensor, the
    reference's CPU arithmetic) -- over 4 train steps of LIFFireNet at C = 8 (4,994 parameters: one
    block) and C = 32 (75,266: the two-launch multi-block form) with large gradients
    (so that the clip is active), plus weight decay on a second run.  Both copies see the same
    gradients at every step (the torch copy's gradients are copied from ours before clipping), so
    the comparison isolates the optimizer: clipped gradients and the reported norm within 1e-6 /
    1e-5 relative; moments within 1e-6 of their scale; parameters within 1e-6 relative or 1e-4 of
    the largest Adam step."""
    import copy

    import snnflow
    from snnflow.parser import train_snn_model_kwargs
    from snnflow.synthetic import make_window

    for wd in (0.0, 1e-2):
        torch.manual_seed(0)
        model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=C)).to(dev).train()
        twin = [p.detach().clone() for p in model.parameters()]
        opt = snnflow.ClipAdam(model.parameters(), lr=2e-4, weight_decay=wd, max_norm=1.0)
        tw = [torch.nn.Parameter(t) for t in twin]
        topt = torch.optim.Adam(tw, lr=2e-4, weight_decay=wd, foreach=False)
        cfg = {"loader": {"resolution": [64, 64]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
               "model": {"mask_output": True}}
        lf = snnflow.EventWarping(cfg, dev)
        gen = torch.Generator(device=dev).manual_seed(5)
        is_thr = [n.endswith("threshold") for n, _ in model.named_parameters()]
        for it in range(4):
            wins = [make_window(2, 500, 64, 64, gen, dev) for _ in range(3)]
            with torch.no_grad():  # the forward clamps thresholds at 0.01 in place (weight preparation)
                for t, th in zip(tw, is_thr):
                    if th:
                        t.clamp_(min=0.01)
            lf.reset()
            outs = model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
            for w, o in zip(wins, outs):
                lf.event_flow_association(o["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            (lf() * 1e3).backward()
            for t, p in zip(tw, model.parameters()):
                t.grad = p.grad.detach().clone()
            want_norm = torch.nn.utils.clip_grad_norm_(tw, 1.0)
            opt.step()
            topt.step()
            assert abs(float(opt.last_total_norm) - float(want_norm)) <= 1e-5 * float(want_norm)
            assert float(want_norm) > 1.0  # the clip is active
            for p, t in zip(model.parameters(), tw):
                # the largest Adam step is lr / bc1 = 2e-3 (step 1); near-zero first moments round
                # differently in the two lerps: 1e-4 of that step
                np.testing.assert_allclose(p.detach().cpu().numpy(), t.detach().cpu().numpy(), rtol=1e-6, atol=2e-7)
                np.testing.assert_allclose(p.grad.cpu().numpy(), t.grad.cpu().numpy(), rtol=1e-6, atol=1e-12)
                so, st = opt.state[p], topt.state[t]
                for k in ("exp_avg", "exp_avg_sq"):  # lerp / fma rounding: relative to the tensor's scale
                    want = st[k].cpu().numpy()
                    np.testing.assert_allclose(so[k].cpu().numpy(), want, rtol=1e-6, atol=1e-6 * np.abs(want).max())
                assert float(so["step"]) == float(st["step"]) == it + 1
            opt.zero_grad(set_to_none=True)
            model.detach_states()
        # state dict round trip: a fresh optimizer continues from the saved moments
        sd = copy.deepcopy(opt.state_dict())
        opt2 = snnflow.ClipAdam(model.parameters(), lr=2e-4, weight_decay=wd, max_norm=1.0)
        opt2.load_state_dict(sd)
        m = opt2._state([p for p in model.parameters()])
        assert float(m[3]) == 4.0
        np.testing.assert_array_equal(m[1].cpu().numpy(), opt._moments[1].cpu().numpy())


def _window_run(dev, wins, C, keep, bits=True):
    """forward_sequence + EventWarping + backward of one window at full size, with the engine either
    keeping every step's states (capture_states: nothing skipped, as test_cfg2_train_step_vs_oracle
    runs it) or not (the bench: the unread spike planes and state-gradient halves are skipped); `bits`:
    the spike bit planes between the kernels (ABI 39) or the fp32 spike half of the states."""
    import snnflow

    model = _new_model(C).to(dev).train()
    B, _, H, W = wins[0]["event_cnt"].shape
    model.engine.capture_states = keep
    model.engine.spk_bits = bits
    outs = model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
    if keep:
        model.engine.seq_states = None
    ew = snnflow.EventWarping(_cfg(H, W), dev)
    for o, w in zip(outs, wins):
        ew.event_flow_association(o["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
    loss = ew()
    loss.backward()
    return ([o["flow"][0].detach().cpu() for o in outs], loss.item(),
            [p.grad.detach().cpu().clone() for p in model.parameters()], [s.detach().cpu() for s in model._states])


@pytest.mark.parametrize("tag,B,H", [("cfg2", 8, 128), ("cfg3", 4, 256)], ids=["cfg2", "cfg3"])
def test_bench_window_skips_bit_identical(dev, tag, B, H):
    """The bench's exact window at full size: test_cfg2_train_step_vs_oracle runs forward_sequence with
    capture_states on, which keeps every write; the bench runs it off, which skips the spike half of the
    feed-forward layers' intermediate states (state_spk_skip) and the membrane half of the internal
    state gradients.  Same windows as the oracle test (seed 1, T = 10 x 1000 events, C = 8): flows, loss,
    every parameter gradient and the final states must be the same bits.  (Run-to-run, the fp64
    batch-sum atomics could reorder; the sums round to fp32 identically in practice -- a mismatch here
    names the tensor.)"""
    from snnflow.synthetic import make_window

    T, N, C = 10, 1000, 8
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, N, H, H, gen, dev) for _ in range(T)]
    keep = _window_run(dev, wins, C, True)
    skip = _window_run(dev, wins, C, False)
    for t, (a, b) in enumerate(zip(keep[0], skip[0])):
        assert torch.equal(a, b), f"flow of step {t}"
    assert keep[1] == skip[1], (keep[1], skip[1])
    names = [n for n, _ in _new_model(C).named_parameters()]
    for n, a, b in zip(names, keep[2], skip[2]):
        assert torch.equal(a, b), f"gradient of {n}: max |d| {float((a - b).abs().max()):.3e}"
    for l, (a, b) in enumerate(zip(keep[3], skip[3])):
        assert torch.equal(a, b), f"final state of layer {l}"
    print(f"\n[{tag}] capture on / off: loss {keep[1]:.9g}, {len(names)} gradients, {len(keep[3])} final states identical")


@pytest.mark.parametrize("C,B", [(16, 4), (32, 8)], ids=["C16", "C32"])
def test_spike_bit_planes_bit_identical(dev, C, B):
    """The spike bit planes (ABI 39, C = 16 / 32: the forward writes each layer's spikes as one C-bit word
    per pixel; the recurrent convs and the deferred weight gradients read them, and the fp32 spike half
    of the intermediate states is no longer stored)
    against the fp32 spike planes (engine.spk_bits off, every state written): one full window at 128x128,
    T = 10 x 1000 events -- flows, loss, every parameter gradient and the final states the same bits."""
    from snnflow.synthetic import make_window

    T, N, H = 10, 1000, 128
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, N, H, H, gen, dev) for _ in range(T)]
    ref = _window_run(dev, wins, C, True, bits=False)
    got = _window_run(dev, wins, C, False, bits=True)
    for t, (a, b) in enumerate(zip(ref[0], got[0])):
        assert torch.equal(a, b), f"flow of step {t}"
    assert ref[1] == got[1], (ref[1], got[1])
    names = [n for n, _ in _new_model(C).named_parameters()]
    worst = 0.0
    for n, a, b in zip(names, ref[2], got[2]):
        d = float((a - b).abs().max() / a.abs().max().clamp_min(1e-30))
        worst = max(worst, d)
        # the fp64 batch-sum atomics may reorder between two runs and round a BatchNorm-backward
        # coefficient to a neighbouring fp32 value (C = 16: 1.5e-7 measured); a wrong spike bit would
        # move a gradient by orders of magnitude more
        assert d <= 1e-5, f"gradient of {n}: max rel |d| {d:.3e}"
    for l, (a, b) in enumerate(zip(ref[3], got[3])):
        assert torch.equal(a, b), f"final state of layer {l}"
    print(f"\n[C={C} B={B}] bit planes vs fp32 spikes: loss {ref[1]:.9g}, worst gradient rel diff {worst:.3e}")


def test_bench_graph_pingpong_matches_eager(dev):
    """The bench's timed step itself (bench.py main, N = 1): one HIP graph per resident batch and state
    parity holding forward_sequence + EventWarping + backward + ClipAdam, the states handed over
    copy-free through bench.StatePingPong -- replayed twice at cfg2 (128x128, B = 8, T = 10 x 1000
    events, C = 8) against the same two steps run eagerly (forward_sequence, loss, backward,
    ClipAdam.step, detach_states) from the same initial parameters, moments and (zero) states.  Loss,
    every parameter, the Adam moments and the handed-over states must be the same bits after each step."""
    import bench
    import snnflow
    from snnflow.parser import train_snn_model_kwargs
    from snnflow.synthetic import make_window

    B, R, T, N = 8, 128, 10, 1000
    gen = torch.Generator(device=dev).manual_seed(11)
    pool = [bench._pack([make_window(B, N, R, R, gen, dev) for _ in range(T)]) for _ in range(2)]
    seed = torch.ones((), device=dev)

    def build():
        torch.manual_seed(0)
        m = snnflow.LIFFireNet(train_snn_model_kwargs("LIFFireNet", base_num_channels=8)).to(dev).train()
        return m, snnflow.EventWarping(_cfg(R, R), dev), snnflow.ClipAdam(list(m.parameters()), lr=2e-4, max_norm=1.0)

    def fwd_bwd(m, lf, views):
        lf.reset()
        outs = m.forward_sequence([w["event_voxel"] for w in views], [w["event_cnt"] for w in views])
        for t in range(T):
            w = views[t]
            lf.event_flow_association(outs[t]["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = lf()
        loss.backward(seed)
        return loss

    def snap(m, opt):
        _, ea, es, _, _ = opt._moments
        return [p.detach().cpu().clone() for p in m.parameters()], ea.cpu().clone(), es.cpu().clone()

    # eager reference: two steps from the fresh model (zero initial states)
    me, lfe, oe = build()
    want = []
    for j in range(2):
        oe.zero_grad(set_to_none=True)
        loss = fwd_bwd(me, lfe, pool[j][1])
        oe.step()
        want.append((loss.item(), snap(me, oe), [s.detach().cpu() for s in me._states]))
        me.detach_states()

    # the bench's graphs: warm up eagerly (workspaces, optimizer state), capture, then restore the
    # initial parameters / buffers / moments in place and zero both ping-pong buffers
    mg, lfg, og = build()
    init = {k: v.detach().clone() for k, v in mg.state_dict().items()}
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for j in range(3):
            og.zero_grad(set_to_none=True)
            fwd_bwd(mg, lfg, pool[j % 2][1])
            og.step()
            mg.detach_states()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    pingpong = bench.StatePingPong(dev, mg._states)
    graphs, losses = [], []
    for j in range(pingpong.cycle(len(pool))):
        og.zero_grad(set_to_none=True)
        pingpong.arm(mg, j)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            losses.append(fwd_bwd(mg, lfg, pool[j % len(pool)][1]))
            og.step()
        graphs.append(g)
    with torch.no_grad():
        for k, v in mg.state_dict().items():
            v.copy_(init[k])
        for t in og._moments[1:4]:
            t.zero_()
        for b in pingpong.bufs:
            b.zero_()
    torch.cuda.synchronize(dev)
    for j in range(2):
        graphs[j].replay()
        torch.cuda.synchronize(dev)
        wl, (wp, wea, wes), wst = want[j]
        assert losses[j].item() == wl, (j, losses[j].item(), wl)
        gp, gea, ges = snap(mg, og)
        for (n, _), a, b in zip(mg.named_parameters(), gp, wp):
            assert torch.equal(a, b), f"step {j}: parameter {n}"
        assert torch.equal(gea, wea) and torch.equal(ges, wes), f"step {j}: Adam moments"
        for l, (v, w) in enumerate(zip(pingpong.views[(j + 1) % 2], wst)):
            assert torch.equal(v.detach().cpu(), w), f"step {j}: handed-over state of layer {l}"
    print(f"\n[cfg2 graph ping-pong] 2 replays == 2 eager steps: losses {[w[0] for w in want]}")
