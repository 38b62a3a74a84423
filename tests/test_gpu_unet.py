"""GPU parity of the spiking U-Net (SpikingRecEVFlowNet, BASELINE cfg5's model) on the
implicit-GEMM matrix-core kernels (csrc/unet.hip) against the reference-generated fixture
(tests/golden/unet_case.npz, produced by the reference model itself) and the CPU oracle
(oracle/unet_ref.py, pinned by that fixture in tests/test_oracle_golden.py).

Tolerances: flows and membranes rtol 1e-4 (fp32, summation order: oneDNN conv vs the GEMM's
k-ordered fp32 accumulation of exact bf16-split products); spikes identical except where the
membrane lies within 1e-4 of the threshold; loss rtol 1e-5; parameter gradients relative-L2
GRAD_TOL (measured worst case printed by each test).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-4


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _kw(base, activations=("arctanspike", "arctanspike"), hard=True):
    return {"name": "SpikingRecEVFlowNet", "encoding": "cnt", "round_encoding": False, "norm_input": False,
            "num_bins": 2, "base_num_channels": base, "kernel_size": 3, "activations": list(activations),
            "mask_output": True,
            "spiking_neuron": {"leak": [0.0, 1.0], "thresh": [0.0, 0.8], "learn_leak": True, "learn_thresh": True,
                               "hard_reset": hard}}


def _cfg(H, W):
    return {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
            "model": {"mask_output": True}}


def _spk(st):
    s = st.detach().cpu()
    return s[:, 1] if s.dim() == 6 else s[1]


def test_unet_vs_golden(golden, dev):
    """3 steps of the base-4 U-Net at 32x32 (B=2): every flow map and state, the EventWarping loss
    over the 4 flows and every parameter gradient against the reference's own outputs."""
    import snnflow

    g = golden("unet_case.npz")
    T, (H, W), base = int(g["T"]), list(g["res"]), int(g["base"])
    torch.manual_seed(17)
    model = snnflow.SpikingRecEVFlowNet(_kw(base)).to(dev)
    model.load_state_dict({k[3:]: torch.from_numpy(v).to(dev) for k, v in g.items() if k.startswith("p0.")})
    ew = snnflow.EventWarping(_cfg(H, W), dev)
    worst_flow = 0.0
    for t in range(T):
        out = model(None, torch.from_numpy(g[f"cnt_{t}"]).to(dev))
        assert len(out["flow"]) == 4
        for i, f in enumerate(out["flow"]):
            ref = g[f"flow_{t}_{i}"]
            worst_flow = max(worst_flow, float(np.abs(f.detach().cpu().numpy() - ref).max()))
            np.testing.assert_allclose(f.detach().cpu().numpy(), ref, rtol=1e-4, atol=1e-6, err_msg=f"flow {t} {i}")
        for i, st in enumerate(model.states):
            ref = g[f"state_{t}_{i}"]
            ours = st.detach().cpu().numpy()
            np.testing.assert_array_equal(_spk(st).numpy(), ref[:, 1] if ref.ndim == 6 else ref[1], err_msg=f"spk {t} {i}")
            np.testing.assert_allclose(ours, ref, rtol=1e-4, atol=1e-5, err_msg=f"state {t} {i}")
        ew.event_flow_association(out["flow"], torch.from_numpy(g[f"events_{t}"]).to(dev),
                                  torch.from_numpy(g[f"pol_{t}"]).to(dev), torch.from_numpy(g[f"mask_{t}"]).to(dev))
    loss = ew()
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-5)
    errs = {n: _rel(p.grad.cpu().numpy(), g[f"g.{n}"]) for n, p in model.named_parameters()}
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"\n[unet golden] max |dflow| {worst_flow:.2e}; grad rel-L2 worst {worst[0]} {worst[1]:.2e}")
    for n, e in errs.items():
        assert e < GRAD_TOL, (n, e)


@pytest.mark.parametrize("base,H,acts,hard", [(8, 64, ("arctanspike", "arctanspike"), True),
                                              (16, 64, ("superspike", "trianglespike"), False),
                                              (32, 32, ("mgspike", "arctanspike"), True)])
def test_unet_vs_oracle(dev, base, H, acts, hard):
    """Random weights and event windows (B=2, T=3, 1000 events) through the HIP U-Net and the
    oracle: per-step flows and spikes (flips counted, only near-threshold ones tolerated), loss and
    every parameter gradient (compared when no spike differs)."""
    import snnflow
    from oracle import iwe_ref
    from oracle.unet_ref import SpikingRecEVFlowNetRef
    from snnflow.synthetic import make_window

    torch.manual_seed(5)
    model = snnflow.SpikingRecEVFlowNet(_kw(base, acts, hard)).to(dev)
    torch.manual_seed(5)
    ref = SpikingRecEVFlowNetRef(_kw(base, acts, hard))
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    W = H
    ew, rew = snnflow.EventWarping(_cfg(H, W), dev), None
    gen = torch.Generator(device=dev).manual_seed(3)
    flows, wins, ours = [], [], []
    for t in range(3):
        w = make_window(2, 1000, H, W, gen, dev)
        wins.append(w)
        flows.append(model(None, w["event_cnt"])["flow"])
        ours.append([s.detach().cpu() for s in model.states])
    # flip-corrected oracle (as test_unet_cfg5_shapes_vs_oracle): where its spike differs from ours and
    # its membrane lies within 1e-4 of the threshold it adopts ours straight-through; a spike that
    # differs away from the threshold fails
    counters = {"flips": 0, "hard": 0}
    step = _patch_flips(ref, ours, 1e-4, counters)
    rflows = []
    for t, w in enumerate(wins):
        step(t)
        rflows.append(ref(None, w["event_cnt"].cpu())["flow"])
        for k, (a, b) in enumerate(zip(ours[t], ref.states)):
            np.testing.assert_allclose(a.numpy(), b.detach().numpy(), rtol=1e-4, atol=1e-4, err_msg=f"state {t} {k}")
    print(f"\n[unet base={base} {H}x{W} {acts} hard={hard}] spike flips {counters['flips']} "
          f"(away from the threshold: {counters['hard']})")
    assert counters["hard"] == 0
    for t in range(3):
        for i in range(4):
            np.testing.assert_allclose(flows[t][i].detach().cpu().numpy(), rflows[t][i].detach().numpy(), rtol=1e-4,
                                       atol=1e-6, err_msg=f"flow {t} {i}")
    for i in range(4):
        lf = iwe_ref.EventWarpingRef([H, W], weight=0.001)
        for t in range(3):
            lf.event_flow_association([rflows[t][i]], wins[t]["event_list"].cpu(), wins[t]["event_list_pol_mask"].cpu(),
                                      wins[t]["event_mask"].cpu())
        rew = lf() if rew is None else rew + lf()
    rloss = rew / 4
    for t in range(3):
        ew.event_flow_association(flows[t], wins[t]["event_list"], wins[t]["event_list_pol_mask"], wins[t]["event_mask"])
    loss = ew()
    np.testing.assert_allclose(loss.item(), rloss.item(), rtol=1e-5)
    loss.backward()
    rloss.backward()
    errs = {n: _rel(a.grad.cpu().numpy(), b.grad.numpy()) for (n, a), (_, b) in
            zip(model.named_parameters(), ref.named_parameters())}
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"[unet base={base}] grad rel-L2 worst {worst[0]} {worst[1]:.2e}")
    for n, e in errs.items():
        assert e < GRAD_TOL, (n, e)


@pytest.mark.parametrize("recurrent,stride,cin,C,act,hard,detach",
                         [(False, 2, 2, 16, "arctanspike", True, True), (True, 1, 24, 24, "superspike", False, True),
                          (False, 1, 40, 64, "mgspike", True, False), (True, 1, 64, 64, "trianglespike", True, False)])
def test_convlif_general_cell_vs_oracle(dev, recurrent, stride, cin, C, act, hard, detach):
    """ConvLIF / ConvLIFRecurrent configurations outside the fixed one-kernel path (stride 2, other
    widths, the four surrogates, soft reset, detach=False) through the implicit-GEMM cell path:
    outputs, states and the gradients of input, previous state and parameters over 2 steps."""
    import snnflow
    from oracle.unet_ref import _Cell

    torch.manual_seed(9)
    if recurrent:
        cell = snnflow.ConvLIFRecurrent(cin, C, 3, activation=act, leak=(0.0, 1.0), thresh=(0.5, 0.2),
                                        hard_reset=hard, detach=detach).to(dev)
    else:
        cell = snnflow.ConvLIF(cin, C, 3, stride=stride, activation=act, leak=(0.0, 1.0), thresh=(0.5, 0.2),
                               hard_reset=hard, detach=detach).to(dev)
    ref = _Cell(cin, C, 3, stride=stride, recurrent=recurrent, activation=act, leak=(0.0, 1.0), thresh=(0.5, 0.2),
                hard_reset=hard, detach=detach)
    ref.load_state_dict({k: v.detach().cpu() for k, v in cell.state_dict().items()})
    gen = torch.Generator().manual_seed(4)
    B, H, W = 2, 16, 24
    Ho, Wo = H // stride, W // stride
    s0 = torch.randn(2, B, C, Ho, Wo, generator=gen) * 0.5
    s0[1] = (s0[1] > 0).float()
    sd, sc = s0.to(dev).requires_grad_(True), s0.clone().requires_grad_(True)
    x0 = [(torch.rand(B, cin, H, W, generator=gen) < 0.5).float() * 1.5 for _ in range(2)]
    xd = [x.to(dev).requires_grad_(True) for x in x0]
    xc = [x.clone().requires_grad_(True) for x in x0]
    std, stc, lossd, lossc = sd, sc, 0, 0
    for t in range(2):
        zd, std = cell(xd[t], std)
        zc, stc = ref(xc[t], stc)
        assert torch.equal(zd.detach().cpu(), zc.detach()), "spike flip (near threshold): change the seed"
        np.testing.assert_allclose(std.detach().cpu().numpy(), stc.detach().numpy(), rtol=1e-5, atol=1e-5)
        wz = torch.randn(B, C, Ho, Wo, generator=gen)
        lossd = lossd + (zd * wz.to(dev)).sum() + 0.3 * std[0].sum()
        lossc = lossc + (zc * wz).sum() + 0.3 * stc[0].sum()
    lossd.backward()
    lossc.backward()
    errs = {"x0": _rel(xd[0].grad.cpu().numpy(), xc[0].grad.numpy()), "x1": _rel(xd[1].grad.cpu().numpy(), xc[1].grad.numpy()),
            "state0": _rel(sd.grad.cpu().numpy(), sc.grad.numpy())}
    errs.update({n: _rel(p.grad.cpu().numpy(), q.grad.numpy())
                 for (n, p), (_, q) in zip(cell.named_parameters(), ref.named_parameters())})
    print(f"\n[cell rec={recurrent} s={stride} {cin}->{C} {act}] " + ", ".join(f"{k}={v:.1e}" for k, v in errs.items()))
    for n, e in errs.items():
        assert e < 1e-4, (n, e)


def _ref_cells(ref):
    """The oracle U-Net's cells in the order of the model's 10 states, as (cell, state index,
    sub-index or None) (encoders: ff + recurrent cell, resblocks: conv1 + conv2, decoders)."""
    u = ref.multires_unetrec
    out = []
    for i, e in enumerate(u.encoders):
        out += [(e.conv, i, 0), (e.recurrent_block, i, 1)]
    for j, r in enumerate(u.resblocks):
        out += [(r.conv1, 4 + j, 0), (r.conv2, 4 + j, 1)]
    for i, d in enumerate(u.decoders):
        out.append((d.conv2d, 6 + i, None))
    return out


def _patch_flips(ref, ours_states, eps, counters):
    """Flip correction of the oracle U-Net (see test_unet_cfg5_shapes_vs_oracle): every cell adopts
    our spike straight-through where its own differs; the ones whose membrane is not within eps of
    the threshold are counted as hard.  Returns the per-step target setter."""
    cells = _ref_cells(ref)
    targets = []
    for cell, i, j in cells:
        tgt = {}
        orig = type(cell).forward

        def fwd(x, prev, residual=0, cell=cell, tgt=tgt, orig=orig):
            out, st = orig(cell, x, prev, residual)
            v, s = st[0], st[1]
            o = tgt["state"].to(s.dtype)
            diff = s.detach() != o
            n = int(diff.sum())
            if n:
                th = cell.thresh.detach().clamp_min(0.01)
                near = (v.detach() - th).abs() <= eps
                counters["flips"] += n
                counters["hard"] += int((diff & ~near).sum())
                s = s + ((o - s.detach()) * diff).detach()
                st = torch.stack([v, s])
                out = s + residual
            return out, st
        cell.forward = fwd
        targets.append((tgt, i, j))

    def set_step(t):
        for tgt, i, j in targets:
            st = ours_states[t][i]
            tgt["state"] = (st[j] if j is not None else st)[1]
    return set_step


def _bslice(st, sl):
    """Batch slice of a U-Net state ([2, B, ...], or [2, 2, B, ...] for the encoders' pairs)."""
    return st[:, sl] if st.dim() == 5 else st[:, :, sl]


def _unet_plans(model, B, H, T, dev, seed):
    """Forward + loss + backward of the U-Net at batch B, returning the split plans of every GEMM
    launch (snnflow.unet.PLAN_LOG) and the run's flows / states / windows."""
    import snnflow
    import snnflow.unet as un
    from snnflow.synthetic import make_window

    gen = torch.Generator(device=dev).manual_seed(seed)
    wins = [make_window(B, 1000, H, H, gen, dev) for _ in range(T)]
    model.reset_states()
    un.PLAN_LOG = []
    try:
        flows, ours = [], []
        for w in wins:
            flows.append(model(None, w["event_cnt"])["flow"])
            ours.append([st.detach().cpu() for st in model.states])
        plans = list(un.PLAN_LOG)
    finally:
        un.PLAN_LOG = None
    return plans, flows, ours, wins


def test_unet_cfg5_shapes_vs_oracle(dev):
    """BASELINE cfg5 itself: SpikingRecEVFlowNet at 256x256, base 32 (20.4 M parameters, 64..512
    channels) at the bench's batch B=16, T=2 windows of 1000 events -- so every conv, input-gradient
    and weight-gradient launch runs the split-K factors and pixel-split plans the cfg5 bench runs (the
    plans depend on B * H * W: csrc/unet.hip snnflow_unet_conv_ksplit, wgrad_plan; the test prints the
    plans that differ from B=2's and requires some to).  The U-Net has no BatchNorm, so samples are
    independent: the oracle (oracle/unet_ref.py) runs samples 0 and 1 only, and the loss is the
    EventWarping loss of those two samples' flows, back-propagated through the B=16 graph (the
    other 14 samples' flow gradients are zero, their pixels still flow through every split plan).
    Flip-corrected like test_gpu_fullsize.py: where an oracle spike differs from ours and the oracle
    membrane lies within 1e-4 of the threshold, the oracle adopts our spike straight-through (its
    graph kept); any other differing spike fails.  Flows, states and the loss must then match (rtol
    1e-4 / 1e-5).  Parameter gradients: at this size the fp32 oracle's own summation error reaches
    1e-4 on the deep, low-resolution layers, so both are measured against an fp64 run of the oracle
    (same flip correction); all three network backwards are seeded with our dL/dflow, and ours must
    be within max(2 x the fp32 oracle's error, 2e-5) of fp64."""
    import copy

    import snnflow
    from oracle import iwe_ref
    from oracle.unet_ref import SpikingRecEVFlowNetRef

    base, H, B, T, eps = 32, 256, 16, 2, 1e-4
    S = slice(0, 2)
    torch.manual_seed(5)
    model = snnflow.SpikingRecEVFlowNet(_kw(base)).to(dev)
    ref = SpikingRecEVFlowNetRef(_kw(base))
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    ref64 = copy.deepcopy(ref).double()

    # the split plans at B=2 (forward, input and weight gradients of one step) against the bench's B=16
    p2, f2, _, w2 = _unet_plans(model, 2, H, 1, dev, 9)
    ew2 = snnflow.EventWarping(_cfg(H, H), dev)
    ew2.event_flow_association(f2[0], w2[0]["event_list"], w2[0]["event_list_pol_mask"], w2[0]["event_mask"])
    import snnflow.unet as un
    un.PLAN_LOG = []
    ew2().backward()
    p2 += un.PLAN_LOG
    un.PLAN_LOG = None
    model.zero_grad(set_to_none=True)

    plans, flows, ours, wins = _unet_plans(model, B, H, T, dev, 3)
    ours2 = [[_bslice(st, S) for st in sts] for sts in ours]
    counters = {"flips": 0, "hard": 0}
    step32 = _patch_flips(ref, ours2, eps, counters)
    c64 = {"flips": 0, "hard": 0}
    step64 = _patch_flips(ref64, ours2, eps, c64)
    rflows, rflows64 = [], []
    for t, w in enumerate(wins):
        x = w["event_cnt"][S].cpu()
        step32(t)
        rflows.append(ref(None, x)["flow"])
        step64(t)
        rflows64.append(ref64(None, x.double())["flow"])
        for k, (a, b) in enumerate(zip(ours2[t], ref.states)):
            np.testing.assert_allclose(a.numpy(), b.detach().numpy(), rtol=1e-4, atol=1e-4, err_msg=f"state {t} {k}")
    print(f"\n[unet cfg5 B={B}] spike flips {counters['flips']} (away from the threshold: {counters['hard']}); "
          f"fp64 oracle: {c64['flips']} ({c64['hard']})")
    assert counters["hard"] == 0 and c64["hard"] == 0
    worst = 0.0
    for t in range(T):
        for i in range(4):
            a, b = flows[t][i][S].detach().cpu().numpy(), rflows[t][i].detach().numpy()
            worst = max(worst, float(np.abs(a - b).max()))
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5, err_msg=f"flow {t} {i}")
    ew = snnflow.EventWarping(_cfg(H, H), dev)
    for t in range(T):
        ew.event_flow_association([f[S] for f in flows[t]], wins[t]["event_list"][S], wins[t]["event_list_pol_mask"][S],
                                  wins[t]["event_mask"][S])
    loss = ew()
    rloss = 0
    for i in range(4):
        lf = iwe_ref.EventWarpingRef([H, H], weight=0.001)
        for t in range(T):
            lf.event_flow_association([rflows[t][i]], wins[t]["event_list"][S].cpu(),
                                      wins[t]["event_list_pol_mask"][S].cpu(), wins[t]["event_mask"][S].cpu())
        rloss = rloss + lf()
    rloss = rloss / 4
    np.testing.assert_allclose(loss.item(), rloss.item(), rtol=1e-5)
    allo = [f for fs in flows for f in fs]
    for f in allo:
        f.retain_grad()
    un.PLAN_LOG = []
    loss.backward()
    plans += un.PLAN_LOG
    un.PLAN_LOG = None

    # the plans: every launch shape of B=16 against the same layer's plan at B=2 (P scales by 8)
    by2 = {}
    for kind, M, K, P, plan in p2:
        by2.setdefault((kind, M, K, P * 8), plan)
    changed = sorted({(kind, M, K, P, by2[(kind, M, K, P)], plan) for kind, M, K, P, plan in plans
                      if (kind, M, K, P) in by2 and by2[(kind, M, K, P)] != plan})
    print(f"[unet cfg5 B={B}] {len(plans)} GEMM launches, {len(changed)} launch shapes with another split plan than "
          "at B=2 (kind, M, K, P, plan@B2 -> plan@B16): " + "; ".join(f"{c[0]} M{c[1]} K{c[2]} P{c[3]} {c[4]}->{c[5]}"
                                                                        for c in changed))
    assert changed, "B=16 runs the same split plans as B=2: this test would not cover the bench's plans"

    seeds_full = [f.grad.detach() for f in allo]
    seeds = [g[S].cpu() for g in seeds_full]
    for g in seeds_full:  # the other samples' flows do not reach the loss
        assert float(g[2:].abs().max()) == 0.0
    allr = [f for fs in rflows for f in fs]
    rseeds = torch.autograd.grad(rloss, allr, retain_graph=True)
    # the network backward of all three is seeded with OUR dL/dflow: the contrast loss is
    # ill-conditioned in the flows (a corner weight 1 - |dx| ~ 1e-4 enters the count image as the
    # denominator of ts/count), so flows equal to 6e-8 can give dL/dflow that differ by 1e-4; the
    # loss gradient itself is checked at 256^2 by test_event_warping_bands_and_empty_windows_vs_oracle
    gl = _rel(torch.cat([g.reshape(-1) for g in seeds]).numpy(), torch.cat([g.reshape(-1) for g in rseeds]).numpy())
    print(f"[unet cfg5 B={B}] dL/dflow rel-L2 ours vs fp32 oracle {gl:.2e}")
    torch.autograd.backward(allr, seeds)
    sur = sum((f * g.double()).sum() for f, g in zip([f for fs in rflows64 for f in fs], seeds))
    sur.backward()
    e_ours, e_32 = {}, {}
    for (n, a), (_, b), (_, c) in zip(model.named_parameters(), ref.named_parameters(), ref64.named_parameters()):
        g64 = c.grad.numpy()
        e_ours[n] = _rel(a.grad.cpu().numpy(), g64)
        e_32[n] = _rel(b.grad.numpy(), g64)
    w = max(e_ours.items(), key=lambda kv: kv[1])
    print(f"[unet cfg5 B={B}] max |dflow| {worst:.2e}; loss {loss.item():.9g} vs {rloss.item():.9g}; "
          f"grad rel-L2 vs fp64: ours worst {w[0]} {w[1]:.2e} (fp32 oracle there {e_32[w[0]]:.2e}; "
          f"fp32 oracle worst {max(e_32.values()):.2e}) over {len(e_ours)} tensors")
    print(f"[unet cfg5 B={B}] ours/oracle32 vs fp64: " + ", ".join(
        f"{n}={e_ours[n]:.1e}/{e_32[n]:.1e}" for n in sorted(e_ours, key=lambda k: -e_ours[k])[:20]))
    for n in e_ours:
        assert e_ours[n] <= max(2 * e_32[n], 2e-5), (n, e_ours[n], e_32[n])


def _cell_variants():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "cell_variants.json")) as f:
        return [tuple(v) for v in json.load(f)["variants"]]


CELL_VARIANTS = _cell_variants()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", CELL_VARIANTS, ids=[v[0] for v in CELL_VARIANTS])
def test_convlif_variants_vs_golden(golden, dev, variant):
    """HIP ConvLIF / ConvLIFRecurrent against the REFERENCE-generated fixture of the cell options
    outside the default one (make_golden.py:spiking_cell_variants_case: SuperSpike, MultiGauss,
    Triangle surrogates with their widths, soft reset, detach=False, stride 2): spikes exact, states
    rtol 1e-5, gradients of inputs, initial state and parameters rel-L2 < 1e-4."""
    import snnflow
    tag, recurrent, stride, cin, C, act, width, hard, detach = variant
    g = golden("spiking_cell_variants_case.npz")
    kw = dict(activation=act, act_width=width, hard_reset=hard, detach=detach)
    cell = (snnflow.ConvLIFRecurrent(cin, C, 3, **kw) if recurrent
            else snnflow.ConvLIF(cin, C, 3, stride=stride, **kw)).to(dev)
    cell.load_state_dict({k[len(tag) + 3:]: torch.from_numpy(v).to(dev) for k, v in g.items()
                          if k.startswith(f"{tag}.p.")})
    s0 = torch.from_numpy(g[f"{tag}.s0"]).to(dev).requires_grad_(True)
    xs = [torch.from_numpy(g[f"{tag}.x_{t}"]).to(dev).requires_grad_(True) for t in range(2)]
    state, loss = s0, 0
    for t in range(2):
        z, state = cell(xs[t], state)
        np.testing.assert_array_equal(z.detach().cpu().numpy(), g[f"{tag}.z_{t}"])
        np.testing.assert_allclose(state.detach().cpu().numpy(), g[f"{tag}.state_{t}"], rtol=1e-5, atol=1e-5)
        loss = loss + (z * torch.from_numpy(g[f"{tag}.wz_{t}"]).to(dev)).sum() + 0.3 * state[0].sum()
    loss.backward()
    errs = {"state0": _rel(s0.grad.cpu().numpy(), g[f"{tag}.gs0"])}
    errs.update({f"x{t}": _rel(xs[t].grad.cpu().numpy(), g[f"{tag}.gx_{t}"]) for t in range(2)})
    errs.update({n: _rel(p.grad.cpu().numpy(), g[f"{tag}.g.{n}"]) for n, p in cell.named_parameters()})
    print(f"\n[variant {tag}] " + ", ".join(f"{k}={v:.1e}" for k, v in errs.items()))
    for n, e in errs.items():
        assert e < 1e-4, (n, e)


def test_unet_bit_reproducible(dev):
    """Two identical U-Net train steps (same weights, windows and states) give bit-identical flows,
    loss and parameter gradients: every cross-block sum of the backward (LIF / prediction parameter
    sums, split-K and split-pixel partial tiles, the IWE splat) is reduced in a fixed order."""
    import snnflow
    from snnflow.synthetic import make_window

    H = W = 64
    gen = torch.Generator(device=dev).manual_seed(11)
    wins = [make_window(2, 1000, H, W, gen, dev) for _ in range(3)]
    runs = []
    for _ in range(2):
        torch.manual_seed(7)
        model = snnflow.SpikingRecEVFlowNet(_kw(16)).to(dev)
        ew = snnflow.EventWarping(_cfg(H, W), dev)
        flows = []
        for w in wins:
            out = model(None, w["event_cnt"])
            flows.append(torch.cat([f.detach().flatten() for f in out["flow"]]))
            ew.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = ew()
        loss.backward()
        runs.append((torch.cat(flows).cpu(), loss.detach().cpu(),
                     {n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()}))
    (f0, l0, g0), (f1, l1, g1) = runs
    assert torch.equal(f0, f1)
    assert torch.equal(l0, l1), (l0.item(), l1.item())
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n


def test_unet_cfg5_b16_gradients_equal_sum_of_b2_pairs(dev):
    """cfg5's bench batch with the loss on ALL 16 samples: the U-Net has no BatchNorm and the
    EventWarping loss is a sum of per-sample terms (loss/flow.py:178-303: per-sample IWE terms summed,
    the smoothness term a sum over pixels), so the B = 16 parameter gradients must equal the sum of
    eight B = 2 runs on the same sample pairs.  B = 16 runs other split-K and pixel-split plans than
    B = 2 (test_unet_cfg5_shapes_vs_oracle lists them) and B = 2 is pinned to the oracle, so a B = 16
    plan that dropped or mis-indexed the pixels of samples 2..15 fails here.  256 x 256, base 32, T = 2
    windows of 1000 events.  Split-K is capped at 1 in both runs (snnflow.unet.KSPLIT_MAX: split-K
    partitions K, not pixels, and test_unet_cfg5_shapes_vs_oracle covers it), so every conv sums in the
    same order at both batch sizes and the spikes must agree exactly (a free-running near-threshold flip
    cascades through the recurrence); the weight gradients keep their own pixel-split plans.  Loss rtol
    1e-5, every gradient within rel-L2 1e-5 (fp32 summation order)."""
    import snnflow
    import snnflow.unet as un
    from snnflow.synthetic import make_window

    base, H, B, T = 32, 256, 16, 2
    torch.manual_seed(5)
    model = snnflow.SpikingRecEVFlowNet(_kw(base)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(3)
    wins = [make_window(B, 1000, H, H, gen, dev) for _ in range(T)]

    def run(sl):
        model.reset_states()
        model.zero_grad(set_to_none=True)
        ew = snnflow.EventWarping(_cfg(H, H), dev)
        spikes, flows = [], []
        for w in wins:
            out = model(None, w["event_cnt"][sl])
            ew.event_flow_association(out["flow"], w["event_list"][sl], w["event_list_pol_mask"][sl], w["event_mask"][sl])
            spikes.append([_spk(st) for st in model.states])
            flows.append([f.detach().cpu() for f in out["flow"]])
        loss = ew()
        loss.backward()
        return loss.item(), {n: p.grad.detach().double().cpu() for n, p in model.named_parameters()}, spikes, flows

    un.KSPLIT_MAX, un.PLAN_LOG = 1, []
    try:
        l16, g16, s16, f16 = run(slice(0, B))
        p16 = {(k, M, K, P // 8): n for k, M, K, P, n in un.PLAN_LOG if k == "wgrad"}
        un.PLAN_LOG = []
        runs2 = [run(slice(2 * k, 2 * k + 2)) for k in range(B // 2)]
        p2 = {(k, M, K, P): n for k, M, K, P, n in un.PLAN_LOG if k == "wgrad"}
    finally:
        un.KSPLIT_MAX, un.PLAN_LOG = None, None
    changed = sum(1 for key, n in p16.items() if key in p2 and p2[key] != n)
    print(f"\n[unet cfg5 B=16 vs 8 x B=2] {changed} weight-gradient launch shapes with another pixel-split plan")
    assert changed
    lsum, gsum, flips, where = 0.0, None, 0, []
    for k in range(B // 2):
        sl = slice(2 * k, 2 * k + 2)
        l2, g2, s2, f2 = runs2[k]
        lsum += l2
        gsum = g2 if gsum is None else {n: gsum[n] + g2[n] for n in gsum}
        for t in range(T):
            for i, (a, b) in enumerate(zip(s16[t], s2[t])):
                a = a[:, sl] if a.dim() == 5 else a[sl]
                n = int((a != b).sum())
                flips += n
                if n:
                    where.append((k, t, i, n))
            for i, (a, b) in enumerate(zip(f16[t], f2[t])):
                d = float((a[sl] - b).abs().max())
                if d > 1e-5:
                    where.append((k, t, f"flow{i}", round(d, 6)))
    print(f"\n[unet cfg5 B=16 vs 8 x B=2] spike differences {flips}; loss {l16:.9g} vs {lsum:.9g}; "
          f"(pair, step, state, count): {where[:40]}")
    assert flips == 0, f"{flips} spike differences between the batch sizes (near-threshold flips: change the seed)"
    np.testing.assert_allclose(l16, lsum, rtol=1e-5)
    errs = {n: _rel(g16[n].numpy(), gsum[n].numpy()) for n in g16}
    worst = max(errs.items(), key=lambda kv: kv[1])
    print(f"[unet cfg5 B=16 vs 8 x B=2] gradient rel-L2 worst {worst[0]} {worst[1]:.2e} over {len(errs)} tensors")
    for n, e in errs.items():
        assert e <= 1e-5, (n, e)
