"""GPU unit tests of the C = 8 tile pipelines of the wavefront launches (csrc/lif_layers.hip
fwd_lif8_pipe / bwd_lif8_pipe) at the level of one task through the C-ABI: the same random task
arguments run once through the one-tile-per-block bodies (snnflow_set_pipe(0, 0)) and once through
the pipelines, and every output buffer is compared -- the forward's pre-BN current, both state
halves, the batch sums, statistics and running statistics; the backward's gradients of layer l-1
(current, membrane), the recurrent state gradient, layer l-1's batch sums, layer l's neuron
gradients and BN-backward coefficients, and the fused weight-gradient slabs (summed over rows, the
pipeline keeps one row per block).

Tolerances: the convs run in another summation order inside the matrix cores (swapped operands) and
the batch sums add in another order, so real-valued outputs agree to 1e-5 relative (measured worst
printed); the recomputed spikes (0/1) must match exactly wherever the membrane is not within 1e-4 of
the threshold.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _neuron(lib_, dev, gen, C, train=True, zero_reset=True):
    n = lib_.Neuron()
    keep = {
        "w": 0.5 + torch.rand(C, device=dev, generator=gen),
        "b": 0.2 * torch.randn(C, device=dev, generator=gen),
        "rm": 0.1 * torch.randn(C, device=dev, generator=gen),
        "rv": 0.5 + torch.rand(C, device=dev, generator=gen),
        "nbt": torch.zeros(1, dtype=torch.int64, device=dev),
        "beta": 0.3 + 0.6 * torch.rand(C, device=dev, generator=gen),
        "th": 0.4 + 0.6 * torch.rand(C, device=dev, generator=gen),
    }
    n.bn_weight, n.bn_bias = keep["w"].data_ptr(), keep["b"].data_ptr()
    n.running_mean, n.running_var = keep["rm"].data_ptr(), keep["rv"].data_ptr()
    n.num_batches_tracked = keep["nbt"].data_ptr()
    n.beta, n.threshold = keep["beta"].data_ptr(), keep["th"].data_ptr()
    n.momentum, n.eps, n.bn_train, n.zero_reset = 0.1, 1e-5, 1 if train else 0, 1 if zero_reset else 0
    return n, keep


def _weights(dev, gen, C):
    w = 0.3 * torch.randn(C, C, 3, 3, device=dev, generator=gen)
    wt_fwd = w.permute(2, 3, 1, 0).contiguous()  # [tap][ci][co]
    wt_bwd = w.permute(2, 3, 0, 1).contiguous()  # [tap][co][ci]
    return wt_fwd, wt_bwd


def _run(lib_, fn, tasks, n, tf, tb, tile=0):
    old = (lib_.lib.snnflow_get_pipe(0), lib_.lib.snnflow_get_pipe(1))
    old_tile = lib_.lib.snnflow_get_bwd_tile()
    try:
        assert lib_.lib.snnflow_set_pipe(tf, tb) == 0
        assert lib_.lib.snnflow_set_bwd_tile(tile) == 0
        arr = (type(tasks[0]) * len(tasks))(*tasks)
        lib_.check(fn(arr, n, None, lib_.stream_ptr(torch.device("cuda:0"))), "slot")
        torch.cuda.synchronize()
    finally:
        lib_.lib.snnflow_set_pipe(*old)
        lib_.lib.snnflow_set_bwd_tile(old_tile)


@pytest.mark.parametrize("rec,B,H,W,tb,zr,acc", [(False, 8, 32, 32, 2, True, 0), (True, 8, 32, 32, 2, True, 0),
                                                (True, 3, 40, 72, 3, False, 0), (False, 2, 24, 96, 1, True, 0),
                                                (True, 8, 32, 32, "tile", True, 0), (False, 8, 32, 32, "tile", True, 1),
                                                (True, 3, 40, 72, "tile", False, 1), (False, 2, 24, 96, "tile", True, 0),
                                                (True, 1, 13, 50, "tile", True, 1)])
def test_bwd_pipe_task_vs_one_tile(dev, rec, B, H, W, tb, zr, acc):
    """One LIF-fed backward task (fused weight gradients, prev_g_state given, recurrent input gradient
    when rec) through k_bwd_slot<8> (layer_bwd_body) and through k_bwd_slot_p8 (bwd_lif8_pipe, tb
    tiles per block) or, tb = "tile", k_bwd_slot_t8 (bwd_lif8_tile: one tile per block, swapped-operand
    input gradients); acc: the weight-gradient slabs accumulate onto their old values."""
    from snnflow import _lib

    C = 8
    gen = torch.Generator(device=dev).manual_seed(11)
    P = B * H * W
    keep = []

    def t(*shape, scale=1.0):
        x = scale * torch.randn(*shape, device=dev, generator=gen)
        keep.append(x)
        return x

    y, gcur = t(P, C), t(P, C, scale=0.05)
    stats = torch.stack([0.1 * torch.randn(C, device=dev, generator=gen), 0.8 + 0.4 * torch.rand(C, device=dev, generator=gen)])
    prev_y, prev_mem = t(P, C), t(P, C, scale=0.5)
    prev_stats = torch.stack([0.1 * torch.randn(C, device=dev, generator=gen), 0.8 + 0.4 * torch.rand(C, device=dev, generator=gen)])
    prev_gs = t(2, P, C, scale=0.02)
    acc_in = torch.zeros(_lib.acc_storage(5 * C + 2), dtype=torch.float64, device=dev)
    acc_in.view(32, -1)[:, :5 * C + 2] = 0.01 * torch.randn(32, 5 * C + 2, device=dev, generator=gen).double()
    wf, wb = _weights(dev, gen, C)
    wfr, wbr = _weights(dev, gen, C)
    s_prev = (torch.rand(P, C, device=dev, generator=gen) < 0.3).float()
    n, kn = _neuron(_lib, dev, gen, C, zero_reset=zr)
    pn, kp = _neuron(_lib, dev, gen, C, zero_reset=zr)
    ntiles = _lib.lib.snnflow_conv_blocks(B, H, W)

    slab0 = torch.randn(ntiles, C * C * 9, device=dev, generator=gen)
    outs = {}
    for tag, tbb in (("one", 0), ("pipe", tb)):
        o = {"g_cur": torch.full((P, C), 7.0, device=dev), "g_mem": torch.full((P, C), 7.0, device=dev),
             "acc_out": torch.zeros(_lib.acc_storage(5 * C + 2), dtype=torch.float64, device=dev),
             "ng": torch.zeros(4, C, device=dev), "bnc": torch.zeros(2, C, device=dev),
             "gsp": torch.full((2, P, C), 7.0, device=dev),
             "slab_ff": torch.full((ntiles, C * C * 9), 7.0, device=dev),
             "slab_rec": torch.full((ntiles, C * C * 9), 7.0, device=dev)}
        a = _lib.LayerBwdArgs()
        a.B, a.H, a.W, a.cin, a.c = B, H, W, C, C
        a.y, a.stats, a.g_cur, a.acc_in, a.n = y.data_ptr(), stats.data_ptr(), gcur.data_ptr(), acc_in.data_ptr(), n
        ng = _lib.NeuronGrad()
        ng.bn_weight, ng.bn_bias = o["ng"][0].data_ptr(), o["ng"][1].data_ptr()
        ng.beta, ng.threshold = o["ng"][2].data_ptr(), o["ng"][3].data_ptr()
        a.ng, a.accumulate, a.bnc_out = ng, 0, o["bnc"].data_ptr()
        a.wt_bwd_ff, a.wt_fwd_ff, a.lif_in = wb.data_ptr(), wf.data_ptr(), 1
        if rec:
            a.wt_bwd_rec, a.wt_fwd_rec = wbr.data_ptr(), wfr.data_ptr()
            a.g_state_prev, a.zero_mem_half = o["gsp"].data_ptr(), 1
            a.wslab_rec, a.s_prev = o["slab_rec"].data_ptr(), s_prev.data_ptr()
        a.prev_y, a.prev_mem, a.prev_stats, a.prev = prev_y.data_ptr(), prev_mem.data_ptr(), prev_stats.data_ptr(), pn
        a.prev_g_state, a.prev_g_cur, a.prev_g_mem = prev_gs.data_ptr(), o["g_cur"].data_ptr(), o["g_mem"].data_ptr()
        a.acc_out = o["acc_out"].data_ptr()
        if acc:
            o["slab_ff"].copy_(slab0)
            o["slab_rec"].copy_(slab0.flip(0))
        a.wslab_ff, a.wslab_accumulate = o["slab_ff"].data_ptr(), acc
        if tbb == "tile":
            _run(_lib, _lib.lib.snnflow_bwd_slot, [a], 1, 0, 0, tile=1)
        else:
            _run(_lib, _lib.lib.snnflow_bwd_slot, [a], 1, 0, tbb)
        outs[tag] = o
    errs = {}
    for k in ("g_cur", "g_mem", "ng", "bnc") + (("gsp",) if rec else ()):
        errs[k] = _rel(outs["pipe"][k].cpu().numpy(), outs["one"][k].cpu().numpy())
    sums = [outs[x]["acc_out"].view(32, -1)[:, :3 * C].sum(0).cpu().numpy() for x in ("pipe", "one")]
    errs["acc_out"] = _rel(*sums)
    for k in ("slab_ff",) + (("slab_rec",) if rec else ()):
        if tb == "tile":  # one slab row per tile in both: row by row
            errs[k] = _rel(outs["pipe"][k].cpu().numpy(), outs["one"][k].cpu().numpy())
        else:
            errs[k] = _rel(outs["pipe"][k].sum(0).cpu().numpy(), outs["one"][k].sum(0).cpu().numpy())
    if tb == "tile":  # the recomputed spikes: g_cur is zero exactly where no surrogate gradient flows
        errs["g_cur_max"] = float((outs["pipe"]["g_cur"] - outs["one"]["g_cur"]).abs().max() /
                                  outs["one"]["g_cur"].abs().max())
    print(f"\n[bwd pipe rec={rec} {B}x{H}x{W} tb={tb}] " + ", ".join(f"{k} {v:.1e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v < 1e-5, (k, v)


def test_bwd_pipe_set_get():
    """snnflow_set_pipe / snnflow_get_pipe and snnflow_set_bwd_tile / get round trips; negative tile
    counts are refused."""
    from snnflow import _lib

    old = (_lib.lib.snnflow_get_pipe(0), _lib.lib.snnflow_get_pipe(1))
    old_tile = _lib.lib.snnflow_get_bwd_tile()
    try:
        assert _lib.lib.snnflow_set_pipe(3, 2) == 0
        assert (_lib.lib.snnflow_get_pipe(0), _lib.lib.snnflow_get_pipe(1)) == (3, 2)
        assert _lib.lib.snnflow_set_pipe(-1, 0) != 0
        assert _lib.lib.snnflow_set_bwd_tile(5) == 0 and _lib.lib.snnflow_get_bwd_tile() == 1
        assert _lib.lib.snnflow_set_bwd_tile(0) == 0 and _lib.lib.snnflow_get_bwd_tile() == 0
    finally:
        _lib.lib.snnflow_set_pipe(*old)
        _lib.lib.snnflow_set_bwd_tile(old_tile)


def test_bwd_pipe_debug_dgrad(dev):
    """(debug build only: SNNFLOW_PIPE_DEBUG_GX) the raw input gradient of the pipeline vs torch."""
    import os
    if not os.environ.get("SNNFLOW_LIB", "").endswith("_dbg.so"):
        pytest.skip("debug build only")
    from snnflow import _lib
    C, B, H, W = 8, 2, 32, 32
    gen = torch.Generator(device=dev).manual_seed(3)
    P = B * H * W
    y = torch.randn(P, C, device=dev, generator=gen)
    gcur = torch.randn(P, C, device=dev, generator=gen)
    stats = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev)])
    acc_in = torch.zeros(_lib.acc_storage(5 * C + 2), dtype=torch.float64, device=dev)
    wf, wb = _weights(dev, gen, C)
    n, kn = _neuron(_lib, dev, gen, C)
    pn, kp = _neuron(_lib, dev, gen, C)
    n.bn_train = 0  # G = g_cur * gamma * invstd
    kn["w"].fill_(1.0)
    out = torch.zeros(P, C, device=dev)
    ng = _lib.NeuronGrad()
    tmp = torch.zeros(6, C, device=dev)
    ng.bn_weight, ng.bn_bias, ng.beta, ng.threshold = [tmp[i].data_ptr() for i in range(4)]
    a = _lib.LayerBwdArgs()
    a.B, a.H, a.W, a.cin, a.c = B, H, W, C, C
    a.y, a.stats, a.g_cur, a.acc_in, a.n, a.ng = y.data_ptr(), stats.data_ptr(), gcur.data_ptr(), acc_in.data_ptr(), n, ng
    a.bnc_out = tmp[4].data_ptr()
    a.wt_bwd_ff, a.wt_fwd_ff, a.lif_in = wb.data_ptr(), wf.data_ptr(), 1
    a.prev_y, a.prev_mem, a.prev_stats, a.prev = y.data_ptr(), y.data_ptr(), stats.data_ptr(), pn
    a.prev_g_cur = out.data_ptr()
    acc_out = torch.zeros(_lib.acc_storage(5 * C + 2), dtype=torch.float64, device=dev)
    a.acc_out = acc_out.data_ptr()
    _run(_lib, _lib.lib.snnflow_bwd_slot, [a], 1, 0, 2)
    w = wf.permute(3, 2, 0, 1)  # [co][ci][ky][kx]
    g = gcur.view(B, H, W, C).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv_transpose2d(g, w, padding=1).permute(0, 2, 3, 1).reshape(P, C)
    print("\nrel", _rel(out.cpu().numpy(), ref.cpu().numpy()))
    print(out[:3].cpu().numpy())
    print(ref[:3].cpu().numpy())
    assert _rel(out.cpu().numpy(), ref.cpu().numpy()) < 1e-5
