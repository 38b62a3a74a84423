"""Drivers of the HIP C-ABI: the fused per-time-step LIFFireNet Function, the
per-cell Function and their scratch workspaces.

One time step of the network (reference ``models/model.py:135-207``: head, G1, R1a,
R1b, G2, R2a, R2b, pred) is ONE autograd node here:

  forward  (L+1 kernels)  conv(head) | LIF(l)+conv(l+1) ... | LIF(L-1)+pred
  backward (L+1 kernels)  LIF(L-1)+pred bwd | BN-bwd+dgrad+wgrad(l)+LIF-bwd(l-1) ... | wgrad(head)

States are the only tensors that cross time steps.  The spike halves of the
recurrent cells' states carry gradients backward in time (the membrane half is
detached, ``SNNtorch_spiking_submodules.py:554-556``).  Parameter gradients of all
T steps of a truncated-BPTT window are accumulated on the device (weight
gradients in per-block slabs, neuron/BN gradients in place) and returned once,
by the first step of the window ("root"), so autograd performs no per-step
gradient additions.
"""
import ctypes
import operator
import os

import torch

from . import _lib
from ._lib import check, lib, ptr



def nhwc_state_strides(B, C, H, W):
    """Strides of a [2,B,C,H,W] state whose storage is [2][B][H][W][C]."""
    return (B * H * W * C, H * W * C, 1, W * C, C)


def empty_state(B, C, H, W, device):
    return torch.empty_strided((2, B, C, H, W), nhwc_state_strides(B, C, H, W), device=device, dtype=torch.float32)


def as_nhwc_state(s):
    """Any [2,B,C,H,W] state -> tensor with [2][B][H][W][C] storage (no copy if already)."""
    two, B, C, H, W = s.shape
    if s.stride() == nhwc_state_strides(B, C, H, W) and s.dtype == torch.float32:
        return s
    out = empty_state(B, C, H, W, s.device)
    out.copy_(s)
    return out


def as_nhwc(t):
    """[B,C,H,W] -> channels_last storage (no copy if already)."""
    B, C, H, W = t.shape
    if t.stride() == (H * W * C, 1, W * C, C) and t.dtype == torch.float32:
        return t
    return t.contiguous(memory_format=torch.channels_last).float()


def neuron_struct(cell, weight=None, bias=None):
    """Neuron parameters of a cell for the kernels; weight/bias override the BatchNorm affine
    parameters (TEBN folds its temporal weight into them, cells.py)."""
    bn, lif = getattr(cell, "batch_norm", cell.bn), cell.lif
    train = bn.training or not bn.track_running_stats
    return _lib.Neuron(
        ptr(bn.weight if weight is None else weight), ptr(bn.bias if bias is None else bias),
        ptr(bn.running_mean) if bn.track_running_stats else None,
        ptr(bn.running_var) if bn.track_running_stats else None,
        ptr(bn.num_batches_tracked) if (bn.training and bn.track_running_stats) else None,
        ptr(lif.beta), ptr(lif.threshold),
        float(bn.momentum if bn.momentum is not None else 0.0), float(bn.eps),
        1 if train else 0, 1 if cell.hard_reset else 0)


class Workspace:
    """Device scratch sized for one (B, H, W, C) problem; reused across steps.

    fwd_acc[l] / bwd_acc[l]: fp64 batch-sum accumulators of layer l (BatchNorm forward
    sums; LIF/BN backward sums + pred sums).  Zero when idle; each is re-zeroed by a
    kernel that runs after its consumer (see FireNetStep)."""

    def __init__(self, B, H, W, C, layers, device):
        self.key = (B, H, W, C, device)
        self.B, self.H, self.W, self.C = B, H, W, C
        self.nblk = lib.snnflow_conv_blocks(B, H, W)
        self.fwd_acc = torch.zeros(max(layers, 1), _lib.acc_storage(2 * C), dtype=torch.float64, device=device)
        self.bwd_acc = torch.zeros(max(layers, 1), _lib.acc_storage(_lib.bwd_acc_len(C)), dtype=torch.float64,
                                   device=device)
        self.slab_ff = []
        self.slab_rec = []
        self.device = device

    def reset_acc(self):
        self.fwd_acc.zero_()
        self.bwd_acc.zero_()

    def slabs(self, layer_shapes):
        """layer_shapes: list of (cin, recurrent)."""
        if len(self.slab_ff) != len(layer_shapes):
            dev = self.device
            self.slab_ff = [torch.empty(self.nblk, self.C * cin * 9, device=dev) for cin, _ in layer_shapes]
            self.slab_rec = [torch.empty(self.nblk, self.C * self.C * 9, device=dev) if rec else None
                             for _, rec in layer_shapes]
        return self.slab_ff, self.slab_rec


class PreppedWeights:
    """Transposed conv weights [3][3][Cin][C] / [3][3][C][Cin] + in-place threshold clamp
    (reference: ``threshold.data.clamp_(min=0.01)`` at every cell forward,
    SNNtorch_spiking_submodules.py:284 / :516).

    Refreshed by one batched launch at the first forward after a completed backward
    pass (the optimizer step sits between them) and whenever a parameter's version
    counter moved (load_state_dict, in-place edits through autograd-visible ops).  Version
    counters alone cannot key the cache: fused optimizers update weights without bumping
    them.  The backward pass reuses the buffers of the last forward (same weights)."""

    def __init__(self):
        self.fwd = {}
        self.bwd = {}
        self.frag = {}   # i -> uint16 [snnflow_frag_halfs] forward-conv bf16 fragments (C = 16, 32) or None
        self.fragb = {}  # i -> the same for the input-gradient conv
        self.key = None
        self.gen = 0  # bumped whenever the buffers are re-allocated

    def weight_version(self):
        """The version-counter sum ensure() last prepared from (-1 before the first preparation)."""
        src = self.__dict__.get("src")
        if src is None:
            return -1
        return sum(w._version for w in src) + sum(t._version for t in self.__dict__.get("th", ()))

    def ensure(self, weights, thresholds, stream, refresh=True, zero=None):
        """`weights` / `thresholds` are the engine's cached lists (re-built when a parameter is replaced
        or moved): a new list re-checks pointers and buffers, the same list only the version counters.
        `zero`: an fp64 tensor zeroed by the same launch (a zero-only launch if nothing is re-prepared)."""
        ver = sum(w._version for w in weights) + sum(t._version for t in thresholds)
        same = self.__dict__.get("src") is weights
        if not same:
            key = tuple((w.data_ptr(), w._version) for w in weights) + tuple((t.data_ptr(), t._version) for t in thresholds)
            if key != self.key:
                refresh = True
            self.key = key
            self.src = weights
            self.th = thresholds
        elif ver != self.__dict__.get("ver"):
            refresh = True
        self.ver = ver
        fresh = False
        shapes = tuple((w.data_ptr(), w.numel()) for w in weights) if not same else self.shapes
        for i, w in enumerate(weights if shapes != self.__dict__.get("shapes") else ()):
            f = self.fwd.get(i)
            if f is None or f.numel() != w.numel() or f.device != w.device:
                self.fwd[i] = torch.empty(w.numel(), device=w.device)
                self.bwd[i] = torch.empty(w.numel(), device=w.device)
                c, cin = w.shape[0], w.shape[1]
                nf = lib.snnflow_frag_halfs(c, cin) if c >= 16 else 0  # C = 8 splits in LDS
                self.frag[i] = torch.empty(nf, dtype=torch.int16, device=w.device) if nf else None
                self.fragb[i] = torch.empty(nf, dtype=torch.int16, device=w.device) if nf else None
                fresh = True
        self.shapes = shapes
        if fresh:
            self.gen += 1
        if not (refresh or fresh):
            if zero is not None:
                d = _lib.PrepDesc()
                d.zero, d.zero_n = zero.data_ptr(), zero.numel()
                _lib.call("prep_weights", lib.snnflow_prep_weights_batch, (_lib.PrepDesc * 1)(d), 1, stream)
            return
        descs = []
        for i, w in enumerate(weights):
            c, cin = w.shape[0], w.shape[1]
            if not w.is_contiguous():
                raise _lib.SnnflowError("conv weight must be contiguous")
            descs.append(_lib.PrepDesc(ptr(w), c, cin, ptr(self.fwd[i]), ptr(self.bwd[i]), None, 0,
                                       _ptr_t(self.frag.get(i)), _ptr_t(self.fragb.get(i))))
        for i, t in enumerate(thresholds):  # ride along with the weight descriptors
            if i < len(descs):
                descs[i].threshold, descs[i].thr_n = ptr(t), t.numel()
            else:
                descs.append(_lib.PrepDesc(None, 0, 0, None, None, ptr(t), t.numel()))
        if zero is not None:
            if not descs:
                descs.append(_lib.PrepDesc())
            descs[0].zero, descs[0].zero_n = zero.data_ptr(), zero.numel()
        for i0 in range(0, len(descs), _lib.MAX_BATCH):
            chunk = descs[i0:i0 + _lib.MAX_BATCH]
            _lib.call("prep_weights", lib.snnflow_prep_weights_batch, (_lib.PrepDesc * len(chunk))(*chunk),
                      len(chunk), stream)


# ---------------------------------------------------------------------------
# Fused time step of the LIFFireNet family
# ---------------------------------------------------------------------------
class FireNetEngine:
    """Owns the cells' device-side bookkeeping for one model instance."""

    def __init__(self, model):
        self.cells = [getattr(model, name) for name, _ in model.layer_spec]
        self.rec = [rec for _, rec in model.layer_spec]
        self.pred = model.pred.conv2d
        self.L = len(self.cells)
        self.C = self.cells[0].hidden_size
        self.ws = None
        self.prep = PreppedWeights()
        self.bwd_open = False
        self.flat = None
        self.flat_views = None
        self.pending = []   # per-step tensors of the open backward chain (deferred wgrad)
        self.pending_layers = []  # per pending step: the layers whose weight gradients are still deferred
        self.slab_live = [False] * self.L      # slab rows of layer l hold partial sums of this chain
        self.fuse_wgrad = self.C == 8          # wavefront backward computes layers >= 1's dW in place
        # wavefront backward adds the head's dW of each step inside the head's backward task (ABI 40).
        # Measured (profiles/r06/fuse_head_ab.txt): C = 32 -35 us per step (the deferred k_wgrad<2, 32> gone,
        # the slots +2-4 us per launch); C = 8 neutral to +5 us, so off there.  SNNFLOW_FUSE_HEAD=0 / 1 forces.
        fh = os.environ.get("SNNFLOW_FUSE_HEAD")
        self.fuse_head = (self.C >= 16) if fh is None else fh != "0"
        # forward_sequence: spike bit planes between its kernels (ABI 39; SNNFLOW_SPK_BITS=0: the fp32 spike
        # half of the states everywhere, as before)
        self.spk_bits = os.environ.get("SNNFLOW_SPK_BITS", "1") != "0"
        # per-step autograd nodes of one BPTT chain (the reference loop's T model() calls): their backwards
        # are collected and issued at the chain's first step as wavefront launches (FireNetStep, _Chain);
        # SNNFLOW_DEFER_BWD=0: every node runs its own step's backward
        self.defer_backward = os.environ.get("SNNFLOW_DEFER_BWD", "1") != "0"
        self.keep_seq_states = False  # FireNetSequence: expose every step's states (activity log)
        self.capture_states = False   # tests: keep every step's states of forward_sequence in seq_states
        # forward_sequence, one-shot: a flat fp32 buffer of L x 2BHWC floats that receives the final
        # step's states (the states the call returns are views into it) instead of a fresh
        # allocation.  A graph-replay loop that alternates two such buffers hands the states from
        # one step to the next with no copy; the buffer must not alias the states passed in.
        self.final_state_out = None
        self.seq_states = None
        self.prep_stale = True  # re-prepare weights at the next forward (set after each backward)
        self.lifs = [c.lif for c in self.cells]
        self.bns = [getattr(c, "batch_norm", c.bn) for c in self.cells]
        self._plist = None     # cached param_list() (+ identity checks), see param_list
        self._neurons = None   # cached neuron structs, re-validated per call (neurons())
        self._gen = 0          # bumped whenever the neuron structs are rebuilt or invalidate() runs

    def __deepcopy__(self, memo):  # (copy.deepcopy(model)): ctypes caches are rebuilt, not copied
        import copy
        new = self.__class__.__new__(self.__class__)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            new.__dict__[k] = None if k in ("_neurons", "_nk_src", "_plist", "_prep_ws", "_prep_map", "_plan", "_gviews", "_layout",
                                            "_anchor") \
                else copy.deepcopy(v, memo)
        return new

    def invalidate(self):
        """Drop cached parameter lists / neuron structs / step-driver plans (the model's _apply moved
        or replaced tensors)."""
        self._plist = None
        self._neurons = None
        self._prep_ws = None
        self._prep_map = None
        self._plan = None
        self._gen = self.__dict__.get("_gen", 0) + 1

    def _neuron_key(self):
        """Everything neuron_struct reads, per cell: the tensors themselves (held by the cache, so a
        replaced tensor can never alias a freed one's identity) and the scalar options.  Read from
        the modules' _parameters / _buffers dicts directly (nn.Module.__getattr__ costs ~0.3 us a
        lookup; this runs three times per time step on the eager path)."""
        src = self.__dict__.get("_nk_src")
        if src is None:
            src = [(c, bn, bn._parameters, bn._buffers, lif._parameters, lif._buffers)
                   for c, bn, lif in zip(self.cells, self.bns, self.lifs)]
            self._nk_src = src
        tens, scal = [], []
        for c, bn, bp, bb, lp, lb in src:
            tens += (bp.get("weight"), bp.get("bias"), bb.get("running_mean"), bb.get("running_var"),
                     bb.get("num_batches_tracked"), lp["beta"] if "beta" in lp else lb.get("beta"),
                     lp["threshold"] if "threshold" in lp else lb.get("threshold"))
            scal += (bn.training, bn.track_running_stats, bn.momentum, bn.eps, c.hard_reset)
        return tens, scal

    def neurons(self):
        """neuron_struct of every cell, cached and re-validated on every call against the tensors and
        options it was built from (identity for tensors, equality for scalars).  A rebuild bumps the
        engine generation, which keys the C step driver's plan (it holds copies of the structs)."""
        tens, scal = self._neuron_key()
        n = self._neurons
        if n is None or n[1] != scal or not all(map(operator.is_, n[0], tens)):
            self._neurons = (tens, scal, [neuron_struct(c) for c in self.cells])
            self._gen = self.__dict__.get("_gen", 0) + 1
        return self._neurons[2]

    def any_subtract(self):
        """True if some cell uses the subtract reset (theta_subtract has work)."""
        return any(lif.reset_mechanism == "subtract" for lif in self.lifs)

    def sequence_ok(self, cin0):
        """True if FireNetSequence's wavefront launches take this model (C = 8, 16, 32; cin0 2 or 4)."""
        return bool(lib.snnflow_slot_supported(self.C, cin0))

    # parameter order = Function input order after the states
    def param_list(self):
        """Cached; re-validated per call by identity against the owning modules' _parameters dicts."""
        pl = self._plist
        if pl is not None and all(d.get(k) is v for d, k, v in pl[1]):
            return pl[0]
        ps = self._param_list()
        checks = []
        for cell, rec in zip(self.cells, self.rec):
            checks.append((cell.ff._parameters, "weight", cell.ff.weight))
            if rec:
                checks.append((cell.rec._parameters, "weight", cell.rec.weight))
            bn = getattr(cell, "batch_norm", cell.bn)
            checks += [(bn._parameters, "weight", bn.weight), (bn._parameters, "bias", bn.bias),
                       (cell.lif._parameters, "beta", cell.lif._parameters.get("beta")),
                       (cell.lif._parameters, "threshold", cell.lif._parameters.get("threshold"))]
        checks += [(self.pred._parameters, "weight", self.pred.weight), (self.pred._parameters, "bias", self.pred.bias)]
        self._plist = (tuple(ps), checks)
        self._neurons = None
        self._prep_ws = None
        return self._plist[0]

    def _param_list(self):
        ps = []
        for cell, rec in zip(self.cells, self.rec):
            ps.append(cell.ff.weight)
            if rec:
                ps.append(cell.rec.weight)
            ps += [cell.bn.weight, cell.bn.bias, cell.lif.beta, cell.lif.threshold]
        ps += [self.pred.weight, self.pred.bias]
        return ps

    def workspace(self, B, H, W, device):
        key = (B, H, W, self.C, device)
        if self.ws is None or self.ws.key != key:
            self.ws = Workspace(B, H, W, self.C, self.L, device)
            self.ws.slabs([(c.input_size, r) for c, r in zip(self.cells, self.rec)])
        return self.ws

    def prep_weights(self, stream, refresh=True, zero=None):
        ws = self.__dict__.get("_prep_ws")
        if ws is None or self._plist is None:  # conv weights in PreppedWeights order (param_list validates)
            ws = []
            for cell, rec in zip(self.cells, self.rec):
                ws.append(cell.ff.weight)
                if rec:
                    ws.append(cell.rec.weight)
            self._prep_ws = ws
            self._prep_th = [c.lif.threshold for c in self.cells]
            self._prep_map = None
        self.prep.ensure(ws, self._prep_th, stream, refresh, zero)
        m = self._prep_map
        if m is not None and m[0] == self.prep.gen:
            return m[1], m[2]
        # map layer -> prepped buffers
        fwd, bwd, frag, fragb, i = [], [], [], [], 0
        for rec in self.rec:
            ff = (self.prep.fwd[i], self.prep.bwd[i], self.prep.frag.get(i), self.prep.fragb.get(i))
            i += 1
            rc = (None, None, None, None)
            if rec:
                rc = (self.prep.fwd[i], self.prep.bwd[i], self.prep.frag.get(i), self.prep.fragb.get(i))
                i += 1
            fwd.append((ff[0], rc[0]))
            bwd.append((ff[1], rc[1]))
            frag.append((ff[2], rc[2]))
            fragb.append((ff[3], rc[3]))
        self.frags, self.fragsb = frag, fragb
        self._prep_map = (self.prep.gen, fwd, bwd)
        return fwd, bwd

    def flat_layout_for(self, params):
        """[(offset, numel, shape)] of `params` packed back to back (the flat gradient buffer)."""
        layout = self.__dict__.get("_layout")
        if layout is None or layout[0] != [id(p) for p in params]:
            lay, off = [], 0
            for p in params:
                lay.append((off, p.numel(), p.shape))
                off += p.numel()
            layout = ([id(p) for p in params], lay, off)
            self._layout = layout
        return layout[1]

    def anchor(self, states):
        """The ParamAnchor of the BPTT chain a step with previous `states` belongs to: the current
        one if a recurrent state carries this engine's graph (the chain continues), else a new one
        (None without autograd)."""
        params = self.param_list()
        if not torch.is_grad_enabled() or not any(p.requires_grad for p in params):
            return None
        cont = False
        for p, rec in zip(states, self.rec):
            if rec and p is not None and p.requires_grad and getattr(p.grad_fn, "eng", None) is self:
                cont = True
                break
        a = self.__dict__.get("_anchor")
        if not cont or a is None or a[0] is not params:
            self._anchor = (params, ParamAnchor.apply(self, *params))
        return self._anchor[1]

    def prepped(self):
        """The prepared weight buffers of the last forward (no re-validation: the backward of a step
        runs on the weights its forward saw)."""
        m = self.__dict__.get("_prep_map")
        if m is None:
            raise _lib.SnnflowError("backward before any forward of this model")
        return m[1], m[2]

    def open_chain(self, device):
        self.bwd_task = torch._C._current_graph_task_id()
        self.slab_live = [False] * self.L
        self.flat_layout = self.flat_layout_for(self.param_list())
        o, n, _ = self.flat_layout[-1]
        self.flat = torch.empty(o + n, device=device)
        self.flat_views = True  # (gradient destinations are addressed through flat_layout)
        self.bwd_open = True

    def drop_stale_chain(self):
        """A backward chain left open by an earlier backward pass that never reached the chain's first step
        (autograd.grad / backward(inputs=...) on an intermediate state) is abandoned: its partial weight
        gradients and pending steps would otherwise be added to this pass's."""
        if self.bwd_open and getattr(self, "bwd_task", None) != torch._C._current_graph_task_id():
            if self.ws is not None:
                self.ws.reset_acc()
            self.bwd_open = False
            self.pending, self.pending_layers = [], []
            self.prep_stale = True

    def launch_wgrad(self, l, B, H, W, cin0, ws, stream, steps=None):
        """Deferred weight gradients of layer l over the given pending time steps (default: all;
        one snnflow_wgrad launch per <= 32 steps) into the layer's per-block slabs (SURVEY
        Appendix D: x, s_prev, y, stats saved per step), added to what the chain's fused steps
        already left there."""
        C, rec = self.C, self.rec[l]
        steps = self.pending if steps is None else steps
        for i0 in range(0, len(steps), _lib.MAX_WGRAD_STEPS):
            chunk = steps[i0:i0 + _lib.MAX_WGRAD_STEPS]
            a = _lib.WgradArgs()
            a.B, a.H, a.W, a.c = B, H, W, C
            a.cin = cin0 if l == 0 else C
            a.nsteps, a.rec = len(chunk), 1 if rec else 0
            a.accumulate = 1 if (i0 or self.slab_live[l]) else 0
            # layers >= 1: x and s_prev are spikes of this engine (0/1, exact in bf16)
            a.exact_inputs = 1 if l > 0 else 0
            a.bn_weight = ptr(self.cells[l].bn.weight)
            a.slab_ff, a.slab_rec = ptr(ws.slab_ff[l]), _ptr_t(ws.slab_rec[l])
            for k, (gcur, bnc, ys, stats, x, states, s_prev, _, bits) in enumerate(chunk):
                st = a.steps[k]
                st.g_cur, st.y, st.stats, st.bnc = gcur[l], ys[l], stats[l], bnc[l]
                xb, sb = bits if bits is not None else (None, None)
                if l == 0:
                    st.x = ptr(x)
                    st.xs_b, st.xs_c, st.xs_h, st.xs_w = _x_strides(x)
                elif xb is not None and xb[l - 1] is not None:  # layer l-1's spikes as a bit plane (ABI 39)
                    st.x_bits = xb[l - 1]
                else:
                    st.x, (st.xs_b, st.xs_c, st.xs_h, st.xs_w) = _spk_half(states[l - 1])
                if rec and sb is not None and sb[l] is not None:
                    st.s_prev_bits = sb[l]
                else:
                    st.s_prev = _ptr_t(s_prev[l]) if rec else None
            _lib.call(f"wgrad[{l}]", lib.snnflow_wgrad, ctypes.byref(a), stream)
            self.slab_live[l] = True

    def launch_slab_reduce(self, ws, glayers, stream):
        """Fixed-order fp64 sum of every layer's per-block slabs into the flat gradient buffer."""
        descs = []
        for l in range(self.L):
            gff, grec, _ = glayers[l]
            cin = self.cells[l].input_size
            descs.append(_lib.SlabDesc(ptr(ws.slab_ff[l]), gff, self.C * cin * 9))
            if grec is not None:
                descs.append(_lib.SlabDesc(ptr(ws.slab_rec[l]), grec, self.C * self.C * 9))
        for i0 in range(0, len(descs), 16):
            chunk = (_lib.SlabDesc * len(descs[i0:i0 + 16]))(*descs[i0:i0 + 16])
            _lib.call("slab_reduce", lib.snnflow_slab_reduce, chunk, len(descs[i0:i0 + 16]), ws.nblk, stream)

    def flush_weight_grads(self, B, H, W, cin0, ws, glayers, stream, plan=None):
        """All deferred weight gradients on `stream` (serial form of the root step's tail): one
        snnflow_firenet_wgrad call given the step driver's plan, else (per-kernel timing) the
        per-layer launches from Python."""
        partial = any(len(ls) < self.L for ls in self.pending_layers) or any(self.slab_live)
        if plan is None or _lib.TIMER is not None or partial:
            for l in range(self.L):
                steps = [e for e, ls in zip(self.pending, self.pending_layers) if l in ls]
                if steps:
                    self.launch_wgrad(l, B, H, W, cin0, ws, stream, steps)
            self.launch_slab_reduce(ws, glayers, stream)
            self.pending, self.pending_layers = [], []
            return
        L = self.L
        steps = (_lib.FireNetWgradStep * len(self.pending))()
        for k, (gcur, bnc, ys, stats, x, states, s_prev, _, bits) in enumerate(self.pending):
            assert bits is None, "the step driver's deferred weight gradients read fp32 spike planes"
            st = steps[k]
            st.g_cur, st.bnc, st.ys, st.stats = gcur.base, bnc.base, ys.base, stats.base
            st.x = x.data_ptr()
            st.xs[0], st.xs[1], st.xs[2], st.xs[3] = x.stride()
            st.states = states[0].data_ptr()
            for l in range(L):
                st.s_prev[l] = _ptr_t(s_prev[l])
        gff = (ctypes.c_void_p * L)(*[glayers[l][0] for l in range(L)])
        grec = (ctypes.c_void_p * L)(*[glayers[l][1] for l in range(L)])
        _lib.call("firenet_wgrad", lib.snnflow_firenet_wgrad, ctypes.byref(plan), steps, len(self.pending), gff, grec,
                  stream)
        self.pending, self.pending_layers = [], []

    def plan(self, B, H, W, cin0, ws, wfwd, wbwd):
        """The C step driver's constant arguments (snnflow_firenet_plan), cached per model state."""
        neurons = self.neurons()
        train = tuple(bn.training or not bn.track_running_stats for bn in self.bns)
        key = (B, H, W, cin0, id(ws), ws.fwd_acc.data_ptr(), self.prep.gen, self._gen, train,
               self.pred.weight.data_ptr(), self.pred.bias.data_ptr())
        pl = self.__dict__.get("_plan")
        if pl is not None and pl[0] == key:
            return pl[1]
        L = self.L
        if L > _lib.MAX_LAYERS:
            raise _lib.SnnflowError(f"at most {_lib.MAX_LAYERS} layers")
        p = _lib.FireNetPlan()
        p.L, p.B, p.H, p.W, p.c, p.cin0 = L, B, H, W, self.C, cin0
        for l in range(L):
            p.rec[l] = 1 if self.rec[l] else 0
            p.train[l] = 1 if train[l] else 0
            p.n[l] = neurons[l]
            p.wt_fwd_ff[l], p.wt_fwd_rec[l] = _ptr_t(wfwd[l][0]), _ptr_t(wfwd[l][1])
            p.wt_bwd_ff[l], p.wt_bwd_rec[l] = _ptr_t(wbwd[l][0]), _ptr_t(wbwd[l][1])
            p.wf_ff[l], p.wf_rec[l] = _ptr_t(self.frags[l][0]), _ptr_t(self.frags[l][1])
            p.wd_ff[l], p.wd_rec[l] = _ptr_t(self.fragsb[l][0]), _ptr_t(self.fragsb[l][1])
            p.slab_ff[l], p.slab_rec[l] = _ptr_t(ws.slab_ff[l]), _ptr_t(ws.slab_rec[l])
        p.fwd_acc, p.fwd_acc_stride = ws.fwd_acc.data_ptr(), ws.fwd_acc.stride(0)
        p.bwd_acc, p.bwd_acc_stride = ws.bwd_acc.data_ptr(), ws.bwd_acc.stride(0)
        p.pred_w, p.pred_b = ptr(self.pred.weight), ptr(self.pred.bias)
        p.nblk = ws.nblk
        self._plan = (key, p)
        return p

    def grad_views(self):
        """Per-layer gradient destinations inside the flat buffer (cached per chain)."""
        gv = self.__dict__.get("_gviews")
        if gv is not None and gv[0] is self.flat:
            return gv[1]
        gv = self._grad_views()
        self._gviews = (self.flat, gv)
        return gv

    def _grad_views(self):
        """(per layer: (dW_ff ptr, dW_rec ptr or None, NeuronGrad), pred dW ptr, pred db ptr) by offset
        into the flat buffer (param_list order)."""
        base = self.flat.data_ptr()
        v = iter(self.flat_layout)

        def nxt():
            return base + 4 * next(v)[0]
        layers = []
        for rec in self.rec:
            gff = nxt()
            grec = nxt() if rec else None
            gbw, gbb, gbeta, gth = nxt(), nxt(), nxt(), nxt()
            layers.append((gff, grec, _lib.NeuronGrad(gbw, gbb, gbeta, gth)))
        gpw, gpb = nxt(), nxt()
        return layers, gpw, gpb


def _x_strides(x):
    return x.stride(0), x.stride(1), x.stride(2), x.stride(3)


def _spk_half(state_nhwc):
    """Spike half of a [2][B][H][W][C] state as (pointer, strides (b,c,h,w))."""
    two, B, C, H, W = state_nhwc.shape
    base = state_nhwc.data_ptr() + 4 * (B * H * W * C)
    return base, (H * W * C, 1, W * C, C)



class _Rows:
    """Device pointers of t[0], t[1], ... by address arithmetic (indexing a tensor builds a view,
    a few microseconds each; the eager per-step path needs ~100 of them per time step)."""
    __slots__ = ("base", "step")

    def __init__(self, t):
        self.base = t.data_ptr()
        self.step = t.stride(0) * t.element_size()

    def __getitem__(self, i):
        return self.base + i * self.step


def _rows(t):
    return t if isinstance(t, _Rows) else _Rows(t)


def theta_subtract(cell, g_cur, mem, npix, g_theta, stream):
    """Subtract-reset cells (``hard_reset=False``): the threshold's gradient through the reset term
    of v = beta*m + I - r*theta (snn.Leaky, r detached), -sum [m > theta] * dL/dv, added to
    g_theta after the fused LIF backward has written the zero-reset part.  g_cur / mem: device
    pointers (NHWC); no-op for zero-reset cells or a step without an incoming membrane."""
    if cell.lif.reset_mechanism != "subtract" or mem is None:
        return
    dev = cell.lif.threshold.device
    scratch = torch.empty(_lib.THETA_SCRATCH, device=dev)  # stream-ordered reuse by the caching allocator
    _lib.call("lif_theta_subtract", lib.snnflow_lif_theta_subtract, _ptr_t(g_cur), _ptr_t(mem),
              ptr(cell.lif.threshold), npix, cell.hidden_size, g_theta, ptr(scratch), stream)


# ---------------------------------------------------------------------------
# Kernel arguments of one time step (shared by the per-step and the sequence Functions)
# ---------------------------------------------------------------------------
def _fwd_conv_args(eng, l, B, H, W, cin0, x, ys, stats, states, mem_in, s_prev, facc, neurons, train, wfwd, wbwd):
    """Forward kernel K_l (l < L) of one step: conv(head) for l == 0, else LIF(l-1) on the
    halo + conv(l).  facc[l]: layer l's BatchNorm batch-sum accumulator."""
    ys, stats, facc = _rows(ys), _rows(stats), _rows(facc)
    a = _lib.ConvFwdArgs()
    a.B, a.H, a.W, a.c = B, H, W, eng.C
    if l == 0:
        a.cin, a.lif_in = cin0, 0
        a.x = ptr(x)
        a.xs_b, a.xs_c, a.xs_h, a.xs_w = _x_strides(x)
    else:
        a.cin, a.lif_in = eng.C, 1
        a.prev_y, a.prev_mem = ys[l - 1], _ptr_t(mem_in[l - 1])
        a.prev_acc, a.prev_stats = facc[l - 1], stats[l - 1]
        a.prev, a.prev_state = neurons[l - 1], ptr(states[l - 1])
    a.wt_ff, a.wt_rec = ptr(wfwd[l][0]), ptr(wfwd[l][1])
    a.wt_ff_t, a.wt_rec_t = ptr(wbwd[l][0]), ptr(wbwd[l][1])  # MFMA B operand layout
    a.s_prev = _ptr_t(s_prev[l])
    a.y, a.acc = ys[l], (facc[l] if train[l] else None)
    fr = getattr(eng, "frags", None)
    if fr is not None:  # pre-split bf16 fragments of the spike convs (C = 16, 32)
        a.wf_ff, a.wf_rec = _ptr_t(fr[l][0]), _ptr_t(fr[l][1])
    return a


def _fwd_top_args(eng, B, H, W, ys, stats, states, mem_in, facc, neurons, flow):
    """Forward kernel K_L of one step: LIF of the last layer + pred."""
    L = eng.L
    ys, stats, facc = _rows(ys), _rows(stats), _rows(facc)
    f = _lib.LifFwdArgs()
    f.B, f.H, f.W, f.c = B, H, W, eng.C
    f.y, f.mem, f.acc, f.stats = ys[L - 1], _ptr_t(mem_in[L - 1]), facc[L - 1], stats[L - 1]
    f.n, f.state = neurons[L - 1], ptr(states[L - 1])
    f.pred_w, f.pred_b, f.flow = ptr(eng.pred.weight), ptr(eng.pred.bias), ptr(flow)
    return f


def _bwd_top_args(eng, B, H, W, ys, stats, mem_in, neurons, gst, g_flow, flow, gcur, gmem, bacc):
    """Backward kernel of the top of one step: pred backward + LIF backward of layer L-1.
    g_flow: dL/dflow with unit W and channel-plane strides, or None."""
    top = eng.L - 1
    ys, stats, gcur, bacc = _rows(ys), _rows(stats), _rows(gcur), _rows(bacc)
    b = _lib.LifBwdArgs()
    b.B, b.H, b.W, b.c = B, H, W, eng.C
    b.y, b.mem, b.stats, b.n = ys[top], _ptr_t(mem_in[top]), stats[top], neurons[top]
    b.g_state = _ptr_t(gst[top])
    b.pred_w, b.flow = ptr(eng.pred.weight), ptr(flow)
    if g_flow is not None:
        b.g_flow, b.gflow_sb, b.gflow_sc = ptr(g_flow), g_flow.stride(0), g_flow.stride(1)
    b.g_cur, b.g_mem = gcur[top], _ptr_t(gmem[top])
    b.acc = bacc[top]
    return b


def _bwd_layer_args(eng, l, B, H, W, cin0, ys, stats, mem_in, neurons, gst, gcur, gmem, bacc, bnc, glayers, gpw, gpb,
                    acc, wfwd, wbwd, g_prev, ext, gx):
    """Backward kernel of layer l of one step: BN backward + dgrad of layer l's convs
    [+ LIF backward of layer l-1]; gx: input gradient of the head (l == 0) or None."""
    C, L = eng.C, eng.L
    ys, stats, gcur, bacc, bnc = _rows(ys), _rows(stats), _rows(gcur), _rows(bacc), _rows(bnc)
    a = _lib.LayerBwdArgs()
    a.B, a.H, a.W, a.c = B, H, W, C
    a.y, a.stats, a.g_cur, a.acc_in, a.n = ys[l], stats[l], gcur[l], bacc[l], neurons[l]
    a.ng, a.accumulate, a.bnc_out = glayers[l][2], acc, bnc[l]
    if l == L - 1:
        a.has_pred, a.g_pred_w, a.g_pred_b = 1, gpw, gpb
    if eng.rec[l]:
        a.wt_bwd_rec, a.wt_fwd_rec = ptr(wbwd[l][1]), ptr(wfwd[l][1])
        if g_prev[l] is not None:
            a.g_state_prev = ptr(g_prev[l])
            a.zero_mem_half = 0 if ext[l] else 1
    fb = getattr(eng, "fragsb", None)
    if fb is not None:  # pre-split bf16 fragments of the input-gradient convs (C = 16, 32)
        a.wd_ff, a.wd_rec = _ptr_t(fb[l][0]), _ptr_t(fb[l][1])
    if l > 0:
        a.cin, a.lif_in = C, 1
        a.wt_bwd_ff, a.wt_fwd_ff = ptr(wbwd[l][0]), ptr(wfwd[l][0])
        a.prev_y, a.prev_mem, a.prev_stats, a.prev = ys[l - 1], _ptr_t(mem_in[l - 1]), stats[l - 1], neurons[l - 1]
        a.prev_g_state = _ptr_t(gst[l - 1])
        a.prev_g_cur, a.prev_g_mem = gcur[l - 1], _ptr_t(gmem[l - 1])
        a.acc_out = bacc[l - 1]
    else:
        a.cin, a.lif_in = cin0, 0
        if gx is not None:
            a.wt_bwd_ff, a.wt_fwd_ff = ptr(wbwd[0][0]), ptr(wfwd[0][0])
            a.g_x = ptr(gx)
            a.gxs_b, a.gxs_c, a.gxs_h, a.gxs_w = _x_strides(gx)
    return a


def _fwd_step_kernels(eng, B, H, W, cin0, x, ys, stats, states, mem_in, s_prev, flow, ws, wfwd, wbwd, s):
    """The L+1 forward kernels of one step launched one by one (what snnflow_firenet_fwd does)."""
    L = eng.L
    neurons = eng.neurons()
    train = [bn.training or not bn.track_running_stats for bn in eng.bns]
    facc = _Rows(ws.fwd_acc)
    zn = ws.fwd_acc.shape[1]
    ys, stats = _Rows(ys), _Rows(stats)
    # K0: conv(head)  (zeroes fwd_acc[L-1], consumed by the previous step's last kernel)
    # K_l: LIF(l-1) on the halo + conv(l)  (zeroes fwd_acc[l-2], consumed by K_{l-1})
    for l in range(L):
        a = _fwd_conv_args(eng, l, B, H, W, cin0, x, ys, stats, states, mem_in, s_prev, facc, neurons, train, wfwd,
                           wbwd)
        if l == 0:
            a.zero0, a.zero_n = facc[L - 1], zn
        elif l >= 2:
            a.zero0, a.zero_n = facc[l - 2], zn
        _lib.call(f"conv_fwd[{l}]" if l else "conv_fwd[0]", lib.snnflow_conv_fwd, ctypes.byref(a), s)
    # K_L: LIF of the last layer + pred  (zeroes fwd_acc[L-2])
    f = _fwd_top_args(eng, B, H, W, ys, stats, states, mem_in, facc, neurons, flow)
    if L >= 2:
        f.zero0, f.zero_n = facc[L - 2], zn
    _lib.call("lif_fwd", lib.snnflow_lif_fwd, ctypes.byref(f), s)


class ParamAnchor(torch.autograd.Function):
    """One autograd node standing for all parameters of a FireNet model within one BPTT chain.

    Every FireNetStep of the chain takes the anchor instead of the ~32 parameter tensors (the
    per-call cost of an autograd Function grows with its inputs); the chain's root step returns
    the engine's flat gradient buffer as the anchor's gradient, and this node hands out
    per-parameter views of it -- fresh views, no other reference, which AccumulateGrad adopts as
    ``.grad`` without a copy (all gradients then live in one flat buffer, dp.flat_grad_buffer)."""

    @staticmethod
    def forward(ctx, eng, *params):
        ctx.layout = eng.flat_layout_for(params)
        ctx.set_materialize_grads(False)
        return torch.empty(ctx.layout[-1][0] + ctx.layout[-1][1], device=params[0].device)

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return (None,) * (1 + len(ctx.layout))
        return (None, *[g[o:o + n].view(shp) if ctx.needs_input_grad[1 + i] else None
                        for i, (o, n, shp) in enumerate(ctx.layout)])


class FireNetStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, eng, x, *rest):
        L, C = eng.L, eng.C
        prev = list(rest[:L])
        B, cin0, H, W = x.shape
        dev = x.device
        _lib.require_device(x, "event tensor")
        s = _lib.stream_ptr(dev)
        # one allocation per step: the L states back to back (a state hand-over, e.g. the bench's
        # graph-replay detach, is then a single contiguous copy), then the pre-BN currents, the flow
        # and the statistics (views; the per-window loop pays one allocator call instead of four)
        n1 = 2 * B * H * W * C
        ny = L * B * H * W * C
        buf = torch.empty(L * n1 + ny + 2 * B * H * W + L * 2 * C, device=dev)
        st_all = buf[:L * n1]
        ys = buf[L * n1:L * n1 + ny].view(L, B, H, W, C)
        flow = buf[L * n1 + ny:L * n1 + ny + 2 * B * H * W].view(B, 2, H, W)
        stats = buf[L * n1 + ny + 2 * B * H * W:].view(L, 2, C)
        # [L][2][B][H][W][C] storage as L states [2, B, C, H, W] (nhwc_state_strides), in one unbind
        states = list(st_all.view(L, 2, B, H, W, C).permute(0, 1, 2, 5, 3, 4).unbind(0))

        # incoming membranes / previous spikes as pointers; `keep` holds their tensors (the whole
        # previous state, or the cell's membrane cache) for the backward and the deferred wgrad
        mem_in, s_prev, keep = [], [], []
        half = 4 * (n1 // 2)
        root = True
        chain = None
        ext = [False] * L  # prev state requiring grad that this engine did not produce
        for l in range(L):
            p = prev[l]
            if p is None:
                cache = eng.lifs[l].mem
                ok = cache is not None and cache.shape == (B, C, H, W) and cache.device == dev
                mem_in.append(cache.data_ptr() if ok else None)
                s_prev.append(None)
                keep.append(cache if ok else None)
            else:
                pn = as_nhwc_state(p)
                base = pn.data_ptr()
                mem_in.append(base)
                s_prev.append(base + half if eng.rec[l] else None)
                keep.append(pn)
                ours = getattr(p.grad_fn, "eng", None) is eng
                if eng.rec[l] and p.requires_grad and ours:
                    root = False
                    chain = chain or getattr(p.grad_fn, "chain", None)
                ext[l] = p.requires_grad and not ours
        # the BPTT chain of this step: a new one at its first step (root); the chain's backwards can be
        # batched if no step needs an event-tensor gradient and only the first step sees external states
        if root:
            chain = _Chain(eng.defer_backward and not x.requires_grad and eng.sequence_ok(cin0))
        elif chain is None:  # continues a forward_sequence window: per-step backwards
            chain = _Chain(False)
        elif x.requires_grad or any(ext) or chain.last is None or any(
                p is None or mem_in[l] != chain.last + 4 * l * n1 for l, p in enumerate(prev)):
            # the batched form reads step t's incoming states as step t-1's output states
            chain.defer = False
        # workspace, prepared weights and the step driver's plan: validated at the chain's first step
        # (and whenever the shapes, the stream or the engine's state changed), then reused by its later
        # steps -- the per-call re-validation of the cached parameter / neuron / weight state was most of
        # the per-window loop's host time.  Still checked per step: the weights' version counters (an
        # in-place edit re-prepares), the train / eval mode and the engine generation (invalidate()).
        ckey = (B, H, W, cin0, dev, s, tuple(bn.training for bn in eng.bns))
        cc = chain.cached
        if not root and cc is not None and cc[0] == ckey and not eng.prep_stale and _lib.TIMER is None \
                and cc[5] == eng.__dict__.get("_gen") and cc[6] == eng.prep.gen \
                and cc[7] == eng.prep.weight_version() and cc[1] is eng.ws:
            ws, wfwd, wbwd, plan = cc[1:5]
        else:
            ws = eng.workspace(B, H, W, dev)
            wfwd, wbwd = eng.prep_weights(s, refresh=eng.prep_stale)
            eng.prep_stale = False
            plan = None if _lib.TIMER is not None else eng.plan(B, H, W, cin0, ws, wfwd, wbwd)
            chain.cached = (ckey, ws, wfwd, wbwd, plan, eng.__dict__.get("_gen"), eng.prep.gen,
                            eng.prep.weight_version())
        ys_t, stats_t = ys, stats
        try:
            if plan is not None:  # one call of the C step driver
                io = _lib.FireNetFwdIo()
                io.x = x.data_ptr()
                io.xs[0], io.xs[1], io.xs[2], io.xs[3] = x.stride()
                io.ys, io.stats, io.states, io.flow = ys.data_ptr(), stats.data_ptr(), st_all.data_ptr(), flow.data_ptr()
                for l in range(L):
                    io.mem_in[l] = mem_in[l]
                    io.s_prev[l] = s_prev[l]
                _lib.call("firenet_fwd", lib.snnflow_firenet_fwd, ctypes.byref(plan), ctypes.byref(io), s)
            else:  # per-kernel launches (KernelTimer attribution): the same kernels and arguments
                _fwd_step_kernels(eng, B, H, W, cin0, x, ys, stats, states, mem_in, s_prev, flow, ws, wfwd, wbwd, s)
        except Exception:
            ws.reset_acc()
            raise

        mst = (H * W * C, 1, W * C, C)
        for l in range(L):  # snn.Leaky's membrane cache, materialised on first read (cells.Leaky.mem)
            eng.lifs[l].__dict__["_mem_lazy"] = (st_all, (B, C, H, W), mst, l * n1)

        chain.last = st_all.data_ptr()
        ctx.eng = eng
        ctx.root = root
        ctx.chain = chain
        # (deferred backward) the incoming recurrent states a caller may read the gradient of, and the
        # chain's parameter anchor, whose node runs only in backward passes that want parameter gradients
        ctx.prev_rec = [p for l, p in enumerate(prev) if p is not None and eng.rec[l] and p.requires_grad]
        ctx.anchor_fn = getattr(rest[L], "grad_fn", None) if len(rest) > L else None
        ctx.ext = ext
        ctx.shape = (B, H, W, cin0)
        ctx.has_prev = [p is not None for p in prev]
        ctx.keep = [k is not None for k in keep]
        ctx.ptrs = (mem_in, s_prev)
        saved = [x, ys_t, stats_t, flow] + states
        saved += [k for k in keep if k is not None]
        ctx.save_for_backward(*saved)
        ctx.set_materialize_grads(False)
        return (flow, *states)

    @staticmethod
    def backward(ctx, g_flow, *g_states):
        eng, chain = ctx.eng, ctx.chain
        eng.drop_stale_chain()
        st = _StepBwd(ctx, g_flow, g_states)
        if chain.defer:
            if chain.steps and chain.steps[0].task != st.task:  # left by an earlier pass that stopped early
                chain.steps = []
            if not ctx.root:
                if _defer_ok(ctx):  # collected; the chain's first step (the last node autograd calls) runs them
                    chain.steps.append(st)
                    return (None,) * (3 + eng.L)
                # the gradient of this step's incoming states is read (retain_grad, a hook), or this pass will
                # not reach the chain's first step (autograd.grad / backward(inputs=...) of an intermediate
                # state): this step and the later ones collected so far run now, one after the other, and
                # return their input gradients to autograd
                steps = [st] + chain.steps[::-1]
                chain.steps = []
                return _chain_backward(eng, steps, batched=False)
            steps = [st] + chain.steps[::-1]  # time order
            chain.steps = []
            if len(steps) > 1:
                return _chain_backward(eng, steps)
        return _step_backward(eng, st)


def _defer_ok(ctx):
    """May a non-first step of a chain hand its backward to the chain's first step?  Not when a caller
    reads the gradient of one of its incoming recurrent states (retain_grad or a tensor hook: the
    batched form never hands those to autograd), and not when this backward pass will not run the
    parameter anchor's node (no parameter gradients wanted: autograd.grad or backward(inputs=...) of an
    intermediate state -- the first step may then never run)."""
    for p in ctx.prev_rec:
        if p.retains_grad or p._backward_hooks:
            return False
    a = ctx.anchor_fn
    return a is None or torch._C._will_engine_execute_node(a)


class _Chain:
    """The BPTT chain of FireNetStep nodes linked by this engine's recurrent states (one truncated
    window of the reference loop, train_flow.py:232-262: T model() calls, one loss.backward()).  With
    ``defer`` the later steps' nodes only record their backward inputs (``steps``) and the chain's first
    step -- the last node autograd calls -- issues every step's backward at once (_chain_backward)."""
    __slots__ = ("defer", "steps", "last", "cached")

    def __init__(self, defer):
        self.defer = defer
        self.steps = []
        self.last = None  # the latest step's state allocation (its L output states back to back)
        self.cached = None  # (key, workspace, prepared weights fwd / bwd, plan, engine generation, prep generation)


class _StepBwd:
    """One FireNetStep's backward inputs, unpacked from its ctx (autograd frees a node's saved tensors
    once its backward returns; these references keep them for the chain's first step)."""
    __slots__ = ("saved", "ptrs", "shape", "root", "ext", "has_prev", "needs", "g_flow", "g_states", "task")

    def __init__(self, ctx, g_flow, g_states):
        self.task = torch._C._current_graph_task_id()
        self.saved = list(ctx.saved_tensors)
        self.ptrs, self.shape, self.root, self.ext = ctx.ptrs, ctx.shape, ctx.root, ctx.ext
        self.has_prev, self.needs = ctx.has_prev, ctx.needs_input_grad
        self.g_flow, self.g_states = g_flow, g_states


def _chain_backward(eng, steps, batched=True):
    """The backwards of a chain's steps (time order; steps[0] is the chain's first step), issued by the
    first step's node.  Without external gradients on intermediate states, one snnflow_firenet_bwd_seq
    call: the T x (L+1) layer-steps as 2(T-1)+L+1 wavefront launches (FireNetSequence's schedule and
    kernels, the per-step tensors read in place).  Otherwise, or under per-kernel timing, the steps'
    backwards one after the other (last first), each step's state-input gradient added to the external
    gradient of the previous step's states -- what autograd would have summed.  Returns the first
    step's input gradients."""
    L = eng.L
    T = len(steps)
    B, H, W, _ = steps[0].shape
    n1 = 2 * B * H * W * eng.C
    for t in range(1, T):  # step t reads step t-1's states (one allocation, L states back to back)
        base = steps[t - 1].saved[4].data_ptr()
        if any(steps[t].ptrs[0][l] != base + 4 * l * n1 for l in range(L)):
            eng.drop_stale_chain()
            raise _lib.SnnflowError("deferred chain backward: the collected steps are not one BPTT chain "
                                    "(set model.engine.defer_backward = False for this use)")
    if batched and _lib.TIMER is None and all(g is None for st in steps[:-1] for g in st.g_states):
        return _chain_backward_batched(eng, steps)
    nxt = None
    for t in range(T - 1, -1, -1):
        st = steps[t]
        gs = list(st.g_states)
        if nxt is not None:
            gs = [a if b is None else (b if a is None else a + b) for a, b in zip(gs, nxt)]
        res = _step_backward(eng, st, gs)
        nxt = res[2:2 + L]
    return res


def _chain_backward_batched(eng, steps):
    L, C = eng.L, eng.C
    T = len(steps)
    first = steps[0]
    B, H, W, cin0 = first.shape
    dev = first.saved[0].device
    s = _lib.stream_ptr(dev)
    ws = eng.workspace(B, H, W, dev)
    wfwd, wbwd = eng.prepped()
    plan = eng.plan(B, H, W, cin0, ws, wfwd, wbwd)
    fresh = not eng.bwd_open
    if fresh:
        eng.open_chain(dev)
    glayers, gpw, gpb = eng.grad_views()
    npix = B * H * W
    nrec = sum(1 for r in eng.rec if r)
    nacc = _lib.acc_storage(_lib.bwd_acc_len(C))
    # one allocation: [T][L] g_cur, [T][L][2][C] bnc, (T-1) x recurrent-layer state gradients (spike half
    # written, the membrane half never read inside the chain)
    ng_, nb_, no_ = T * L * npix * C, T * L * 2 * C, (T - 1) * nrec * 2 * npix * C
    buf = torch.empty(ng_ + nb_ + no_, device=dev)
    gcur, bnc = buf[:ng_].view(T, L, B, H, W, C), buf[ng_:ng_ + nb_].view(T, L, 2, C)
    bacc = torch.zeros(T * L * nacc, dtype=torch.float64, device=dev)
    g0 = [None] * L
    for l in range(L):
        if not (first.has_prev[l] and first.needs[2 + l]):
            continue
        if first.ext[l]:
            g0[l] = torch.zeros((2, B, C, H, W), device=dev).as_strided(
                (2, B, C, H, W), (B * H * W * C, H * W * C, 1, W * C, C))
        elif eng.rec[l]:
            g0[l] = empty_state(B, C, H, W, dev)
    q = _lib.FireNetSeqBwd()
    q.T, q.fresh = T, 1 if fresh else 0
    fuse = bool(eng.fuse_wgrad) and C == 8
    q.fused = 1 if fuse else 0
    xs0 = [st.saved[0] for st in steps]
    fuse_head = (bool(eng.fuse_head) and not eng.rec[0] and cin0 in (2, 4)
                 and all(x.dim() == 4 and x.dtype == torch.float32 for x in xs0))
    q.fuse_head = 1 if fuse_head else 0
    if fuse_head:
        for t, x in enumerate(xs0):
            q.x[t] = x.data_ptr()
            q.xs[t][0], q.xs[t][1], q.xs[t][2], q.xs[t][3] = _x_strides(x)
    q.ys[:T] = [st.saved[1].data_ptr() for st in steps]
    q.stats[:T] = [st.saved[2].data_ptr() for st in steps]
    q.flow[:T] = [st.saved[3].data_ptr() for st in steps]
    q.states[:T] = [st.saved[4].data_ptr() for st in steps]  # (the step's L states: one allocation)
    gfl = []
    for t, st in enumerate(steps):
        g = st.g_flow
        if g is not None:
            if g.stride(3) != 1 or g.stride(2) != W or g.dtype != torch.float32:
                g = g.contiguous().float()
            q.g_flow[t], q.gflow_sb[t], q.gflow_sc[t] = g.data_ptr(), g.stride(0), g.stride(1)
        gfl.append(g)
    mem0, sp0 = first.ptrs
    gl = [as_nhwc_state(g) if g is not None else None for g in steps[-1].g_states]
    for l in range(L):
        q.mem_in0[l], q.s_prev0[l], q.g_prev0[l] = mem0[l], sp0[l], _ptr_t(g0[l])
        q.ext0[l] = 1 if first.ext[l] else 0
        q.g_state_last[l] = _ptr_t(gl[l])
        q.ng[l] = glayers[l][2]
    q.g_out = buf.data_ptr() + 4 * (ng_ + nb_) if no_ else None
    q.g_cur, q.bnc = gcur.data_ptr(), bnc.data_ptr()
    q.bwd_acc, q.acc_stride = bacc.data_ptr(), nacc
    q.g_pred_w, q.g_pred_b = gpw, gpb
    live = (ctypes.c_int * L)(*[1 if v else 0 for v in eng.slab_live])
    try:
        _lib.call("firenet_bwd_seq", lib.snnflow_firenet_bwd_seq, ctypes.byref(plan), ctypes.byref(q), live, s)
        eng.slab_live = [bool(v) for v in live]
        if eng.any_subtract():
            for t, st in enumerate(steps):
                for l in range(L):
                    theta_subtract(eng.cells[l], gcur[t][l].data_ptr(), st.ptrs[0][l], B * H * W,
                                   glayers[l][2].threshold, s)
        # the deferred weight gradients (layer 0 with the fused form) see the steps last first
        for t in range(T - 1, -1, -1):
            st = steps[t]
            x, ys, stats = st.saved[:3]
            eng.pending.append((_Rows(gcur[t]), _Rows(bnc[t]), _Rows(ys), _Rows(stats), x, st.saved[4:4 + L],
                                st.ptrs[1], (st.saved, buf), None))
            eng.pending_layers.append(tuple(l for l in range(L) if not ((fuse and l > 0) or (fuse_head and l == 0))))
        eng.flush_weight_grads(B, H, W, cin0, ws, glayers, s, plan)
    except Exception:
        eng.ws.reset_acc()
        eng.bwd_open = False
        eng.pending, eng.pending_layers = [], []
        eng.prep_stale = True
        raise
    g_anchor = eng.flat if first.needs[2 + L] else None
    eng.flat_views = None
    eng.bwd_open = False
    eng.last_flat = eng.flat
    eng.prep_stale = True
    del gfl
    return (None, None, *g0, g_anchor)


def _step_backward(eng, ctx, g_states=None):
    """One step's backward (snnflow_firenet_bwd), ``ctx`` a _StepBwd; g_states overrides its state
    gradients (the chain's sequential form)."""
    g_flow = ctx.g_flow
    if g_states is None:
        g_states = ctx.g_states
    L, C = eng.L, eng.C
    B, H, W, cin0 = ctx.shape
    saved = ctx.saved
    x, ys, stats, flow = saved[:4]
    states = saved[4:4 + L]
    keep = saved[4 + L:]  # tensors behind the mem_in / s_prev pointers (alive while saved here)
    mem_in, s_prev = ctx.ptrs

    dev = x.device
    s = _lib.stream_ptr(dev)
    ws = eng.workspace(B, H, W, dev)
    wfwd, wbwd = eng.prepped()  # the buffers of the forward (same weights)
    if not eng.bwd_open:
        eng.open_chain(dev)
        acc = 0
    else:
        acc = 1
    glayers, gpw, gpb = eng.grad_views()
    neurons = eng.neurons()
    bacc = _Rows(ws.bwd_acc)
    zn = ws.bwd_acc.shape[1]
    gst = [as_nhwc_state(g) if g is not None else None for g in g_states]
    # gradients of the previous states: the spike half of recurrent cells (rec dgrad);
    # for states that did not come from this engine also the membrane half
    # (v depends on the incoming membrane, SNNtorch_spiking_submodules.py:305 / snn.Leaky).
    g_prev = [None] * L
    for l in range(L):
        if not (ctx.has_prev[l] and ctx.needs[2 + l]):
            continue
        if ctx.ext[l]:
            g_prev[l] = torch.zeros((2, B, C, H, W), device=dev).as_strided(
                (2, B, C, H, W), (B * H * W * C, H * W * C, 1, W * C, C))
        elif eng.rec[l]:
            g_prev[l] = empty_state(B, C, H, W, dev)
    gmem = [g_prev[l] if (g_prev[l] is not None and ctx.ext[l]) else None for l in range(L)]

    # per-step buffers kept until the deferred weight gradients run (root step)
    gcur_t = torch.empty(L, B, H, W, C, device=dev)   # dL/d BN-output of every layer
    bnc_t = torch.empty(L, 2, C, device=dev)           # BN backward coefficients (grad_mean, k)
    gcur, bnc, ys, stats = _Rows(gcur_t), _Rows(bnc_t), _Rows(ys), _Rows(stats)
    # pending: row pointers for the deferred wgrad + the tensors behind them (kept alive)
    eng.pending.append((gcur, bnc, ys, stats, x, states, s_prev, (keep, gcur_t, bnc_t, saved), None))
    eng.pending_layers.append(tuple(range(L)))
    # (the deferred weight gradients stay on this stream after the chain: a side stream
    # overlapping them with the root step's chain measured slower under graph replay,
    # 2.48 -> 2.72 ms per cfg2 train step)
    try:
        if g_flow is not None and (g_flow.stride(3) != 1 or g_flow.stride(2) != W or g_flow.dtype != torch.float32):
            g_flow = g_flow.contiguous().float()
        gx = None
        if ctx.needs[1]:
            gx = torch.empty_like(x)
        plan = None if _lib.TIMER is not None else eng.plan(B, H, W, cin0, ws, wfwd, wbwd)
        if plan is not None:  # one call of the C step driver
            io = _lib.FireNetBwdIo()
            io.ys, io.stats, io.flow = ys.base, stats.base, flow.data_ptr()
            for l in range(L):
                io.mem_in[l] = mem_in[l]
                io.g_state[l] = _ptr_t(gst[l])
                io.g_prev[l] = _ptr_t(g_prev[l])
                io.ext[l] = 1 if ctx.ext[l] else 0
                io.ng[l] = glayers[l][2]
            if g_flow is not None:
                io.g_flow, io.gflow_sb, io.gflow_sc = g_flow.data_ptr(), g_flow.stride(0), g_flow.stride(1)
            io.g_cur, io.bnc = gcur.base, bnc.base
            if gx is not None:
                io.g_x = gx.data_ptr()
                io.gxs[0], io.gxs[1], io.gxs[2], io.gxs[3] = gx.stride()
            io.g_pred_w, io.g_pred_b, io.accumulate = gpw, gpb, acc
            _lib.call("firenet_bwd", lib.snnflow_firenet_bwd, ctypes.byref(plan), ctypes.byref(io), s)
        else:  # per-kernel launches (KernelTimer attribution): the same kernels and arguments
            # top: pred backward + LIF backward of layer L-1  (zeroes bwd_acc[0])
            b = _bwd_top_args(eng, B, H, W, ys, stats, mem_in, neurons, gst, g_flow, flow, gcur, gmem, bacc)
            b.zero0, b.zero_n = bacc[0], zn
            _lib.call("lif_bwd", lib.snnflow_lif_bwd, ctypes.byref(b), s)
            for l in range(L - 1, -1, -1):
                a = _bwd_layer_args(eng, l, B, H, W, cin0, ys, stats, mem_in, neurons, gst, gcur, gmem, bacc, bnc,
                                    glayers, gpw, gpb, acc, wfwd, wbwd, g_prev, ctx.ext, gx)
                if l + 1 <= L - 1:
                    a.zero0, a.zero_n = bacc[l + 1], zn
                _lib.call(f"layer_bwd[{l}]", lib.snnflow_layer_bwd, ctypes.byref(a), s)
        if eng.any_subtract():
            for l in range(L):
                theta_subtract(eng.cells[l], gcur[l], mem_in[l], B * H * W, glayers[l][2].threshold, s)
        if ctx.root:
            eng.flush_weight_grads(B, H, W, cin0, ws, glayers, s, plan)
    except Exception:
        ws.reset_acc()
        eng.bwd_open = False
        eng.pending, eng.pending_layers = [], []
        eng.prep_stale = True
        raise

    g_anchor = None
    if ctx.root:
        # the whole flat gradient buffer to the chain's parameter anchor (ParamAnchor splits it
        # into per-parameter views once every step of the chain is done)
        g_anchor = eng.flat if ctx.needs[2 + L] else None
        eng.flat_views = None
        eng.bwd_open = False
        eng.last_flat = eng.flat
        eng.prep_stale = True
    return (None, gx, *g_prev, g_anchor)


def _ptr_t(t):
    """Device pointer of a tensor, an int pointer passed through, None -> NULL."""
    if t is None or isinstance(t, int):
        return t
    return t.data_ptr()


# ---------------------------------------------------------------------------
# A whole truncated-BPTT window in one autograd node, launched in wavefront order
# ---------------------------------------------------------------------------
def wavefront_slots(T, K):
    """Launch order of a (kernel k < K, step t < T) grid whose task (k, t) reads the outputs of
    (k-1, t), (k, t-1) and (k+1, t-1) (the spikes of a recurrent layer come out of the next
    kernel of the previous step): task (k, t) runs in launch k + 2t, so every launch holds
    mutually independent tasks and follows all of its inputs' launches.
    Returns [[(k, t), ...] per launch]."""
    slots = [[] for _ in range(K + 2 * (T - 1))]
    for t in range(T):
        for k in range(K):
            slots[k + 2 * t].append((k, t))
    return slots


def _state_rows(st_all, fin, T):
    """Flat per-step state rows of a FireNetSequence call: st_all's rows, the last one replaced by
    the caller's final_state_out buffer when there is one (st_all then has T - 1 rows)."""
    rows = [st_all[t] for t in range(st_all.shape[0])]
    return rows + [fin] if fin is not None else rows


class FireNetSequence(torch.autograd.Function):
    """T fused time steps of the network as one autograd node (``forward_sequence``).

    Same arithmetic per (layer, step) as T FireNetStep calls; the L+1 kernels of every step are
    issued as wavefront launches (``wavefront_slots``, ``snnflow_fwd_slot`` /
    ``snnflow_bwd_slot``) that each run up to four independent layer-steps: a single
    layer-step of C = 8 at 128x128 occupies the chip for one latency-bound block round, so
    the (L+1) x T launches of the per-step path are replaced by 2(T-1)+L+1.  Batch-sum
    accumulators are per (step, layer) and zeroed once per call.  Inputs: eng, T, x_0..x_{T-1},
    initial states (L), parameters; outputs: flow_0..flow_{T-1}, final states (L)."""

    @staticmethod
    def forward(ctx, eng, T, *rest):
        L, C = eng.L, eng.C
        xs = list(rest[:T])
        prev = list(rest[T:T + L])
        B, cin0, H, W = xs[0].shape
        dev = xs[0].device
        for x in xs:
            _lib.require_device(x, "event tensor")
            if tuple(x.shape) != (B, cin0, H, W):
                raise _lib.SnnflowError("forward_sequence: every step's input must have the same shape")
        s = _lib.stream_ptr(dev)
        ws = eng.workspace(B, H, W, dev)
        # the batch-sum accumulators of this forward (facc) and of its backward (bacc), one fp64
        # allocation zeroed by the weight-preparation launch
        nf, nb = T * L * _lib.acc_storage(2 * C), T * L * _lib.acc_storage(_lib.bwd_acc_len(C))
        accs = torch.empty(nf + nb, dtype=torch.float64, device=dev)
        facc = accs[:nf].view(T, L, -1)
        ctx.bacc = accs[nf:].view(T, L, -1)
        wfwd, wbwd = eng.prep_weights(s, refresh=eng.prep_stale, zero=accs)
        eng.prep_stale = False
        cells = eng.cells

        ys = torch.empty(T, L, B, H, W, C, device=dev)
        stats = torch.empty(T, L, 2, C, device=dev)
        n1 = 2 * B * H * W * C
        fin = eng.final_state_out
        eng.final_state_out = None
        if fin is not None:
            if (fin.device != dev or fin.dtype != torch.float32 or fin.numel() != L * n1 or not fin.is_contiguous()
                    or any(p is not None and p.untyped_storage().data_ptr() == fin.untyped_storage().data_ptr()
                           for p in prev)):
                raise _lib.SnnflowError("final_state_out: a contiguous fp32 buffer of L*2*B*H*W*C floats on the "
                                        "input's device, not aliasing the initial states")
            fin = fin.view(L * n1)
        st_all = torch.empty(T - (fin is not None), L * n1, device=dev)
        rows = _state_rows(st_all, fin, T)
        states = [[rows[t][l * n1:(l + 1) * n1].as_strided((2, B, C, H, W), nhwc_state_strides(B, C, H, W))
                   for l in range(L)] for t in range(T)]
        flows = [torch.empty(B, 2, H, W, device=dev) for _ in range(T)]

        # step 0 reads the initial states (as FireNetStep); step t > 0 the states of step t-1
        mem0, sprev0 = [], []
        root = True
        ext = [False] * L
        for l in range(L):
            p = prev[l]
            if p is None:
                cache = cells[l].lif.mem
                mem0.append(cache if (cache is not None and tuple(cache.shape) == (B, C, H, W)
                                      and cache.device == dev) else None)
                sprev0.append(None)
            else:
                pn = as_nhwc_state(p)
                mem0.append(pn[0])
                sprev0.append(pn[1] if eng.rec[l] else None)
                ours = getattr(p.grad_fn, "eng", None) is eng
                if eng.rec[l] and p.requires_grad and ours:
                    root = False
                ext[l] = p.requires_grad and not ours
        mem_in = [mem0] + [[states[t - 1][l][0] for l in range(L)] for t in range(1, T)]
        s_prev = [sprev0] + [[states[t - 1][l][1] if eng.rec[l] else None for l in range(L)] for t in range(1, T)]
        neurons = eng.neurons()
        train = [bn.training or not bn.track_running_stats for bn in eng.bns]

        # with the weight gradients fused into the backward (C = 8) the spike half of a feed-forward
        # layer's state at steps t < T-1 is never read (the next step's LIF reads the membrane half,
        # the backward recomputes the spikes, only recurrent layers read s_prev; the deferred weight
        # gradients of the other widths read the spikes), so it is not stored unless the caller
        # keeps every step's states
        fuse = bool(eng.fuse_wgrad)  # decided once: the backward must see the same choice (ctx.fuse)

        # spike bit planes (ABI 39, C = 16 / 32, whose weight gradients are deferred): task l >= 1 of step t
        # writes layer l-1's spikes of step t as one C-bit word per pixel (the top layer's are not
        # written); the recurrent convs at t >= 1 and the deferred weight gradients read those instead of
        # the fp32 spike half of the states.  (C = 8 fuses the weight gradients into the backward, which
        # recomputes the spikes; there the bit planes measured no faster: the recurrent layers' fp32
        # planes stay.)
        bits_on = eng.spk_bits and C in (16, 32) and not fuse
        need_bits = [bits_on and l < L - 1 for l in range(L)]
        bits = (torch.empty(T, L, B * H * W * C // 8, dtype=torch.uint8, device=dev) if any(need_bits)
                else None)
        bptr = [[bits[t, l].data_ptr() if need_bits[l] else None for l in range(L)] for t in range(T)]

        def spk_skip(l, t):
            # the spike half of layer l's state at t < T-1 is read by nobody when its readers take the bit
            # plane, or (fused weight gradients) when the layer is feed-forward: the next step's LIF reads
            # the membrane half and the backward recomputes the spikes
            return t < T - 1 and not eng.keep_seq_states and ((fuse and not eng.rec[l]) or need_bits[l])
        for tasks in wavefront_slots(T, L + 1):
            convs, top = [], None
            for k, t in tasks:
                if k < L:
                    a = _fwd_conv_args(eng, k, B, H, W, cin0, xs[t], ys[t], stats[t], states[t], mem_in[t],
                                       s_prev[t], facc[t], neurons, train, wfwd, wbwd)
                    if k >= 1 and spk_skip(k - 1, t):
                        a.state_spk_skip = 1
                    if k >= 1 and need_bits[k - 1]:
                        a.prev_spk_bits = bptr[t][k - 1]
                    if eng.rec[k] and t >= 1 and need_bits[k]:
                        a.s_prev_bits, a.s_prev = bptr[t - 1][k], None
                    convs.append(a)
                else:
                    top = _fwd_top_args(eng, B, H, W, ys[t], stats[t], states[t], mem_in[t], facc[t], neurons,
                                        flows[t])
                    if spk_skip(L - 1, t):
                        top.state_spk_skip = 1
            arr = (_lib.ConvFwdArgs * max(len(convs), 1))(*convs)
            _lib.call("fwd_slot", lib.snnflow_fwd_slot, arr, len(convs), ctypes.byref(top) if top is not None else None,
                      s)
        _lib.timer_close()

        if eng.capture_states:  # tests / diagnostics: the window's pre-BN currents, statistics, batch sums
            eng.seq_debug = (ys, stats, facc)
        for l in range(L):
            cells[l].lif.mem = states[T - 1][l][0].detach()
        # per-step states for the caller's activity log (forward_sequence(log=True)); views only
        eng.seq_states = [[st.detach() for st in sts] for sts in states] if eng.keep_seq_states else None

        ctx.eng = eng
        ctx.T = T
        ctx.fuse = fuse
        ctx.bptr = bptr
        ctx.bits = bits  # (the backward's readers run before the next forward can reuse it: a plain attribute)
        ctx.root = root
        ctx.ext = ext
        ctx.shape = (B, H, W, cin0)
        ctx.has_prev = [p is not None for p in prev]
        ctx.has_mem = [m is not None for m in mem0]
        saved = xs + flows + [ys, stats, st_all]
        ctx.has_fin = fin is not None
        if fin is not None:
            saved.append(fin)
        saved += [m for m in mem0 if m is not None]
        saved += [sp for sp in sprev0 if sp is not None]
        ctx.save_for_backward(*saved)
        ctx.set_materialize_grads(False)
        return (*flows, *states[T - 1])

    @staticmethod
    def backward(ctx, *grads):
        eng, T = ctx.eng, ctx.T
        L, C = eng.L, eng.C
        B, H, W, cin0 = ctx.shape
        g_flows, g_final = list(grads[:T]), list(grads[T:T + L])
        saved = list(ctx.saved_tensors)
        xs, flows = saved[:T], saved[T:2 * T]
        ys, stats, st_all = saved[2 * T:2 * T + 3]
        rest = saved[2 * T + 3:]
        fin = rest.pop(0) if ctx.has_fin else None
        rows = _state_rows(st_all, fin, T)
        n1 = 2 * B * H * W * C
        states = [[rows[t][l * n1:(l + 1) * n1].as_strided((2, B, C, H, W), nhwc_state_strides(B, C, H, W))
                   for l in range(L)] for t in range(T)]
        mem0 = [rest.pop(0) if ctx.has_mem[l] else None for l in range(L)]
        sprev0 = [rest.pop(0) if (ctx.has_prev[l] and eng.rec[l]) else None for l in range(L)]
        mem_in = [mem0] + [[states[t - 1][l][0] for l in range(L)] for t in range(1, T)]
        s_prev = [sprev0] + [[states[t - 1][l][1] if eng.rec[l] else None for l in range(L)] for t in range(1, T)]

        dev = xs[0].device
        s = _lib.stream_ptr(dev)
        eng.drop_stale_chain()
        eng.workspace(B, H, W, dev)
        ws = eng.ws
        wfwd, wbwd = eng.prep_weights(s, refresh=False)
        fresh = not eng.bwd_open
        if fresh:
            eng.open_chain(dev)
        glayers, gpw, gpb = eng.grad_views()
        neurons = eng.neurons()
        bacc = ctx.bacc  # zeroed in the forward (prep launch); a second backward (retain_graph) gets a fresh one
        ctx.bacc = None
        if bacc is None:
            bacc = torch.zeros(T, L, _lib.acc_storage(_lib.bwd_acc_len(C)), dtype=torch.float64, device=dev)
        gcur = torch.empty(T, L, B, H, W, C, device=dev)
        bnc = torch.empty(T, L, 2, C, device=dev)

        # gradients flowing into the states of step t: from the caller for the last step, from
        # step t+1's recurrent dgrad (spike half; membrane half zero-filled) for the others
        g_into = [None] * T   # g_into[t][l]: dL/d state_t[l]
        g_into[T - 1] = [as_nhwc_state(g) if g is not None else None for g in g_final]
        g_out = [None] * T    # g_out[t][l]: dL/d (state input of step t)[l], written by step t's backward
        for t in range(T - 1, 0, -1):
            g_out[t] = [empty_state(B, C, H, W, dev) if eng.rec[l] else None for l in range(L)]
            g_into[t - 1] = g_out[t]
        g0 = [None] * L
        for l in range(L):
            if not (ctx.has_prev[l] and ctx.needs_input_grad[2 + T + l]):
                continue
            if ctx.ext[l]:
                g0[l] = torch.zeros((2, B, C, H, W), device=dev).as_strided(
                    (2, B, C, H, W), (B * H * W * C, H * W * C, 1, W * C, C))
            elif eng.rec[l]:
                g0[l] = empty_state(B, C, H, W, dev)
        g_out[0] = g0
        ext = [list(ctx.ext)] + [[False] * L for _ in range(T - 1)]  # only step 0 sees external states
        gmem = [[None] * L for _ in range(T)]
        gmem[0] = [g0[l] if (g0[l] is not None and ctx.ext[l]) else None for l in range(L)]
        gxs = [torch.empty_like(xs[t]) if ctx.needs_input_grad[2 + t] else None for t in range(T)]
        gfl = []
        for g in g_flows:
            if g is not None and (g.stride(3) != 1 or g.stride(2) != W or g.dtype != torch.float32):
                g = g.contiguous().float()
            gfl.append(g)

        # the deferred weight gradients see the steps in the per-step path's order (last first)
        # layers >= 1: dW inside the backward slot tasks (wslab_*); the forward's choice (it skipped the
        # spike planes the fused form never reads), not the engine flag's value now
        fuse = ctx.fuse
        # the head's dW inside its backward tasks (ABI 40): a feed-forward 2- / 4-channel head
        fuse_head = (bool(eng.fuse_head) and not eng.rec[0] and cin0 in (2, 4)
                     and all(x.dim() == 4 and x.dtype == torch.float32 for x in xs))
        bptr = ctx.bptr
        for t in range(T - 1, -1, -1):
            eng.pending.append((_Rows(gcur[t]), _Rows(bnc[t]), _Rows(ys[t]), _Rows(stats[t]), xs[t], states[t], s_prev[t],
                                (gcur, bnc, ys, stats, ctx.bits), (bptr[t], bptr[t - 1] if t >= 1 else [None] * L)))
            eng.pending_layers.append(tuple(l for l in range(L) if not ((fuse and l > 0) or (fuse_head and l == 0))))
        try:
            # backward kernel j of step t: j = 0 top (pred + LIF of layer L-1), j >= 1 layer L-j;
            # in reversed time tau = T-1-t the dependencies have the forward's shape: (j-1, tau)
            # (the BN-backward sums of layer L-j), (j, tau-1) (the membrane gradient from step t+1),
            # and (j+1, tau-1) where layer L-j-1 is recurrent (its spikes' gradient from the
            # recurrent dgrad of step t+1)
            for tasks in wavefront_slots(T, L + 1):
                layers, top = [], None
                for j, tau in tasks:
                    t = T - 1 - tau
                    acc = 0 if (fresh and t == T - 1) else 1
                    if j == 0:
                        top = _bwd_top_args(eng, B, H, W, ys[t], stats[t], mem_in[t], neurons, g_into[t], gfl[t],
                                            flows[t], gcur[t], gmem[t], bacc[t])
                    else:
                        l = L - j
                        a = _bwd_layer_args(eng, l, B, H, W, cin0, ys[t], stats[t], mem_in[t], neurons,
                                            g_into[t], gcur[t], gmem[t], bacc[t], bnc[t], glayers, gpw, gpb,
                                            acc, wfwd, wbwd, g_out[t], ext[t], gxs[t] if l == 0 else None)
                        if t > 0:
                            # g_out[t] (t >= 1) stays inside the chain, and its membrane half is never
                            # read (the engine's cells detach the reset: step t-1's kernels read only
                            # the spike half of g_into), so that plane is not zero-filled; step 0's is
                            # returned to autograd and is
                            a.zero_mem_half = 0
                        if fuse_head and l == 0:
                            a.x = xs[t].data_ptr()
                            a.xs_b, a.xs_c, a.xs_h, a.xs_w = _x_strides(xs[t])
                            a.wslab_ff = ws.slab_ff[0].data_ptr()
                            a.wslab_accumulate = 1 if eng.slab_live[0] else 0
                            eng.slab_live[0] = True
                        if fuse and l > 0:
                            a.wslab_ff = ws.slab_ff[l].data_ptr()
                            if eng.rec[l]:
                                a.wslab_rec = ws.slab_rec[l].data_ptr()
                                a.s_prev = _ptr_t(s_prev[t][l])
                            a.wslab_accumulate = 1 if eng.slab_live[l] else 0
                            eng.slab_live[l] = True
                        layers.append(a)
                arr = (_lib.LayerBwdArgs * max(len(layers), 1))(*layers)
                _lib.call("bwd_slot", lib.snnflow_bwd_slot, arr, len(layers),
                          ctypes.byref(top) if top is not None else None, s)
            _lib.timer_close()
            for l in range(L):
                for t in range(T):
                    theta_subtract(eng.cells[l], gcur[t][l], mem_in[t][l], B * H * W, glayers[l][2].threshold, s)
            if ctx.root:
                eng.flush_weight_grads(B, H, W, cin0, ws, glayers, s)
        except Exception:
            ws.reset_acc()
            eng.bwd_open = False
            eng.pending, eng.pending_layers = [], []
            eng.prep_stale = True
            raise

        pgrads = [None] * len(eng.flat_layout)
        if ctx.root:
            pgrads = [eng.flat[o:o + n].view(shp) for o, n, shp in eng.flat_layout]
            eng.flat_views = None
            eng.bwd_open = False
            eng.last_flat = eng.flat
            eng.prep_stale = True
        return (None, None, *gxs, *g0, *pgrads)


def eval_fused_ok(eng, xs, prev=()):
    """True if forward_sequence may take the fused evaluation launches (eval_sequence): C = 8, every
    BatchNorm on running statistics, no autograd needed -- neither the parameters nor any input or
    initial state require grad while grad mode is on (saliency / adversarial evaluation keeps the
    autograd path) --, 2- or 4-bin input on the GPU, and not disabled by SNNFLOW_EVAL_FUSED=0 (the
    train-path split launches then run in eval mode too)."""
    import os
    x = xs[0]
    if os.environ.get("SNNFLOW_EVAL_FUSED", "1") == "0" or eng.C != 8 or not x.is_cuda or x.shape[1] not in (2, 4):
        return False
    if any(bn.training or not bn.track_running_stats for bn in eng.bns):
        return False
    if not torch.is_grad_enabled():
        return True
    return not (any(p.requires_grad for p in eng.param_list()) or any(t.requires_grad for t in xs)
                or any(p is not None and p.requires_grad for p in prev))


def eval_sequence(eng, xs, prev):
    """T steps of the network in evaluation mode (eval_flow.py:208-338 under torch.no_grad(),
    BatchNorm on running statistics) through snnflow_eval_slot: task (l, t) = conv + BatchNorm + LIF
    of layer l at step t (+ the prediction for the last layer) reads layer l-1's spikes at t and its
    own state at t-1, so the T x L tasks run in T + L - 1 wavefront launches.  Same results as the
    train-path kernels in eval mode (forward_sequence with SNNFLOW_EVAL_FUSED=0) up to the conv's
    summation order.  Returns (flows [T], final states [L]); no autograd."""
    L, C = eng.L, eng.C
    T = len(xs)
    B, cin0, H, W = xs[0].shape
    dev = xs[0].device
    for x in xs:
        _lib.require_device(x, "event tensor")
        if tuple(x.shape) != (B, cin0, H, W):
            raise _lib.SnnflowError("forward_sequence: every step's input must have the same shape")
    s = _lib.stream_ptr(dev)
    wfwd, wbwd = eng.prep_weights(s, refresh=eng.prep_stale)
    eng.prep_stale = False
    neurons = eng.neurons()
    n1 = 2 * B * H * W * C
    fin = eng.final_state_out
    eng.final_state_out = None
    if fin is not None:
        if (fin.device != dev or fin.dtype != torch.float32 or fin.numel() != L * n1 or not fin.is_contiguous()
                or any(p is not None and p.untyped_storage().data_ptr() == fin.untyped_storage().data_ptr()
                       for p in prev)):
            raise _lib.SnnflowError("final_state_out: a contiguous fp32 buffer of L*2*B*H*W*C floats on the "
                                    "input's device, not aliasing the initial states")
        fin = fin.view(L * n1)
    st_all = torch.empty(T - (fin is not None), L * n1, device=dev)
    rows = _state_rows(st_all, fin, T)
    sst = nhwc_state_strides(B, C, H, W)
    states = [[rows[t][l * n1:(l + 1) * n1].as_strided((2, B, C, H, W), sst) for l in range(L)] for t in range(T)]
    flows = [torch.empty(B, 2, H, W, device=dev) for _ in range(T)]
    half = 4 * (n1 // 2)
    keep, mem0, sp0 = [], [], []
    for l in range(L):
        p = prev[l]
        if p is None:
            cache = eng.lifs[l].mem
            ok = cache is not None and tuple(cache.shape) == (B, C, H, W) and cache.device == dev
            if ok and cache.stride() != (H * W * C, 1, W * C, C):
                cache = cache.permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)
            mem0.append(cache.data_ptr() if ok else None)
            sp0.append(None)
            keep.append(cache if ok else None)
        else:
            pn = as_nhwc_state(p.detach())
            mem0.append(pn.data_ptr())
            sp0.append(pn.data_ptr() + half if eng.rec[l] else None)
            keep.append(pn)
    base = [r.data_ptr() for r in rows]

    def targs(l, t):
        a = _lib.EvalFwdArgs()
        a.B, a.H, a.W, a.c = B, H, W, C
        if l == 0:
            x = xs[t]
            a.cin, a.x = cin0, x.data_ptr()
            a.xs_b, a.xs_c, a.xs_h, a.xs_w = _x_strides(x)
        else:
            a.cin, a.s_in = C, base[t] + 4 * (l - 1) * n1 + half
        a.mem_prev = mem0[l] if t == 0 else base[t - 1] + 4 * l * n1
        if eng.rec[l]:
            a.s_prev = sp0[l] if t == 0 else base[t - 1] + 4 * l * n1 + half
        a.wt_ff, a.wt_rec = ptr(wfwd[l][0]), _ptr_t(wfwd[l][1])
        a.wt_ff_t, a.wt_rec_t = ptr(wbwd[l][0]), _ptr_t(wbwd[l][1])
        a.n = neurons[l]
        a.state = base[t] + 4 * l * n1
        if l == L - 1:
            a.pred_w, a.pred_b, a.flow = ptr(eng.pred.weight), ptr(eng.pred.bias), flows[t].data_ptr()
        return a

    for d in range(T + L - 1):  # wavefront: task (l, t) in launch l + t
        tasks = [(l, d - l) for l in range(L) if 0 <= d - l < T]
        for i0 in range(0, len(tasks), _lib.EVAL_MAX_TASKS):
            chunk = [targs(l, t) for l, t in tasks[i0:i0 + _lib.EVAL_MAX_TASKS]]
            _lib.call("eval_slot", lib.snnflow_eval_slot, (_lib.EvalFwdArgs * len(chunk))(*chunk), len(chunk), s)
    _lib.timer_close()
    del keep  # (the initial states are read by the launches above: stream-ordered)
    for l in range(L):
        eng.cells[l].lif.mem = states[T - 1][l][0]
    eng.seq_states = [list(sts) for sts in states] if eng.keep_seq_states else None
    return flows, states[T - 1]
