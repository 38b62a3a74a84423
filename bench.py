"""LIFFireNet train-step throughput on MI355X (events/s), the BASELINE.json metric.

One step = the reference training loop's inner iteration (train_flow.py:231-279):
T=10 forwards of LIFFireNet on 1000-event windows, EventWarping loss, backward,
SUM all-reduce of gradients across ranks (data parallel, weak scaling), clip_grad_norm_
(1.0), Adam (lr 2e-4), truncated-BPTT state detach, loss reset.  Synthetic seeded
event windows resident in HBM (configs/train_SNN.yml shapes: 128x128, batch 8 per
GPU, base_num_channels 8).  The whole step is captured into a HIP graph (torch.cuda.graph),
one graph per resident batch of the pool and state parity, each reading its batch in place, and the
graphs are replayed in turn (N > 1: per batch a forward + backward graph, the SUM all-reduce of its
gradient buffer, an update graph); every kernel on the path is in libsnnflow.so.

    python bench.py [--gpus N --steps K --warmup W --channels C --res R --batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...        (one rank per GPU, RCCL)

Rank 0 prints one JSON line.  `roofline` is for the dominant kernel, timed live with
HIP events around each of its launches in one extra eager step after the timed
region; `cpu_baseline` times the CPU oracle (oracle/, a restatement of the
reference's PyTorch path) on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "snn_event-based_optical_flow_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--channels", type=int, default=None, help="base_num_channels (LIFFireNet: 8, U-Net: 32)")
    p.add_argument("--res", type=int, default=None, help="LIFFireNet: 128 (cfg2), U-Net: 256 (cfg5)")
    p.add_argument("--batch", type=int, default=None, help="per-GPU batch (cfg2/cfg4: 8; cfg5: 16)")
    p.add_argument("--T", type=int, default=None, help="windows per loss (window_loss / window; cfg5: 20)")
    p.add_argument("--events", type=int, default=1000, help="events per window (data.window)")
    p.add_argument("--model", default="LIFFireNet")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--per-step", action="store_true",
                   help="T model() calls (FireNetStep) instead of model.forward_sequence (wavefront launches)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--pool", type=int, default=3, help="distinct synthetic batches cycled in HBM")
    p.add_argument("--dist-backend", default=None,
                   help="nccl (= RCCL; the default when a GPU is present) or gloo (rehearsals, CPU, "
                        "SNNFLOW_SHARE_GPU=1)")
    p.add_argument("--bn-broadcast", action="store_true",
                   help="N>1: after the timed steps, broadcast rank 0's BatchNorm running statistics to every rank "
                        "(snnflow.dp.broadcast_bn_stats; not part of the timed step)")
    p.add_argument("--torch-adam", action="store_true",
                   help="LIFFireNet: snnflow's clip + torch's fused Adam (two launches + torch's) instead of "
                        "snnflow.ClipAdam (one launch)")
    p.add_argument("--eval", action="store_true",
                   help="LIFFireNet evaluation pass instead of the train step (eval_flow.py:208-338): model.eval(), "
                        "no autograd, T windows forward + rounded per-polarity IWE + AEE per window")
    p.add_argument("--force-dist", action="store_true",
                   help="run the N>1 step path (process group, forward + backward graph, SUM all-reduce of the flat "
                        "gradient buffer, update graph) even at one rank: the RCCL code path rehearsed at world size 1")
    p.add_argument("--dp-check", action="store_true",
                   help="N>1 correctness check of this very step path (gloo rehearsal): the all-reduced "
                        "gradient == the sum of the ranks' own gradients, parameters identical after the update")
    a = p.parse_args()
    unet = a.model == "SpikingRecEVFlowNet"
    for k, lif, un in (("channels", 8, 32), ("res", 128, 256), ("batch", 8, 16), ("T", 10, 20)):
        if getattr(a, k) is None:
            setattr(a, k, un if unet else lif)
    return a


def algorithmic_bytes(name, C, P, cin0):
    """Algorithmic HBM bytes of one launch (each tensor read/written once; fp32)."""
    f = 4 * P
    if name.startswith("conv_fwd[0]"):
        return f * (cin0 + C)                      # x in, y out
    if name.startswith("conv_fwd_rec"):
        return f * (2 * C + 2 * C + C + C)         # prev y, prev mem in; prev state out; s_prev in; y out
    if name.startswith("conv_fwd"):
        return f * (2 * C + 2 * C + C)
    if name == "lif_fwd":
        return f * (2 * C + 2 * C + 2)             # y, mem in; state out; flow out
    if name == "lif_bwd":
        return f * (2 * C + 4 + C)                 # y, mem, flow, g_flow in; g_cur out
    if name.startswith("layer_bwd_head"):
        return f * (2 * C + cin0)                  # g_cur, y, x in
    if name.startswith("layer_bwd_rec"):
        return f * (3 * C + C + 2 * C + 2 * C + C)  # g_cur,y,x ; s_prev ; g_state_prev out ; prev y,mem ; prev g_cur
    if name.startswith("layer_bwd"):
        return f * (3 * C + 2 * C + C)
    return None


def slot_pass_bytes(kind, C, P, cin0, T, layer_spec, g0=False):
    """Algorithmic bytes of all T x (L+1) layer-steps of a forward (fwd_slot) or backward
    (bwd_slot) pass: the per-kernel formulas of algorithmic_bytes, summed, less the writes the
    sequence path leaves out: at C = 8 (weight gradients fused into the backward) the spike half of
    a feed-forward layer's state at steps t < T-1 (state_spk_skip), at every width the membrane half
    of the recurrent state gradients of steps t >= 1 (never read); step 0 of the backward writes no state
    gradient at all when the initial states need none (g0=False: the bench's detached hand-over)."""
    rec = [r for _, r in layer_spec]
    L, f = len(rec), 4 * P
    if kind == "fwd_slot":
        names = ["conv_fwd[0]"] + ["conv_fwd_rec" if r else "conv_fwd" for r in rec[1:]] + ["lif_fwd"]
        total = T * sum(algorithmic_bytes(n, C, P, cin0) for n in names)
        if C == 8:  # task l >= 1 writes layer l-1's state, the top task layer L-1's
            total -= (T - 1) * sum(f * C for l in range(L) if not rec[l])
        return total
    # the head's backward reads no pixels without an input gradient (one block: neuron grads only)
    names = ["lif_bwd"] + ["layer_bwd_rec" if r else "layer_bwd" for r in rec[1:]]
    total = T * sum(algorithmic_bytes(n, C, P, cin0) for n in names)
    nrec = sum(1 for l in range(1, L) if rec[l])
    total -= (T - 1) * nrec * f * C
    if not g0:
        total -= nrec * f * 2 * C
    return total


def eval_pass_bytes(C, P, cin0, T, layer_spec):
    """Algorithmic bytes of the fused evaluation launches over T steps (snnflow_eval_slot): per
    layer-step the input (event tensor, or layer l-1's spikes), the layer's membrane at t-1 (and its
    spikes at t-1 for a recurrent cell) in, its state (membrane, spikes) out; the flow out once per
    step."""
    f = 4 * P
    per = f * (cin0 + C + 2 * C)
    for _, r in layer_spec[1:]:
        per += f * (C + C + (C if r else 0) + 2 * C)
    return T * (per + f * 2)


def classify(name, rec_layers):
    """Map engine launch names to kernel classes with one byte formula each."""
    if name.startswith("conv_fwd["):
        l = int(name[9:-1])
        if l == 0:
            return "conv_fwd[0]"
        return "conv_fwd_rec" if l in rec_layers else "conv_fwd"
    if name.startswith("layer_bwd["):
        l = int(name[10:-1])
        if l == 0:
            return "layer_bwd_head"
        return "layer_bwd_rec" if l in rec_layers else "layer_bwd"
    return name


def resolve_backend(requested, n_devices, share_gpu):
    """The process-group backend: an explicit --dist-backend wins; ranks sharing one GPU
    (SNNFLOW_SHARE_GPU=1 rehearsals) need gloo; otherwise RCCL ("nccl") whenever a GPU is
    visible, gloo on a CPU-only host."""
    if requested:
        return requested
    if share_gpu:
        return "gloo"
    return "nccl" if n_devices > 0 else "gloo"


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, n):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the environment): start N
    fresh rank processes through torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) and
    pass their output through.  This parent never touches the GPU (torch.cuda.device_count() does
    not initialise it on this image) and never re-execs itself: the ranks are children, and the
    parent exits with their exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the launched world size",
              file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    share = os.environ.get("SNNFLOW_SHARE_GPU") == "1"
    if share:  # rehearsal: several ranks on one device (gloo)
        local = local % torch.cuda.device_count()
    backend = None
    dist_on = world > 1 or args.force_dist
    if dist_on:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if "MASTER_ADDR" not in os.environ:  # --force-dist without a launcher: a one-rank group on this host
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
                              LOCAL_RANK="0")
        torch.cuda.set_device(local)
        backend = resolve_backend(args.dist_backend, torch.cuda.device_count(), share)
        dist.init_process_group(backend, init_method="env://")
    dev = torch.device("cuda", local)
    if args.eval:
        if args.model != "LIFFireNet":
            raise SystemExit("bench.py --eval: LIFFireNet only")
        return eval_main(args, world, rank, dev, backend, dist_on)

    import snnflow
    from snnflow import _lib
    from snnflow import dp
    from snnflow.synthetic import make_window

    torch.manual_seed(0)  # configs/parser.py:92-96 (loader.seed = 0): identical init on every rank
    from snnflow.parser import train_snn_model_kwargs
    kw = train_snn_model_kwargs(args.model, base_num_channels=args.channels)  # configs/train_SNN.yml
    model = getattr(snnflow, args.model)(kw).to(dev).train()
    R, B, T, N = args.res, args.batch, args.T, args.events
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    loss_fn = snnflow.EventWarping(cfg, dev)
    params = list(model.parameters())
    # LIFFireNet: clip_grad_norm_ + Adam in one launch (snnflow.ClipAdam over the engine's flat
    # gradient buffer); the U-Net (and --torch-adam): torch's fused Adam after snnflow's clip
    fused_opt = args.model != "SpikingRecEVFlowNet" and not args.torch_adam
    if fused_opt:
        opt = snnflow.ClipAdam(params, lr=2e-4, max_norm=1.0)
    else:
        opt = torch.optim.Adam(params, lr=2e-4, capturable=not args.no_graph, fused=True)

    # synthetic data, resident in HBM; per-rank stream seeded by (seed, rank)
    gen = torch.Generator(device=dev).manual_seed(dp.stream_seed(1, rank))
    pool = [_pack([make_window(B, N, R, R, gen, dev) for _ in range(T)]) for _ in range(args.pool)]
    static_flat, static_views = _pack_like(pool[0])
    cur = {"views": static_views}  # the windows fwd_bwd reads (graph capture: one resident batch each)

    def load_batch(i):  # eager steps: one device copy of the next resident batch into the input buffer
        static_flat.copy_(pool[i % len(pool)][0], non_blocking=True)
        cur["views"] = static_views

    unet = args.model == "SpikingRecEVFlowNet"

    def get_states():
        return model.multires_unetrec.states if unet else model._states

    def set_states(st):
        if unet:
            model.multires_unetrec.states = st
        else:
            model._states = st

    seed = torch.ones((), device=dev)

    def fwd_bwd():
        static = cur["views"]
        loss_fn.reset()
        if unet:  # the reference loop: one forward per window (train_flow.py:232), 4 flow maps each
            outs = [model(w["event_voxel"], w["event_cnt"]) for w in static]
        elif args.per_step:
            outs = [model(w["event_voxel"], w["event_cnt"]) for w in static]
        else:  # the same T steps, kernels issued as wavefront launches (C = 8, 16, 32; else per step)
            outs = model.forward_sequence([w["event_voxel"] for w in static], [w["event_cnt"] for w in static])
        for t in range(T):
            w = static[t]
            loss_fn.event_flow_association(outs[t]["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = loss_fn()
        loss.backward(seed)  # == loss.backward(): the unit seed is a persistent tensor, not a fill per step
        return loss

    sync_grads = dp.GradAllReduce(params)  # one SUM all-reduce over the engine's flat gradient buffer

    handover = StateHandover(dev, get_states, set_states)
    pingpong = None  # graph replays of forward_sequence: copy-free hand-over (StatePingPong)

    def update():
        if not fused_opt:
            dp.clip_grad_norm_(params, 1.0)
        opt.step()
        if args.no_graph:  # the reference loop's hand-over (train_flow.py:262-279)
            model.detach_states()
            return
        if pingpong is None:
            handover()

    def step_eager():
        opt.zero_grad(set_to_none=True)
        fwd_bwd()
        sync_grads()
        update()

    # warmup (eager; builds workspaces, optimizer state, persistent state buffers).  Before a graph
    # capture it runs on a side stream; the eager loop warms up on the stream it is timed on (autograd's
    # AccumulateGrad nodes keep the stream they were created on: a side-stream warmup would put a
    # cross-stream wait behind every parameter's gradient in each timed backward)
    s_side = torch.cuda.Stream(dev) if not args.no_graph else torch.cuda.current_stream(dev)
    s_side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s_side):
        for i in range(max(args.warmup, 3)):
            load_batch(i)
            step_eager()
    torch.cuda.current_stream(dev).wait_stream(s_side)
    torch.cuda.synchronize(dev)

    # HIP graphs, one per resident batch of the pool (and state parity: StatePingPong), each reading
    # its batch in place.  N = 1: forward, backward, clip, Adam and the state hand-over in one graph.
    # N > 1: the same forward + backward graph per batch, the eager SUM all-reduce of that graph's
    # flat gradient buffer, then that batch's update graph (clip + Adam read the graph's gradients).
    # Every capture starts from set_to_none gradients, so each graph owns its gradient buffer.
    graphs, upds, flats = [], [], []
    multi = not dist_on  # one graph holds the whole step (no collective between forward+backward and update)
    if not args.no_graph:
        n_graphs = len(pool)
        if not unet and not args.per_step:
            pingpong = StatePingPong(dev, get_states())
            n_graphs = pingpong.cycle(len(pool))
        for j in range(n_graphs):
            opt.zero_grad(set_to_none=True)
            cur["views"] = pool[j % len(pool)][1]
            if pingpong is not None:
                pingpong.arm(model, j)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fwd_bwd()
                if multi:
                    update()
            graphs.append(g)
            if not multi:
                flats.append(dp.flat_grad_buffer(params))
                u = torch.cuda.CUDAGraph()
                with torch.cuda.graph(u, pool=g.pool()):
                    update()
                upds.append(u)

    def step(i):
        if not graphs:
            load_batch(i)
            step_eager()
        elif multi:
            graphs[i % len(graphs)].replay()
        else:
            j = i % len(graphs)
            graphs[j].replay()
            if flats[j] is not None:
                dist.all_reduce(flats[j], op=dist.ReduceOp.SUM)
            else:
                sync_grads()
            upds[j].replay()

    for i in range(2):  # graph warm replays
        step(i)
    if args.dp_check:
        _dp_check(world, rank, step_parts=(graphs, upds, flats, fwd_bwd, sync_grads, update, opt), params=params)
        dist.destroy_process_group()
        return
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    prof = None
    if os.environ.get("SNNFLOW_BENCH_PROFILE") == "1":  # host-side profile of the timed loop (stderr)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(30)
    if dist_on:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    if world > 1 and args.bn_broadcast:
        dp.broadcast_bn_stats(model)
    ms_per_step = 1000.0 * elapsed / args.steps
    events_per_step = world * B * T * N
    value = events_per_step * args.steps / elapsed

    # live per-kernel timing: one extra eager step with HIP events around every launch
    # (the stream is first held by a ~40 ms device-side sleep so the host enqueues the
    # whole step ahead of the GPU: the events then bracket kernel execution only)
    timer = _lib.KernelTimer()
    _lib.TIMER = timer
    load_batch(0)
    if pingpong is not None:  # the states the graphs hand over (detached views), not a capture's outputs
        set_states(list(pingpong.views[0]))
    torch.cuda._sleep(100_000_000)
    step_eager()
    _lib.TIMER = None
    kern = timer.summary()
    if unet:
        roofline, kernels = _unet_roofline(kern)
    else:
        roofline, kernels = _firenet_roofline(kern, model, args, B, R, T)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_unet(args, pool[0][1]) if unet else cpu_baseline(args, pool[0][1])

    if rank == 0:
        line = {
            "metric": (f"events/sec (train step) SpikingRecEVFlowNet T={T} {R}x{R}" if unet
                       else f"events/sec (train step) LIFFireNet T={T} {R}x{R}"
                       + (f" C={args.channels}" if args.channels != 8 else "")),
            "value": round(value, 1), "unit": "events/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": f"{args.model} train step: T={T} x {N}-event windows, {R}x{R}, "
                                   f"batch {B}/GPU, base_num_channels {args.channels}, EventWarping + Adam",
                       "global_batch": B * world, "parallelism": f"dp{world}", "collective": backend,
                       "hip_graph": not args.no_graph,
                       "launch_order": "per-step" if (args.per_step or unet) else "wavefront"},
            "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


def _dp_check(world, rank, step_parts, params):
    """One step of the N>1 path exactly as timed (batch 1's forward + backward graph; the eager
    all-reduce of that graph's flat gradient buffer; its update graph: clip + Adam), checked: the
    all-reduced flat gradient equals the SUM of every rank's own gradient (gathered through the
    host), and after the update every rank holds the same parameters.  Rank 0 prints one JSON line."""
    from snnflow import dp

    graphs, upds, flats, fwd_bwd, sync_grads, update, opt = step_parts
    if graphs:  # batch 1's graphs (the gradients of a replay live in that graph's own flat buffer)
        graphs[1 % len(graphs)].replay()
        flat = flats[1 % len(graphs)]
    else:
        opt.zero_grad(set_to_none=True)
        fwd_bwd()
        flat = dp.flat_grad_buffer(params)
    torch.cuda.synchronize()

    def grads():
        return flat.detach().cpu().clone() if flat is not None else torch.cat(
            [p.grad.detach().reshape(-1).cpu() for p in params])

    local = grads()
    if flat is not None:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    else:
        sync_grads()
    torch.cuda.synchronize()
    reduced = grads()
    # (gathered through device tensors: the nccl backend has no CPU collectives)
    cdev = flat.device if flat is not None else params[0].device
    locals_ = [torch.empty_like(local, device=cdev) for _ in range(world)]
    dist.all_gather(locals_, local.to(cdev))
    locals_ = [t.cpu() for t in locals_]
    want = locals_[0].double()
    for t in locals_[1:]:
        want = want + t.double()
    err = float((reduced.double() - want).abs().max() / max(float(want.abs().max()), 1e-30))
    distinct = float(max((t - locals_[0]).abs().max() for t in locals_[1:])) if world > 1 else 0.0
    if graphs:
        upds[1 % len(graphs)].replay()
    else:
        update()
    torch.cuda.synchronize()
    pflat = torch.cat([p.detach().reshape(-1) for p in params])
    ps = [torch.empty_like(pflat) for _ in range(world)]
    dist.all_gather(ps, pflat)
    ps = [t.cpu() for t in ps]
    pdiff = float(max((t - ps[0]).abs().max() for t in ps[1:])) if world > 1 else 0.0
    if rank == 0:
        print(json.dumps({"dp_check": {"world": world, "backend": dist.get_backend(), "grad_numel": local.numel(), "allreduce_rel_err": err,
                                       "ranks_local_grads_differ_by": distinct, "param_max_diff_after_update": pdiff}}),
              flush=True)


def perturb_running_stats(model, seed=3):
    """Seeded BatchNorm running statistics away from (0, 1), as a trained model carries them: the
    eval-mode BatchNorm is then not the identity (the same perturbation as
    tests/test_gpu_fullsize.py::test_cfg2_eval_vs_oracle)."""
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.running_mean.copy_(0.2 * torch.randn(m.running_mean.shape, generator=g))
            m.running_var.copy_(0.5 + torch.rand(m.running_var.shape, generator=g))


def eval_main(args, world, rank, dev, backend, dist_on=False):
    """`--eval`: the reference's evaluation loop (eval_flow.py:208-338) on synthetic windows.  One
    step = T windows of B sequences: model.eval() forward (BatchNorm on running statistics, no
    autograd; forward_sequence's wavefront launches), then per window the rounded per-polarity IWE
    (compute_pol_iwe, eval_flow.py:227-235) and AEE against a synthetic ground-truth flow
    (loss/flow.py:597-649), the per-sample AEE / outlier percentage left on the device (the
    reference moves them to the host per window for its result table; the line reports the last
    pass's mean).  Visualisation is not part
    of the step.  HIP graphs as the train bench: one per resident batch, the state hand-over inside.
    A second, smaller measurement covers configs[0] of BASELINE.json (T=5, B=1, forward only) on
    the GPU and with the CPU oracle."""
    import snnflow
    from snnflow import _lib, dp
    from snnflow.iwe import compute_pol_iwe
    from snnflow.parser import train_snn_model_kwargs
    from snnflow.synthetic import make_window

    R, B, T, N = args.res, args.batch, args.T, args.events
    kw = train_snn_model_kwargs(args.model, base_num_channels=args.channels)

    def new_model():
        torch.manual_seed(0)
        m = snnflow.LIFFireNet(kw)
        perturb_running_stats(m)
        return m.to(dev).eval()

    model = new_model()
    gen = torch.Generator(device=dev).manual_seed(dp.stream_seed(1, rank))
    pool = [_pack([make_window(B, N, R, R, gen, dev) for _ in range(T)]) for _ in range(args.pool)]
    gts = [[(torch.rand(B, 2, R, R, generator=gen, device=dev) - 0.5) * 8.0 for _ in range(T)]
           for _ in range(args.pool)]
    one = torch.ones(1, device=dev)
    metric = snnflow.AEE({"loader": {"resolution": [R, R]}, "loss": {"overwrite_intermediate": False}}, dev,
                         flow_scaling=128)
    last = {}  # the last pass's per-window AEE / outlier % (device tensors; read after timing)

    pingpong = []  # set after the warm-up: graph replays hand the states over copy-free

    def set_states(st):
        model._states = st

    handover = StateHandover(dev, lambda: model._states, set_states)

    def eval_pass(j):
        views, gt = pool[j % len(pool)][1], gts[j % len(pool)]
        outs = model.forward_sequence([w["event_voxel"] for w in views], [w["event_cnt"] for w in views])
        for t, w in enumerate(views):
            pol = w["event_list_pol_mask"]
            compute_pol_iwe(outs[t]["flow"][-1], w["event_list"], (R, R), pol[:, :, 0:1], pol[:, :, 1:2],
                            flow_scaling=128, round_idx=True)
            metric.event_flow_association(outs[t]["flow"], {"event_list": w["event_list"], "event_list_pol_mask": pol,
                                                            "event_mask": w["event_mask"], "gtflow": gt[t],
                                                            "dt_input": one, "dt_gt": one})
            last[t] = metric()
            metric.reset()
        if not pingpong:
            handover()

    def arm(j):
        if not pingpong:
            pingpong.append(StatePingPong(dev, model._states))
        pingpong[0].arm(model, j)

    graphs, elapsed = _timed_passes(args, dev, world, eval_pass, arm=arm)
    aee_mean = (torch.stack([last[t][0] for t in range(T)]).mean(0)).tolist()  # the last timed pass
    events_per_step = world * B * T * N
    value = events_per_step * args.steps / elapsed

    timer = _lib.KernelTimer()
    _lib.TIMER = timer
    torch.cuda._sleep(100_000_000)
    with torch.no_grad():
        eval_pass(0)
    _lib.TIMER = None
    roofline, kernels = _firenet_roofline(timer.summary(), model, args, B, R, T)

    # configs[0]: T = 5 windows of one sequence, forward only, GPU and CPU oracle
    cfg1 = None
    if rank == 0 and world == 1:
        m1 = new_model()
        g1 = torch.Generator(device=dev).manual_seed(11)
        wins1 = [make_window(1, N, R, R, g1, dev) for _ in range(5)]
        h1 = StateHandover(dev, lambda: m1._states, lambda st: setattr(m1, "_states", st))
        pp1 = []

        def fwd1(j):
            m1.forward_sequence([w["event_voxel"] for w in wins1], [w["event_cnt"] for w in wins1])
            if not pp1:
                h1()

        def arm1(j):
            if not pp1:
                pp1.append(StatePingPong(dev, m1._states))
            pp1[0].arm(m1, j)

        a1 = argparse.Namespace(**vars(args))
        a1.steps, a1.pool = max(args.steps, 50), 1
        _, el1 = _timed_passes(a1, dev, 1, fwd1, arm=arm1)
        cfg1 = {"workload": f"configs[0]: LIFFireNet {R}x{R}, T=5, batch 1, forward only (eval mode)",
                "gpu": {"value": round(5 * N * a1.steps / el1, 1), "unit": "events/s",
                        "ms_per_pass": round(1000.0 * el1 / a1.steps, 4)}}
        if not args.no_cpu_baseline:
            cfg1["cpu"] = cpu_baseline_forward(args, wins1)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_eval(args, pool[0][1], gts[0])

    if rank == 0:
        line = {
            "metric": f"events/sec (eval: forward + IWE + AEE) LIFFireNet T={T} {R}x{R}",
            "value": round(value, 1), "unit": "events/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": f"LIFFireNet eval pass: T={T} x {N}-event windows, {R}x{R}, batch {B}/GPU, "
                                   f"base_num_channels {args.channels}, model.eval() (running statistics), "
                                   "rounded per-polarity IWE + AEE per window",
                       "global_batch": B * world, "parallelism": f"dp{world}" if world > 1 else "none",
                       "collective": backend, "hip_graph": not args.no_graph, "launch_order": "wavefront"},
            "aee_last_pass_mean_per_sample": [round(v, 6) for v in aee_mean],
            "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu, "configs0": cfg1,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


def _timed_passes(args, dev, world, run, reset=None, arm=None):
    """Warm-up (eager, side stream), one HIP graph per resident batch (unless --no-graph; with
    `arm(j)`, called before capture j, StatePingPong.cycle(pool) graphs), then args.steps timed
    passes bracketed by barrier + synchronize; returns (graphs, max-over-ranks seconds).  `run(j)`
    enqueues pass j; it runs under torch.no_grad()."""
    s_side = torch.cuda.Stream(dev)
    s_side.wait_stream(torch.cuda.current_stream(dev))
    with torch.no_grad(), torch.cuda.stream(s_side):
        for i in range(max(args.warmup, 3)):
            run(i)
    torch.cuda.current_stream(dev).wait_stream(s_side)
    torch.cuda.synchronize(dev)
    graphs = []
    if not args.no_graph:
        for j in range(args.pool if arm is None else StatePingPong.cycle(args.pool)):
            if arm is not None:
                arm(j)
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g):
                run(j)
            graphs.append(g)

    def step(i):
        if graphs:
            graphs[i % len(graphs)].replay()
        else:
            with torch.no_grad():
                run(i)

    for i in range(2):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if reset is not None:  # accumulators count the timed passes only
        reset()
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    return graphs, elapsed


def _firenet_roofline(kern, model, args, B, R, T):
    """HBM roofline of the dominant LIFFireNet kernel class (algorithmic bytes / HIP-event time)."""
    rec_layers = {i for i, (_, r) in enumerate(model.layer_spec) if r}
    classes = {}
    for name, v in kern.items():
        c = classify(name, rec_layers)
        n, tot = classes.get(c, (0, 0.0))
        classes[c] = (n + v["launches"], tot + v["total_ms"])
    P = B * R * R
    dominant = max(classes, key=lambda k: classes[k][1])
    n_dom, tot_dom = classes[dominant]
    avg_us = 1000.0 * tot_dom / n_dom
    abytes = algorithmic_bytes(dominant, args.channels, P, 2)
    if dominant in ("fwd_slot", "bwd_slot"):  # wavefront launches: the pass's layer-step bytes / its launches
        abytes = slot_pass_bytes(dominant, args.channels, P, 2, T, model.layer_spec) / n_dom
    elif dominant == "eval_slot":
        abytes = eval_pass_bytes(args.channels, P, 2, T, model.layer_spec) / n_dom
    achieved = abytes / (avg_us * 1e-6) / 1e9 if abytes else None
    kernels = {k: {"launches": n, "avg_us": round(1000.0 * t / n, 2), "share": round(t / sum(x[1] for x in classes.values()), 3)}
               for k, (n, t) in sorted(classes.items(), key=lambda kv: -kv[1][1])}
    roofline = {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": _pmc_traffic(dominant, args),
                "traffic_source": "committed PMC (profiles/pmc_traffic.json, separate rocprofv3 --pmc passes), not live",
                "bytes_per_launch": abytes, "avg_us": round(avg_us, 2)}
    return roofline, kernels


# bf16 dense MFMA peak (MI355X_MICROARCH.md) over the three bf16 products that make one exact fp32 product
# (weights split hi/mid/lo, operands exact in bf16): the peak rate of fp32-exact convolution FLOPs
BF16_PEAK_TFLOPS = 2500.0
BF16X3_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 3


# bf16 matrix-core products each U-Net GEMM class issues per exact fp32 product: the forward conv and
# the weight gradient multiply an exact-in-bf16 operand (spikes, spike sums) by a 3-part split, the
# input gradient multiplies two 3-part splits (six products above 2^-24 relative)
UNET_PRODUCTS = {"unet_conv": 3, "unet_wgrad": 3, "unet_dgrad": 6}


def _unet_roofline(kern):
    """MFMA roofline of the dominant U-Net GEMM class: algorithmic (reference fp32 conv) FLOPs per
    launch / HIP-event time, against the bf16x3 peak; every class listed with its own rate, and with
    its issued rate (algorithmic x the bf16 products it issues) against the dense bf16 peak."""
    kernels = {}
    total = sum(v["total_ms"] for v in kern.values())
    for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"]):
        e = {"launches": v["launches"], "avg_us": round(v["avg_us"], 2), "share": round(v["total_ms"] / total, 3)}
        if v["work"]:
            tf = v["work"] / (v["total_ms"] * 1e-3) / 1e12
            e["tflops"] = round(tf, 1)
            if k in UNET_PRODUCTS:
                e["issued_tflops"] = round(tf * UNET_PRODUCTS[k], 1)
                e["issued_frac"] = round(tf * UNET_PRODUCTS[k] / BF16_PEAK_TFLOPS, 4)
        kernels[k] = e
    gemm = {k: v for k, v in kern.items() if v["work"]}
    dominant = max(gemm, key=lambda k: gemm[k]["total_ms"])
    d = gemm[dominant]
    achieved = d["work"] / (d["total_ms"] * 1e-3) / 1e12
    roofline = {"bound": "mfma", "kernel": dominant, "achieved": round(achieved, 1), "peak": round(BF16X3_PEAK_TFLOPS, 1),
                "unit": "TFLOP/s", "frac": round(achieved / BF16X3_PEAK_TFLOPS, 4), "traffic": None,
                "flops_per_launch": d["work"] / d["launches"], "avg_us": round(d["avg_us"], 2),
                "peak_note": "bf16 dense 2.5 PF / 3 (hi/mid/lo weight products per exact fp32 product)",
                "issued_frac": kernels.get(dominant, {}).get("issued_frac")}
    return roofline, kernels


_KEYS = ("event_cnt", "event_list", "event_list_pol_mask", "event_mask")


def _flat_span(tensors):
    """1-D view over the storage range of `tensors` if they are fp32 views laid back to back
    in one storage (each exactly covering its numel), else None."""
    if not tensors or any(t is None for t in tensors):
        return None
    st = tensors[0].untyped_storage()
    off = tensors[0].storage_offset()
    base = off
    for t in tensors:
        if t.untyped_storage().data_ptr() != st.data_ptr() or t.storage_offset() != off or t.dtype != torch.float32:
            return None
        off += t.numel()
    flat = torch.empty(0, device=tensors[0].device)
    flat.set_(st, base, (off - base,), (1,))
    return flat


class StateHandover:
    """The reference loop's state hand-over (detach_states, train_flow.py:262-279) for HIP-graph
    replays: persistent state buffers, and detach == one copy of the step's final states into them
    (one contiguous copy when the engine's states lie back to back), so that every replay of a
    captured step reads the states the previous replay left."""

    def __init__(self, dev, get_states, set_states):
        self.dev, self.get, self.set = dev, get_states, set_states
        self.bufs = None
        self.flat = None

    def __call__(self):
        states = self.get()
        src = _flat_span(states)
        if self.bufs is None:
            if src is not None:  # persistent buffers with the same back-to-back layout
                self.flat = src.clone()
                base = src.data_ptr()
                self.bufs = [torch.empty(0, device=self.dev).set_(self.flat.untyped_storage(),
                                                                  (s.data_ptr() - base) // 4, s.shape, s.stride())
                             for s in states]
            else:
                self.bufs = [s.detach().clone() for s in states]
        if src is not None and self.flat is not None:
            self.flat.copy_(src)
        else:
            torch._foreach_copy_(self.bufs, [s.detach() for s in states])
        self.set(list(self.bufs))


class StatePingPong:
    """Copy-free state hand-over for HIP-graph replays of forward_sequence: two persistent state
    buffers; the graph of replay j reads buffer j % 2 as its initial states while the engine writes
    the final step's states straight into buffer (j + 1) % 2 (FireNetEngine.final_state_out), so the
    reference's detach (a clone, train_flow.py:262-279) costs nothing.  Replays must alternate
    parity: `cycle(n)` is the number of graphs to capture for n resident batches (2n when n is odd)."""

    def __init__(self, dev, states):
        src = _flat_span(states)
        if src is None:
            raise RuntimeError("StatePingPong: the engine's states are not one flat row")
        base = src.data_ptr()
        self.bufs = [src.clone(), src.clone()]
        self.views = [[torch.empty(0, device=dev).set_(b.untyped_storage(), (s.data_ptr() - base) // 4, s.shape,
                                                       s.stride()) for s in states] for b in self.bufs]

    @staticmethod
    def cycle(n):
        return n if n % 2 == 0 else 2 * n

    def arm(self, model, j):
        model._states = list(self.views[j % 2])
        model.engine.final_state_out = self.bufs[(j + 1) % 2]


def _pack(windows):
    """Pack T windows into one flat device buffer; returns (flat, list of dict views)."""
    sizes = [w[k].numel() for w in windows for k in _KEYS]
    flat = torch.empty(sum(sizes), device=windows[0]["event_cnt"].device)
    views, off = [], 0
    for w in windows:
        d = {}
        for k in _KEYS:
            n = w[k].numel()
            flat[off:off + n].copy_(w[k].reshape(-1))
            d[k] = flat[off:off + n].view(w[k].shape)
            off += n
        d["event_voxel"] = d["event_cnt"]
        views.append(d)
    return flat, views


def _pack_like(packed):
    flat = packed[0].clone()
    views, off = [], 0
    for w in packed[1]:
        d = {}
        for k in _KEYS:
            n = w[k].numel()
            d[k] = flat[off:off + n].view(w[k].shape)
            off += n
        d["event_voxel"] = d["event_cnt"]
        views.append(d)
    return flat, views


def _pmc_traffic(kernel, args):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from separate --pmc passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM), if it was measured on this config."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    key = f"C{args.channels}_R{args.res}_B{args.batch}"
    return d.get(key, {}).get(kernel)


_THREADS_NOTE = ("threads = min(affinity, 16): a GPU box grants each GPU a 16-CPU share (OMP_NUM_THREADS=16 "
                 "there) while os.cpu_count() / the affinity mask show the whole machine")


def _cpu_threads():
    return max(1, min(len(os.sched_getaffinity(0)), 16))


def _cpu_model():
    """Host CPU model name (/proc/cpuinfo), recorded beside cpu_baseline.cores."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args, windows):
    """The CPU oracle (pure-PyTorch restatement of the reference path, same op sequence)
    timed on this host: one full train step of the same workload after one warm-up
    step, then whole train steps until ~10 s of CPU work (bounded sample, >= 1 step)."""
    from oracle import iwe_ref, lif_ref

    threads = _cpu_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    kw = lif_ref.make_unet_kwargs(base_num_channels=args.channels)
    model = lif_ref.LIFFireNetRef(kw, args.model).train()
    opt = torch.optim.Adam(model.parameters(), lr=2e-4)
    cpu_w = [{k: v.cpu() for k, v in w.items()} for w in windows]
    R = args.res

    def one():
        lf = iwe_ref.EventWarpingRef([R, R])
        for w in cpu_w:
            out = model(None, w["event_cnt"])
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = lf()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad()
        model.detach_states()

    one()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:  # bounded sample: whole train steps until ~10 s of CPU work (>= 1 step)
        one()
        n += 1
        if time.perf_counter() - t0 > 10.0:
            break
    dt = time.perf_counter() - t0
    ev = n * args.batch * args.T * args.events
    return {"value": round(ev / dt, 1), "unit": "events/s", "cores": threads, "cpu_model": _cpu_model(),
            "threads_note": _THREADS_NOTE, "kind": "port",
            "sample": f"{n} timed train steps (after 1 warm-up) of the same workload: {args.batch}x{args.T} windows "
                      f"of {args.events} events, {R}x{R}, C={args.channels}, Adam; oracle/ pure-PyTorch CPU "
                      f"restatement of the reference path, {threads} threads", "seconds": round(dt, 3)}


def _oracle_eval_model(args):
    from oracle import lif_ref

    torch.manual_seed(0)
    model = lif_ref.LIFFireNetRef(lif_ref.make_unet_kwargs(base_num_channels=args.channels), args.model)
    perturb_running_stats(model)
    return model.eval()


def _bounded(run, seconds):
    """run() once as warm-up, then until `seconds` of CPU work have passed (>= 1 run)."""
    run()
    n, t0 = 0, time.perf_counter()
    while n == 0 or time.perf_counter() - t0 < seconds:
        run()
        n += 1
    return n, time.perf_counter() - t0


def cpu_baseline_eval(args, windows, gts):
    """The CPU oracle's evaluation pass of the --eval workload: eval-mode forward of every window,
    rounded per-polarity IWE (oracle/iwe_ref.py compute_pol_iwe_t) and AEE (oracle/metrics_ref.py),
    whole T-window passes until ~10 s of CPU work."""
    from oracle import iwe_ref
    from oracle.metrics_ref import flow_metrics_ref

    threads = _cpu_threads()
    torch.set_num_threads(threads)
    model = _oracle_eval_model(args)
    R = args.res
    cpu_w = [{k: v.cpu() for k, v in w.items()} for w in windows]
    cpu_gt = [g.cpu() for g in gts]
    one = torch.ones(1)

    def one_pass():
        with torch.no_grad():
            for w, gt in zip(cpu_w, cpu_gt):
                flow = model(None, w["event_cnt"])["flow"][-1]
                pol = w["event_list_pol_mask"]
                iwe_ref.compute_pol_iwe_t(flow, w["event_list"], [R, R], pol[:, :, 0:1], pol[:, :, 1:2], 128, True)
                flow_metrics_ref(flow, gt, w["event_mask"], one, one, 128)

    n, dt = _bounded(one_pass, 10.0)
    ev = n * args.batch * args.T * args.events
    return {"value": round(ev / dt, 1), "unit": "events/s", "cores": threads, "cpu_model": _cpu_model(),
            "threads_note": _THREADS_NOTE, "kind": "port",
            "sample": f"{n} timed eval passes (after 1 warm-up) of the same workload: {args.batch}x{args.T} windows "
                      f"of {args.events} events, {R}x{R}, C={args.channels}; oracle/ CPU restatement (eval-mode "
                      f"forward, rounded IWE, AEE), {threads} threads", "seconds": round(dt, 3)}


def cpu_baseline_forward(args, windows):
    """configs[0] of BASELINE.json on the CPU oracle: T = len(windows) eval-mode forwards of one
    sequence (batch 1), repeated until ~5 s of CPU work."""
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    model = _oracle_eval_model(args)
    cpu_w = [w["event_cnt"].cpu() for w in windows]

    def one_pass():
        with torch.no_grad():
            for x in cpu_w:
                model(None, x)

    n, dt = _bounded(one_pass, 5.0)
    ev = n * len(cpu_w) * args.events
    return {"value": round(ev / dt, 1), "unit": "events/s", "cores": threads, "kind": "port",
            "sample": f"{n} timed passes of {len(cpu_w)} windows x 1 sequence, forward only (oracle/lif_ref.py)",
            "seconds": round(dt, 3)}


def cpu_baseline_unet(args, windows):
    """The U-Net oracle (oracle/unet_ref.py, pinned by the reference-generated fixture) on the host
    cores: one sample's train step over 2 windows at the bench resolution and width (~10-30 s of CPU
    work), scaled to events/s."""
    from oracle import iwe_ref
    from oracle.unet_ref import SpikingRecEVFlowNetRef

    threads = _cpu_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    from snnflow.parser import train_snn_model_kwargs
    model = SpikingRecEVFlowNetRef(train_snn_model_kwargs("SpikingRecEVFlowNet", base_num_channels=args.channels))
    opt = torch.optim.Adam(model.parameters(), lr=2e-4)
    R, nw = args.res, 2
    cpu_w = [{k: v[:1].cpu() for k, v in w.items()} for w in windows[:nw]]

    def step():
        flows = [model(None, w["event_cnt"])["flow"] for w in cpu_w]
        loss = 0
        for i in range(4):
            lf = iwe_ref.EventWarpingRef([R, R])
            for t, w in enumerate(cpu_w):
                lf.event_flow_association([flows[t][i]], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
            loss = loss + lf()
        opt.zero_grad(set_to_none=True)
        (loss / 4).backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        model.reset_states()

    step()  # warm-up (first-touch allocations)
    n, t0 = 0, time.perf_counter()
    while n == 0 or time.perf_counter() - t0 < 10.0:
        step()
        n += 1
    dt = time.perf_counter() - t0
    ev = n * nw * args.events
    return {"value": round(ev / dt, 1), "unit": "events/s", "cores": threads, "cpu_model": _cpu_model(),
            "threads_note": _THREADS_NOTE, "kind": "port",
            "sample": f"{n} timed train steps (after 1 warm-up) of 1 sample x {nw} windows of {args.events} events, "
                      f"{R}x{R}, base {args.channels}; "
                      f"oracle/unet_ref.py (CPU restatement of the reference U-Net), {threads} threads",
            "seconds": round(dt, 3)}


if __name__ == "__main__":
    main()
