"""Data parallelism of the train step.

The reference trains one model on one device (train_flow.py:232-279).  Its batch
slots are independent event sequences with their own recurrent state and the
event-warping loss is a per-sample SUM (loss/flow.py:228, 261, 291), so the
step shards along the batch axis with exactly one exchange per optimizer step:
a SUM all-reduce of the parameter gradients before clip_grad_norm_
(train_flow.py:265-266).  One process per GPU, torch.distributed over RCCL
("nccl" backend) on the GPU box, gloo in the CPU tests.

BatchNorm statistics stay rank-local (batch statistics of the rank's B slots,
i.e. the reference's own semantics for a batch of B): a single-device run with
the global batch would normalise over all slots and differ.
"""
import torch
import torch.distributed as dist


def shard_slots(global_batch, rank, world):
    """Batch slots owned by `rank`: [rank*B/P, (rank+1)*B/P)."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} does not split over {world} ranks")
    per = global_batch // world
    return range(rank * per, (rank + 1) * per)


def stream_seed(seed, rank):
    """Seed of rank `rank`'s synthetic event stream (identical weights, distinct data)."""
    return int(seed) * 1000 + int(rank)


def flat_grad_buffer(params):
    """If the p.grad are contiguous views that tile one range of one storage exactly (in any
    order: FireNetEngine's buffer follows its own parameter order, not the module's
    registration order) -- the layout FireNetEngine hands to AccumulateGrad -- return one
    1-D tensor over that range, else None."""
    grads = [p.grad for p in params]
    if not grads or any(g is None or not g.is_contiguous() for g in grads):
        return None
    st = grads[0].untyped_storage()
    if any(g.untyped_storage().data_ptr() != st.data_ptr() or g.dtype != grads[0].dtype for g in grads):
        return None
    spans = sorted((g.storage_offset(), g.numel()) for g in grads)
    base = off = spans[0][0]
    for o, n in spans:
        if o != off:
            return None
        off += n
    flat = torch.empty(0, dtype=grads[0].dtype, device=grads[0].device)
    flat.set_(st, base, (off - base,), (1,))
    return flat


class GradAllReduce:
    """SUM all-reduce of the gradients of `params` in one flat bucket.

    Gradients living in one flat buffer (the engine's layout) are reduced in place
    with a single collective; otherwise they are packed into a bucket, reduced and
    copied back.  The parameter set is small (C=8: 4,994 floats, C=32: 75,266), so a
    single bucket is latency-bound and needs no overlap with the backward pass."""

    def __init__(self, params, group=None):
        self.params = list(params)
        self.group = group

    def __call__(self):
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        flat = flat_grad_buffer(self.params)
        if flat is not None:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            return
        grads = [p.grad for p in self.params if p.grad is not None]
        bucket = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=self.group)
        off = 0
        for g in grads:
            g.copy_(bucket[off:off + g.numel()].view_as(g))
            off += g.numel()


def bn_buffers(model):
    """The BatchNorm running statistics of `model` (running_mean, running_var, num_batches_tracked
    of every BatchNorm module, in module order)."""
    out = []
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.track_running_stats:
            out += [m.running_mean, m.running_var, m.num_batches_tracked]
    return [b for b in out if b is not None]


def broadcast_bn_stats(model, src=0, group=None):
    """Opt-in: overwrite every rank's BatchNorm running statistics with rank
    `src`'s, so that an evaluation after data-parallel training sees one set (the batch statistics
    of the train step itself stay rank-local either way).  One flat broadcast of the float buffers
    (running means and variances) and one of the int64 counters; a no-op without a process group
    or with one rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    bufs = bn_buffers(model)
    for dtype in (torch.float32, torch.int64):
        part = [b for b in bufs if b.dtype == dtype]
        if not part:
            continue
        flat = torch.cat([b.reshape(-1) for b in part])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        for b in part:
            b.copy_(flat[off:off + b.numel()].view_as(b))
            off += b.numel()


_CLIP_SCRATCH = {}


def clip_grad_norm_(params, max_norm, eps=1e-6):
    """torch.nn.utils.clip_grad_norm_ (2-norm) with the flat-buffer fast path: one
    norm and one scale over the engine's gradient buffer instead of per-tensor
    foreach launches.  Same math: coef = clamp(max_norm / (total + eps), max=1)."""
    params = [p for p in params if p.grad is not None]
    flat = flat_grad_buffer(params)
    if flat is None:
        return torch.nn.utils.clip_grad_norm_(params, max_norm)
    if flat.is_cuda and flat.dtype == torch.float32:
        # one HIP launch: norm (fp64 accumulation) + scale in place; grid-wide for large vectors
        from . import _lib
        total = torch.empty((), device=flat.device)
        if flat.numel() <= (1 << 20):
            _lib.call("clip_grad_norm", _lib.lib.snnflow_clip_grad_norm, flat.data_ptr(), flat.numel(), float(max_norm),
                      float(eps), total.data_ptr(), _lib.stream_ptr(flat.device))
        else:
            scratch = _CLIP_SCRATCH.get(flat.device)
            if scratch is None:
                scratch = torch.empty(513, dtype=torch.float64, device=flat.device)
                _CLIP_SCRATCH[flat.device] = scratch
            _lib.call("clip_grad_norm_large", _lib.lib.snnflow_clip_grad_norm_large, flat.data_ptr(), flat.numel(),
                      float(max_norm), float(eps), total.data_ptr(), scratch.data_ptr(), _lib.stream_ptr(flat.device))
        return total
    total = torch.linalg.vector_norm(flat, 2.0)  # host tensors (gloo tests): same math in torch
    coef = torch.clamp(max_norm / (total + eps), max=1.0)
    flat.mul_(coef)
    return total
