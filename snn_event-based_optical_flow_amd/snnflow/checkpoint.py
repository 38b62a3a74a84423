"""Checkpoint interchange with the reference's training loop (format row f4).

``train_flow.py:131-150`` saves ``{'model_state_dict', 'optimizer_state_dict', ...}`` with
``torch.save``; ``utils/utils.py:9-87`` (``load_model``) accepts that dict, a bare state dict,
or a pickled model object.  The module tree and parameter/buffer names of this package are
the reference's (``head.ff.weight``, ``G1.rec.weight``, ``*.lif.beta``, ``*.bn.running_var``,
snntorch's ``*.lif.graded_spikes_factor`` / ``reset_mechanism_val`` buffers ...), so a
reference checkpoint loads with ``strict=True``.  Loading never unpickles code:
``torch.load(..., weights_only=True)``; a pickled whole-model checkpoint is refused (the
reference's 'old format').  MLflow run lookup (``mlflow.get_run``) is not part of this path:
pass the ``model.pth`` path.
"""
import torch


def load_model(path, model, device="cpu", strict=True):
    """``utils/utils.py:load_model`` for a checkpoint file: returns the model with the weights
    loaded.  ``strict=False`` also applies the reference's PTQ key mapping (``*.lif.beta`` ->
    ``*.beta``, ``*.lif.threshold`` -> ``*.threshold``, :44-68) before a non-strict load."""
    ckpt = torch.load(path, map_location=device, weights_only=True)
    if not isinstance(ckpt, dict):
        raise TypeError("checkpoint is not a state dict (pickled model objects are not loaded)")
    state = ckpt.get("model_state_dict", ckpt)
    if not strict:
        extra = {}
        for k, v in state.items():
            if ".lif.beta" in k:
                extra[k.replace(".lif.beta", ".beta")] = v.clone()
            elif ".lif.threshold" in k:
                extra[k.replace(".lif.threshold", ".threshold")] = v.clone()
        state = dict(state, **extra)
    model.load_state_dict(state, strict=strict)
    return model


def save_checkpoint(path, model, optimizer=None, **extra):
    """The dict ``train_flow.py:132-140`` writes (model / optimizer state + user fields)."""
    data = {"model_state_dict": model.state_dict()}
    if optimizer is not None:
        data["optimizer_state_dict"] = optimizer.state_dict()
    data.update(extra)
    torch.save(data, path)
