"""Checkpoint / resume in the reference schema (survey §2.8, C1).

File: ``./checkpoint/resnet_ckpt.pth`` / ``transformer_ckpt.pth``; payload
``{'net': state_dict, 'acc': float percent, 'epoch': int}`` (``resnet50_test.py:664-675``).
Compatibility details kept: parameter names identical to the reference; DataParallel/
DDP checkpoints carry a ``module.`` prefix — we *write* that prefix when
``module_prefix=True`` (what a reference DDP/DP run produces) and *accept* both forms when
loading (the reference's distributed resume fails on the prefix mismatch).

Extras live under additional keys the reference loader ignores: ``optimizer``
(incl. NGD state), ``scheduler``, ``scaler``, ``rng``; plus a rolling "last" file.
Writes are rank-0 only, atomic (tmp + rename), followed by a barrier (Q16).
Loads use ``weights_only=True``.
"""
from __future__ import annotations

import os

import torch

from ..parallel.dist import barrier
from ..utils.env import is_rank0


def _compact(sd):
    """Clone tensors so saved storages are compact (our params are views into one flat
    buffer; saving the views would serialise the whole buffer per tensor group)."""
    return {k: (v.detach().clone().cpu() if isinstance(v, torch.Tensor) else v) for k, v in sd.items()}


def _sharded(model):
    """The FullyShardedDP (parallel/fsdp.py) owning ``model``'s parameters, if any."""
    return getattr(model, "_fsdp_sharded", None)


def model_state(model, module_prefix=False):
    """Full state_dict (compact CPU copies).  Under FSDP this gathers every unit: it is a
    collective and must run on every rank."""
    fs = _sharded(model)
    if fs is not None:
        sd = fs.full_state_dict()  # (compact CPU copies, unit by unit on the full-shard ring)
    else:
        sd = _compact(model.state_dict())
    if module_prefix:
        sd = {"module." + k: v for k, v in sd.items()}
    return sd


def strip_prefix(sd, prefix="module."):
    if all(k.startswith(prefix) for k in sd):
        return {k[len(prefix):]: v for k, v in sd.items()}
    return sd


def save_checkpoint(path, model, acc, epoch, module_prefix=False, extra=None):
    net = model_state(model, module_prefix) if (is_rank0() or _sharded(model) is not None) else None
    if is_rank0():
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        state = {"net": net, "acc": float(acc), "epoch": int(epoch)}
        if extra:
            state.update(extra)
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)
    barrier()


def load_checkpoint(path, map_location="cpu"):
    return torch.load(path, map_location=map_location, weights_only=True)


def load_model_state(model, sd, strict=True):
    """Load a reference-schema state_dict (with or without ``module.``) in place
    (copies into the existing, possibly flat-buffer-backed, parameters)."""
    sd = strip_prefix(sd)
    fs = _sharded(model)
    if fs is not None:
        return fs.load_full_state_dict(sd, strict=strict)
    missing, unexpected = model.load_state_dict(sd, strict=strict)
    return missing, unexpected


def load_best_performance(path, num_class, resume):
    """Reference ``load_best_performance`` (``resnet50_test.py:680-690``):
    (best_acc, start_epoch); resume re-runs the saved epoch like the reference."""
    best_acc, start_epoch = 1.0 / num_class, 0
    if resume:
        if not os.path.isfile(path):
            raise FileNotFoundError(f"no checkpoint at {path}")
        ck = load_checkpoint(path)
        best_acc = max(best_acc, float(ck["acc"]))
        start_epoch = int(ck["epoch"])
    return best_acc, start_epoch
